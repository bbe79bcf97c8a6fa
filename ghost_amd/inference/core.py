"""Per-identity swap loop of model_inference (utils/inference/core.py:13-26, :57-88).

Only the per-frame part is here: crops in, swapped crops out with the reference's
``present`` bookkeeping (frames without a face yield ``[]``).  Detection, alignment,
landmarks and blending stay on the host pipeline of the reference (out of scope).
"""
from __future__ import annotations

from typing import List, Sequence

import numpy as np
import torch

from .. import _lib


def transform_target_to_torch(resized_frs: np.ndarray, half: bool = True, device=None) -> torch.Tensor:
    """core.py:13-26: uint8 BGR NHWC crops -> RGB, /255, (x-0.5)/0.5, returned as an NCHW view.

    Runs on the GPU kernel ``ghost_crops_to_input_nhwc``; ``half=True`` yields float16 as in the
    reference (core.py:20-21: fp32 /255, then fp16); ``half=False`` float32.
    """
    device = torch.device(device or "cuda")
    crops = torch.from_numpy(np.ascontiguousarray(resized_frs)).to(device)
    _lib.require_gpu(crops, "transform_target_to_torch")
    B, H, W, _ = crops.shape
    dt = torch.float16 if half else torch.float32
    y = torch.empty(B, H, W, 3, dtype=dt, device=device)
    lib = _lib.load()
    _lib.check(lib.ghost_crops_to_input_nhwc(crops.data_ptr(), crops.stride(0), B, H, W, _lib.gdtype(dt),
                                             y.data_ptr(), _lib.stream_ptr(device)), "transform_target_to_torch")
    return y.permute(0, 3, 1, 2)


def swap_identity_frames(resized_frs: np.ndarray, present: Sequence[int], source_embed: torch.Tensor, G,
                         BS: int = 60, device=None) -> List:
    """core.py:57-88 for one identity: batched swap of the present crops, then re-insert ``[]``
    for frames without a face so the result is indexed by frame (bit-exact crop indices)."""
    device = torch.device(device or "cuda")
    crops = torch.from_numpy(np.ascontiguousarray(resized_frs)).to(device) if len(resized_frs) else None
    outputs = []
    if crops is not None:
        for i in range(0, crops.shape[0], BS):
            outputs.append(G.swap_u8(crops[i:i + BS], source_embed).cpu().numpy())
    model_output = np.concatenate(outputs) if outputs else np.zeros((0, 256, 256, 3), np.uint8)
    return reinsert_present(model_output, present)


def reinsert_present(model_output: np.ndarray, present: Sequence[int]) -> List:
    """core.py:79-88: frames with a face take the next swapped crop, the others get ``[]``."""
    final_frames, idx_fs = [], 0
    for pres in present:
        if pres == 1:
            final_frames.append(model_output[idx_fs])
            idx_fs += 1
        else:
            final_frames.append([])
    return final_frames
