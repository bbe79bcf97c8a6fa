"""Per-identity swap loop of model_inference (utils/inference/core.py:13-26, :57-88).

Only the per-frame part is here: crops in, swapped crops out with the reference's
``present`` bookkeeping (frames without a face yield ``[]``).  Detection, alignment and
landmarks stay on the host pipeline of the reference (out of scope).

* ``resize_frames`` — video_processing.py:174-188 on the device: the 224x224 aligned crops of one identity
  (``[]`` where no face was found) -> ``present`` and the 256x256 crops, resized by the cv2 INTER_LINEAR
  fixed-point kernel (``ghost_resize_u8_linear``) instead of one cv2.resize per frame on the host;
* ``swap_identity_frames`` — core.py:57-88 for one identity on already-resized crops (host or device);
* ``swap_crop_frames`` — both: crop_frames of one identity in, the per-frame list out.
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
    cstride = crops.stride(0) if B > 1 else H * W * 3
    _lib.check(lib.ghost_crops_to_input_nhwc(crops.data_ptr(), cstride, B, H, W, _lib.gdtype(dt),
                                             y.data_ptr(), _lib.stream_ptr(device)), "transform_target_to_torch")
    return y.permute(0, 3, 1, 2)


def resize_frames(crop_frames: Sequence, new_size=(256, 256), device=None):
    """video_processing.py:174-188 with the resize on the device.  ``crop_frames``: one entry per video frame,
    a uint8 [h, w, 3] crop (crop_frames_and_get_transforms' 224x224 warpAffine output) or ``[]`` where the
    identity had no face (cv2.resize raises on it and the reference marks the frame absent).  Returns
    (resized device uint8 [n, 256, 256, 3] of the present frames in frame order, present: float64 [F] of 1/0,
    as ``np.ones`` then ``present[i] = 0`` make it).  All crops of one call must share one size (the reference's
    crops are all crop_size x crop_size)."""
    device = torch.device(device or "cuda")
    present = np.ones(len(crop_frames))
    keep = []
    for i, fr in enumerate(crop_frames):
        a = np.asarray(fr) if not isinstance(fr, list) else None
        if a is None or a.ndim != 3 or a.size == 0:
            present[i] = 0
        else:
            keep.append(a)
    Wd, Hd = new_size
    if not keep:
        return torch.empty(0, Hd, Wd, 3, dtype=torch.uint8, device=device), present
    shapes = {k.shape for k in keep}
    if len(shapes) != 1 or keep[0].dtype != np.uint8 or keep[0].shape[2] != 3:
        raise RuntimeError(f"ghost_amd: resize_frames needs uint8 crops of one [h,w,3] shape, got {sorted(shapes)}")
    host = torch.from_numpy(np.stack(keep))
    src = host.pin_memory().to(device, non_blocking=True)
    if tuple(src.shape[1:3]) == (Hd, Wd):
        return src, present
    from .blend import resize_u8
    return resize_u8(src, (Wd, Hd)), present


def swap_crop_frames(crop_frames: Sequence, source_embed: torch.Tensor, G, BS: int = 60, device=None,
                     return_device: bool = False):
    """core.py:57-88 for one identity from its crop_frames: ``resize_frames`` on the device (224 -> 256, the
    ``present`` vector), then ``swap_identity_frames`` on the device-resident crops.  Returns the per-frame list
    (swapped uint8 crop, or ``[]``), plus the device swaps with ``return_device``."""
    crops, present = resize_frames(crop_frames, device=device)
    return swap_identity_frames(crops, present, source_embed, G, BS=BS, device=device, return_device=return_device)


def swap_identity_frames(resized_frs, present: Sequence[int], source_embed: torch.Tensor, G,
                         BS: int = 60, device=None, return_device: bool = False):
    """core.py:57-88 for one identity: batched swap of the present crops, then re-insert ``[]``
    for frames without a face so the result is indexed by frame (bit-exact crop indices).

    ``resized_frs``: host uint8 [n,256,256,3] (numpy) or a device tensor of them (``resize_frames``' output).
    The crops go to the device once (core.py:63 transfers the identity's frames at once); each
    batch of BS is swapped into a device buffer and copied to pinned host memory on a copy stream
    while the next batch is swapped (the reference's per-batch ``.cpu()``, faceshifter_run.py:22,
    without serialising the GPU on it).  ``return_device=True`` also returns the device-resident
    uint8 swaps [N,256,256,3] (for a device paste-back, ``blend.blend_swaps``)."""
    device = torch.device(device or "cuda")
    n = len(resized_frs)
    if n == 0:
        final = reinsert_present(np.zeros((0, 256, 256, 3), np.uint8), present)
        return (final, None) if return_device else final
    if torch.is_tensor(resized_frs):
        crops = resized_frs.to(device)
    else:
        crops = torch.from_numpy(np.ascontiguousarray(resized_frs)).pin_memory().to(device, non_blocking=True)
    z = source_embed.to(device)
    out = torch.empty(n, 256, 256, 3, dtype=torch.uint8, device=device)
    host = torch.empty(n, 256, 256, 3, dtype=torch.uint8, pin_memory=True)
    cur = torch.cuda.current_stream(device)
    from .streams import stream_set
    copy = stream_set(device).d2h
    # the identity's projections once for all its batches (AEI_Net.identity_table; core.py recomputes them in every
    # faceshifter_batch call), gathered per sample with an all-zero index
    z_rows = z.reshape(z.shape[0], -1)
    table = G.identity_table(z_rows) if hasattr(G, "identity_table") and z_rows.shape[0] == 1 else None
    zero = torch.zeros(min(BS, n), dtype=torch.int32, device=device) if table is not None else None
    for i in range(0, n, BS):
        j = min(n, i + BS)
        if table is not None:
            G.swap_u8_indexed(crops[i:j], table, zero[:j - i], out=out[i:j])
        else:
            G.swap_u8(crops[i:j], z, out=out[i:j])
        done = torch.cuda.Event()
        done.record(cur)
        with torch.cuda.stream(copy):
            copy.wait_event(done)
            host[i:j].copy_(out[i:j], non_blocking=True)
    copy.synchronize()
    out.record_stream(copy)
    final = reinsert_present(host.numpy(), present)
    return (final, out) if return_device else final


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
