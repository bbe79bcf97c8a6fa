"""Paste-back of swapped faces into full frames on the device.

``blend_swaps`` is the tensor part of get_final_video (utils/inference/video_processing.py:191-243)
for one identity over many frames at once: kornia.invert_affine_transform + warp_affine of the
swapped crop and its mask, then ``(mask_t*swap_t + (1-mask_t)*frame).type(uint8)``, computed by
one native launch (``ghost_blend_swaps_u8``) in place on device-resident uint8 frames.  Producing
the mask (landmark model + cv2 erode/blur, masks.py) and resizing the 256x256 swap to the crop size
(cv2.resize) stay on the host as in the reference; their outputs are the inputs here.
"""
from __future__ import annotations

from typing import Optional

import numpy as np
import torch

from .. import _lib


def blend_swaps(frames: torch.Tensor, swaps: torch.Tensor, masks: torch.Tensor, tfms,
                valid: Optional[torch.Tensor] = None) -> torch.Tensor:
    """frames u8 [F,H,W,3] (modified in place and returned), swaps u8 [F,S,S,3], masks f32 [F,S,S],
    tfms [F,2,3] crop <- frame transforms (numpy or tensor), valid bool/int [F] (frames to skip = 0)."""
    _lib.require_gpu(frames, "blend_swaps")
    dev = frames.device
    if frames.dtype != torch.uint8 or frames.ndim != 4 or frames.shape[3] != 3 or not frames.is_contiguous():
        raise RuntimeError("ghost_amd: frames must be a contiguous uint8 [F,H,W,3] device tensor")
    F_, H, W = frames.shape[:3]
    swaps = swaps.to(dev).contiguous()
    masks = masks.to(dev, torch.float32).contiguous()
    if swaps.dtype != torch.uint8 or swaps.shape[0] != F_ or swaps.shape[3] != 3:
        raise RuntimeError("ghost_amd: swaps must be uint8 [F,S,S,3]")
    S_h, S_w = swaps.shape[1:3]
    if tuple(masks.shape) != (F_, S_h, S_w):
        raise RuntimeError("ghost_amd: masks must be [F,S,S] matching the swaps")
    m = torch.as_tensor(np.asarray(tfms, dtype=np.float32) if not torch.is_tensor(tfms) else tfms)
    m = m.to(dev, torch.float32).reshape(F_, 6).contiguous()
    v = None if valid is None else valid.to(dev, torch.int32).contiguous()
    lib = _lib.load()
    _lib.check(lib.ghost_blend_swaps_u8(frames.data_ptr(), frames.stride(0), F_, H, W, swaps.data_ptr(),
                                        swaps.stride(0), S_h, S_w, masks.data_ptr(), masks.stride(0), m.data_ptr(),
                                        None if v is None else v.data_ptr(), _lib.stream_ptr(dev)), "blend_swaps")
    return frames
