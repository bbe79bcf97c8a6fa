"""Drop-in for utils/inference/masks.py on MI355X: the paste-back masks built on the device.

``face_mask_static(image, landmarks, landmarks_tgt, params=None)`` keeps the reference signature and return
convention (masks.py:38-86: ``(mask, [erode, sigmaX, sigmaY])`` when params is None, else ``mask``), with the
mask a float32 device tensor [H, W] instead of a float64 numpy array (it feeds the device blend directly;
``.cpu().numpy()`` gives the reference's values as float32).  ``face_masks`` does a whole batch of frames
in three launches (``ghost_face_masks``): the video path builds every frame's mask of an identity at once.

Split as in the reference: the parameter choice (masks.py:43-65) and, in the native library's host code,
the eyebrow expansion on int32 landmarks and the convex hull (``ghost_mask_polygons``, C++ on the CPU);
the raster (cv2.fillConvexPoly), the box erode / dilate, the border fade and the Gaussian blur run on the GPU
(ghost_amd/csrc/masks.hip).  The OpenCV calls are restated from OpenCV 4.x's published algorithms; cv2 is
absent here, so the masks are checked against the CPU restatement oracle/mask_ref.py (parity unpinned).
"""
from __future__ import annotations

import ctypes as C
from typing import Optional, Sequence

import numpy as np
import torch

from .. import _lib

MAX_V = 128   # hull vertices per frame (masks.hip kMaxV)


def mask_params(landmarks, landmarks_tgt):
    """face_mask_static's (erode, sigmaX, sigmaY) when params is None (masks.py:43-65)."""
    lm, lt = np.asarray(landmarks), np.asarray(landmarks_tgt)
    left = np.sum((lm[1][0] - lt[1][0], lm[2][0] - lt[2][0], lm[13][0] - lt[13][0]))
    right = np.sum((lt[17][0] - lm[17][0], lt[18][0] - lm[18][0], lt[29][0] - lm[29][0]))
    offset = max(left, right)
    if offset > 6:
        return [15, 15, 10]
    if offset > 3:
        return [10, 10, 8]
    if offset < -3:
        return [-5, 5, 10]
    return [5, 5, 5]


def mask_polygons(landmarks: np.ndarray, params: np.ndarray):
    """Host half (ghost_mask_polygons): eyebrow expansion + convex hull -> (poly int32 [F,128,2], nv int32 [F])."""
    lib = _lib.load()
    lm = np.ascontiguousarray(np.asarray(landmarks, dtype=np.float32).reshape(-1, 106, 2))
    F = lm.shape[0]
    pr = np.ascontiguousarray(np.asarray(params, dtype=np.int32).reshape(F, 3))
    poly = np.zeros((F, MAX_V, 2), dtype=np.int32)
    nv = np.zeros(F, dtype=np.int32)
    _lib.check(lib.ghost_mask_polygons(lm.ctypes.data, F, 106, pr.ctypes.data, poly.ctypes.data, nv.ctypes.data),
               "ghost_mask_polygons")
    return poly, nv


def face_masks(landmarks, params, H: int = 224, W: int = 224, device=None,
               out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Masks of F frames: landmarks [F,106,2] (the swap's, as the landmark model returns them), params [F,3]
    (erode, sigmaX, sigmaY) -> float32 [F,H,W] on ``device`` (face_mask_static's mask / 255 per frame)."""
    dev = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
    if dev.type != "cuda":
        raise RuntimeError("ghost_amd: face_masks runs on the GPU only (no CPU path)")
    pr = np.asarray(params, dtype=np.int32).reshape(-1, 3)
    poly, nv = mask_polygons(landmarks, pr)
    F = poly.shape[0]
    if F == 0:
        return torch.empty(0, H, W, dtype=torch.float32, device=dev)
    if out is None:
        out = torch.empty(F, H, W, dtype=torch.float32, device=dev)
    elif out.shape != (F, H, W) or out.dtype != torch.float32 or not out.is_contiguous() or out.device != dev:
        raise RuntimeError(f"ghost_amd: out must be a contiguous float32 [{F},{H},{W}] tensor on {dev}")
    lib = _lib.load()
    with torch.cuda.device(dev):
        d_poly = torch.from_numpy(poly).to(dev, non_blocking=True)
        d_nv = torch.from_numpy(nv).to(dev, non_blocking=True)
        d_pr = torch.from_numpy(pr).to(dev, non_blocking=True)
        ws = torch.empty(int(lib.ghost_face_masks_workspace_bytes(F, H, W)), dtype=torch.uint8, device=dev)
        _lib.check(lib.ghost_face_masks(d_poly.data_ptr(), d_nv.data_ptr(), d_pr.data_ptr(), F, H, W, out.data_ptr(),
                                        H * W, ws.data_ptr(), ws.numel(), _lib.stream_ptr(dev)), "ghost_face_masks")
    return out


def face_mask_static(image, landmarks, landmarks_tgt=None, params: Optional[Sequence[int]] = None, device=None):
    """masks.py:38-86 for one frame: ``image`` gives the mask size ([H,W,...] array or tensor)."""
    H, W = int(image.shape[0]), int(image.shape[1])
    p = mask_params(landmarks, landmarks_tgt) if params is None else list(params)
    if device is None and isinstance(image, torch.Tensor) and image.is_cuda:
        device = image.device
    m = face_masks(np.asarray(landmarks)[None], np.asarray(p)[None], H, W, device)[0]
    return (m, p) if params is None else m
