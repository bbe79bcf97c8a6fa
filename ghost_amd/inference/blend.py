"""Paste-back of swapped faces into full frames on the device.

* ``blend_swaps`` — the tensor part of get_final_video (utils/inference/video_processing.py:191-243) for
  one identity over many frames at once: the swap's cv2.resize to the crop size (:212; ``resize_to``),
  kornia.invert_affine_transform + warp_affine of the swap and its mask, then
  ``(mask_t*swap_t + (1-mask_t)*frame).type(uint8)``, in place on device-resident uint8 frames.
* ``blend_image`` — get_final_image (utils/inference/image_processing.py:51-76), the image-to-image path:
  cv2.resize to 224, cv2.warpAffine with BORDER_REPLICATE for the swap and a constant 0 border for the
  mask, identities accumulated in float64 (the mask is ``mask/255`` of a uint8 array: numpy float64) and cast
  to uint8 once.
Producing the masks (landmark model + cv2 erode/blur, masks.py) stays on the host as in the reference;
the masks are inputs here.  cv2 / kornia are absent in this container: the kernels follow restatements
of their published algorithms (oracle/blend_ref.py), parity unpinned.
"""
from __future__ import annotations

from typing import Optional, Sequence

import numpy as np
import torch

from .. import _lib


def _fstride(t: torch.Tensor) -> int:
    """Elements between consecutive items of dim 0; for a single item any stride is valid (numpy's a[None] and
    torch's size-1 dims may report 0), so report the dense size the native checks expect."""
    return t.stride(0) if t.shape[0] > 1 else int(np.prod(t.shape[1:]))


def resize_u8(src: torch.Tensor, size=(224, 224)) -> torch.Tensor:
    """cv2.resize(src, size) INTER_LINEAR for uint8 [F,H,W,3] device images -> [F,size[1],size[0],3]."""
    _lib.require_gpu(src, "resize_u8")
    if src.dtype != torch.uint8 or src.ndim != 4 or src.shape[3] != 3:
        raise RuntimeError("ghost_amd: resize_u8 takes uint8 [F,H,W,3]")
    src = src.contiguous()
    F_, Hs, Ws = src.shape[:3]
    Wd, Hd = size
    dst = torch.empty(F_, Hd, Wd, 3, dtype=torch.uint8, device=src.device)
    if F_:
        _lib.check(_lib.load().ghost_resize_u8_linear(src.data_ptr(), _fstride(src), F_, Hs, Ws, dst.data_ptr(),
                                                      dst.stride(0), Hd, Wd, _lib.stream_ptr(src.device)), "resize_u8")
    return dst


def blend_swaps(frames: torch.Tensor, swaps: torch.Tensor, masks: torch.Tensor, tfms,
                valid: Optional[torch.Tensor] = None, resize_to: Optional[int] = None) -> torch.Tensor:
    """frames u8 [F,H,W,3] (modified in place and returned), swaps u8 [F,S,S,3], masks f32 [F,M,M],
    tfms [F,2,3] crop <- frame transforms (numpy or tensor), valid bool/int [F] (frames to skip = 0).
    resize_to=M: the swaps are first resized to M x M as the reference does (cv2.resize(final_frames[j][i],
    (224, 224)), video_processing.py:212); without it the swaps are already crop-sized (S == M)."""
    _lib.require_gpu(frames, "blend_swaps")
    dev = frames.device
    if frames.dtype != torch.uint8 or frames.ndim != 4 or frames.shape[3] != 3 or not frames.is_contiguous():
        raise RuntimeError("ghost_amd: frames must be a contiguous uint8 [F,H,W,3] device tensor")
    F_, H, W = frames.shape[:3]
    swaps = swaps.to(dev).contiguous()
    if resize_to is not None and tuple(swaps.shape[1:3]) != (resize_to, resize_to):
        swaps = resize_u8(swaps, (resize_to, resize_to))
    masks = masks.to(dev, torch.float32).contiguous()
    if swaps.dtype != torch.uint8 or swaps.shape[0] != F_ or swaps.shape[3] != 3:
        raise RuntimeError("ghost_amd: swaps must be uint8 [F,S,S,3]")
    S_h, S_w = swaps.shape[1:3]
    if tuple(masks.shape) != (F_, S_h, S_w):
        raise RuntimeError("ghost_amd: masks must be [F,S,S] matching the (resized) swaps")
    m = torch.as_tensor(np.asarray(tfms, dtype=np.float32) if not torch.is_tensor(tfms) else tfms)
    m = m.to(dev, torch.float32).reshape(F_, 6).contiguous()
    v = None if valid is None else valid.to(dev, torch.int32).contiguous()
    lib = _lib.load()
    _lib.check(lib.ghost_blend_swaps_u8(frames.data_ptr(), _fstride(frames), F_, H, W, swaps.data_ptr(),
                                        _fstride(swaps), S_h, S_w, masks.data_ptr(), _fstride(masks), m.data_ptr(),
                                        None if v is None else v.data_ptr(), _lib.stream_ptr(dev)), "blend_swaps")
    return frames


def _invert_affine_cv(m: np.ndarray) -> np.ndarray:
    """cv2.invertAffineTransform of a float64 [2,3] matrix (double arithmetic, imgwarp.cpp)."""
    m = np.asarray(m, np.float64).reshape(2, 3)
    D = m[0, 0] * m[1, 1] - m[0, 1] * m[1, 0]
    D = 1.0 / D if D != 0 else 0.0
    A11, A22, A12, A21 = m[1, 1] * D, m[0, 0] * D, -m[0, 1] * D, -m[1, 0] * D
    return np.array([[A11, A12, -A11 * m[0, 2] - A12 * m[1, 2]], [A21, A22, -A21 * m[0, 2] - A22 * m[1, 2]]])


def cv_warp_map(tfm: np.ndarray) -> np.ndarray:
    """The destination -> source map cv2.warpAffine(src, invertAffineTransform(tfm), ...) samples with:
    warpAffine inverts the matrix it is given (no WARP_INVERSE_MAP), so twice-inverted tfm, in double."""
    return _invert_affine_cv(_invert_affine_cv(tfm))


def blend_image(full_frame: torch.Tensor, swaps: torch.Tensor, masks: torch.Tensor,
                tfms: Sequence[np.ndarray]) -> torch.Tensor:
    """get_final_image on the device: full_frame u8 [H,W,3] (modified in place and returned), swaps u8
    [J,256,256,3] (or already 224), masks [J,224,224] — face_mask_static's float64 ``mask/255`` as the reference
    returns it, or the float32 masks of ``masks.face_masks`` (q/255 of a uint8 q, rebuilt exactly as q/255.0 in
    float64) — tfms J crop <- frame [2,3] matrices (estimate_norm's, float64)."""
    _lib.require_gpu(full_frame, "blend_image")
    dev = full_frame.device
    if full_frame.dtype != torch.uint8 or full_frame.ndim != 3 or full_frame.shape[2] != 3 or \
            not full_frame.is_contiguous():
        raise RuntimeError("ghost_amd: full_frame must be a contiguous uint8 [H,W,3] device tensor")
    J = swaps.shape[0]
    swaps = swaps.to(dev).contiguous()
    if tuple(swaps.shape[1:3]) != (224, 224):
        swaps = resize_u8(swaps, (224, 224))          # image_processing.py:63
    masks = torch.as_tensor(masks).to(dev)
    if masks.dtype != torch.float64:
        # a float32 / float16 q/255 mask (masks.face_masks) -> the float64 q/255.0 numpy computes: a 256-entry table
        # of numpy's correctly rounded q / 255 (torch's device division by a scalar multiplies by the reciprocal,
        # which is not), indexed by the recovered q.  Only when every value is such a q/255: any other
        # soft mask is promoted to float64 unchanged
        m32 = masks.to(torch.float32)
        q = torch.round(m32 * 255.0)
        if bool(((m32 * 255.0 - q).abs() <= 1e-3).all()) and bool(((q >= 0) & (q <= 255)).all()):
            lut = torch.from_numpy(np.arange(256, dtype=np.float64) / 255).to(dev)
            masks = lut[q.to(torch.int64)]
        else:
            masks = masks.to(torch.float64)
    masks = masks.contiguous()
    if tuple(masks.shape) != (J, 224, 224) or len(tfms) != J:
        raise RuntimeError("ghost_amd: blend_image needs J masks [224,224] and J transforms")
    maps = torch.from_numpy(np.stack([cv_warp_map(t) for t in tfms]).reshape(J, 6) if J else
                            np.zeros((0, 6))).to(dev, torch.float64).contiguous()
    H, W = full_frame.shape[:2]
    _lib.check(_lib.load().ghost_blend_image_u8(full_frame.data_ptr(), H, W, swaps.data_ptr(),
                                                _fstride(swaps) if J else 0, J, 224, masks.data_ptr(),
                                                _fstride(masks) if J else 0, maps.data_ptr(),
                                                _lib.stream_ptr(dev)), "blend_image")
    return full_frame
