"""ORACLE — CPU restatement of GHOST's paste-back blend (test infrastructure only).

Imported only by ``tests/``; the product (``ghost_amd.inference.blend``) never imports it.

What it restates: the per-(frame, identity) composite of get_final_video
(utils/inference/video_processing.py:210-227):

    mat_rev = kornia.invert_affine_transform(mat)
    swap_t  = kornia.warp_affine(swap, mat_rev, size)        # bilinear, zeros, align_corners=True
    mask_t  = kornia.warp_affine(mask, mat_rev, size)
    final   = (mask_t*swap_t + (1-mask_t)*full_frame).type(torch.uint8)

kornia is a third-party dependency absent from this container: requirements.txt:13 pins
``kornia==0.5.4``.  Its published 0.5.4 algorithm is restated here with torch ops:
``invert_affine_transform`` = inverse of the 3x3 homography, top two rows;
``warp_affine(src, M, dsize)`` = normalize_homography(M) (pixel -> [-1, 1] with
2/(W-1), 2/(H-1) scales, align_corners=True) -> inverse -> F.affine_grid -> F.grid_sample
(bilinear, padding 'zeros', align_corners=True).  Parity anchor: the reference call sites above;
no fixture of the reference covers them (cv2 / kornia / the landmark model are absent), so the
blend is pinned only to this restatement of kornia's published algorithm.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F


def _homography(m2x3: torch.Tensor) -> torch.Tensor:
    out = torch.zeros(m2x3.shape[0], 3, 3, dtype=m2x3.dtype)
    out[:, :2, :] = m2x3
    out[:, 2, 2] = 1.0
    return out


def invert_affine_transform(m: torch.Tensor) -> torch.Tensor:
    """kornia.invert_affine_transform: [B,2,3] -> [B,2,3]."""
    return torch.inverse(_homography(m))[:, :2, :3]


def _normal_transform_pixel(h: int, w: int, eps: float = 1e-14) -> torch.Tensor:
    tr = torch.tensor([[1.0, 0.0, -1.0], [0.0, 1.0, -1.0], [0.0, 0.0, 1.0]])
    tr[0, 0] = tr[0, 0] * 2.0 / (eps if w == 1 else w - 1.0)
    tr[1, 1] = tr[1, 1] * 2.0 / (eps if h == 1 else h - 1.0)
    return tr.unsqueeze(0)


def warp_affine(src: torch.Tensor, m: torch.Tensor, dsize) -> torch.Tensor:
    """kornia.warp_affine(src [B,C,H,W], M [B,2,3], dsize=(h, w)), bilinear / zeros / align_corners=True."""
    B, C, H, W = src.shape
    dst_pix_trans_src_pix = _homography(m)
    src_norm_trans_src_pix = _normal_transform_pixel(H, W)
    src_pix_trans_src_norm = torch.inverse(src_norm_trans_src_pix)
    dst_norm_trans_dst_pix = _normal_transform_pixel(dsize[0], dsize[1])
    dst_norm_trans_src_norm = dst_norm_trans_dst_pix @ (dst_pix_trans_src_pix @ src_pix_trans_src_norm)
    src_norm_trans_dst_norm = torch.inverse(dst_norm_trans_src_norm)
    grid = F.affine_grid(src_norm_trans_dst_norm[:, :2, :], [B, C, dsize[0], dsize[1]], align_corners=True)
    return F.grid_sample(src, grid, align_corners=True, mode="bilinear", padding_mode="zeros")


def paste_back(full_frame_u8: np.ndarray, swap_u8: np.ndarray, mask: np.ndarray, mat: np.ndarray) -> np.ndarray:
    """One (frame, identity) composite of video_processing.py:218-227 on CPU: returns the new u8 frame."""
    size = (full_frame_u8.shape[0], full_frame_u8.shape[1])
    swap = torch.from_numpy(swap_u8).permute(2, 0, 1).unsqueeze(0).type(torch.float32)
    msk = torch.from_numpy(mask).unsqueeze(0).unsqueeze(0).type(torch.float32)
    full = torch.from_numpy(full_frame_u8).permute(2, 0, 1).unsqueeze(0)
    m = torch.from_numpy(mat).unsqueeze(0).type(torch.float32)
    m_rev = invert_affine_transform(m)
    swap_t = warp_affine(swap, m_rev, size)
    mask_t = warp_affine(msk, m_rev, size)
    final = (mask_t * swap_t + (1 - mask_t) * full).type(torch.uint8).squeeze().permute(1, 2, 0)
    return final.numpy()


def make_case(seed: int, H: int = 270, W: int = 480, S: int = 224):
    """A synthetic frame, swapped crop, soft mask and an estimate_norm-like similarity transform
    (frame -> crop: scale, rotation, translation) that puts the face inside the frame."""
    g = np.random.Generator(np.random.PCG64(seed))
    frame = g.integers(0, 256, size=(H, W, 3), dtype=np.uint8)
    swap = g.integers(0, 256, size=(S, S, 3), dtype=np.uint8)
    yy, xx = np.mgrid[0:S, 0:S].astype(np.float32)
    r = np.sqrt((yy - S / 2) ** 2 + (xx - S / 2) ** 2) / (S / 2)
    mask = np.clip(1.3 - r, 0.0, 1.0).astype(np.float32)   # 1 in the centre, 0 near the border
    scale = g.uniform(1.2, 2.5)
    ang = g.uniform(-0.4, 0.4)
    cx, cy = g.uniform(0.35 * W, 0.65 * W), g.uniform(0.35 * H, 0.65 * H)
    c, s = scale * np.cos(ang), scale * np.sin(ang)
    # crop = A (frame - centre) + S/2
    mat = np.array([[c, -s, S / 2 - (c * cx - s * cy)], [s, c, S / 2 - (s * cx + c * cy)]], dtype=np.float32)
    return frame, swap, mask, mat
