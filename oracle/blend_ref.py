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


def make_case(seed: int, H: int = 270, W: int = 480, S: int = 224, scale_range=(1.2, 2.5)):
    """A synthetic frame, swapped crop, soft mask and an estimate_norm-like similarity transform
    (frame -> crop: scale, rotation, translation) that puts the face inside the frame."""
    g = np.random.Generator(np.random.PCG64(seed))
    frame = g.integers(0, 256, size=(H, W, 3), dtype=np.uint8)
    swap = g.integers(0, 256, size=(S, S, 3), dtype=np.uint8)
    yy, xx = np.mgrid[0:S, 0:S].astype(np.float32)
    r = np.sqrt((yy - S / 2) ** 2 + (xx - S / 2) ** 2) / (S / 2)
    mask = np.clip(1.3 - r, 0.0, 1.0).astype(np.float32)   # 1 in the centre, 0 near the border
    scale = g.uniform(*scale_range)
    ang = g.uniform(-0.4, 0.4)
    cx, cy = g.uniform(0.35 * W, 0.65 * W), g.uniform(0.35 * H, 0.65 * H)
    c, s = scale * np.cos(ang), scale * np.sin(ang)
    # crop = A (frame - centre) + S/2
    mat = np.array([[c, -s, S / 2 - (c * cx - s * cy)], [s, c, S / 2 - (s * cx + c * cy)]], dtype=np.float32)
    return frame, swap, mask, mat


# ----------------------------------------------------------------------------------------------------
# OpenCV pieces of the paste-back (cv2 is absent here: requirements.txt pins opencv-python; restated from
# OpenCV's published imgproc algorithms, so these are unpinned too):
#   cv2.resize(img, (224, 224))                          INTER_LINEAR, uint8 (video_processing.py:212,
#                                                        image_processing.py:63)
#   cv2.invertAffineTransform / cv2.warpAffine            INTER_LINEAR, BORDER_REPLICATE for the swap,
#                                                        BORDER_CONSTANT 0 for the mask (image_processing.py:69-72)
# ----------------------------------------------------------------------------------------------------
RESIZE_COEF_BITS = 11                 # INTER_RESIZE_COEF_BITS: 11-bit fixed-point resize weights
INTER_BITS = 5                        # warp sub-pixel grid: 32 positions per pixel
AB_BITS = 10                          # warpAffine's coordinate fixed point (max(10, INTER_BITS))
REMAP_COEF_BITS = 15                  # INTER_REMAP_COEF_BITS: 15-bit bilinear weights for uint8


def _cv_round(v):
    """cvRound / saturate_cast<int> of a double: round half to even (lrint)."""
    return np.rint(v).astype(np.int64)


def resize_linear_tables(src_n: int, dst_n: int):
    """Per destination index: source index and the two 11-bit weights of cv2 INTER_LINEAR (resize.cpp:
    fx = (float)((dx + 0.5) * scale - 0.5), sx = floor(fx), clamped at both borders with the weight on
    the edge pixel; alpha = saturate_cast<short>(w * 2048))."""
    scale = 1.0 / (float(dst_n) / float(src_n))
    fx = ((np.arange(dst_n, dtype=np.float64) + 0.5) * scale - 0.5).astype(np.float32)
    sx = np.floor(fx).astype(np.int64)
    fx = (fx - sx.astype(np.float32)).astype(np.float32)
    lo = sx < 0
    fx[lo], sx[lo] = 0.0, 0
    hi = sx >= src_n - 1
    fx[hi], sx[hi] = 0.0, src_n - 1
    a0 = _cv_round((np.float32(1.0) - fx).astype(np.float32) * np.float32(1 << RESIZE_COEF_BITS))
    a1 = _cv_round(fx * np.float32(1 << RESIZE_COEF_BITS))
    sx1 = np.minimum(sx + 1, src_n - 1)
    return sx, sx1, a0, a1


def resize_linear_u8(img: np.ndarray, dsize) -> np.ndarray:
    """cv2.resize(img, dsize=(W, H)) INTER_LINEAR for uint8 [H, W, C]: horizontal pass in int (pixel x
    11-bit weight), vertical pass as OpenCV's vector VResizeLinear (the path every row of a 224-wide
    3-channel image takes): (((D0 >> 4) * b0 >> 16) + ((D1 >> 4) * b1 >> 16) + 2) >> 2, saturated."""
    Wd, Hd = dsize
    Hs, Ws = img.shape[:2]
    sx, sx1, a0, a1 = resize_linear_tables(Ws, Wd)
    sy, sy1, b0, b1 = resize_linear_tables(Hs, Hd)
    s = img.astype(np.int64)
    D = s[:, sx, :] * a0[None, :, None] + s[:, sx1, :] * a1[None, :, None]     # [Hs, Wd, C]
    D0, D1 = D[sy] >> 4, D[sy1] >> 4
    v = (((D0 * b0[:, None, None]) >> 16) + ((D1 * b1[:, None, None]) >> 16) + 2) >> 2
    return np.clip(v, 0, 255).astype(np.uint8)


def invert_affine_cv(m: np.ndarray) -> np.ndarray:
    """cv2.invertAffineTransform of a float64 [2, 3] matrix (double arithmetic)."""
    m = np.asarray(m, np.float64)
    D = m[0, 0] * m[1, 1] - m[0, 1] * m[1, 0]
    D = 1.0 / D if D != 0 else 0.0
    A11, A22, A12, A21 = m[1, 1] * D, m[0, 0] * D, -m[0, 1] * D, -m[1, 0] * D
    b1 = -A11 * m[0, 2] - A12 * m[1, 2]
    b2 = -A21 * m[0, 2] - A22 * m[1, 2]
    return np.array([[A11, A12, b1], [A21, A22, b2]], np.float64)


def warp_affine_map(m_dst_to_src_given: np.ndarray) -> np.ndarray:
    """warpAffine without WARP_INVERSE_MAP inverts its matrix first (imgwarp.cpp, double): the map from
    destination to source pixel coordinates it actually samples with."""
    return invert_affine_cv(m_dst_to_src_given)


def warp_affine_cv(src: np.ndarray, M: np.ndarray, dsize, border: str) -> np.ndarray:
    """cv2.warpAffine(src, M, dsize=(W, H), INTER_LINEAR, border) for uint8 [H, W, 3] or float32 / float64 [H, W]
    (border 'replicate' or 'constant' with 0).  Fixed point as imgwarp.cpp: X = (round(M1*y + M2)*1024 + 16 +
    round(M0*x*1024)) >> 5 (sub-pixel index X & 31, pixel X >> 5), 32 x 32 bilinear table; uint8: 15-bit
    integer weights, (sum + 2^14) >> 15; float32 / float64: the float table weights, a left-to-right sum in the
    source's type (remapBilinear's work type: float for CV_32F, double for CV_64F)."""
    W, H = dsize
    A = warp_affine_map(M)
    x = np.arange(W, dtype=np.float64)
    y = np.arange(H, dtype=np.float64)
    adelta = _cv_round(A[0, 0] * x * (1 << AB_BITS))
    bdelta = _cv_round(A[1, 0] * x * (1 << AB_BITS))
    rd = (1 << AB_BITS) >> INTER_BITS >> 1
    X0 = _cv_round((A[0, 1] * y + A[0, 2]) * (1 << AB_BITS)) + rd
    Y0 = _cv_round((A[1, 1] * y + A[1, 2]) * (1 << AB_BITS)) + rd
    X = (X0[:, None] + adelta[None, :]) >> (AB_BITS - INTER_BITS)
    Y = (Y0[:, None] + bdelta[None, :]) >> (AB_BITS - INTER_BITS)
    sx, sy = X >> INTER_BITS, Y >> INTER_BITS
    fx = (X & ((1 << INTER_BITS) - 1)).astype(np.float32) / np.float32(1 << INTER_BITS)
    fy = (Y & ((1 << INTER_BITS) - 1)).astype(np.float32) / np.float32(1 << INTER_BITS)
    wx = [np.float32(1.0) - fx, fx]
    wy = [np.float32(1.0) - fy, fy]
    Hs, Ws = src.shape[:2]
    is_u8 = src.dtype == np.uint8
    C = src.shape[2] if src.ndim == 3 else 1
    s = src.reshape(Hs, Ws, C)
    ft = np.float64 if src.dtype == np.float64 else np.float32
    acc = np.zeros((H, W, C), np.int64 if is_u8 else ft)
    inside_any = np.zeros((H, W), bool)
    for ky in range(2):
        for kx in range(2):
            w = (wy[ky] * wx[kx]).astype(np.float32)
            tx, ty = sx + kx, sy + ky
            ok = (tx >= 0) & (tx < Ws) & (ty >= 0) & (ty < Hs)
            inside_any |= ok
            if border == "replicate":
                v = s[np.clip(ty, 0, Hs - 1), np.clip(tx, 0, Ws - 1)]
            else:
                v = np.where(ok[..., None], s[np.clip(ty, 0, Hs - 1), np.clip(tx, 0, Ws - 1)], 0)
            if is_u8:
                wi = _cv_round(w * np.float32(1 << REMAP_COEF_BITS))
                acc = acc + v.astype(np.int64) * wi[..., None]
            else:
                acc = (acc + v.astype(ft) * w[..., None].astype(ft)).astype(ft)
    if is_u8:
        out = np.clip((acc + (1 << (REMAP_COEF_BITS - 1))) >> REMAP_COEF_BITS, 0, 255).astype(np.uint8)
    else:
        out = acc
    if border == "constant":
        out = np.where(inside_any[..., None], out, 0).astype(out.dtype)
    return out.reshape((H, W, C) if src.ndim == 3 else (H, W))


def get_final_image(final_frames, full_frame: np.ndarray, tfm_arrays, masks) -> np.ndarray:
    """image_processing.py:51-76 (get_final_image) with the masks given (face_mask_static needs the
    landmark model, absent here): per identity i, frame = cv2.resize(swap_i, 224); swap_t = warpAffine
    (frame, invertAffineTransform(tfm_i), BORDER_REPLICATE); mask_t = warpAffine(mask_i, ..., constant 0);
    final = mask_t*swap_t + (1-mask_t)*final, identities in order; one uint8 cast at the end.  The mask is
    face_mask_static's ``mask/255`` (masks.py:83-85) of a uint8 array — numpy float64 — so the mask warp and the
    composite are float64, as numpy promotes them (``masks`` given as uint8 are divided here; float arrays are
    taken as they are)."""
    H, W = full_frame.shape[:2]
    final = full_frame.copy()
    for sw, tfm, mask in zip(final_frames, tfm_arrays, masks):
        mask = np.asarray(mask)
        if mask.dtype == np.uint8:
            mask = mask / 255
        frame = resize_linear_u8(sw, (224, 224))
        mat_rev = invert_affine_cv(tfm)
        swap_t = warp_affine_cv(frame, mat_rev, (W, H), "replicate")
        mask_t = warp_affine_cv(mask, mat_rev, (W, H), "constant")[..., None]
        final = mask_t * swap_t + (1 - mask_t) * final
    return np.array(final, dtype="uint8")


def paste_back_video(full_frame_u8: np.ndarray, swap256_u8: np.ndarray, mask224: np.ndarray, mat: np.ndarray):
    """video_processing.py:212-227 for one (frame, identity): cv2.resize(swap, (224, 224)) first, then the
    kornia warp + composite of paste_back."""
    return paste_back(full_frame_u8, resize_linear_u8(swap256_u8, (224, 224)), mask224, mat)
