"""ORACLE — CPU restatement of GHOST's face-mask construction (test infrastructure only).

Imported only by ``tests/``; the product (``ghost_amd.inference.masks``) never imports it.

What it restates: utils/inference/masks.py — ``face_mask_static`` (masks.py:38-86: the erode / blur
parameters from the source-target landmark offset, ``expand_eyebrows`` (masks.py:5-20), ``get_mask``
(masks.py:23-35: convex hull of the 106 landmarks filled with 255) and ``erode_and_blur`` (masks.py:89-107:
box erode or dilate, the border fade, Gaussian blur), returned as mask / 255 in float.

cv2 is a third-party dependency absent from this container (requirements.txt pins opencv-python); the
calls are restated from OpenCV 4.x's published algorithms:
* ``cv2.convexHull``: the set of hull vertices (no collinear points); the fill below does not depend on the
  vertex order or start;
* ``cv2.fillConvexPoly(mask, hull, 255)`` (drawing.cpp FillConvexPoly, shift 0, LINE_8): every polygon edge
  drawn with the 8-connected Bresenham of LineIterator (left to right, the segment clipped to the image by
  clipLine), then the scanline spans of the two vertex chains from the topmost vertex in 16.16 fixed point
  (x advanced by dx = ((xe - xs)*2 + (ty - y)) / (2*(ty - y)) per row, span ends rounded by + 0.5);
* ``cv2.erode`` / ``cv2.dilate`` with ``np.ones((k, k))``: the window [x - k//2, x - k//2 + k - 1] per axis,
  pixels outside the image ignored (morphologyDefaultBorderValue);
* ``cv2.GaussianBlur(mask, (0, 0), sigmaX, sigmaY)``: kernel size cvRound(sigma*6 + 1) | 1 per axis (8-bit
  input), getGaussianKernel's normalised exp(-x^2 / (2 sigma^2)) taps, BORDER_REFLECT_101, rows then columns in
  fp32, one rounding to uint8 (cvRound: half to even).  OpenCV's 8-bit path evaluates this filter in fixed point
  (8-bit fractional coefficients), which can differ from the fp32 evaluation by about one LSB.
No fixture of the reference covers masks (the landmark model and cv2 are absent), so the device masks are
pinned only to this restatement: **parity unpinned**.
"""
from __future__ import annotations

import math

import numpy as np

XY_SHIFT = 16
XY_ONE = 1 << XY_SHIFT


def mask_params(landmarks: np.ndarray, landmarks_tgt: np.ndarray):
    """face_mask_static's (erode, sigmaX, sigmaY) when params is None (masks.py:43-65)."""
    left = np.sum((landmarks[1][0] - landmarks_tgt[1][0], landmarks[2][0] - landmarks_tgt[2][0],
                   landmarks[13][0] - landmarks_tgt[13][0]))
    right = np.sum((landmarks_tgt[17][0] - landmarks[17][0], landmarks_tgt[18][0] - landmarks[18][0],
                    landmarks_tgt[29][0] - landmarks[29][0]))
    offset = max(left, right)
    if offset > 6:
        return 15, 15, 10
    if offset > 3:
        return 10, 10, 8
    if offset < -3:
        return -5, 5, 10
    return 5, 5, 5


def expand_eyebrows(lmrks: np.ndarray, eyebrows_expand_mod: float = 1.0) -> np.ndarray:
    """masks.py:5-20 (int32 landmarks; the float update assigned back truncates toward zero)."""
    lmrks = np.array(lmrks.copy(), dtype=np.int32)
    bot_l, bot_r = lmrks[[35, 41, 40, 42, 39]], lmrks[[89, 95, 94, 96, 93]]
    top_l, top_r = lmrks[[43, 48, 49, 51, 50]], lmrks[[102, 103, 104, 105, 101]]
    lmrks[[43, 48, 49, 51, 50]] = top_l + eyebrows_expand_mod * 0.5 * (top_l - bot_l)
    lmrks[[102, 103, 104, 105, 101]] = top_r + eyebrows_expand_mod * 0.5 * (top_r - bot_r)
    return lmrks


def eyebrow_mod(erode: int) -> float:
    return 2.7 if erode == 15 else 0.5 if erode == -5 else 2.0


def convex_hull(points: np.ndarray) -> np.ndarray:
    """Hull vertices of integer points (Andrew's monotone chain, collinear points dropped)."""
    pts = sorted(set(map(tuple, np.asarray(points, dtype=np.int64).tolist())))
    if len(pts) <= 2:
        return np.array(pts, dtype=np.int64)

    def cross(o, a, b):
        return (a[0] - o[0]) * (b[1] - o[1]) - (a[1] - o[1]) * (b[0] - o[0])
    lower, upper = [], []
    for p in pts:
        while len(lower) >= 2 and cross(lower[-2], lower[-1], p) <= 0:
            lower.pop()
        lower.append(p)
    for p in reversed(pts):
        while len(upper) >= 2 and cross(upper[-2], upper[-1], p) <= 0:
            upper.pop()
        upper.append(p)
    return np.array(lower[:-1] + upper[:-1], dtype=np.int64)


def _tdiv(a: int, b: int) -> int:
    """C integer division (truncation toward zero)."""
    q = abs(a) // abs(b)
    return q if (a >= 0) == (b >= 0) else -q


def clip_line(W: int, H: int, x1: int, y1: int, x2: int, y2: int):
    """OpenCV clipLine (drawing.cpp) on integer endpoints; returns (inside, x1, y1, x2, y2)."""
    right, bottom = W - 1, H - 1

    def code(x, y):
        return (x < 0) + (x > right) * 2 + (y < 0) * 4 + (y > bottom) * 8
    c1, c2 = code(x1, y1), code(x2, y2)
    if (c1 & c2) == 0 and (c1 | c2) != 0:
        if c1 & 12:
            a = 0 if c1 < 8 else bottom
            x1 += int(float(a - y1) * (x2 - x1) / (y2 - y1))
            y1 = a
            c1 = (x1 < 0) + (x1 > right) * 2
        if c2 & 12:
            a = 0 if c2 < 8 else bottom
            x2 += int(float(a - y2) * (x2 - x1) / (y2 - y1))
            y2 = a
            c2 = (x2 < 0) + (x2 > right) * 2
        if (c1 & c2) == 0 and (c1 | c2) != 0:
            if c1:
                a = 0 if c1 == 1 else right
                y1 += int(float(a - x1) * (y2 - y1) / (x2 - x1))
                x1 = a
                c1 = 0
            if c2:
                a = 0 if c2 == 1 else right
                y2 += int(float(a - x2) * (y2 - y1) / (x2 - x1))
                x2 = a
                c2 = 0
    return (c1 | c2) == 0, x1, y1, x2, y2


def draw_line(img: np.ndarray, x1: int, y1: int, x2: int, y2: int, v: int = 255) -> None:
    """cv2 Line, LINE_8 (LineIterator, left to right)."""
    H, W = img.shape
    if not (0 <= x1 < W and 0 <= y1 < H and 0 <= x2 < W and 0 <= y2 < H):
        ok, x1, y1, x2, y2 = clip_line(W, H, x1, y1, x2, y2)
        if not ok:
            return
    if x2 < x1:
        x1, y1, x2, y2 = x2, y2, x1, y1
    dx, dy = x2 - x1, y2 - y1
    sy = -1 if dy < 0 else 1
    dy = abs(dy)
    if dy > dx:                       # y major
        M, m, maj_x = dy, dx, False
    else:
        M, m, maj_x = dx, dy, True
    err = M - 2 * m
    x, y = x1, y1
    for _ in range(M + 1):
        img[y, x] = v
        if err < 0:                   # step along both axes
            err += 2 * M - 2 * m
            x += 1
            y += sy
        else:                         # step along the major axis
            err -= 2 * m
            if maj_x:
                x += 1
            else:
                y += sy
    return


def fill_convex_poly(img: np.ndarray, pts: np.ndarray, v: int = 255) -> None:
    """cv2.fillConvexPoly(img, pts, v) with shift 0, LINE_8 (drawing.cpp FillConvexPoly)."""
    H, W = img.shape
    pts = [(int(p[0]), int(p[1])) for p in pts]
    n = len(pts)
    if n == 0:
        return
    delta1 = delta2 = XY_ONE >> 1
    imin = 0
    ymin = ymax = pts[0][1]
    xmin = xmax = pts[0][0]
    p0 = pts[n - 1]
    for i, p in enumerate(pts):
        if p[1] < ymin:
            ymin, imin = p[1], i
        ymax, xmax, xmin = max(ymax, p[1]), max(xmax, p[0]), min(xmin, p[0])
        draw_line(img, p0[0], p0[1], p[0], p[1], v)
        p0 = p
    if n < 3 or xmax < 0 or ymax < 0 or xmin >= W or ymin >= H:
        return
    ymax = min(ymax, H - 1)
    edge = [{"idx": imin, "di": 1, "x": -XY_ONE, "dx": 0, "ye": ymin},
            {"idx": imin, "di": n - 1, "x": -XY_ONE, "dx": 0, "ye": ymin}]
    edges = n
    y = ymin
    while True:
        for e in edge:
            if y >= e["ye"]:
                idx0 = e["idx"]
                idx = (idx0 + e["di"]) % n
                while True:
                    edges -= 1
                    if edges < 0:
                        break
                    ty = pts[idx][1]
                    if ty > y:
                        xs, xe = pts[idx0][0] << XY_SHIFT, pts[idx][0] << XY_SHIFT
                        e["ye"] = ty
                        e["dx"] = _tdiv((xe - xs) * 2 + (ty - y), 2 * (ty - y))
                        e["x"] = xs
                        e["idx"] = idx
                        break
                    idx0 = idx
                    idx = (idx + e["di"]) % n
        if edges < 0:
            break
        if y >= 0:
            left, right = (1, 0) if edge[0]["x"] > edge[1]["x"] else (0, 1)
            xx1 = (edge[left]["x"] + delta1) >> XY_SHIFT
            xx2 = (edge[right]["x"] + delta2) >> XY_SHIFT
            if xx2 >= 0 and xx1 < W:
                img[y, max(xx1, 0):min(xx2, W - 1) + 1] = v
        edge[0]["x"] += edge[0]["dx"]
        edge[1]["x"] += edge[1]["dx"]
        y += 1
        if y > ymax:
            break


def box_morph(mask: np.ndarray, k: int, dilate: bool) -> np.ndarray:
    """cv2.erode / cv2.dilate with np.ones((k, k)), anchor k//2, pixels outside the image ignored."""
    H, W = mask.shape
    a = k // 2
    big = np.full((H + k, W + k), 0 if dilate else 255, dtype=np.int32)
    big[a:a + H, a:a + W] = mask
    f = np.maximum if dilate else np.minimum
    out = big[:H, a:a + W].copy()             # rows y - a ... y - a + k - 1
    for d in range(1, k):
        out = f(out, big[d:d + H, a:a + W])
    res = out
    big2 = np.full((H, W + k), 0 if dilate else 255, dtype=np.int32)
    big2[:, a:a + W] = res
    out = big2[:, :W].copy()
    for d in range(1, k):
        out = f(out, big2[:, d:d + W])
    return out.astype(np.uint8)


def gaussian_kernel(sigma: float) -> np.ndarray:
    """getGaussianKernel(n, sigma): exp(-x^2 / (2 sigma^2)) in double, summed in tap order, normalised, as float."""
    n = int(math.floor(sigma * 6 + 1 + 0.5)) | 1       # cvRound(sigma*3*2 + 1) | 1 for 8-bit input
    sc = -0.5 / (sigma * sigma)
    t = [math.exp(sc * (i - (n - 1) * 0.5) * (i - (n - 1) * 0.5)) for i in range(n)]
    s = 0.0
    for v in t:
        s += v
    return np.array([v / s for v in t], dtype=np.float64).astype(np.float32)


def _reflect101(i: np.ndarray, n: int) -> np.ndarray:
    if n == 1:
        return np.zeros_like(i)
    p = 2 * (n - 1)
    i = np.abs(i) % p
    return np.where(i >= n, p - i, i)


def gaussian_blur(mask: np.ndarray, sx: float, sy: float) -> np.ndarray:
    H, W = mask.shape
    kx, ky = gaussian_kernel(sx), gaussian_kernel(sy)
    m = mask.astype(np.float32)
    rx, ry = len(kx) // 2, len(ky) // 2
    cols = _reflect101(np.arange(W)[:, None] + np.arange(-rx, rx + 1)[None, :], W)
    tmp = np.zeros((H, W), dtype=np.float32)
    for t in range(len(kx)):
        tmp = tmp + kx[t] * m[:, cols[:, t]]
    rows = _reflect101(np.arange(H)[:, None] + np.arange(-ry, ry + 1)[None, :], H)
    out = np.zeros((H, W), dtype=np.float32)
    for t in range(len(ky)):
        out = out + ky[t] * tmp[rows[:, t], :]
    return np.clip(np.rint(out), 0, 255).astype(np.uint8)


def face_mask_static(H: int, W: int, landmarks: np.ndarray, landmarks_tgt=None, params=None):
    """masks.py:38-86 on an H x W image: returns (mask / 255 as float32, [erode, sigmaX, sigmaY])."""
    if params is None:
        params = list(mask_params(landmarks, landmarks_tgt))
    erode, sx, sy = params
    lm = expand_eyebrows(landmarks, eyebrow_mod(erode))
    m = np.zeros((H, W), dtype=np.uint8)
    fill_convex_poly(m, convex_hull(lm), 255)
    m = box_morph(m, abs(erode), dilate=erode <= 0)
    c = sy * 2
    m[:c, :] = 0
    m[-c:, :] = 0
    m[:, :c] = 0
    m[:, -c:] = 0
    m = gaussian_blur(m, sx, sy)
    return (m.astype(np.float64) / 255).astype(np.float32), [erode, sx, sy]
