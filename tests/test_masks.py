"""Face masks for the paste-back (utils/inference/masks.py: face_mask_static, get_mask, erode_and_blur).

CPU: the restatement oracle (oracle/mask_ref.py) against independent checks — a filled axis-aligned box and a
triangle against point-in-polygon, the box erode / dilate against scipy.ndimage's rank filters, the Gaussian
kernel sizes — and the native library's host half (ghost_mask_polygons: eyebrow expansion + convex hull) against
the oracle's.  GPU: the device masks (ghost_face_masks) against the oracle, frame by frame, for all four
parameter regimes of face_mask_static and landmark sets that leave the image (clipLine paths).
cv2 and the landmark model are absent, so this is parity unpinned: the oracle restates OpenCV 4.x's published
algorithms and nothing of the reference's own output covers masks.
"""
import numpy as np
import pytest
import torch

from oracle import mask_ref as M

DEV = torch.device("cuda:0")
REGIMES = [[15, 15, 10], [10, 10, 8], [-5, 5, 10], [5, 5, 5]]


def landmarks(seed, shift=(0.0, 0.0), scale=1.0):
    """106 face-like points: a 33-point jaw/forehead contour on an ellipse + 73 interior points (float32, as the
    landmark model returns them)."""
    g = np.random.Generator(np.random.PCG64(seed))
    t = np.linspace(0.15 * np.pi, 0.85 * np.pi, 33) + np.pi
    cx, cy = 112 + shift[0], 118 + shift[1]
    contour = np.stack([cx + 78 * scale * np.cos(-t), cy + 92 * scale * np.sin(-t)], 1)
    inner = np.stack([cx + g.uniform(-60, 60, 73) * scale, cy + g.uniform(-70, 60, 73) * scale], 1)
    pts = np.concatenate([contour, inner]) + g.normal(0, 1.5, (106, 2))
    return pts.astype(np.float32)


def test_oracle_fill_box_and_triangle():
    img = np.zeros((40, 50), np.uint8)
    M.fill_convex_poly(img, np.array([[5, 7], [30, 7], [30, 20], [5, 20]]))
    ref = np.zeros_like(img)
    ref[7:21, 5:31] = 255
    assert np.array_equal(img, ref)
    img = np.zeros((64, 64), np.uint8)
    tri = np.array([[10, 50], [55, 40], [20, 5]])
    M.fill_convex_poly(img, tri)
    yy, xx = np.mgrid[:64, :64]

    def side(a, b):
        return (b[0] - a[0]) * (yy - a[1]) - (b[1] - a[1]) * (xx - a[0])
    s = [side(tri[i], tri[(i + 1) % 3]) / np.hypot(*(tri[(i + 1) % 3] - tri[i])) for i in range(3)]
    inside = np.minimum.reduce([x * np.sign(s[0][20, 25]) for x in s])
    assert (img[inside > 1.0] == 255).all() and (img[inside < -1.0] == 0).all()


def test_oracle_lines_and_clipping():
    img = np.zeros((10, 10), np.uint8)
    M.draw_line(img, 0, 0, 9, 9)
    assert np.array_equal(img, np.eye(10, dtype=np.uint8) * 255)
    img = np.zeros((10, 10), np.uint8)
    M.draw_line(img, -5, 3, 20, 3)                 # clipped to the row
    assert (img[3] == 255).all() and img.sum() == 255 * 10
    img = np.zeros((10, 10), np.uint8)
    M.draw_line(img, -5, -5, -1, 20)               # entirely outside
    assert img.sum() == 0


@pytest.mark.parametrize("k,dilate", [(15, False), (10, False), (5, False), (5, True)])
def test_oracle_box_morph_matches_rank_filters(k, dilate):
    from scipy import ndimage
    g = np.random.Generator(np.random.PCG64(k))
    m = (g.uniform(size=(60, 70)) > 0.35).astype(np.uint8) * 255
    m[20:40, 10:50] = 255
    ref = (ndimage.maximum_filter(m, size=k, mode="constant", cval=0) if dilate
           else ndimage.minimum_filter(m, size=k, mode="constant", cval=255))
    assert np.array_equal(M.box_morph(m, k, dilate), ref)


def test_oracle_gaussian_kernel():
    for s, n in ((15, 91), (10, 61), (8, 49), (5, 31)):
        k = M.gaussian_kernel(s)
        assert len(k) == n and abs(float(k.astype(np.float64).sum()) - 1.0) < 1e-6 and k[n // 2] == k.max()
    flat = np.full((32, 40), 200, np.uint8)
    assert np.array_equal(M.gaussian_blur(flat, 5, 8), flat)   # reflect-101 borders keep a constant image


def test_host_polygons_match_oracle():
    """ghost_mask_polygons (C++, CPU) = the oracle's expand_eyebrows + convex hull."""
    from ghost_amd.inference.masks import mask_polygons
    lms = np.stack([landmarks(s, shift=(s * 7 - 20, -40 if s == 3 else 0)) for s in range(6)])
    params = np.array([REGIMES[s % 4] for s in range(6)], np.int32)
    poly, nv = mask_polygons(lms, params)
    for f in range(6):
        hull = M.convex_hull(M.expand_eyebrows(lms[f], M.eyebrow_mod(params[f][0])))
        assert nv[f] == len(hull)
        assert set(map(tuple, poly[f, :nv[f]].tolist())) == set(map(tuple, hull.tolist()))


def test_mask_params_follow_reference():
    from ghost_amd.inference.masks import mask_params
    for s in range(8):
        a, b = landmarks(s), landmarks(s + 100, shift=(s - 4, 0))
        assert list(mask_params(a, b)) == list(M.mask_params(a, b))


@pytest.mark.gpu
def test_face_masks_match_oracle():
    from ghost_amd.inference.masks import face_masks
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    cases = [(landmarks(s), REGIMES[s % 4]) for s in range(8)]
    cases += [(landmarks(20, shift=(-70, 0)), [10, 10, 8]),        # off the left edge
              (landmarks(21, shift=(0, -80), scale=1.2), [-5, 5, 10]),   # eyebrows far above the image
              (landmarks(22, scale=0.2), [5, 5, 5])]                # a small face
    lms = np.stack([c[0] for c in cases])
    params = np.array([c[1] for c in cases], np.int32)
    got = face_masks(lms, params, 224, 224, DEV).cpu().numpy()
    for f, (lm, p) in enumerate(cases):
        ref, _ = M.face_mask_static(224, 224, lm, params=p)
        d = np.abs(got[f] - ref)
        # exp / normalisation of the Gaussian taps in double on both sides: a rounding tie may land on the
        # other side once in a while
        assert d.max() <= 1.0 / 255 + 1e-7 and (d > 0).mean() < 1e-3, (f, float(d.max()), float((d > 0).mean()))


@pytest.mark.gpu
def test_face_mask_static_dropin_returns_params():
    from ghost_amd.inference.masks import face_mask_static
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    swap = np.zeros((224, 224, 3), np.uint8)
    a, b = landmarks(1), landmarks(2, shift=(5, 0))
    m, p = face_mask_static(swap, a, b, device=DEV)
    assert p == list(M.mask_params(a, b)) and m.shape == (224, 224) and m.dtype == torch.float32
    m2 = face_mask_static(swap, a, b, params=p, device=DEV)
    assert torch.equal(m, m2)
    ref, _ = M.face_mask_static(224, 224, a, b)
    assert float(np.abs(m.cpu().numpy() - ref).max()) <= 1.0 / 255 + 1e-7
