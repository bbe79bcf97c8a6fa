"""GPU parity tests (MI355X): the HIP path through the C ABI against the oracle and the
reference golden vectors.

Gates
* fp32 path: max|dY| <= 1e-3 against the reference CPU fp32 forward (BASELINE.json
  north_star), u8 output within 1 LSB (truncation flips at integer boundaries).
* per-op fp32 kernels: against torch fp32 CPU ops of the same op, max abs <= 1e-4
  relative to the output scale.
* bf16 path: bf16 storage of weights and activations cannot meet 1e-3 (SURVEY.md §7
  "Hard parts" 1).  Its error against the fp32 oracle must not exceed the error of the
  bf16-storage-emulating oracle (oracle/aei_ref.aei_forward_bf16_storage: the same stored
  roundings, fp32 in between) by more than 25 % in mean and 99.9th percentile; the tight
  per-stage gates against that oracle are in tests/test_bf16_parity.py.
"""
import os

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from oracle import aei_ref

pytestmark = pytest.mark.gpu

GOLD = os.path.join(os.path.dirname(__file__), "golden")
DEV = torch.device("cuda:0")


def gold(name):
    return np.load(os.path.join(GOLD, name + ".npz"))


@pytest.fixture(scope="module")
def lib():
    from ghost_amd import _lib
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return _lib.load()


_WEIGHTS = {}


def weights(backbone, nb):
    key = (backbone, nb)
    if key not in _WEIGHTS:
        _WEIGHTS[key] = aei_ref.make_weights(aei_ref.param_specs(backbone, nb))
    return _WEIGHTS[key]


def model(backbone, nb, compute_dtype=None):
    from ghost_amd.network import AEI_Net
    G = AEI_Net(backbone, num_blocks=nb, c_id=512, compute_dtype=compute_dtype).eval()
    G.load_state_dict(weights(backbone, nb))
    return G.to(DEV)


def stream(lib):
    return torch.cuda.current_stream().cuda_stream


# ----------------------------------------------------------------------------------------
# single operators
# ----------------------------------------------------------------------------------------
def nhwc(x):
    return x.permute(0, 2, 3, 1).contiguous()


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("cin,cout,k,s,p,H", [(32, 64, 4, 2, 1, 32), (3, 32, 4, 2, 1, 64), (64, 64, 3, 1, 1, 40),
                                              (128, 3, 3, 1, 1, 32), (96, 200, 1, 1, 0, 9),
                                              # halo-tiled 3x3 kernel shapes (bf16, H % 16, W % 32, N % 64)
                                              (64, 64, 3, 1, 1, 64), (96, 128, 3, 1, 1, 32), (256, 64, 3, 1, 1, 32),
                                              (128, 192, 3, 1, 1, 16)])
def test_conv2d_op(lib, dt, cin, cout, k, s, p, H):
    from ghost_amd import _lib
    from ghost_amd.network.pack import pack_conv, rup
    g = torch.Generator().manual_seed(cin * 7 + cout)
    x = torch.randn(2, cin, H, H, generator=g)
    w = torch.randn(cout, cin, k, k, generator=g) * (2.0 / (cin * k * k)) ** 0.5
    sc = torch.rand(cout, generator=g) + 0.5
    sh = torch.randn(cout, generator=g) * 0.1
    Ho = (H + 2 * p - k) // s + 1
    res = torch.randn(2, cout, Ho, Ho, generator=g)
    xr = x.to(dt).float()
    wr = w.to(dt).float()
    ref = F.leaky_relu(F.conv2d(xr, wr, stride=s, padding=p) * sc.view(1, -1, 1, 1) + sh.view(1, -1, 1, 1), 0.1)
    ref = ref + res.to(dt).float()
    wp = pack_conv(w, dt).to(DEV)
    xd = nhwc(x).to(dt).to(DEV)
    rd = nhwc(res).to(dt).to(DEV)
    y = torch.empty(2, Ho, Ho, cout, dtype=dt, device=DEV)
    scp = torch.zeros(rup(cout, 128), device=DEV); scp[:cout] = sc.to(DEV)
    shp = torch.zeros(rup(cout, 128), device=DEV); shp[:cout] = sh.to(DEV)
    ws = torch.empty(64 << 20, dtype=torch.uint8, device=DEV)
    _lib.check(lib.ghost_conv2d_nhwc(_lib.gdtype(dt), xd.data_ptr(), 2, H, H, cin, cin, wp.data_ptr(), cout,
                                     wp.shape[0], wp.shape[1], k, k, s, p, scp.data_ptr(), shp.data_ptr(), 0.1,
                                     rd.data_ptr(), cout, 0, y.data_ptr(), cout, ws.data_ptr(), ws.numel(),
                                     stream(lib)))
    got = y.float().cpu().permute(0, 3, 1, 2)
    tol = 1e-4 if dt == torch.float32 else 3e-2
    assert float((got - ref).abs().max()) <= tol * max(1.0, float(ref.abs().max()))


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
@pytest.mark.parametrize("H,B", [(256, 2), (256, 1), (64, 3), (128, 1)])
def test_conv3x3_64_op(lib, dt, H, B):
    """The persistent halo conv at 64 -> 64 with resident weights (AADBlk8's first conv at 256 x 256) against
    torch's fp32 conv of the same 16-bit operands, bf16 and fp16 storage; B = 1 at 128 x 128 and B = 3 at
    64 x 64 give workgroups with uneven tile counts."""
    from ghost_amd import _lib
    from ghost_amd.network.pack import pack_conv, rup
    g = torch.Generator().manual_seed(H + B)
    x = torch.randn(B, 64, H, H, generator=g)
    w = torch.randn(64, 64, 3, 3, generator=g) * (2.0 / (64 * 9)) ** 0.5
    sc = torch.rand(64, generator=g) + 0.5
    sh = torch.randn(64, generator=g) * 0.1
    xr, wr = x.to(dt).float(), w.to(dt).float()
    ref = F.leaky_relu(F.conv2d(xr, wr, padding=1) * sc.view(1, -1, 1, 1) + sh.view(1, -1, 1, 1), 0.2)
    wp = pack_conv(w, dt).to(DEV)
    xd = nhwc(x).to(dt).to(DEV)
    y = torch.full((B, H, H, 64), float("nan"), dtype=dt, device=DEV)
    scp = torch.zeros(128, device=DEV); scp[:64] = sc.to(DEV)
    shp = torch.zeros(128, device=DEV); shp[:64] = sh.to(DEV)
    ws = torch.empty(64 << 20, dtype=torch.uint8, device=DEV)
    _lib.check(lib.ghost_conv2d_nhwc(_lib.gdtype(dt), xd.data_ptr(), B, H, H, 64, 64, wp.data_ptr(), 64,
                                     wp.shape[0], wp.shape[1], 3, 3, 1, 1, scp.data_ptr(), shp.data_ptr(), 0.2,
                                     None, 0, 0, y.data_ptr(), 64, ws.data_ptr(), ws.numel(), stream(lib)))
    got = y.float().cpu().permute(0, 3, 1, 2)
    assert torch.isfinite(got).all()
    ulp = 2.0 ** -7 if dt == torch.bfloat16 else 2.0 ** -10
    d = (got - ref).abs()
    assert float((d / ref.abs().clamp_min(1.0)).max()) <= 1.01 * ulp, float(d.max())


@pytest.mark.parametrize("cin,cout,H,B,xoff,yoff,bn", [(32, 64, 32, 2, 32, 64, True), (64, 128, 64, 2, 0, 0, True),
                                                 (128, 256, 32, 3, 128, 256, True), (32, 64, 64, 1, 0, 0, False),
                                                 (256, 64, 32, 2, 256, 0, True)])
def test_conv4x4s2_patch_kernel(lib, cin, cout, H, B, xoff, yoff, bn):
    """The encoder's 4x4/s2 convs with Cin % 32 == 0 (conv2..conv4) on the LDS input-patch kernel: the input read
    from a channel slice of a 2*Cin-wide buffer (the unet concat layout) and the output written into a channel
    slice of a wider buffer, against torch's fp32 conv of the same bf16 operands."""
    from ghost_amd import _lib
    from ghost_amd.network.pack import pack_conv, rup
    dt = torch.bfloat16
    g = torch.Generator().manual_seed(cin + 3 * cout + H)
    x = torch.randn(B, cin, H, H, generator=g)
    w = torch.randn(cout, cin, 4, 4, generator=g) * (2.0 / (cin * 16)) ** 0.5
    sc = torch.rand(cout, generator=g) + 0.5
    sh = torch.randn(cout, generator=g) * 0.1
    Ho = H // 2
    xr, wr = x.to(dt).float(), w.to(dt).float()
    v = F.conv2d(xr, wr, stride=2, padding=1)
    if bn:
        v = v * sc.view(1, -1, 1, 1) + sh.view(1, -1, 1, 1)
    ref = F.leaky_relu(v, 0.1)
    ldx, ldy = cin + xoff, cout + yoff
    xbuf = torch.randn(B, H, H, ldx, generator=g).to(dt).to(DEV)
    xbuf[..., xoff:] = nhwc(x).to(dt).to(DEV)
    ybuf = torch.full((B, Ho, Ho, ldy), 7.0, dtype=dt, device=DEV)
    wp = pack_conv(w, dt).to(DEV)
    scp = torch.zeros(rup(cout, 128), device=DEV); scp[:cout] = sc.to(DEV)
    shp = torch.zeros(rup(cout, 128), device=DEV); shp[:cout] = sh.to(DEV)
    ws = torch.empty(64 << 20, dtype=torch.uint8, device=DEV)
    _lib.check(lib.ghost_conv2d_nhwc(_lib.gdtype(dt), xbuf[..., xoff:].data_ptr(), B, H, H, cin, ldx, wp.data_ptr(),
                                     cout, wp.shape[0], wp.shape[1], 4, 4, 2, 1,
                                     scp.data_ptr() if bn else None, shp.data_ptr() if bn else None, 0.1, None, 0, 0,
                                     ybuf[..., yoff:].data_ptr(), ldy, ws.data_ptr(), ws.numel(), stream(lib)))
    torch.cuda.synchronize()
    got = ybuf[..., yoff:].float().cpu().permute(0, 3, 1, 2)
    err = float((got - ref).abs().max())
    assert err <= 2e-2 * max(1.0, float(ref.abs().max())), err
    # bf16 rounding of the fp32 result: at most 1 ulp away almost everywhere
    assert float(((got - ref).abs() > 2 ** -7 * ref.abs() + 1e-3).float().mean()) < 1e-3
    if yoff:   # the channels before the slice are untouched
        assert bool((ybuf[..., :yoff] == 7.0).all())


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("cin,ldx,cout,k,s,p,H,mode", [
    (3, 4, 64, 7, 1, 3, 32, "relu"),          # resnet encoder conv0 on the 4-channel input layout
    (64, 64, 64, 7, 2, 3, 32, "relu"),        # resnet encoder conv1 7x7/s2
    (64, 64, 32, 1, 2, 0, 16, "relu"),        # Bottleneck conv1 1x1/s2
    (128, 128, 512, 1, 2, 0, 16, "none"),     # downsample 1x1/s2 + BN
    (32, 32, 128, 1, 1, 0, 16, "res_relu"),   # Bottleneck tail relu(bn3(conv3) + residual)
    (64, 64, 64, 3, 1, 1, 28, "prelu_y2"),    # IBasicBlock conv + BN + PReLU, with a BN'd second output
    (64, 64, 128, 3, 2, 1, 28, "res_y2"),     # IBasicBlock conv2/s2 + BN + residual, second output = next BN
    # 3x3/s1 shapes the halo kernel takes in bf16 with overhanging 16x16 tiles (ArcFace stages)
    (64, 64, 64, 3, 1, 1, 112, "prelu_y2"),   # layer1 block-0 conv1 at 112x112 (7 x 7 exact tiles)
    (64, 64, 128, 3, 1, 1, 56, "prelu_y2"),   # layer2 block-0 conv1 at 56x56
    (128, 128, 128, 3, 1, 1, 28, "res_y2"),   # layer2 conv2 + residual + next BN
    (256, 256, 256, 3, 1, 1, 14, "prelu_y2"), # layer3 conv1
    (256, 256, 256, 3, 1, 1, 14, "res_y2"),   # layer3 conv2
    (64, 64, 64, 3, 1, 1, 48, "res_relu"),    # residual before the activation on the halo path
    (512, 512, 512, 3, 1, 1, 7, "res_y2"),    # 7x7 stays on the implicit GEMM
    (3, 4, 64, 3, 1, 1, 112, "prelu_y2"),     # ArcFace stem (bf16: the 4-channel MFMA stem kernel)
    (3, 4, 64, 3, 1, 1, 9, "prelu_y2"),       # stem with a partial last 64-pixel chunk (B*81 = 162)
    # 3x3/s2 on the LDS input-patch kernel in bf16 (conv_s2.hip, 8 x 16 output tiles overhanging 56/28/14)
    (64, 64, 64, 3, 2, 1, 112, "res_y2"),     # layer1 block-0 conv2 112 -> 56
    (128, 128, 128, 3, 2, 1, 56, "res_y2"),   # layer2 block-0 conv2 56 -> 28
    (256, 256, 256, 3, 2, 1, 28, "res_y2"),   # layer3 block-0 conv2 28 -> 14
    (64, 96, 64, 3, 2, 1, 32, "prelu_y2"),    # exact tiles, PReLU, padded input channels
    (64, 64, 64, 3, 2, 1, 34, "relu"),        # 17 x 17 output: too much overhang, the implicit GEMM
])
def test_conv2d_ex_epilogues(lib, dt, cin, ldx, cout, k, s, p, H, mode):
    """ghost_conv2d_ex_nhwc: residual-before-activation, per-channel PReLU and the dual output."""
    from ghost_amd import _lib
    from ghost_amd.network.pack import pack_conv, rup
    g = torch.Generator().manual_seed(cin * 13 + cout + k)
    B = 2
    x = torch.randn(B, cin, H, H, generator=g)
    w = torch.randn(cout, cin, k, k, generator=g) * (2.0 / (cin * k * k)) ** 0.5
    sc, sh = torch.rand(cout, generator=g) + 0.5, torch.randn(cout, generator=g) * 0.1
    pr = torch.rand(cout, generator=g) * 0.5
    sc2, sh2 = torch.rand(cout, generator=g) + 0.5, torch.randn(cout, generator=g) * 0.1
    Ho = (H + 2 * p - k) // s + 1
    res = torch.randn(B, cout, Ho, Ho, generator=g)
    xr, wr, rr = x.to(dt).float(), w.to(dt).float(), res.to(dt).float()
    v = F.conv2d(xr, wr, stride=s, padding=p) * sc.view(1, -1, 1, 1) + sh.view(1, -1, 1, 1)
    if mode == "relu":
        ref = F.relu(v)
    elif mode == "none":
        ref = v
    elif mode == "res_relu":
        ref = F.relu(v + rr)
    elif mode == "prelu_y2":
        ref = F.prelu(v, pr)
    else:
        ref = v + rr
    ref2 = ref * sc2.view(1, -1, 1, 1) + sh2.view(1, -1, 1, 1)
    xin = torch.zeros(B, H, H, ldx)
    xin[..., :cin] = nhwc(x)
    if ldx > cin:
        xin[..., cin:] = 7.0          # padding channels must not contribute
    xd = xin.to(dt).to(DEV)
    wp = pack_conv(w, dt).to(DEV)

    def padv(t):
        o = torch.zeros(rup(cout, 128), device=DEV)
        o[:cout] = t.to(DEV)
        return o
    scp, shp, prp, sc2p, sh2p = padv(sc), padv(sh), padv(pr), padv(sc2), padv(sh2)
    rd = nhwc(res).to(dt).to(DEV)
    y = torch.empty(B, Ho, Ho, cout, dtype=dt, device=DEV)
    y2 = torch.empty(B, Ho, Ho, cout, dtype=dt, device=DEV)
    e = _lib.ConvEpi()
    e.scale, e.shift = scp.data_ptr(), shp.data_ptr()
    e.slope = 0.0 if mode in ("relu", "res_relu") else 1.0
    if mode == "prelu_y2":
        e.prelu = prp.data_ptr()
    if mode in ("res_relu", "res_y2"):
        e.res, e.ldres, e.res_first = rd.data_ptr(), cout, 1
    if mode.endswith("y2"):
        e.y2, e.ldy2, e.scale2, e.shift2 = y2.data_ptr(), cout, sc2p.data_ptr(), sh2p.data_ptr()
    ws = torch.empty(64 << 20, dtype=torch.uint8, device=DEV)
    _lib.check(lib.ghost_conv2d_ex_nhwc(_lib.gdtype(dt), xd.data_ptr(), B, H, H, cin, ldx, wp.data_ptr(), cout,
                                        wp.shape[0], wp.shape[1], k, k, s, p, C_byref(e), y.data_ptr(), cout,
                                        ws.data_ptr(), ws.numel(), stream(lib)))
    tol = 1e-4 if dt == torch.float32 else 3e-2
    got = y.float().cpu().permute(0, 3, 1, 2)
    assert float((got - ref).abs().max()) <= tol * max(1.0, float(ref.abs().max()))
    if mode.endswith("y2"):
        got2 = y2.float().cpu().permute(0, 3, 1, 2)
        assert float((got2 - ref2).abs().max()) <= tol * max(1.0, float(ref2.abs().max()))


def C_byref(x):
    import ctypes
    return ctypes.byref(x)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_first_conv_padded_input(lib, dt):
    """Encoder conv1 (3 -> 32, 4x4/s2) on the runtime's 4-channel input layout (channel 3 is padding
    and must not contribute: filled with finite junk here); bf16 runs the MFMA kernel."""
    from ghost_amd import _lib
    from ghost_amd.network.pack import pack_conv, rup
    g = torch.Generator().manual_seed(5)
    B, H, cout = 2, 128, 32
    x = torch.randn(B, 3, H, H, generator=g)
    w = torch.randn(cout, 3, 4, 4, generator=g) * 0.3
    sc = torch.rand(cout, generator=g) + 0.5
    sh = torch.randn(cout, generator=g) * 0.1
    ref = F.leaky_relu(F.conv2d(x.to(dt).float(), w.to(dt).float(), stride=2, padding=1) * sc.view(1, -1, 1, 1)
                       + sh.view(1, -1, 1, 1), 0.1)
    x4 = torch.cat([nhwc(x), torch.randn(B, H, H, 1, generator=g) * 100], -1).to(dt).to(DEV).contiguous()
    wp = pack_conv(w, dt).to(DEV)
    scp = torch.zeros(rup(cout, 128), device=DEV); scp[:cout] = sc.to(DEV)
    shp = torch.zeros(rup(cout, 128), device=DEV); shp[:cout] = sh.to(DEV)
    y = torch.empty(B, H // 2, H // 2, cout, dtype=dt, device=DEV)
    ws = torch.empty(1 << 20, dtype=torch.uint8, device=DEV)
    _lib.check(lib.ghost_conv2d_nhwc(_lib.gdtype(dt), x4.data_ptr(), B, H, H, 3, 4, wp.data_ptr(), cout, wp.shape[0],
                                     wp.shape[1], 4, 4, 2, 1, scp.data_ptr(), shp.data_ptr(), 0.1, None, 0, 0,
                                     y.data_ptr(), cout, ws.data_ptr(), ws.numel(), stream(lib)))
    got = y.float().cpu().permute(0, 3, 1, 2)
    tol = 1e-4 if dt == torch.float32 else 3e-2
    assert float((got - ref).abs().max()) <= tol * max(1.0, float(ref.abs().max()))


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("cin,cout,H,ldy_extra,skip_add", [(64, 32, 8, 32, False), (1024, 1024, 2, 1024, False),
                                                           (128, 64, 16, 0, True), (32, 48, 5, 16, False),
                                                           # halo ConvT shapes (bf16): N = 32 slice, two N tiles
                                                           (64, 32, 16, 32, False), (96, 128, 32, 64, False)])
def test_convT_op(lib, dt, cin, cout, H, ldy_extra, skip_add):
    """ConvT4x4/s2/p1 + BN + LReLU, written into a channel slice (unet concat) or + skip (linknet)."""
    from ghost_amd import _lib
    from ghost_amd.network.pack import pack_convT4x4, rup
    g = torch.Generator().manual_seed(cin + H)
    x = torch.randn(2, cin, H, H, generator=g)
    w = torch.randn(cin, cout, 4, 4, generator=g) * (2.0 / (cin * 16)) ** 0.5
    sc = torch.rand(cout, generator=g) + 0.5
    sh = torch.randn(cout, generator=g) * 0.1
    skip = torch.randn(2, cout, 2 * H, 2 * H, generator=g)
    ref = F.leaky_relu(F.conv_transpose2d(x.to(dt).float(), w.to(dt).float(), stride=2, padding=1)
                       * sc.view(1, -1, 1, 1) + sh.view(1, -1, 1, 1), 0.1)
    if skip_add:
        ref = ref + skip.to(dt).float()
    wp = pack_convT4x4(w, dt).to(DEV)
    ld = cout + ldy_extra
    y = torch.full((2, 2 * H, 2 * H, ld), 7.0, dtype=dt, device=DEV)
    scp = torch.zeros(rup(cout, 128), device=DEV); scp[:cout] = sc.to(DEV)
    shp = torch.zeros(rup(cout, 128), device=DEV); shp[:cout] = sh.to(DEV)
    sk = nhwc(skip).to(dt).to(DEV)
    ws = torch.empty(256 << 20, dtype=torch.uint8, device=DEV)
    xd = nhwc(x).to(dt).to(DEV)
    _lib.check(lib.ghost_conv_transpose4x4s2_nhwc(_lib.gdtype(dt), xd.data_ptr(), 2, H, H, cin, cin, wp.data_ptr(),
                                                  cout, wp.shape[1], wp.shape[2], scp.data_ptr(), shp.data_ptr(), 0.1,
                                                  sk.data_ptr() if skip_add else None, cout, y.data_ptr(), ld,
                                                  ws.data_ptr(), ws.numel(), stream(lib)))
    got = y.float().cpu()
    assert torch.all(got[..., cout:] == 7.0), "wrote outside its channel slice"
    got = got[..., :cout].permute(0, 3, 1, 2)
    tol = 1e-4 if dt == torch.float32 else 3e-2
    assert float((got - ref).abs().max()) <= tol * max(1.0, float(ref.abs().max()))


@pytest.mark.parametrize("split", [1, 3, 8])
def test_conv3x3_splitk_residual_tanh(lib, split):
    """conv3x3 with forced split-K (the low-resolution AADBlk path), residual add and tanh epilogue."""
    from ghost_amd import _lib
    from ghost_amd.network.pack import pack_conv
    # drive split-K through the generic entry by a shape whose tile count is small (B*H*W = 128)
    g = torch.Generator().manual_seed(split)
    cin, cout, H = 512, 256, 8
    x = torch.randn(2, cin, H, H, generator=g)
    w = torch.randn(cout, cin, 3, 3, generator=g) * (1.0 / (cin * 9)) ** 0.5
    res = torch.randn(2, cout, H, H, generator=g)
    ref = torch.tanh(F.conv2d(x, w, padding=1) + res)
    wp = pack_conv(w, torch.float32).to(DEV)
    y = torch.empty(2, H, H, cout, device=DEV)
    ws = torch.empty(256 << 20, dtype=torch.uint8, device=DEV)
    xd, rd = nhwc(x).to(DEV), nhwc(res).to(DEV)
    e = _lib.ConvEpi()
    e.slope, e.res, e.ldres, e.tanh_out, e.split_k = 1.0, rd.data_ptr(), cout, 1, split
    _lib.check(lib.ghost_conv2d_ex_nhwc(_lib.F32, xd.data_ptr(), 2, H, H, cin, cin, wp.data_ptr(), cout, wp.shape[0],
                                        wp.shape[1], 3, 3, 1, 1, C_byref(e), y.data_ptr(), cout, ws.data_ptr(), ws.numel(),
                                        stream(lib)))
    got = y.cpu().permute(0, 3, 1, 2)
    assert float((got - ref).abs().max()) <= 1e-5


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("B,C,H", [(2, 64, 256), (3, 1024, 2), (2, 256, 32), (1, 32, 5)])
def test_instnorm_stats(lib, dt, B, C, H):
    from ghost_amd import _lib
    g = torch.Generator().manual_seed(C + H)
    x = (torch.randn(B, C, H, H, generator=g) * 0.3 + 5.0).to(dt)   # |mean| >> std: cancellation check
    var, mean = torch.var_mean(x.double(), dim=(2, 3), unbiased=False)
    rstd = 1.0 / torch.sqrt(var + 1e-5)
    stat = torch.empty(B, C, 2, device=DEV)
    ws = torch.empty(64 << 20, dtype=torch.uint8, device=DEV)
    xd = nhwc(x).to(DEV)
    _lib.check(lib.ghost_instnorm_stats_nhwc(_lib.gdtype(dt), xd.data_ptr(), B, H * H, C, C, stat.data_ptr(),
                                             ws.data_ptr(), ws.numel(), stream(lib)))
    st = stat.cpu().double()
    torch.testing.assert_close(st[..., 0], mean, atol=1e-5, rtol=1e-6)
    torch.testing.assert_close(st[..., 1], rstd, atol=0, rtol=2e-4)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("B,C,H,W", [(2, 64, 128, 128), (2, 128, 16, 256), (3, 128, 64, 64), (2, 64, 32, 32),
                                     (2, 256, 32, 16), (2, 32, 16, 16), (1, 64, 7, 5), (2, 1024, 2, 2)])
def test_instnorm_stats_of_virtual_upsample(lib, dt, B, C, H, W):
    """Statistics of upsample2x(x) without materialising it == those of the materialised upsample: the
    per-pixel kernel samples the same bf16-rounded values; the closed form over the source (bf16,
    W % 128 == 0) gives the statistics of the fp32 upsample, so there the storage rounding remains."""
    from ghost_amd import _lib
    g = torch.Generator().manual_seed(C + H + W)
    x = (torch.randn(B, C, H, W, generator=g) * 0.3 + 2.0).to(dt)
    ws = torch.empty(64 << 20, dtype=torch.uint8, device=DEV)
    xd = nhwc(x).to(DEV)
    # the materialised path: our upsample kernel, then the statistics of its output
    upd = torch.empty(B, 2 * H, 2 * W, C, dtype=dt, device=DEV)
    _lib.check(lib.ghost_upsample2x_nhwc(_lib.gdtype(dt), xd.data_ptr(), C, upd.data_ptr(), C, B, H, W, C, stream(lib)))
    st_m = torch.empty(B, C, 2, device=DEV)
    _lib.check(lib.ghost_instnorm_stats_nhwc(_lib.gdtype(dt), upd.data_ptr(), B, 4 * H * W, C, C, st_m.data_ptr(),
                                             ws.data_ptr(), ws.numel(), stream(lib)))
    stat = torch.empty(B, C, 2, device=DEV)
    _lib.check(lib.ghost_instnorm_stats_up2x_nhwc(_lib.gdtype(dt), xd.data_ptr(), B, H, W, C, C, stat.data_ptr(),
                                                  ws.data_ptr(), ws.numel(), stream(lib)))
    st, st_m = stat.cpu().double(), st_m.cpu().double()
    cpb = min(W, 128)   # the closed form's source columns per workgroup (512 / cpb rows)
    quad = dt == torch.bfloat16 and W % 16 == 0 and W % cpb == 0 and H % (512 // cpb) == 0 and C % 64 == 0
    # quad: the materialised side carries bf16 storage rounding (|e| <= half an ulp = 2^-7 at
    # 2 <= |x| < 4), whose mean over N outputs is ~N(0, 2^-7 / sqrt(3 N)): 5 sigma; otherwise the
    # fp32 summation order only
    n_out = 4 * H * W
    tol_m = 5 * 2.0 ** -7 / (3 * n_out) ** 0.5 if quad else 1e-5
    torch.testing.assert_close(st[..., 0], st_m[..., 0], atol=tol_m, rtol=1e-5)
    # rstd: the rounding's variance and its sampled cross term with x (~1/sqrt(N))
    torch.testing.assert_close(st[..., 1], st_m[..., 1], atol=0, rtol=1e-3 + 0.1 / n_out ** 0.5 if quad else 1e-5)
    # and against float64 statistics of the (unrounded) PyTorch upsample: bf16 storage rounding only
    up = F.interpolate(x.double(), scale_factor=2, mode="bilinear", align_corners=True)
    var, mean = torch.var_mean(up, dim=(2, 3), unbiased=False)
    tol = 1e-5 if dt == torch.float32 else 8e-3   # bf16 half-ulp at |x| < 4 (a 4x4 output averages few)
    torch.testing.assert_close(st[..., 0], mean, atol=tol, rtol=0)
    torch.testing.assert_close(st[..., 1], 1.0 / torch.sqrt(var + 1e-5), atol=0, rtol=10 * tol)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("C,H", [(64, 128), (1024, 2), (32, 64), (128, 7)])
def test_upsample2x(lib, dt, C, H):
    from ghost_amd import _lib
    x = torch.randn(2, C, H, H).to(dt)
    ref = F.interpolate(x.float(), scale_factor=2, mode="bilinear", align_corners=True)
    y = torch.empty(2, 2 * H, 2 * H, C, dtype=dt, device=DEV)
    xd = nhwc(x).to(DEV)
    _lib.check(lib.ghost_upsample2x_nhwc(_lib.gdtype(dt), xd.data_ptr(), C, y.data_ptr(), C, 2, H, H, C, stream(lib)))
    got = y.float().cpu().permute(0, 3, 1, 2)
    tol = 2e-6 if dt == torch.float32 else 1e-2   # fp32: same index arithmetic as PyTorch (scale rounded once)
    assert float((got - ref).abs().max()) <= tol * max(1.0, float(ref.abs().max()))


def test_aad_layer_module_vs_reference_golden(lib):
    """ghost_amd.network.AADLayer.forward (native) against the reference AADLayer outputs."""
    from ghost_amd.network import AADLayer
    g = gold("aad_layer_cases")
    for i, (c_x, c_a, n) in enumerate(g["cases"].tolist()):
        layer = AADLayer(c_x, c_a, 512)
        specs = [(f"case{i}.{k}", tuple(v.shape), "lin_w" if k.startswith("fc") and k.endswith("weight")
                  else ("bias" if k.endswith("bias") else "conv")) for k, v in layer.state_dict().items()]
        w = aei_ref.make_weights(specs)
        layer.load_state_dict({k.split(".", 1)[1]: v for k, v in w.items()})
        layer = layer.to(DEV)
        rg = np.random.Generator(np.random.PCG64(100 + i))
        h = torch.from_numpy(rg.normal(0.5, 2.0, size=(2, c_x, n, n)).astype(np.float32)).to(DEV)
        za = torch.from_numpy(rg.normal(0, 1, size=(2, c_a, n, n)).astype(np.float32)).to(DEV)
        zi = torch.from_numpy(rg.normal(0, 1, size=(2, 512)).astype(np.float32)).to(DEV)
        out = layer(h, za, zi).float().cpu()
        ref = torch.from_numpy(g[f"case{i}_out"])
        assert float((out - ref).abs().max()) <= 1e-4 * max(1.0, float(ref.abs().max())), (c_x, c_a, n)


# ----------------------------------------------------------------------------------------
# whole network
# ----------------------------------------------------------------------------------------
@pytest.mark.parametrize("name", ["aei_unet2_b2", "aei_linknet3_b2", "aei_unet1_b1", "aei_unet3_b1",
                                  "aei_resnet2_b1"])
def test_forward_fp32_matches_reference(lib, name):
    g = gold(name)
    backbone, nb, B = str(g["backbone"]), int(g["num_blocks"]), int(g["batch"])
    G = model(backbone, nb)
    xt, z = aei_ref.make_inputs(B, int(g["seed"]))
    Y, attr = G(xt.to(DEV), z.to(DEV))
    torch.cuda.synchronize()
    assert Y.shape == (B, 3, 256, 256) and Y.dtype == torch.float32
    dy = float((Y.cpu() - torch.from_numpy(g["Y"])).abs().max())
    assert dy <= 1e-3, f"max|dY| = {dy}"
    for i, a in enumerate(attr, 1):
        assert tuple(a.shape) == tuple(g[f"attr{i}_shape"])
        flat = a.contiguous().reshape(-1)      # NCHW order, as the reference stored it
        samp = flat.cpu()[torch.from_numpy(g[f"attr{i}_idx"])]
        assert float((samp - torch.from_numpy(g[f"attr{i}_sample"])).abs().max()) <= 1e-4


@pytest.mark.parametrize("name", ["aei_unet2_b2", "aei_linknet3_b2"])
def test_swap_u8_pipeline_matches_reference(lib, name):
    """u8 crops -> normalise -> AEI_Net -> BGR uint8, fp32 path, against faceshifter_batch's output."""
    g = gold(name)
    backbone, nb, B = str(g["backbone"]), int(g["num_blocks"]), int(g["batch"])
    G = model(backbone, nb)
    _, z = aei_ref.make_inputs(B, int(g["seed"]))
    crops = torch.from_numpy(aei_ref.make_u8_crops(B, int(g["crops_seed"]))).to(DEV)
    out = G.swap_u8(crops, z[:1].to(DEV)).cpu().numpy()
    diff = np.abs(out.astype(np.int16) - g["U8"].astype(np.int16))
    assert diff.max() <= 1 and (diff > 0).mean() < 1e-3
    # the faceshifter_batch drop-in (host-side API) gives the same bytes
    from ghost_amd.inference import faceshifter_batch, transform_target_to_torch
    tgt = transform_target_to_torch(aei_ref.make_u8_crops(B, int(g["crops_seed"])), half=False)
    out2 = faceshifter_batch(z[:1].to(DEV), tgt, G)
    d2 = np.abs(out2.astype(np.int16) - g["U8"].astype(np.int16))
    assert d2.max() <= 1 and (d2 > 0).mean() < 1e-3


def bf16_gate(y, ref, emu):
    """y (GPU bf16) is no further from the fp32 oracle than the emulated bf16 arithmetic is."""
    d = (y - ref).abs().flatten()
    de = (emu - ref).abs().flatten()
    k = max(1, d.numel() // 200)       # tail: mean of the largest 0.5 % (steadier than a quantile on one frame)
    t, te = float(d.topk(k).values.mean()), float(de.topk(k).values.mean())
    assert float(d.mean()) <= 1.25 * float(de.mean()) and t <= 1.3 * te, (float(d.mean()), float(de.mean()), t, te)


def emulate(backbone, nb, xt, z):
    return aei_ref.aei_forward_bf16_storage(weights(backbone, nb), xt, z, backbone, nb)[0]


def test_forward_bf16_close_to_oracle(lib):
    g = gold("aei_unet2_b2")
    G = model("unet", 2, compute_dtype=torch.bfloat16)
    xt, z = aei_ref.make_inputs(2, int(g["seed"]))
    Y, attr = G(xt.to(DEV), z.to(DEV))
    assert Y.dtype == torch.bfloat16
    bf16_gate(Y.float().cpu(), torch.from_numpy(g["Y"]), emulate("unet", 2, xt, z))


def test_resnet_backbone_bf16_batch(lib):
    """backbone='resnet' (MLAttrEncoderResnet) on the bf16 path at B=8 against the fp32 oracle."""
    G = model("resnet", 2, compute_dtype=torch.bfloat16)
    xt, z = aei_ref.make_inputs(8, 21)
    Y, attr = G(xt.to(DEV), z.to(DEV))
    y_ref, a_ref = aei_ref.aei_forward(weights("resnet", 2), xt, z, "resnet", 2)
    bf16_gate(Y.float().cpu(), y_ref, emulate("resnet", 2, xt, z))
    for a, r in zip(attr, a_ref):
        assert a.shape == r.shape
        rel = float((a.float().cpu() - r).abs().mean()) / max(1e-6, float(r.abs().mean()))
        assert rel < 0.05, rel


@pytest.mark.parametrize("backbone,nb", [("unet", 2), ("linknet", 3)])
def test_bf16_through_upsample_aad_matches_materialised(lib, backbone, nb):
    """AADBlk8's first AADLayer pair sampling upsample2x(y7) on the fly == the materialised path."""
    G = model(backbone, nb, compute_dtype=torch.bfloat16)
    xt, z = aei_ref.make_inputs(4, 5)
    G.set_option("fuse_upsample", 0)
    Y0, _ = G(xt.to(DEV), z.to(DEV))
    Y0 = Y0.float().cpu()
    G.set_option("fuse_upsample", 1)
    Y1, _ = G(xt.to(DEV), z.to(DEV))
    d = (Y1.float().cpu() - Y0).abs()
    assert float(d.mean()) <= 1e-3 and float(d.max()) <= 0.1, (float(d.mean()), float(d.max()))


@pytest.mark.parametrize("backbone,nb", [("unet", 2), ("linknet", 3)])
def test_bf16_fused_conv_statistics_match_separate_pass(lib, backbone, nb):
    """InstanceNorm statistics from the persistent conv's epilogue partials vs a separate pass: the
    two forwards differ only by bf16 rounding flips downstream of fp-order differences in the
    statistics, so both must meet the bf16 gate against the fp32 oracle and differ from each other
    by no more than their own error against it."""
    G = model(backbone, nb, compute_dtype=torch.bfloat16)
    xt, z = aei_ref.make_inputs(4, 9)
    G.set_option("fuse_stats", 0)
    Y0, _ = G(xt.to(DEV), z.to(DEV))
    Y0 = Y0.float().cpu()
    G.set_option("fuse_stats", 1)
    Y1, _ = G(xt.to(DEV), z.to(DEV))
    Y1 = Y1.float().cpu()
    ref, _ = aei_ref.aei_forward(weights(backbone, nb), xt, z, backbone, nb)
    emu = emulate(backbone, nb, xt, z)
    bf16_gate(Y0, ref, emu)
    bf16_gate(Y1, ref, emu)
    d01 = float((Y1 - Y0).abs().mean())
    d0r = float((Y0 - ref).abs().mean())
    # two bf16 evaluations whose roundings flip in different places drift apart through the decoder
    # about as far as each is from fp32 (tests/test_bf16_parity.py): the forms may not differ by more
    assert d01 <= d0r, (d01, d0r)


def _lib_mod():
    from ghost_amd import _lib
    return _lib


def test_full_batch64_bf16_properties_and_fp32_rows(lib):
    """B=64 (the bench configuration): every one of the 64 fp32 rows (and their 8 attribute maps) against the oracle's
    batched forward within 1e-3 (was 3 sampled rows), then the bf16 gate on four rows."""
    G32 = model("unet", 2)
    xt, z = aei_ref.make_inputs(64, 11)
    Y, attr = G32(xt.to(DEV), z.to(DEV))
    Ycpu = Y.cpu()
    p = weights("unet", 2)
    yr, ar = aei_ref.aei_forward(p, xt, z)          # the whole batch on the CPU (~20 s on the box's 16 threads)
    err = (Ycpu - yr).abs().amax(dim=(1, 2, 3))
    assert float(err.max()) <= 1e-3, (int(err.argmax()), float(err.max()))
    for k, (a, b) in enumerate(zip(attr, ar)):
        assert float((a.cpu() - b).abs().max()) <= 1e-3, k
    Gb = model("unet", 2, compute_dtype=torch.bfloat16)
    Yb, _ = Gb(xt.to(DEV), z.to(DEV))
    # single frames are too few pixels for a steady end-to-end statistic: the B = 1 kernel set is
    # held per stage by tests/test_bf16_parity.py::test_bf16_small_batch_blocks_match_emulation
    bf16_gate(Yb[4:8].float().cpu(), Ycpu[4:8], emulate("unet", 2, xt[4:8], z[4:8]))
    assert torch.isfinite(Yb.float()).all()


def test_get_attr_matches_forward_attr(lib):
    G = model("unet", 2)
    xt, z = aei_ref.make_inputs(2, 3)
    _, attr = G(xt.to(DEV), z.to(DEV))
    attr2 = G.get_attr(xt.to(DEV))
    for a, b in zip(attr, attr2):
        assert torch.equal(a, b)


def test_strided_half_input_view(lib):
    """core.py:24 hands over a permuted (channels-last) fp16 view; it must be read as-is."""
    G = model("unet", 2)
    crops = aei_ref.make_u8_crops(2, 5)
    t = torch.from_numpy(crops).to(DEV)[:, :, :, [2, 1, 0]] / 255.0
    t = ((t.half() - 0.5) / 0.5).permute(0, 3, 1, 2)          # non-contiguous fp16 view
    assert not t.is_contiguous()
    _, z = aei_ref.make_inputs(2, 5)
    Y1, _ = G(t, z.to(DEV))
    Y2, _ = G(t.contiguous().float(), z.to(DEV))
    assert torch.equal(Y1, Y2)


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("c_x,c_a,n,B", [(64, 64, 256, 2), (128, 128, 128, 2), (256, 256, 64, 8), (64, 32, 128, 4)])
def test_aad_layer_fused_path_vs_oracle(lib, dt, c_x, c_a, n, B):
    """The fused AAD kernel (mask pre-pass + MFMA gamma/beta + LDS-staged blend) at pipeline sizes."""
    from ghost_amd.network import AADLayer
    layer = AADLayer(c_x, c_a, 512)
    specs = [(f"fz.{k}", tuple(v.shape), "lin_w" if k.startswith("fc") and k.endswith("weight")
              else ("bias" if k.endswith("bias") else "conv")) for k, v in layer.state_dict().items()]
    w = aei_ref.make_weights(specs)
    sd = {k.split(".", 1)[1]: v for k, v in w.items()}
    layer.load_state_dict(sd)
    if dt == torch.bfloat16:
        layer = layer.to(torch.bfloat16)
    layer = layer.to(DEV)
    g = torch.Generator().manual_seed(c_x + n)
    h = torch.randn(B, c_x, n, n, generator=g) * 1.5 + 0.7
    za = torch.randn(B, c_a, n, n, generator=g)
    zi = torch.randn(B, 512, generator=g)
    out = layer(h.to(DEV), za.to(DEV), zi.to(DEV)).float().cpu()
    p = {f"l.{k}": v.to(dt).float() for k, v in sd.items()}      # the module rounds its params to dt
    h, za = h.to(dt).float(), za.to(dt).float()
    ref = aei_ref.aad_layer(h, za, zi, p, "l")
    scale = max(1.0, float(ref.abs().max()))
    err = float((out - ref).abs().max())
    assert err <= (1e-4 if dt == torch.float32 else 4e-2) * scale, err


@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("cin,cout,H,W,use_res", [(128, 3, 32, 64, False), (64, 3, 16, 32, True), (96, 1, 8, 96, False)])
def test_conv3x3_narrow_op(lib, dt, cin, cout, H, W, use_res):
    """The generator's RGB-output conv: per-tap partial sums on a halo tile, tanh and BGR uint8 epilogue."""
    from ghost_amd import _lib
    from ghost_amd.network.pack import pack_conv3x3_narrow
    g = torch.Generator().manual_seed(cin + W)
    x = torch.randn(2, cin, H, W, generator=g)
    w = torch.randn(cout, cin, 3, 3, generator=g) * (1.0 / (cin * 9)) ** 0.5
    res = torch.randn(2, cout, H, W, generator=g) * 0.3
    ref = F.conv2d(x.to(dt).float(), w.to(dt).float(), padding=1)
    if use_res:
        ref = ref + res.to(dt).float()
    ref = torch.tanh(ref)
    wn = pack_conv3x3_narrow(w, dt).to(DEV)
    xd = nhwc(x).to(dt).to(DEV)
    rd = nhwc(res).to(dt).to(DEV)
    y = torch.empty(2, H, W, cout, dtype=dt, device=DEV)
    u8 = torch.zeros(2, H, W, 3, dtype=torch.uint8, device=DEV)
    _lib.check(lib.ghost_conv3x3_narrow_nhwc(_lib.gdtype(dt), xd.data_ptr(), 2, H, W, cin, cin, wn.data_ptr(),
                                             wn.shape[1], cout, rd.data_ptr() if use_res else None, cout, 1,
                                             y.data_ptr(), cout, u8.data_ptr(), stream(lib)))
    got = y.float().cpu().permute(0, 3, 1, 2)
    tol = 1e-5 if dt == torch.float32 else 1e-2
    assert float((got - ref).abs().max()) <= tol
    ref_u8 = ((ref.permute(0, 2, 3, 1) * 0.5 + 0.5) * 255).type(torch.uint8)
    got_u8 = u8.cpu()[..., [2, 1, 0]][..., :cout] if cout == 3 else u8.cpu()[..., 2:3]
    assert int((got_u8.int() - ref_u8[..., :cout].int()).abs().max()) <= (1 if dt == torch.float32 else 3)


@pytest.mark.parametrize("c_x,c_a,n,B,L,up", [(64, 64, 256, 2, 2, 0), (64, 64, 256, 2, 1, 0), (128, 128, 128, 2, 1, 0),
                                              (64, 32, 128, 4, 2, 0), (128, 64, 64, 8, 1, 0), (128, 32, 64, 8, 1, 0),
                                              (64, 64, 256, 2, 2, 1), (64, 32, 128, 4, 2, 1), (64, 64, 64, 8, 1, 1),
                                              (128, 64, 128, 2, 1, 1), (128, 32, 64, 8, 1, 1), (128, 64, 128, 2, 2, 0),
                                              # aad_v5_wide_kernel (taken when B * HW / 1024 >= 256): AADBlk7's
                                              # block-input pair, L = 1, a 64 x 64 output; B = 2 runs the v3 kernel
                                              (128, 64, 128, 16, 2, 1), (128, 64, 128, 16, 1, 1), (128, 64, 64, 64, 2, 1),
                                              (128, 64, 128, 2, 2, 1),
                                              # C = 256: every channel tile in one workgroup
                                              (256, 64, 64, 8, 1, 0),
                                              # aad_wide: one 64-channel tile per workgroup
                                              (256, 128, 64, 8, 1, 0), (512, 256, 32, 8, 1, 0),
                                              (1024, 256, 16, 16, 1, 0), (512, 64, 32, 4, 1, 0),
                                              (1024, 512, 16, 8, 1, 0)])
def test_aad_layers_v3_vs_oracle(lib, c_x, c_a, n, B, L, up):
    """Register-epilogue AAD kernel (1 or 2 layers sharing h_in / z_attr) against the oracle AADLayer;
    up = 1: h_in is read through the bilinear x2 upsample of an n/2 source (AEI_Net.py:137)."""
    import ctypes as C
    from ghost_amd import _lib
    from ghost_amd.network.pack import pack_aad_v3
    dt = torch.bfloat16
    g = torch.Generator().manual_seed(c_x * 3 + n + L)
    hn = n // 2 if up & 1 else n
    hs = (torch.randn(B, c_x, hn, hn, generator=g) * 1.5 + 0.7).to(dt).float()
    # the materialised path stores the upsample in bf16: the reference sees those values
    up2 = lambda t: F.interpolate(t, scale_factor=2, mode="bilinear", align_corners=True).to(dt).float()  # noqa: E731
    h = up2(hs) if up & 1 else hs
    zs = torch.randn(B, c_a, n, n, generator=g).to(dt).float()
    za = zs
    zi = torch.randn(B, 512, generator=g)
    hd, zad = nhwc(hs).to(dt).to(DEV), nhwc(zs).to(dt).to(DEV)
    keep, w3s, b3s, whs, bhs, ids, outs, refs = [], [], [], [], [], [], [], []
    for l in range(L):
        specs = [(f"v3_{l}.{k}", shp, kind) for k, shp, kind in [
            ("conv1.weight", (c_x, c_a, 1, 1), "conv"), ("conv1.bias", (c_x,), "bias"),
            ("conv2.weight", (c_x, c_a, 1, 1), "conv"), ("conv2.bias", (c_x,), "bias"),
            ("fc1.weight", (c_x, 512), "lin_w"), ("fc1.bias", (c_x,), "bias"),
            ("fc2.weight", (c_x, 512), "lin_w"), ("fc2.bias", (c_x,), "bias"),
            ("conv_h.weight", (1, c_x, 1, 1), "conv"), ("conv_h.bias", (1,), "bias")]]
        p = {k: v.to(dt).float() for k, v in aei_ref.make_weights(specs).items()}
        refs.append(F.relu(aei_ref.aad_layer(h, za, zi, p, f"v3_{l}")))
        pk = pack_aad_v3({k: v.to(DEV) for k, v in p.items()}, f"v3_{l}", dt)
        idgb = torch.cat([F.linear(zi, p[f"v3_{l}.fc1.weight"], p[f"v3_{l}.fc1.bias"]),
                          F.linear(zi, p[f"v3_{l}.fc2.weight"], p[f"v3_{l}.fc2.bias"])], 1).to(DEV).contiguous()
        wh = p[f"v3_{l}.conv_h.weight"].reshape(c_x).to(DEV).contiguous()
        bh = p[f"v3_{l}.conv_h.bias"].reshape(1).to(DEV).contiguous()
        out = torch.empty(B, n, n, c_x, dtype=dt, device=DEV)
        keep += [pk, idgb, wh, bh, out]
        w3s.append(pk["w3"].data_ptr()); b3s.append(pk["b3"].data_ptr()); whs.append(wh.data_ptr())
        bhs.append(bh.data_ptr()); ids.append(idgb.data_ptr()); outs.append(out.data_ptr())
    arr = lambda xs: (C.c_void_p * L)(*xs)  # noqa: E731
    ws = torch.empty(64 << 20, dtype=torch.uint8, device=DEV)
    _lib.check(lib.ghost_aad_layers_v3_nhwc(hd.data_ptr(), c_x, up, zad.data_ptr(), c_a, B, n, n, c_x, c_a, L, arr(w3s),
                                            arr(b3s), arr(whs), arr(bhs), arr(ids), 2 * c_x, 0.0, arr(outs),
                                            (C.c_int * L)(*([c_x] * L)), ws.data_ptr(), ws.numel(), stream(lib)))
    for l in range(L):
        got = keep[5 * l + 4].float().cpu().permute(0, 3, 1, 2)
        ref = refs[l]
        err = float((got - ref).abs().max())
        assert err <= 4e-2 * max(1.0, float(ref.abs().max())), (l, err)
        assert float((got - ref).abs().mean()) <= 2e-3 * max(1.0, float(ref.abs().mean()))


def test_mixed_identity_batch_and_dp_single_rank(lib):
    """Config 5 path: per-sample identity rows in one launch sequence == per-identity batches."""
    from ghost_amd.inference.dp import swap_mixed_identities
    G = model("unet", 2)
    crops = torch.from_numpy(aei_ref.make_u8_crops(4, 9)).to(DEV)
    _, z = aei_ref.make_inputs(2, 9)
    z = z.to(DEV)
    idx = torch.tensor([0, 1, 0, 1], device=DEV)
    mixed = swap_mixed_identities(crops, idx, z, G).cpu().int()
    a = G.swap_u8(crops[0::2].contiguous(), z[0:1]).cpu().int()
    b = G.swap_u8(crops[1::2].contiguous(), z[1:2]).cpu().int()
    assert int((mixed[0::2] - a).abs().max()) <= 1 and int((mixed[1::2] - b).abs().max()) <= 1


def test_half_module_and_half_input_keep_reference_dtypes(lib):
    """inference.py:30 G.half() and core.py:20-21 transform_target_to_torch(half=True): the reference
    hands fp16 in and gets fp16 out.  The drop-in computes with fp16 storage and returns float16 tensors
    (its numerics against the fp16-storage oracle: tests/test_bf16_parity.py)."""
    from ghost_amd.inference import transform_target_to_torch
    G = model("unet", 2).half()
    crops = aei_ref.make_u8_crops(2, 8)
    t = transform_target_to_torch(crops, half=True)
    assert t.dtype == torch.float16 and t.shape == (2, 3, 256, 256) and not t.is_contiguous()
    # (x/255 - 0.5)/0.5 as the reference computes it (fp32 /255, fp16 affine): within one fp16 ulp
    ref = ((torch.from_numpy(crops)[:, :, :, [2, 1, 0]] / 255.0).half().float() - 0.5) / 0.5
    assert float((t.float().cpu() - ref.permute(0, 3, 1, 2)).abs().max()) <= 2 ** -10
    _, z = aei_ref.make_inputs(2, 8)
    Y, attr = G(t, z.to(DEV).half())
    assert Y.dtype == torch.float16 and all(a.dtype == torch.float16 for a in attr)
    Gb = model("unet", 2, compute_dtype=torch.bfloat16).half()    # same fp16-rounded parameters, bf16 storage
    Yb, _ = Gb(t, z.to(DEV).half())
    assert Yb.dtype == torch.bfloat16
    G16 = model("unet", 2, compute_dtype=torch.float16)             # fp32 parameters, fp16 storage
    Y16, _ = G16(t, z.to(DEV).half())
    assert Y16.dtype == torch.float16
    d = (Y.float() - Y16.float()).abs()
    # the two fp16 plans differ only by the parameters' fp16 rounding, compounded through 8 blocks (measured
    # max 0.038 on these inputs)
    assert float(d.max()) <= 0.1 and float(d.mean()) <= 2e-3, (float(d.max()), float(d.mean()))
    assert float((Y.float() - Yb.float()).abs().mean()) <= 5e-2


def test_boundary_rejects_bad_out_and_host_embeddings(lib):
    G = model("unet", 2, compute_dtype=torch.bfloat16)
    crops = torch.from_numpy(aei_ref.make_u8_crops(2, 1)).to(DEV)
    _, z = aei_ref.make_inputs(2, 1)
    with pytest.raises(RuntimeError, match="z_id"):
        G.swap_u8(crops, z[:1])                      # host embedding next to device crops
    for bad in (torch.empty(1, 256, 256, 3, dtype=torch.uint8, device=DEV),
                torch.empty(2, 256, 256, 3, dtype=torch.float32, device=DEV),
                torch.empty(2, 256, 3, 256, dtype=torch.uint8, device=DEV).permute(0, 1, 3, 2)):
        with pytest.raises(RuntimeError, match="out must be"):
            G.swap_u8(crops, z[:1].to(DEV), out=bad)
    with pytest.raises(RuntimeError, match="z_id"):
        G(torch.zeros(2, 3, 256, 256, device=DEV), z)


def test_plan_options_read_back_from_the_handle(lib):
    """get_option reads the native handle: the measured defaults (include/ghost_amd.h) after the first
    forward, and what set_option wrote afterwards (bench.py sizes the roofline kernel's bytes from it)."""
    G = model("unet", 2, compute_dtype=torch.bfloat16)
    xt, z = aei_ref.make_inputs(1, 3)
    G(xt.to(DEV), z.to(DEV))
    assert {n: G.get_option(n) for n in ("fuse_upsample", "fuse_stats", "two_streams", "tap_partials")} == \
        {"fuse_upsample": 1, "fuse_stats": 1, "two_streams": 1, "tap_partials": 2}
    G.set_option("tap_partials", 1)
    assert G.get_option("tap_partials") == 1
    G.set_option("tap_partials", 2)
    with pytest.raises(ValueError):
        G.get_option("no_such_option")
