"""CPU tests of the host side: library exports, runtime plan / slot naming, weight packing.

No GPU compute here: the C ABI is exercised only through calls that touch no device
(handle creation, slot binding with dummy addresses, dry-run workspace sizing).  The
packed layouts are validated by replaying the kernels' index arithmetic with torch on
CPU and comparing against torch's own conv ops.
"""
import ctypes as C
import os

import pytest
import torch
import torch.nn.functional as F

from ghost_amd import _lib
from ghost_amd.network import pack
from oracle import aei_ref

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope="module")
def lib():
    from ghost_amd import build
    build.build(verbose=False)
    return _lib.load()


def test_library_exports_every_header_symbol(lib):
    declared = _lib.header_symbols()
    assert len(declared) >= 20
    for name in declared:
        assert hasattr(lib, name), name
    assert set(declared) == set(_lib._SIGS), "ctypes signature table out of sync with include/ghost_amd.h"


@pytest.mark.parametrize("backbone,nb", [("unet", 2), ("linknet", 3), ("unet", 1), ("unet", 3), ("resnet", 2)])
def test_pack_slots_match_runtime_plan(lib, backbone, nb):
    specs = aei_ref.param_specs(backbone, nb)
    sd = aei_ref.make_weights(specs)
    slots = pack.pack_all(sd, backbone, nb, 512, torch.bfloat16)
    h = C.c_void_p()
    _lib.check(lib.ghost_aei_create(backbone.encode(), nb, 512, _lib.BF16, C.byref(h)))
    try:
        n_before = lib.ghost_aei_missing(h)
        assert n_before == len(slots)
        for i, (name, t) in enumerate(slots.items()):
            _lib.check(lib.ghost_aei_bind(h, name.encode(), 0x100000 + 256 * i, t.numel()), name)
        assert lib.ghost_aei_missing(h) == 0
        assert lib.ghost_aei_bind(h, b"no.such.slot", 0x1000, 1) != 0
        # the identity table rows equal 2*sum(c_x) over the plan
        ntot = sum(2 * sd[f"{pre}.fc1.weight"].shape[0] for _, pre in pack.aad_plan(backbone, nb))
        assert slots["gen.id.w"].shape[0] == pack.rup(ntot, 128)
        for B in (1, 8, 64):
            assert lib.ghost_aei_workspace_bytes(h, B) > 0
            assert lib.ghost_aei_swap_workspace_bytes(h, B) > lib.ghost_aei_workspace_bytes(h, B)
    finally:
        lib.ghost_aei_destroy(h)


def test_resnet_module_state_dict_matches_oracle_specs():
    """AEI_Net('resnet') exposes the reference's 497 state_dict keys (resnet.py:81-149 names)."""
    from ghost_amd.network import AEI_Net
    sd = AEI_Net("resnet", num_blocks=2, c_id=512).state_dict()
    specs = aei_ref.param_specs("resnet", 2)
    assert [(k, tuple(v.shape)) for k, v in sd.items()] == [(k, tuple(s)) for k, s, _ in specs]


def test_create_rejects_bad_arguments(lib):
    h = C.c_void_p()
    assert lib.ghost_aei_create(b"vgg", 2, 512, 0, C.byref(h)) != 0
    assert b"backbone" in lib.ghost_last_error()
    assert lib.ghost_aei_create(b"unet", 0, 512, 0, C.byref(h)) != 0
    assert lib.ghost_aei_create(b"unet", 2, 512, 7, C.byref(h)) != 0


def _gemm_conv(x, wp, cout, k, stride, pad):
    """Replay the implicit GEMM on CPU: rows = output pixels, K = (channel block, tap, c)."""
    B, Cin, H, W = x.shape
    cols = F.unfold(x, k, padding=pad, stride=stride)          # [B, Cin*k*k, L] with (c, ky, kx) order
    L = cols.shape[-1]
    cols = cols.reshape(B, Cin // 32, 32, k * k, L).permute(0, 4, 1, 3, 2).reshape(B, L, k * k * Cin)
    y = cols @ wp[:cout, :k * k * Cin].t()
    Ho = (H + 2 * pad - k) // stride + 1
    return y.reshape(B, Ho, -1, cout).permute(0, 3, 1, 2)


def test_pack_conv_layout():
    g = torch.Generator().manual_seed(0)
    x = torch.randn(2, 32, 12, 12, generator=g, dtype=torch.float64)
    for (co, k, s, p) in [(40, 4, 2, 1), (24, 3, 1, 1), (16, 1, 1, 0)]:
        w = torch.randn(co, 32, k, k, generator=g, dtype=torch.float64)
        wp = pack.pack_conv(w, torch.float64)
        assert wp.shape == (pack.rup(co, 128), pack.rup(32 * k * k, 32))
        torch.testing.assert_close(_gemm_conv(x, wp, co, k, s, p), F.conv2d(x, w, stride=s, padding=p))


def test_pack_convT_subpixel_layout():
    g = torch.Generator().manual_seed(1)
    ci, co, H = 64, 24, 5
    x = torch.randn(2, ci, H, H, generator=g, dtype=torch.float64)
    w = torch.randn(ci, co, 4, 4, generator=g, dtype=torch.float64)
    wp = pack.pack_convT4x4(w, torch.float64)
    ref = F.conv_transpose2d(x, w, stride=2, padding=1)
    out = torch.zeros_like(ref)
    xp = F.pad(x, (1, 1, 1, 1))
    for py in range(2):
        for px in range(2):
            acc = torch.zeros(2, co, H, H, dtype=torch.float64)
            for ty in range(2):
                for tx in range(2):
                    dy, dx = py - ty, px - tx           # input offset = parity - tap (kernel tbase/tsign)
                    patch = xp[:, :, 1 + dy:1 + dy + H, 1 + dx:1 + dx + H]
                    t = ty * 2 + tx     # K order (cb, tap, c): gather this tap's channels block by block
                    wt = wp[2 * py + px, :co, :4 * ci].reshape(co, ci // 32, 4, 32)[:, :, t, :].reshape(co, ci)
                    acc += torch.einsum("bchw,oc->bohw", patch, wt)
            out[:, :, py::2, px::2] = acc
    torch.testing.assert_close(out, ref)


def test_pack_aad_interleave_and_bn_fold():
    sd = aei_ref.make_weights(aei_ref.param_specs("unet", 2))
    pre = "generator.AADBlk6.add_blocks.0"
    p = pack.pack_aad(sd, pre, torch.float32)
    c = sd[f"{pre}.conv1.weight"].shape[0]
    for col in range(2 * c):
        grp, r = divmod(col, 16)
        ch = (grp // 2) * 16 + r
        src = "conv1" if grp % 2 == 0 else "conv2"
        ca = sd[f"{pre}.conv1.weight"].shape[1]
        torch.testing.assert_close(p["gbw"][col, :ca],
                                   sd[f"{pre}.{src}.weight"][ch, :, 0, 0])
        assert float(p["gbb"][col]) == float(sd[f"{pre}.{src}.bias"][ch])
    s, t = pack.bn_fold(sd, "encoder.conv3.1", 128)
    x = torch.randn(4, 128, 3, 3)
    bn = F.batch_norm(x, sd["encoder.conv3.1.running_mean"], sd["encoder.conv3.1.running_var"],
                      sd["encoder.conv3.1.weight"], sd["encoder.conv3.1.bias"], False, 0.0, 1e-5)
    torch.testing.assert_close(x * s.view(1, -1, 1, 1) + t.view(1, -1, 1, 1), bn, atol=1e-5, rtol=1e-5)


def test_pack_up1_and_identity_table():
    sd = aei_ref.make_weights(aei_ref.param_specs("unet", 2))
    slots = pack.pack_all(sd, "unet", 2, 512, torch.float32)
    z = torch.randn(3, 512)
    ref = F.conv_transpose2d(z.reshape(3, 512, 1, 1), sd["generator.up1.weight"], sd["generator.up1.bias"])
    got = (z @ slots["gen.up1.w"][:, :512].t() + slots["gen.up1.shift"]).reshape(3, 2, 2, 1024).permute(0, 3, 1, 2)
    torch.testing.assert_close(got, ref, atol=1e-5, rtol=1e-5)
    tab = z @ slots["gen.id.w"][:, :512].t() + slots["gen.id.shift"]
    off = 0
    for _, pre in pack.aad_plan("unet", 2):
        c = sd[f"{pre}.fc1.weight"].shape[0]
        torch.testing.assert_close(tab[:, off:off + c], F.linear(z, sd[f"{pre}.fc1.weight"], sd[f"{pre}.fc1.bias"]),
                                   atol=1e-5, rtol=1e-5)
        torch.testing.assert_close(tab[:, off + c:off + 2 * c],
                                   F.linear(z, sd[f"{pre}.fc2.weight"], sd[f"{pre}.fc2.bias"]), atol=1e-5, rtol=1e-5)
        off += 2 * c


def test_module_state_dict_matches_reference_keys():
    from ghost_amd.network import AEI_Net
    for backbone, nb in [("unet", 2), ("linknet", 3), ("unet", 1)]:
        G = AEI_Net(backbone, num_blocks=nb, c_id=512)
        mine = [(k, tuple(v.shape)) for k, v in G.state_dict().items()]
        ref = [(k, tuple(s)) for k, s, _ in aei_ref.param_specs(backbone, nb)]
        assert mine == ref
        G.load_state_dict(aei_ref.make_weights(aei_ref.param_specs(backbone, nb)), strict=True)


def test_product_refuses_cpu_tensors():
    from ghost_amd.network import AEI_Net
    G = AEI_Net("unet", num_blocks=2, c_id=512).eval()
    with pytest.raises(RuntimeError, match="ROCm GPU"):
        G(torch.zeros(1, 3, 256, 256), torch.zeros(1, 512))
    with pytest.raises(NotImplementedError):
        G.generator.AADBlk1(torch.zeros(1), None, None)


def test_bench_roofline_bytes_follow_the_stored_outputs():
    """bench.py's minimum bytes of the aad_v4 launch: a tap-partial output is 15 fp16 per pixel, not 64 bf16."""
    import bench
    full, n0, z0 = bench.aad_v4_min_bytes(64, 64, 2, 2, 0)
    assert (n0, z0) == (0, 0) and full == 64 * (128 * 128 * 64 + 65536 * 64 * 3) * 2.0 == 1744830464.0
    part, n2, z2 = bench.aad_v4_min_bytes(64, 64, 2, 2, 2)
    assert (n2, z2) == (1, 2) and full - part == 64 * 65536 * (64 - 15) * 2.0
    assert bench.aad_v4_min_bytes(64, 64, 2, 2, 1)[1:] == (0, 0)          # mode 1: partials in the later layer
    assert bench.aad_v4_min_bytes(64, 32, 2, 1, 2)[1:] == (2, 3)          # nb = 1: both layers feed the RGB conv
    assert bench.aad_v4_min_bytes(64, 32, 2, 1, 1)[1:] == (1, 1)


def test_bench_profile_lookups_match_the_launched_symbol():
    """bench.py finds the roofline kernel's rows in the committed rocprof / PMC summaries by its Itanium
    symbol (the launched instantiation carries the storage type and the ASMW flag)."""
    import bench
    assert bench.mangle("aad_v5_kernel<__bf16, 64, 2, true, 2, true>") == "aad_v5_kernelIDF16bLi64ELi2ELb1ELi2ELb1EE"
    assert bench.mangle("aad_v4_kernel<64, 2, true, true, 2>") == "aad_v4_kernelILi64ELi2ELb1ELb1ELi2EE"
    assert bench.mangle("k<_Float16, false>") == "kIDF16_Lb0EE"


def test_pack_invalidation_rules():
    """_packed.PackedModule: the cached pack survives plain calls and is dropped by every edit it claims to see
    (in-place edits, parameter / buffer / submodule replacement anywhere in the tree, .to/.half of a submodule,
    load_state_dict); ADVICE r03."""
    import copy

    from ghost_amd.network import AEI_Net
    G = AEI_Net("unet", num_blocks=1, c_id=512)
    dev = torch.device("cpu")
    built = []

    def get():
        return G._cached_runtime(dev, torch.float32, lambda sd: built.append(object()) or built[-1])

    def _inplace(p, v):
        with torch.no_grad():
            p.add_(v)

    rt = get()
    assert get() is rt and len(built) == 1
    cases = [
        lambda: _inplace(G.generator.up1.weight, 0.0),                      # in-place: version counter
        lambda: setattr(G.encoder.conv1[0], "weight", torch.nn.Parameter(torch.zeros_like(G.encoder.conv1[0].weight))),
        lambda: G.encoder.conv1[1].register_buffer("running_mean", torch.zeros_like(G.encoder.conv1[1].running_mean)),
        lambda: G.generator.AADBlk1.to(torch.float64),                     # .to on a submodule only
        lambda: G.to(torch.float32),
        lambda: setattr(G.encoder, "conv1", copy.deepcopy(G.encoder.conv1)),   # submodule replaced
        lambda: _inplace(G.encoder.conv1[0].weight, 0.0),                # ... and the new one is owned
        lambda: G.load_state_dict(G.state_dict()),
    ]
    for i, edit in enumerate(cases):
        edit()
        rt2 = get()
        assert rt2 is not rt, f"edit {i} did not invalidate the pack"
        rt = rt2
        assert get() is rt
    assert G._pack_current(rt) and not G._pack_current(object())
    G.invalidate_pack()
    assert get() is not rt


def test_host_code_under_address_sanitizer():
    """SURVEY.md §5 (race detection / sanitizers): the native library's host code — handle creation, the plan's dry
    run and bump allocator at every backbone / num_blocks / dtype / batch size, argument validation, the face-mask
    polygon code — run under AddressSanitizer + UBSan (tools/asan_host.sh builds build/asan/host_main with
    -Xarch_host -fsanitize=address,undefined; CPU only).  Skipped when that binary has not been built here."""
    import subprocess
    exe = os.path.join(REPO, "build", "asan", "host_main")
    if not os.path.exists(exe):
        pytest.skip("build/asan/host_main not built (bash tools/asan_host.sh)")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=300,
                       env=dict(os.environ, ASAN_OPTIONS="detect_leaks=1", UBSAN_OPTIONS="halt_on_error=1"))
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-4000:])
    assert "0 failed checks" in r.stdout and "ERROR: AddressSanitizer" not in r.stderr
