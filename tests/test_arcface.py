"""ArcFace (IResNet) identity encoder: host-side checks on CPU, the HIP path against the oracle on GPU.

PARITY UNPINNED: the reference tree does not contain arcface_model/iresnet.py (a download,
download_models.sh:3) nor its weights, so the oracle (oracle/arcface_ref.py) is a restatement of the
public arcface_torch IResNet and these tests prove self-consistency of the HIP path with it.  The
pipeline arithmetic around the network (normalize_and_torch_batch, the 0.5x align_corners resize,
face matching) is restated from the reference files cited in the oracle.

Gates: fp32 path max|d emb| <= 2e-3 * max|emb| and cosine >= 0.99999 per row (100 residual blocks
of fp32 MFMA in a different summation order).  bf16 path: against the storage-emulating oracle
(arcface_ref.iresnet_forward_storage: every tensor the runtime stores rounded to bf16 where it stores
it), per stage teacher-forced — the stem and every IBasicBlock recomputed from the GPU's own stored
inputs must match the GPU's stored (X, BN(X)) within 2 bf16 ulps of max|ref| and a mean of 5e-3 of
mean|ref|, the head's embedding within 1e-3 relative — and end to end no further from the fp32
forward than the emulated bf16 arithmetic itself (1.25x in the mean and the max).
"""
import ctypes as C

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from ghost_amd import _lib
from oracle import arcface_ref as A

DEV = torch.device("cuda:0")
_W = {}


def weights(arch="iresnet100"):
    if arch not in _W:
        _W[arch] = A.make_weights(A.param_specs(A.LAYERS[arch]))
    return _W[arch]


def net(arch="iresnet100", compute_dtype=None):
    from ghost_amd import arcface
    m = getattr(arcface, arch)(fp16=False, compute_dtype=compute_dtype).eval()
    m.load_state_dict(weights(arch))
    return m.to(DEV)


# ------------------------------------------------------------------------------------------ CPU
@pytest.mark.parametrize("arch", ["iresnet18", "iresnet50", "iresnet100"])
def test_state_dict_matches_arcface_torch_layout(arch):
    from ghost_amd import arcface
    sd = getattr(arcface, arch)().state_dict()
    specs = A.param_specs(A.LAYERS[arch])
    assert [(k, tuple(v.shape)) for k, v in sd.items()] == [(k, tuple(s)) for k, s, _ in specs]


@pytest.mark.parametrize("arch", ["iresnet18", "iresnet100"])
def test_pack_slots_match_native_plan(arch):
    from ghost_amd.arcface.pack import pack_iresnet
    lib = _lib.load()
    layers = A.LAYERS[arch]
    slots = pack_iresnet(weights(arch), layers, torch.bfloat16)
    h = C.c_void_p()
    _lib.check(lib.ghost_arc_create((C.c_int * 4)(*layers), 512, _lib.BF16, C.byref(h)))
    try:
        assert lib.ghost_arc_missing(h) == len(slots)
        for i, (name, t) in enumerate(slots.items()):
            _lib.check(lib.ghost_arc_bind(h, name.encode(), 0x100000 + 256 * i, t.numel()), name)
        assert lib.ghost_arc_missing(h) == 0
        assert lib.ghost_arc_bind(h, b"no.such.slot", 0x1000, 1) != 0
        for n in (1, 8, 64):
            assert lib.ghost_arc_workspace_bytes(h, n) > n * 112 * 112 * 64 * 2 * 5
    finally:
        lib.ghost_arc_destroy(h)


def test_create_rejects_bad_arguments():
    lib = _lib.load()
    h = C.c_void_p()
    assert lib.ghost_arc_create((C.c_int * 4)(3, 0, 30, 3), 512, 0, C.byref(h)) != 0
    assert lib.ghost_arc_create((C.c_int * 4)(3, 13, 30, 3), 500, 0, C.byref(h)) != 0
    assert lib.ghost_arc_create((C.c_int * 4)(3, 13, 30, 3), 512, 9, C.byref(h)) != 0


def test_head_as_valid_conv_equals_flatten_fc_bn():
    """The packed head (7x7 valid conv over NHWC bn2(x), BN1d folded) == flatten -> fc -> features."""
    from ghost_amd.arcface.pack import pack_iresnet
    p = weights("iresnet18")
    slots = pack_iresnet(p, A.LAYERS["iresnet18"], torch.float32)
    g = torch.Generator().manual_seed(0)
    xb = torch.randn(3, 512, 7, 7, generator=g)            # = bn2(x)
    ref = F.batch_norm(F.linear(torch.flatten(xb, 1), p["fc.weight"], p["fc.bias"]), p["features.running_mean"],
                       p["features.running_var"], p["features.weight"], p["features.bias"], False, 0.0, 1e-5)
    # pack_conv K order for Cin % 32 == 0: (channel block of 32, tap, channel)
    cols = xb.reshape(3, 16, 32, 49).permute(0, 1, 3, 2).reshape(3, 512 * 49)
    got = cols @ slots["fc.w"][:512, :512 * 49].t() * slots["fc.scale"][:512] + slots["fc.shift"][:512]
    assert float((got - ref).abs().max()) <= 1e-4 * float(ref.abs().max())


def test_oracle_preprocess_follows_reference_semantics():
    """normalize_and_torch_batch divides by 255 only when the batch max exceeds 1."""
    f = np.zeros((2, 4, 4, 3), np.uint8)
    f[0, 0, 0, 0] = 1
    assert float(A.normalize_batch_u8(f).max()) == 1.0      # (1 - 0.5)/0.5, no /255
    f[1, 1, 1, 1] = 2
    assert abs(float(A.normalize_batch_u8(f).max()) - ((2 / 255 - 0.5) / 0.5)) < 1e-7


# ------------------------------------------------------------------------------------------ GPU
def _close(got, ref, rel, cos_min):
    d = float((got - ref).abs().max())
    assert d <= rel * float(ref.abs().max()), (d, float(ref.abs().max()))
    cos = F.cosine_similarity(got, ref, dim=1)
    assert float(cos.min()) >= cos_min, cos


@pytest.mark.gpu
@pytest.mark.parametrize("arch", ["iresnet18", "iresnet100"])
def test_forward_fp32_vs_oracle(arch):
    m = net(arch)
    x = torch.from_numpy(np.random.Generator(np.random.PCG64(4)).uniform(-1, 1, (3, 3, 112, 112)).astype(np.float32))
    emb = m(x.to(DEV)).cpu()
    ref = A.iresnet_forward(weights(arch), x, A.LAYERS[arch])
    _close(emb, ref, 2e-3, 0.99999)


@pytest.mark.gpu
def test_embed_u8_fp32_vs_oracle_and_strided_input():
    m = net()
    crops = A.make_u8_faces(4, seed=9)
    emb = m.embed_u8(torch.from_numpy(crops).to(DEV)).cpu()
    ref = A.embed_crops(weights("iresnet100"), crops)
    _close(emb, ref, 2e-3, 0.99999)
    # the module call on the reference's own preprocessing (a permuted, non-contiguous view)
    from ghost_amd.arcface import normalize_and_torch_batch
    x = F.interpolate(normalize_and_torch_batch(crops).float(), scale_factor=0.5, mode="bilinear",
                      align_corners=True)
    emb2 = m(x).cpu()
    _close(emb2, ref, 2e-3, 0.99999)


@pytest.mark.gpu
def test_embed_u8_batch_without_values_above_one():
    """A batch whose max is <= 1 is not divided by 255 (image_processing.py:42-43)."""
    m = net("iresnet18")
    crops = (np.random.Generator(np.random.PCG64(2)).uniform(size=(2, 224, 224, 3)) > 0.5).astype(np.uint8)
    emb = m.embed_u8(torch.from_numpy(crops).to(DEV)).cpu()
    ref = A.embed_crops(weights("iresnet18"), crops, A.LAYERS["iresnet18"])
    _close(emb, ref, 2e-3, 0.99999)


def _ulp_bf16(x):
    return 2.0 ** (np.floor(np.log2(max(x, 1e-30))) - 7)


def _stage_close(g, r, what):
    d = (g - r).abs()
    assert float(d.max()) <= 2 * _ulp_bf16(float(r.abs().max())), (what, float(d.max()), float(r.abs().max()))
    assert float(d.mean()) <= 5e-3 * float(r.abs().mean()), (what, float(d.mean()), float(r.abs().mean()))


@pytest.mark.gpu
@pytest.mark.parametrize("arch,B", [("iresnet18", 2), ("iresnet100", 2), ("iresnet100", 128), ("iresnet100", 256)])
def test_bf16_each_stage_matches_storage_emulation(arch, B):
    """Bisection by construction: each stage from the GPU's own stored inputs (ghost_arc_set_taps).  B = 128
    runs the two-sample halo window (HaloPair) at 56x56 / 28x28 / 14x14, B = 256 also the deep LDS-DMA ring at
    7x7 (M = 12 544); two rows of each are checked."""
    m = net(arch, compute_dtype=torch.bfloat16)
    layers, p = A.LAYERS[arch], weights(arch)
    x = torch.from_numpy(np.random.Generator(np.random.PCG64(6)).uniform(-1, 1, (B, 3, 112, 112)).astype(np.float32))
    emb, taps = m.forward_taps(x.to(DEV))
    torch.cuda.synchronize()
    rows = torch.tensor([0, 1] if B == 2 else [0, 77] if B == 128 else [0, 201])
    x = x[rows]
    emb = emb[rows.to(DEV)].cpu()
    assert emb.dtype == torch.float32 and taps[0][0].dtype == torch.bfloat16
    taps = [(a[rows.to(DEV)].float().cpu(), b[rows.to(DEV)].float().cpu()) for a, b in taps]
    nb = A.next_bn_names(layers)
    with torch.no_grad():
        X, XB = A.stem_storage(p, x.bfloat16().float(), torch.bfloat16, nb[0])
        _stage_close(taps[0][0], X, "stem X")
        _stage_close(taps[0][1], XB, "stem XB")
        for i, (li, b, _inp, _planes, stride) in enumerate(A.blocks(layers)):
            X, XB = A.block_storage(p, taps[i][0], taps[i][1], li, b, stride, nb[i + 1])
            _stage_close(taps[i + 1][0], X, f"layer{li}.{b} X")
            _stage_close(taps[i + 1][1], XB, f"layer{li}.{b} XB")
        head = A.head_storage(p, taps[-1][1])
    assert float((emb - head).abs().max()) <= 1e-3 * float(head.abs().max())


@pytest.mark.gpu
def test_bf16_end_to_end_error_is_the_intrinsic_storage_error():
    m = net(compute_dtype=torch.bfloat16)
    p = weights("iresnet100")
    crops = A.make_u8_faces(4, seed=5)
    emb = m.embed_u8(torch.from_numpy(crops).to(DEV)).cpu()
    assert emb.dtype == torch.float32
    ref = A.embed_crops(p, crops)
    with torch.no_grad():
        emu, _ = A.iresnet_forward_storage(p, A.preprocess_crops(crops))
    dg, de = (emb - ref).abs(), (emu - ref).abs()
    assert float(dg.mean()) <= 1.25 * float(de.mean()), (float(dg.mean()), float(de.mean()))
    assert float(dg.max()) <= 1.25 * float(de.max()), (float(dg.max()), float(de.max()))
    assert float(F.cosine_similarity(emb, ref, dim=1).min()) >= 0.999


@pytest.mark.gpu
def test_match_faces_vs_oracle():
    from ghost_amd.arcface import match_faces
    g = torch.Generator().manual_seed(3)
    faces = torch.randn(7, 512, generator=g)
    targets = torch.cat([faces[[4, 1]] * 2.5 + 0.01 * torch.randn(2, 512, generator=g),
                         torch.randn(2, 512, generator=g)])
    faces[6] = faces[4]                                     # tie: the first index wins
    best, sim, ok = match_faces(faces.to(DEV), targets.to(DEV), 0.15)
    rb, rs, rok = A.match_faces(faces, targets, 0.15)
    assert best.cpu().tolist() == rb.tolist()
    assert torch.allclose(sim.cpu(), rs, atol=1e-5)
    assert ok.cpu().tolist() == rok.tolist()


@pytest.mark.gpu
def test_embed_batch_permutation_is_exact():
    """All 128 rows: a permuted batch gives the permuted embeddings bit for bit (the paired halo window,
    overhanging tiles and per-sample records must not mix rows)."""
    m = net(compute_dtype=torch.bfloat16)
    crops = torch.from_numpy(np.random.Generator(np.random.PCG64(12)).integers(0, 256, (128, 224, 224, 3),
                                                                              dtype=np.uint8)).to(DEV)
    perm = torch.randperm(128, generator=torch.Generator().manual_seed(2)).to(DEV)
    e = m.embed_u8(crops)
    ep = m.embed_u8(crops[perm].contiguous())
    torch.cuda.synchronize()
    assert torch.equal(ep, e[perm])
