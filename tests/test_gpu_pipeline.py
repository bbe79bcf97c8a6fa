"""GPU tests of the per-frame loop around the generator (SURVEY.md §8a row a13,
utils/inference/core.py:57-88) and of the multi-identity batch (BASELINE config 5), with the real
AEI_Net on the device:

* ``swap_identity_frames`` (core.py:57-88 for one identity): H2D of the crops, BS-sized swaps, the
  per-batch D2H (faceshifter_run.py:22) and the ``present`` re-insertion (core.py:79-88) — against a
  one-shot ``swap_u8`` and, for two frames, the fp32 oracle's faceshifter_batch bytes;
* ``model_inference_dp`` over a one-rank RCCL process group (its all-gather runs through RCCL on the
  device; the multi-rank ordering is covered by tests/test_dp_cpu.py on gloo);
* config 5: linknet/3, four identities mixed in one bf16 batch through per-sample z_id rows,
  against single-identity batches of the same size and, for two rows, the fp32 oracle with the
  bf16-storage emulation as the error yardstick (the gate of tests/test_gpu_parity.py).
"""
import socket

import numpy as np
import pytest
import torch

from oracle import aei_ref

pytestmark = pytest.mark.gpu
DEV = torch.device("cuda:0")


@pytest.fixture(scope="module")
def lib():
    from ghost_amd import _lib
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return _lib.load()


_W = {}


def model(backbone, nb, compute_dtype=None):
    from ghost_amd.network import AEI_Net
    if (backbone, nb) not in _W:
        _W[(backbone, nb)] = aei_ref.make_weights(aei_ref.param_specs(backbone, nb))
    G = AEI_Net(backbone, num_blocks=nb, c_id=512, compute_dtype=compute_dtype).eval()
    G.load_state_dict(_W[(backbone, nb)])
    return G.to(DEV), _W[(backbone, nb)]


PRESENT = [1, 0, 1, 1, 0, 0, 1, 1]      # 5 frames with a face among 8


def u8_close(a, b, max_lsb=1, frac=1e-3):
    d = np.abs(a.astype(np.int16) - b.astype(np.int16))
    assert d.max() <= max_lsb and (d > 0).mean() < frac, (int(d.max()), float((d > 0).mean()))


def test_swap_identity_frames_fp32(lib):
    from ghost_amd.inference.core import swap_identity_frames
    G, p = model("unet", 2)
    crops = aei_ref.make_u8_crops(sum(PRESENT), 31)
    _, z = aei_ref.make_inputs(1, 31)
    final, dev_out = swap_identity_frames(crops, PRESENT, z.to(DEV), G, BS=2, return_device=True)
    assert len(final) == len(PRESENT)
    assert [isinstance(f, list) and f == [] for f in final] == [pr == 0 for pr in PRESENT]
    swapped = np.stack([f for f in final if not isinstance(f, list)])
    assert swapped.shape == (5, 256, 256, 3) and swapped.dtype == np.uint8
    assert np.array_equal(swapped, dev_out.cpu().numpy())          # the D2H copies carry the device bytes
    one = G.swap_u8(torch.from_numpy(crops).to(DEV), z.to(DEV)).cpu().numpy()
    u8_close(swapped, one)                                          # batches of 2 == one batch of 5
    rows = [0, 4]                                                   # a first-batch and the short last batch frame
    y = aei_ref.aei_forward(p, aei_ref.transform_target(crops[rows]), z.expand(len(rows), -1), "unet", 2)[0]
    u8_close(swapped[rows], aei_ref.y_to_u8_bgr(y))


def test_swap_identity_frames_no_face(lib):
    from ghost_amd.inference.core import swap_identity_frames
    G, _ = model("unet", 2)
    _, z = aei_ref.make_inputs(1, 3)
    final = swap_identity_frames(np.zeros((0, 256, 256, 3), np.uint8), [0, 0, 0], z.to(DEV), G, BS=4)
    assert final == [[], [], []]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def test_model_inference_dp_rccl_one_rank(lib):
    """dp.model_inference_dp with the real G over a one-rank RCCL group: shard, swap in BS batches,
    all_gather_into_tensor on the device, the per-frame list — the bytes of swap_identity_frames."""
    import torch.distributed as dist
    from ghost_amd.inference.core import swap_identity_frames
    from ghost_amd.inference.dp import GatherPipeline, model_inference_dp
    G, _ = model("unet", 2, torch.bfloat16)
    crops = aei_ref.make_u8_crops(sum(PRESENT), 17)
    _, z = aei_ref.make_inputs(1, 17)
    zd = z.to(DEV)
    ref = swap_identity_frames(crops, PRESENT, zd, G, BS=2)
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1)
    try:
        assert dist.get_backend() == "nccl"
        got = model_inference_dp(crops, PRESENT, zd, G, BS=2)
        assert len(got) == len(ref)
        for a, b in zip(got, ref):
            if isinstance(b, list):
                assert a == []
            else:
                assert np.array_equal(a, b)
        # the batch stream of bench.py: tickets, a short last batch with counts
        dc = torch.from_numpy(crops).to(DEV)
        pipe = GatherPipeline(lambda c, o: G.swap_u8(c, zd, out=o), (2, 256, 256, 3), DEV, depth=2)
        t0 = pipe.submit(dc[0:2])
        t1 = pipe.submit(dc[2:4])
        first = pipe.result(t0).cpu().numpy()
        t2 = pipe.submit(dc[4:5], counts=[1])
        last = pipe.result(t2).cpu().numpy()
        with pytest.raises(RuntimeError, match="overwritten"):
            pipe.result(t0)
        mid = pipe.result(t1).cpu().numpy()
        pipe.drain()
        swapped = np.stack([f for f in ref if not isinstance(f, list)])
        assert np.array_equal(np.concatenate([first, mid, last]), swapped)
    finally:
        dist.destroy_process_group()


def test_config5_linknet3_four_identities_bf16(lib):
    """BASELINE config 5's batch: linknet/3, four identities interleaved in one B = 8 bf16 batch via
    per-sample z_id rows (dp.swap_mixed_identities) == the same crops swapped with one identity at a
    time (same batch size, so the same kernels); two rows against the fp32 oracle."""
    from ghost_amd.inference.dp import swap_mixed_identities
    G, p = model("linknet", 3, torch.bfloat16)
    B, nid = 8, 4
    crops_np = aei_ref.make_u8_crops(B, 41)
    crops = torch.from_numpy(crops_np).to(DEV)
    _, zs = aei_ref.make_inputs(nid, 41)
    idx = torch.arange(B) % nid
    mixed = swap_mixed_identities(crops, idx.to(DEV), zs.to(DEV), G).cpu().numpy()
    for i in range(nid):
        zi = zs[i:i + 1].expand(B, -1).contiguous().to(DEV)     # B identical rows: the mixed path's z layout
        single = G.swap_u8(crops, zi).cpu().numpy()
        rows = (idx == i).numpy()
        u8_close(mixed[rows], single[rows], max_lsb=1, frac=1e-4)
    # two rows (identities 0 and 1) against the fp32 oracle: no further from it than bf16 storage is
    rows = [0, 5]
    xt = aei_ref.transform_target(crops_np[rows])
    zr = zs[idx[rows]]
    ref = aei_ref.aei_forward(p, xt, zr, "linknet", 3)[0]
    emu = aei_ref.aei_forward_bf16_storage(p, xt, zr, "linknet", 3)[0]
    d_gpu = np.abs(mixed[rows].astype(np.int16) - aei_ref.y_to_u8_bgr(ref).astype(np.int16))
    d_emu = np.abs(aei_ref.y_to_u8_bgr(emu).astype(np.int16) - aei_ref.y_to_u8_bgr(ref).astype(np.int16))
    assert d_gpu.mean() <= 1.25 * d_emu.mean() + 0.05, (float(d_gpu.mean()), float(d_emu.mean()))
    k = max(1, d_gpu.size // 200)
    tg = np.sort(d_gpu, axis=None)[-k:].mean()
    te = np.sort(d_emu, axis=None)[-k:].mean()
    assert tg <= 1.3 * te + 1.0, (float(tg), float(te))


def _up_stream(G):
    """The up-path stream this module's handle has used on cuda:0 (NULL until its first two-stream call)."""
    import ctypes as C
    ptr = C.c_void_p()
    G._rt.lib.ghost_aei_up_stream(G._rt.h, 0, C.byref(ptr))
    return ptr.value


@pytest.mark.parametrize("backbone,nb,B", [("unet", 2, 8), ("unet", 2, 64), ("linknet", 3, 8)])
def test_two_stream_plan_is_bit_identical(lib, backbone, nb, B):
    """GHOST_AEI_OPT_TWO_STREAMS: the encoder's up path and the identity projections on the shared up-path stream
    give the same bytes as the one-stream plan (forward outputs, attrs and the uint8 swap).  B >= 8, where the plan
    really splits (batches of fewer than 8 frames run on one stream whatever the option says): the handle has used
    the up-path stream after the two-stream calls and not before (at B = 2 / 4 this test
    compared the one-stream plan with itself)."""
    G, _ = model(backbone, nb, torch.bfloat16)
    xt, z = aei_ref.make_inputs(B, 23)
    crops = torch.from_numpy(aei_ref.make_u8_crops(B, 23)).to(DEV)
    res = {}
    for mode in (0, 1):
        G.set_option("two_streams", mode)
        Y, attr = G(xt.to(DEV), z.to(DEV))
        u8 = G.swap_u8(crops, z.to(DEV))
        torch.cuda.synchronize()
        res[mode] = (Y.clone(), [a.clone() for a in attr], u8.clone())
        assert bool(_up_stream(G)) == (mode == 1), mode
    assert torch.equal(res[0][0], res[1][0])
    assert all(torch.equal(a, b) for a, b in zip(res[0][1], res[1][1]))
    assert torch.equal(res[0][2], res[1][2])


@pytest.mark.parametrize("backbone,nb,dt,B,ts", [("unet", 2, torch.bfloat16, 1, 1), ("unet", 2, torch.bfloat16, 64, 1),
                                                 ("linknet", 3, torch.float16, 8, 1), ("unet", 2, None, 2, 1),
                                                 ("unet", 1, torch.bfloat16, 3, 1), ("unet", 2, torch.bfloat16, 8, 0)])
def test_fused_reductions_are_bit_identical(lib, backbone, nb, dt, B, ts):
    """GHOST_AEI_OPT_FUSE_REDUCE: split-K GEMMs summing their partials in the last workgroup of each tile, and
    the InstanceNorm partial kernels merging per sample in their last workgroup, give the bytes of the separate
    reduction kernels (forward outputs, attrs, the uint8 swap), call after call (the arrival counters are
    reused by every launch of a stream and must be left at zero)."""
    G, _ = model(backbone, nb, dt)
    G.set_option("two_streams", ts)
    xt, z = aei_ref.make_inputs(B, 31)
    crops = torch.from_numpy(aei_ref.make_u8_crops(B, 31)).to(DEV)
    res = {}
    for mode in (0, 1, 1):
        G.set_option("fuse_reduce", mode)
        Y, attr = G(xt.to(DEV), z.to(DEV))
        u8 = G.swap_u8(crops, z.to(DEV))
        torch.cuda.synchronize()
        got = (Y.clone(), [a.clone() for a in attr], u8.clone())
        if mode in res:
            assert torch.equal(res[mode][0], got[0]) and torch.equal(res[mode][2], got[2])
        res[mode] = got
    assert G.get_option("fuse_reduce") == 1
    assert torch.equal(res[0][0], res[1][0])
    assert all(torch.equal(a, b) for a, b in zip(res[0][1], res[1][1]))
    assert torch.equal(res[0][2], res[1][2])


@pytest.mark.parametrize("dt", [torch.bfloat16, torch.float16])
def test_swap_into_unaligned_output_views(lib, dt):
    """The RGB conv's gather (tap_sum3x3 over the row-summed tap partials) stores whole dwords only where the
    caller's buffer allows: a uint8 out= view starting 1 byte into its storage gets the same bytes as a fresh
    tensor, and forward's out_u8 likewise."""
    G, _ = model("unet", 2, dt)
    B = 3
    xt, z = aei_ref.make_inputs(B, 37)
    crops = torch.from_numpy(aei_ref.make_u8_crops(B, 37)).to(DEV)
    ref = G.swap_u8(crops, z.to(DEV)).clone()
    n = B * 256 * 256 * 3
    for off in (1, 2, 4):
        buf = torch.full((n + 8,), 7, dtype=torch.uint8, device=DEV)
        view = buf[off:off + n].view(B, 256, 256, 3)
        got = G.swap_u8(crops, z.to(DEV), out=view)
        torch.cuda.synchronize()
        assert got.data_ptr() == view.data_ptr()
        assert torch.equal(got, ref), off
        assert bool((buf[:off] == 7).all()) and bool((buf[off + n:] == 7).all()), off   # nothing outside the view
    o0 = torch.empty(B, 256, 256, 3, dtype=torch.uint8, device=DEV)
    Y0, _ = G(xt.to(DEV), z.to(DEV), out_u8=o0)
    buf = torch.zeros(n + 4, dtype=torch.uint8, device=DEV)
    o1 = buf[3:3 + n].view(B, 256, 256, 3)
    Y1, _ = G(xt.to(DEV), z.to(DEV), out_u8=o1)
    torch.cuda.synchronize()
    assert torch.equal(Y0, Y1) and torch.equal(o0, o1)


@pytest.mark.parametrize("B,nb,indexed", [(4, 5, False), (8, 5, True), (64, 4, True), (64, 3, False)])
def test_gather_pipeline_two_batches_in_flight(lib, B, nb, indexed):
    """dp.GatherPipeline(streams=2) (bench.py's default): consecutive batches swapped on two pipeline streams at
    once (sharing one AEI_Net handle and, at B >= 8, the process's up-path stream) give the bytes of one-at-a-time
    swap_u8 calls, batch by batch, including a short last batch; results read on the caller's stream after the
    batch's stream.  indexed: the headline configuration itself — swap_u8_indexed through the
    identity table built before the loop (bench.py's step), against serial swap_u8 with the z row projected per
    batch (faceshifter_run.py:15-19)."""
    from ghost_amd.inference.dp import GatherPipeline
    G, _ = model("unet", 2, torch.bfloat16)
    crops = torch.from_numpy(aei_ref.make_u8_crops(B * nb - 1, 29)).to(DEV)
    _, z = aei_ref.make_inputs(1, 29)
    zd = z.to(DEV)
    ref = [G.swap_u8(crops[i:i + B], zd).clone() for i in range(0, crops.shape[0], B)]
    torch.cuda.synchronize()
    if indexed:
        table = G.identity_table(zd)
        idx = torch.zeros(B, dtype=torch.int32, device=DEV)

        def swap(c, o):
            return G.swap_u8_indexed(c, table, idx[:c.shape[0]], out=o)
    else:
        def swap(c, o):
            return G.swap_u8(c, zd, out=o)
    pipe = GatherPipeline(swap, (B, 256, 256, 3), DEV, depth=2, streams=2)
    assert pipe.depth == 2 and pipe.nstreams == 2
    for rep in range(2):                       # the second pass reuses both slots and both streams
        got = []
        pending = []
        for i in range(0, crops.shape[0], B):
            c = crops[i:i + B]
            pending.append(pipe.submit(c, counts=[c.shape[0]] if c.shape[0] < B else None))
            if len(pending) == 2:                  # read batch k once k + 1 is in flight
                got.append(pipe.result(pending.pop(0)).clone())
        got += [pipe.result(t).clone() for t in pending]
        pipe.drain()
        torch.cuda.synchronize()
        assert len(got) == len(ref)
        for k, (a, b) in enumerate(zip(got, ref)):
            assert torch.equal(a, b), (rep, k)


@pytest.mark.parametrize("dt,B", [(None, 1), (torch.bfloat16, 1), (torch.bfloat16, 4), (torch.float16, 2),
                                  (torch.bfloat16, 8), (torch.float16, 8)])
def test_graphed_swap_is_bit_identical(lib, dt, B):
    """GraphedSwap (one HIP graph replay of the whole native plan, captured as one chain — the default — or with
    the two-stream plan) gives the bytes of an eager swap_u8, for new inputs copied into the captured buffers on
    every call; the capture leaves the module's own two_streams option as it was.  The plan runs batches of fewer
    than 8 frames on one stream, so only B = 8 captures the cross-stream events and the up-path branch."""
    from ghost_amd.inference import GraphedSwap
    G, _p = model("unet", 2, dt)
    g = GraphedSwap(G, B, DEV)
    g2 = GraphedSwap(G, B, DEV, two_streams=1)
    assert G.get_option("two_streams") == 1
    for seed in (3, 4):
        crops = torch.from_numpy(aei_ref.make_u8_crops(B, seed)).to(DEV)
        z = torch.randn(1, 512, generator=torch.Generator().manual_seed(seed)).to(DEV)
        got2 = g2(crops, z).clone()
        ref = G.swap_u8(crops, z)
        torch.cuda.synchronize()
        assert torch.equal(got2, ref)
    for seed in (3, 4):
        crops = torch.from_numpy(aei_ref.make_u8_crops(B, seed)).to(DEV)
        z = torch.randn(1, 512, generator=torch.Generator().manual_seed(seed)).to(DEV)
        got = g(crops, z).clone()
        ref = G.swap_u8(crops, z)
        torch.cuda.synchronize()
        assert torch.equal(got, ref)


def test_graphed_swap_refuses_a_repacked_module(lib):
    """after the module is re-packed (here load_state_dict), a replay would read the old runtime's
    weights; GraphedSwap keeps that runtime alive and raises instead of returning bytes."""
    from ghost_amd.inference import GraphedSwap
    G, p = model("unet", 2, torch.bfloat16)
    g = GraphedSwap(G, 1, DEV)
    crops = torch.from_numpy(aei_ref.make_u8_crops(1, 5)).to(DEV)
    z = torch.randn(1, 512, generator=torch.Generator().manual_seed(5)).to(DEV)
    g(crops, z)
    G.load_state_dict(p)
    G.swap_u8(crops, z)                      # the eager call re-packs
    with pytest.raises(RuntimeError, match="re-packed"):
        g(crops, z)


def test_resize_frames_on_device(lib):
    """video_processing.py:174-188 on the device: present from the [] entries, the 224 -> 256 cv2 INTER_LINEAR
    resize bit-exact against the OpenCV fixed-point restatement (oracle/blend_ref.resize_linear_u8; cv2 itself is
    absent: parity against cv2 unpinned), and swap_crop_frames == swap_identity_frames on those crops."""
    from oracle import blend_ref as R
    from ghost_amd.inference.core import resize_frames, swap_crop_frames, swap_identity_frames
    g = np.random.default_rng(12)
    crops224 = g.integers(0, 256, (sum(PRESENT), 224, 224, 3), dtype=np.uint8)
    it = iter(crops224)
    crop_frames = [next(it) if p else [] for p in PRESENT]
    dev_crops, present = resize_frames(crop_frames, device=DEV)
    assert present.tolist() == [float(p) for p in PRESENT]
    ref = np.stack([R.resize_linear_u8(c, (256, 256)) for c in crops224])
    assert np.array_equal(dev_crops.cpu().numpy(), ref)
    G, _ = model("unet", 2, torch.bfloat16)
    _, z = aei_ref.make_inputs(1, 12)
    a = swap_crop_frames(crop_frames, z.to(DEV), G, BS=3)
    b = swap_identity_frames(ref, present, z.to(DEV), G, BS=3)
    assert len(a) == len(b)
    for x, y in zip(a, b):
        assert (x == [] and y == []) if isinstance(y, list) else np.array_equal(x, y)


def test_model_inference_multi_rccl_one_rank(lib):
    """dp.model_inference_multi (core.py:56-88 for three identities at once: mixed-identity
    batches through per-sample embedding rows, one-rank RCCL gather to rank 0, final_frames_list) against
    swap_identity_frames run identity by identity (fp32: batch composition moves bytes by at most 1 LSB)."""
    import torch.distributed as dist
    from ghost_amd.inference.core import swap_identity_frames
    from ghost_amd.inference.dp import model_inference_multi
    G, _ = model("unet", 2)
    pres = [[1, 1, 0, 1, 1], [0, 1, 1, 1, 0], [1, 0, 1, 0, 1]]
    g = np.random.default_rng(13)
    idents, refs = [], []
    for q, pr in enumerate(pres):
        crops = g.integers(0, 256, (sum(pr), 256, 256, 3), dtype=np.uint8)
        _, z = aei_ref.make_inputs(1, 100 + q)
        idents.append((crops, np.array(pr, np.float64), z))
        refs.append(swap_identity_frames(crops, pr, z.to(DEV), G, BS=4))
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1)
    try:
        for mode in ("host", "device"):
            got = model_inference_multi(idents, G, BS=4, device=DEV, output=mode)
            assert len(got) == 3
            for fl, rl in zip(got, refs):
                assert len(fl) == len(rl)
                for x, y in zip(fl, rl):
                    if isinstance(y, list):
                        assert isinstance(x, list) and x == []
                    else:
                        u8_close(x if mode == "host" else x.cpu().numpy(), y, max_lsb=1, frac=1e-3)
    finally:
        dist.destroy_process_group()


def test_pipeline_rccl_collectives_two_streams_one_rank(lib):
    """the N > 1 data path on one GPU.  GatherPipeline(streams=2, force_collective=True) over a
    one-rank RCCL group issues bench.py's per-slot async all_gather_into_tensor (dst=None) and the video mux's gather
    to rank 0 (dst=0) from two pipeline streams, waits on each slot's Work on a pipeline stream before the slot is
    rewritten, and must give the bytes of the no-collective two-stream run; a reused slot's ticket raises; drain()
    leaves no collective in flight.  model_inference_multi(collect='rank0'|'all', force_collective=True) must give
    the bytes of the same call without the collective (/root/reference/utils/inference/core.py:72-88)."""
    import torch.distributed as dist
    from ghost_amd.inference.dp import GatherPipeline, model_inference_multi
    G, _ = model("unet", 2, torch.bfloat16)
    B, nb = 8, 5
    crops = torch.from_numpy(aei_ref.make_u8_crops(B * nb - 3, 37)).to(DEV)
    _, z = aei_ref.make_inputs(1, 37)
    zd = z.to(DEV)

    def run(pipe):
        got, pending, stale = [], [], None
        for i in range(0, crops.shape[0], B):
            c = crops[i:i + B]
            pending.append(pipe.submit(c, counts=[c.shape[0]] if c.shape[0] < B else None))
            if len(pending) == 2:
                t = pending.pop(0)
                got.append(pipe.result(t).clone())
                stale = stale or t
        got += [pipe.result(t).clone() for t in pending]
        pipe.drain()
        torch.cuda.synchronize()
        return got, stale

    ref, _ = run(GatherPipeline(lambda c, o: G.swap_u8(c, zd, out=o), (B, 256, 256, 3), DEV, depth=2, streams=2))
    pres = [[1, 1, 0, 1, 1, 1, 1, 0, 1], [0, 1, 1, 1, 0, 1, 1, 1, 1]]
    g = np.random.default_rng(19)
    idents = []
    for q, pr in enumerate(pres):
        _, zq = aei_ref.make_inputs(1, 200 + q)
        idents.append((g.integers(0, 256, (sum(pr), 256, 256, 3), dtype=np.uint8), np.array(pr, np.float64), zq))
    multi_ref = model_inference_multi(idents, G, BS=4, device=DEV, output="device")
    multi_ref = [[x.clone() if torch.is_tensor(x) else x for x in fl] for fl in multi_ref]
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1)
    try:
        for dst in (None, 0):
            pipe = GatherPipeline(lambda c, o: G.swap_u8(c, zd, out=o), (B, 256, 256, 3), DEV, depth=2, streams=2,
                                  dst=dst, force_collective=True)
            assert pipe.collective and pipe.nccl and pipe.nstreams == 2
            assert pipe.gath[0].data_ptr() != pipe.outs[0].data_ptr()
            got, stale = run(pipe)
            assert pipe.in_flight() == 0
            with pytest.raises(RuntimeError, match="overwritten"):
                pipe.result(stale)
            assert len(got) == len(ref)
            for a, b in zip(got, ref):
                assert torch.equal(a, b)
        for collect in ("rank0", "all"):
            for mode in ("device", "host"):
                got = model_inference_multi(idents, G, BS=4, device=DEV, collect=collect, output=mode,
                                            force_collective=True)
                for fl, rl in zip(got, multi_ref):
                    assert len(fl) == len(rl)
                    for x, y in zip(fl, rl):
                        if isinstance(y, list):
                            assert isinstance(x, list) and x == []
                        else:
                            xx = x if mode == "device" else torch.from_numpy(np.asarray(x)).to(DEV)
                            assert torch.equal(xx, y)
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("backbone,nb,dt,B,nid", [("unet", 2, torch.bfloat16, 8, 1), ("unet", 2, torch.bfloat16, 64, 1),
                                                  ("linknet", 3, torch.bfloat16, 8, 4), ("unet", 2, None, 2, 2),
                                                  ("linknet", 3, torch.float16, 8, 3)])
def test_identity_table_indexed_swap_is_bit_identical(lib, backbone, nb, dt, B, nid):
    """VERDICT r04 item 6 (/root/reference/network/AADLayer.py:28-33, faceshifter_run.py:15-16): the
    per-identity projection table (fc1/fc2 of every AADLayer and up1, computed once per identity) gathered by
    identity_index gives the bytes of swap_u8 with per-sample z rows (source_embeds[identity_index]) — one identity
    (B = 8 and the bench's B = 64) and mixed batches of 2-4 identities, bf16 / fp32 / fp16."""
    G, _ = model(backbone, nb, dt)
    if dt == torch.float16:
        G = G.half()
    crops = torch.from_numpy(aei_ref.make_u8_crops(B, 43)).to(DEV)
    _, zs = aei_ref.make_inputs(nid, 43)
    zs = zs.to(DEV)
    if dt == torch.float16:
        zs = zs.half()
    idx = (torch.arange(B) * 7 + 1) % nid
    table = G.identity_table(zs)
    assert len(table) == nid
    got = G.swap_u8_indexed(crops, table, idx)                       # host index: range-checked, then copied
    got_dev = G.swap_u8_indexed(crops, table, idx.to(DEV).to(torch.int32))
    ref = G.swap_u8(crops, zs.index_select(0, idx.to(DEV)).contiguous() if nid > 1 else zs)
    torch.cuda.synchronize()
    assert torch.equal(got, ref)
    assert torch.equal(got_dev, ref)
    with pytest.raises(IndexError):
        G.swap_u8_indexed(crops, table, torch.full((B,), nid))


def test_indexed_swap_refuses_a_short_table(lib):
    """the C ABI checks the table's size against n_ident (the clamped gather never reads past it)."""
    import ctypes as C
    G, _ = model("unet", 2, torch.bfloat16)
    _, z = aei_ref.make_inputs(1, 45)
    table = G.identity_table(z.to(DEV))
    crops = torch.from_numpy(aei_ref.make_u8_crops(1, 45)).to(DEV)
    idx = torch.zeros(1, dtype=torch.int32, device=DEV)
    out = torch.empty(1, 256, 256, 3, dtype=torch.uint8, device=DEV)
    rt = G._rt
    ws = rt.workspace("swap", 1, DEV, 0)
    lib = rt.lib
    rc = lib.ghost_aei_swap_u8_indexed(rt.h, crops.data_ptr(), 196608, 1, table.ptr, 2, table.nbytes, idx.data_ptr(),
                                       out.data_ptr(), ws.data_ptr(), ws.numel(), None)
    assert rc == -1 and b"too small" in lib.ghost_last_error()
    rc = lib.ghost_aei_swap_u8_indexed(rt.h, crops.data_ptr(), 196608, 1, table.ptr, 1, table.nbytes, idx.data_ptr(),
                                       out.data_ptr(), ws.data_ptr(), ws.numel(), None)
    torch.cuda.synchronize()
    assert rc == 0 and torch.equal(out, G.swap_u8_indexed(crops, table, idx))


def test_identity_table_refuses_stale_weights(lib):
    """A table holds the projections of the weights it was built with: after a re-pack it is refused."""
    G, p = model("unet", 2, torch.bfloat16)
    _, z = aei_ref.make_inputs(1, 44)
    table = G.identity_table(z.to(DEV))
    crops = torch.from_numpy(aei_ref.make_u8_crops(1, 44)).to(DEV)
    G.swap_u8_indexed(crops, table, torch.zeros(1, dtype=torch.int32))
    G.load_state_dict(p)
    G.swap_u8(crops, z.to(DEV))                 # re-packs
    with pytest.raises(RuntimeError, match="rebuild"):
        G.swap_u8_indexed(crops, table, torch.zeros(1, dtype=torch.int32))
