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


@pytest.mark.parametrize("backbone,nb,B", [("unet", 2, 4), ("linknet", 3, 2)])
def test_two_stream_plan_is_bit_identical(lib, backbone, nb, B):
    """GHOST_AEI_OPT_TWO_STREAMS: the encoder's up path and the identity projections on the handle's second
    stream give the same bytes as the one-stream plan (forward outputs, attrs and the uint8 swap)."""
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
    assert torch.equal(res[0][0], res[1][0])
    assert all(torch.equal(a, b) for a, b in zip(res[0][1], res[1][1]))
    assert torch.equal(res[0][2], res[1][2])


def test_gather_pipeline_two_batches_in_flight(lib):
    """dp.GatherPipeline(streams=2) (bench.py's default): consecutive batches swapped on two pipeline streams
    at once (sharing one AEI_Net handle) give the bytes of one-at-a-time swaps, batch by batch, including a
    short last batch; results read on the caller's stream after the batch's stream."""
    from ghost_amd.inference.dp import GatherPipeline
    G, _ = model("unet", 2, torch.bfloat16)
    B, nb = 4, 5
    crops = torch.from_numpy(aei_ref.make_u8_crops(B * nb - 1, 29)).to(DEV)
    _, z = aei_ref.make_inputs(1, 29)
    zd = z.to(DEV)
    ref = [G.swap_u8(crops[i:i + B], zd).clone() for i in range(0, crops.shape[0], B)]
    pipe = GatherPipeline(lambda c, o: G.swap_u8(c, zd, out=o), (B, 256, 256, 3), DEV, depth=2, streams=2)
    assert pipe.depth == 2 and pipe.nstreams == 2
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
    for a, b in zip(got, ref):
        assert torch.equal(a, b)


@pytest.mark.parametrize("dt,B", [(None, 1), (torch.bfloat16, 1), (torch.bfloat16, 4), (torch.float16, 2)])
def test_graphed_swap_is_bit_identical(lib, dt, B):
    """GraphedSwap (one HIP graph replay of the whole native plan, two-stream plan included) gives the
    bytes of an eager swap_u8, for new inputs copied into the captured buffers on every call."""
    from ghost_amd.inference import GraphedSwap
    G, _p = model("unet", 2, dt)
    g = GraphedSwap(G, B, DEV)
    for seed in (3, 4):
        crops = torch.from_numpy(aei_ref.make_u8_crops(B, seed)).to(DEV)
        z = torch.randn(1, 512, generator=torch.Generator().manual_seed(seed)).to(DEV)
        got = g(crops, z).clone()
        ref = G.swap_u8(crops, z)
        torch.cuda.synchronize()
        assert torch.equal(got, ref)
