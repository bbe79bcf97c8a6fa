"""Multi-process data-parallel logic on CPU (gloo, world_size 2 and 3): shard bounds, the
all-gather order and the present/[] re-insertion of core.py:79-88.  The swap itself is a
deterministic stand-in here (the GPU swap is covered by tests/test_gpu_parity.py)."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from ghost_amd.inference.core import reinsert_present
from ghost_amd.inference.dp import gather_frames, shard_bounds, swap_frames_dp


def fake_swap(c: torch.Tensor) -> torch.Tensor:
    # per-frame deterministic transform that depends on the frame's own content only
    return (255 - c).flip(-1)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, n, bs, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        g = np.random.Generator(np.random.PCG64(5))
        crops = torch.from_numpy(g.integers(0, 256, size=(n, 4, 4, 3), dtype=np.uint8))
        out = swap_frames_dp(crops, fake_swap, BS=bs)
        q.put((rank, out.numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,n,bs", [(2, 7, 2), (3, 10, 4), (2, 1, 8), (3, 2, 1)])
def test_swap_frames_dp_gloo_order(world, n, bs):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, n, bs, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    g = np.random.Generator(np.random.PCG64(5))
    crops = torch.from_numpy(g.integers(0, 256, size=(n, 4, 4, 3), dtype=np.uint8))
    expect = fake_swap(crops).numpy()
    for r in range(world):
        assert np.array_equal(results[r], expect), r


def _pipe_worker(rank, world, port, depth, q):
    from ghost_amd.inference.dp import GatherPipeline
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        B = 3
        pipe = GatherPipeline(lambda c, o: o.copy_(fake_swap(c)), (B, 4, 4, 3), torch.device("cpu"), depth=depth)
        batches = [torch.full((B, 4, 4, 3), 10 * k + rank, dtype=torch.uint8) + torch.arange(B, dtype=torch.uint8)
                   .view(B, 1, 1, 1) for k in range(5)]
        got, prev, stale = [], None, 0
        for k, bt in enumerate(batches):
            t = pipe.submit(bt)
            if prev is not None:      # batch k-1's gather, read while batch k's is in flight
                try:
                    got.append(pipe.result(prev).clone())
                except RuntimeError:  # depth 1: batch k reused batch k-1's slot
                    got.append(None)
                    stale += 1
            prev = t
        got.append(pipe.result(prev).clone())
        # a short last batch: rank r holds r + 1 valid rows, every rank passes all counts
        counts = [r + 1 for r in range(world)]
        t = pipe.submit(batches[0][:rank + 1], counts=counts)
        short = pipe.result(t).clone()
        pipe.drain()
        q.put((rank, [None if g is None else g.numpy() for g in got], stale, short.numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("depth", [1, 2, 3])
def test_gather_pipeline_gloo(depth):
    """dp.GatherPipeline (bench.py's swap -> all-gather stream): batch k's gathered swaps, in rank
    order, on every rank, with batch k+1 submitted before batch k is read; a ticket whose slot was
    reused raises; a short batch returns only every rank's valid rows."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pipe_worker, args=(r, world, port, depth, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = {r: (got, stale, short) for r, got, stale, short in (q.get(timeout=120) for _ in range(world))}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    B = 3
    for r in range(world):
        got, stale, short = results[r]
        assert stale == (4 if depth == 1 else 0)
        for k in range(5):
            expect = torch.cat([fake_swap(torch.full((B, 4, 4, 3), 10 * k + rr, dtype=torch.uint8)
                                          + torch.arange(B, dtype=torch.uint8).view(B, 1, 1, 1)) for rr in range(world)])
            if depth == 1 and k < 4:
                assert got[k] is None
                continue
            assert np.array_equal(got[k], expect.numpy()), (r, k)
        expect = torch.cat([fake_swap(torch.full((rr + 1, 4, 4, 3), rr, dtype=torch.uint8)
                                      + torch.arange(rr + 1, dtype=torch.uint8).view(rr + 1, 1, 1, 1))
                            for rr in range(world)])
        assert np.array_equal(short, expect.numpy()), r


def test_gather_pipeline_rejects_bad_batches():
    from ghost_amd.inference.dp import GatherPipeline
    pipe = GatherPipeline(lambda c, o: o.copy_(c), (3, 2), torch.device("cpu"), depth=1)
    with pytest.raises(ValueError, match="counts"):
        pipe.submit(torch.zeros(2, 2, dtype=torch.uint8))
    with pytest.raises(ValueError, match="exceeds"):
        pipe.submit(torch.zeros(4, 2, dtype=torch.uint8))
    t0 = pipe.submit(torch.ones(3, 2, dtype=torch.uint8))
    t1 = pipe.submit(torch.full((2, 2), 7, dtype=torch.uint8), counts=[2])
    with pytest.raises(RuntimeError, match="overwritten"):
        pipe.result(t0)
    assert pipe.result(t1).tolist() == [[7, 7], [7, 7]]


def test_shard_bounds_partition():
    for n in range(0, 40):
        for world in (1, 2, 3, 8):
            covered = []
            per = None
            for r in range(world):
                s, e, p = shard_bounds(n, world, r)
                per = p
                assert 0 <= s <= e <= n and e - s <= p
                covered += list(range(s, e))
            assert covered == list(range(n))
            assert per == (n + world - 1) // world


def test_reinsert_present_matches_reference_bookkeeping():
    out = np.arange(3 * 2).reshape(3, 2)
    present = [1, 0, 0, 1, 1, 0]
    frames = reinsert_present(out, present)
    assert [f if isinstance(f, list) else f.tolist() for f in frames] == [[0, 1], [], [], [2, 3], [4, 5], []]


class _FakeG:
    """Stand-in for AEI_Net.swap_u8 on CPU tensors (the GPU swap is covered by the -m gpu tests)."""

    def swap_u8(self, crops, z, out=None):
        y = fake_swap(crops)
        if out is not None:
            out.copy_(y)
            return out
        return y


def _mux_worker(rank, world, port, collect, q):
    from ghost_amd.inference import dp
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    host_copies = []
    orig_cpu = torch.Tensor.cpu

    def spy_cpu(self, *a, **k):   # every device->host copy model_inference_dp makes on this rank
        host_copies.append(tuple(self.shape))
        return orig_cpu(self, *a, **k)
    try:
        g = np.random.Generator(np.random.PCG64(11))
        present = [1, 0, 1, 1, 0, 1, 1, 1, 0]
        frs = g.integers(0, 256, size=(sum(present), 4, 4, 3), dtype=np.uint8)
        torch.Tensor.cpu = spy_cpu
        try:
            out = dp.model_inference_dp(frs, present, torch.zeros(1, 512), _FakeG(), BS=2, device="cpu",
                                        collect=collect)
        finally:
            torch.Tensor.cpu = orig_cpu
        q.put((rank, None if out is None else [f if isinstance(f, list) else f.tolist() for f in out], host_copies))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("collect", ["rank0", "all"])
def test_model_inference_dp_rank0_mux_gloo(collect):
    """core.py:72-88 data-parallel: with collect='rank0' only rank 0 receives the swapped crops and
    copies them to the host (the video mux rank), in frame order with [] re-inserted; rank 1 returns
    None and makes no host copy.  collect='all' gives every rank the list."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_mux_worker, args=(r, world, port, collect, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = {r: (out, cp) for r, out, cp in (q.get(timeout=120) for _ in range(world))}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    g = np.random.Generator(np.random.PCG64(11))
    present = [1, 0, 1, 1, 0, 1, 1, 1, 0]
    frs = g.integers(0, 256, size=(sum(present), 4, 4, 3), dtype=np.uint8)
    sw = fake_swap(torch.from_numpy(frs)).numpy()
    expect = [f if isinstance(f, list) else f.tolist() for f in reinsert_present(sw, present)]
    assert results[0][0] == expect
    assert len(results[0][1]) == 1           # one D2H of the gathered crops
    if collect == "rank0":
        assert results[1] == (None, [])
    else:
        assert results[1][0] == expect


def _bench_worker(rank, world, port, q):
    import time as _t
    import bench
    from ghost_amd.inference.dp import GatherPipeline
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        B, steps, warmup = 3, 4, 2
        calls = []

        def swap(c, o):       # rank 1 is slower: the reported time must be rank 1's (max over ranks)
            calls.append(1)
            _t.sleep(0.02 * (rank + 1))
            o.copy_(fake_swap(c))
        pipe = GatherPipeline(swap, (B, 4, 4, 3), torch.device("cpu"), depth=2)
        crops = torch.full((B, 4, 4, 3), rank, dtype=torch.uint8)
        marks = []
        t0 = _t.perf_counter()
        el = bench.timed_region(lambda: pipe.submit(crops), pipe.drain, steps, warmup, world, torch.device("cpu"),
                                lambda: marks.append(len(calls)))
        total = _t.perf_counter() - t0
        rec = bench.headline_record(world, B, steps, warmup, el, "unet", 2, 1, "bf16", 1)
        q.put((rank, el, total, len(calls), marks, rec))
    finally:
        dist.destroy_process_group()


def test_bench_multi_rank_reporting_gloo():
    """bench.py's N > 1 path with a stand-in swap (gloo world 2): W warm-up steps before the timed region,
    exactly K inside, the reported time is the max over ranks (identical on every rank, >= the slow rank's
    K steps), value = all ranks' frames / that time, global_batch = N*B, parallelism dpN."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bench_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {r: rest for r, *rest in (q.get(timeout=120) for _ in range(world))}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (el0, tot0, n0, m0, rec0), (el1, tot1, n1, m1, rec1) = res[0], res[1]
    assert el0 == el1                         # all-reduce MAX: one time for the job
    assert el1 >= 4 * 0.04 * 0.9              # rank 1's four timed steps at 40 ms each
    assert n0 == n1 == 6 and m0 == m1 == [2]  # 2 warm-up steps, then exactly 4 timed
    assert rec0 == rec1
    assert rec0["n_gpus"] == 2 and rec0["config"]["global_batch"] == 6 and rec0["config"]["parallelism"] == "dp2"
    assert rec0["scaling"] == "weak" and rec0["steps"] == 4 and rec0["warmup"] == 2
    assert abs(rec0["value"] - 2 * 3 * 4 / el0) < 0.01 * rec0["value"]
    assert "all-gather" in rec0["config"]["workload"]


def _pipe_dst_worker(rank, world, port, q):
    from ghost_amd.inference.dp import GatherPipeline
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        B = 2
        pipe = GatherPipeline(lambda c, o: o.copy_(fake_swap(c)), (B, 4, 4, 3), torch.device("cpu"), depth=2, dst=0)
        outs = []
        prev = None
        for k in range(4):
            t = pipe.submit(torch.full((B, 4, 4, 3), 10 * k + rank, dtype=torch.uint8))
            if prev is not None:
                r = pipe.result(prev)
                outs.append(None if r is None else r.clone().numpy())
            prev = t
        r = pipe.result(prev)
        outs.append(None if r is None else r.clone().numpy())
        pipe.drain()
        q.put((rank, outs, pipe.gath[0] is None))
    finally:
        dist.destroy_process_group()


def test_gather_pipeline_dst_rank0_gloo():
    """GatherPipeline(dst=0): batches stream to rank 0 only, in rank order; the other rank holds no
    gather buffers and reads None."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pipe_dst_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {r: (o, nob) for r, o, nob in (q.get(timeout=120) for _ in range(world))}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    outs0, nobuf0 = res[0]
    outs1, nobuf1 = res[1]
    assert not nobuf0 and nobuf1
    assert outs1 == [None] * 4
    for k in range(4):
        expect = torch.cat([fake_swap(torch.full((2, 4, 4, 3), 10 * k + rr, dtype=torch.uint8)) for rr in range(world)])
        assert np.array_equal(outs0[k], expect.numpy()), k


class _FakeGz(_FakeG):
    """Stand-in swap that also depends on each row's identity embedding (z[:, 0] added to the bytes)."""

    def swap_u8(self, crops, z, out=None):
        zz = z.reshape(z.shape[0], -1)[:, 0].round().to(torch.int64)
        y = ((fake_swap(crops).to(torch.int64) + zz.view(-1, 1, 1, 1)) % 256).to(torch.uint8)
        if out is not None:
            out.copy_(y)
            return out
        return y


class _FakeGzTable(_FakeGz):
    """The same stand-in with AEI_Net's identity-table API (identity_table / swap_u8_indexed): the path
    model_inference_multi takes with the real module."""

    def identity_table(self, embeds):
        self.tables = getattr(self, "tables", 0) + 1
        return embeds.reshape(embeds.shape[0], -1).clone()

    def swap_u8_indexed(self, crops, table, idx, out=None):
        assert idx.dtype == torch.int32 and int(idx.max()) < table.shape[0]
        return self.swap_u8(crops, table.index_select(0, idx.to(torch.int64)), out=out)


MULTI_PRESENT = [[1, 1, 0, 1, 1, 1, 0], [0, 1, 1, 1, 0, 0, 1], [1, 0, 0, 0, 0, 1, 1]]


def _multi_case():
    """Three identities of one 7-frame video: identity 0 as crop_frames (a crop or [] per frame), 1 and 2 after
    resize_frames (present crops + present vector); embeddings 7*q + 3."""
    g = np.random.Generator(np.random.PCG64(21))
    idents, crops_of = [], []
    for q, pres in enumerate(MULTI_PRESENT):
        crops = g.integers(0, 256, size=(sum(pres), 256, 256, 3), dtype=np.uint8)
        emb = torch.full((1, 512), 7.0 * q + 3)
        crops_of.append(crops)
        if q == 0:
            it = iter(crops)
            idents.append(([next(it) if p else [] for p in pres], emb))
        else:
            idents.append((crops, np.array(pres, np.float64), emb))
    return idents, crops_of


def _multi_worker(rank, world, port, collect, bs, q):
    from ghost_amd.inference import dp
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        idents, _ = _multi_case()
        out = dp.model_inference_multi(idents, _FakeGz(), BS=bs, device="cpu", collect=collect)
        q.put((rank, None if out is None else [[f if isinstance(f, list) else f.copy() for f in fl] for fl in out]))
    finally:
        dist.destroy_process_group()


def _multi_expect():
    _, crops_of = _multi_case()
    exp = []
    for q, (pres, crops) in enumerate(zip(MULTI_PRESENT, crops_of)):
        sw = ((fake_swap(torch.from_numpy(crops)).to(torch.int64) + (7 * q + 3)) % 256).to(torch.uint8).numpy()
        exp.append(reinsert_present(sw, pres))
    return exp


def _same_lists(got, exp):
    assert len(got) == len(exp)
    for fl, el in zip(got, exp):
        assert len(fl) == len(el)
        for a, b in zip(fl, el):
            if isinstance(b, list):
                assert isinstance(a, list) and a == []
            else:
                assert np.array_equal(a, b)


@pytest.mark.parametrize("world,collect,bs", [(1, "rank0", 4), (2, "rank0", 2), (2, "all", 3), (3, "rank0", 5)])
def test_model_inference_multi_gloo(world, collect, bs):
    """model_inference_multi (core.py:56-88 over every identity at once, config 5) on gloo:
    identities' present crops in one identity-major sequence, contiguous shards, batches that mix identities
    through per-sample embedding rows, gathered to rank 0 (or all) — rank 0 returns final_frames_list equal to the
    single-process per-identity result, the other ranks None (rank0) or the same lists (all)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_multi_worker, args=(r, world, port, collect, bs, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=180) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    exp = _multi_expect()
    _same_lists(res[0], exp)
    for r in range(1, world):
        if collect == "rank0":
            assert res[r] is None
        else:
            _same_lists(res[r], exp)


def _c5_bench_worker(rank, world, port, q):
    import bench
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        calls = []

        class G(_FakeGz):
            def swap_u8(self, crops, z, out=None):
                calls.append(crops.shape[0])
                return super().swap_u8(crops, z, out)
        leg = bench.config5_multi_leg(torch.device("cpu"), world, frames_per_gpu=6, n_ident=4, BS=4, reps=2, G=G(),
                                      crop=256)
        q.put((rank, leg, calls))
    finally:
        dist.destroy_process_group()


def test_bench_config5_multi_leg_reporting_gloo():
    """bench.py's config-5 pipeline leg runs on every rank at N > 1 (gloo world 2, stand-in
    swap): the video grows with N (frames_per_gpu * N), every rank swaps about half of the crops, the reported
    times are the max over ranks (identical on both ranks) for both output modes."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_c5_bench_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = {r: (leg, calls) for r, leg, calls in (q.get(timeout=180) for _ in range(world))}
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (l0, c0), (l1, c1) = res[0], res[1]
    assert l0["frames"] == 12 and l0["crops"] == l1["crops"]
    for mode in ("device", "host"):
        assert l0[mode] == l1[mode] and l0[mode]["crops_per_s"] > 0
    per = (l0["crops"] + 1) // 2               # rank 0's contiguous shard
    # 2 output modes x (1 warm-up + 2 timed) = 6 pipeline calls, each swapping the rank's whole shard
    assert sum(c0) == 6 * per and sum(c1) == 6 * (l0["crops"] - per), (sum(c0), sum(c1), per)


def test_model_inference_multi_identity_forms():
    """model_inference_multi takes each identity as (crop_frames, source_embed), (crop_frames, None,
    source_embed) or (resized_frs, present, source_embed) with resized_frs a numpy array or a tensor (resize_frames'
    output): all forms give the single-process per-identity lists (one process, no process group)."""
    from ghost_amd.inference import dp
    idents, crops_of = _multi_case()
    exp = _multi_expect()
    forms = [
        idents,
        [(idents[0][0], None, idents[0][1])] + idents[1:],
        [idents[0]] + [(torch.from_numpy(c), p, e) for c, p, e in idents[1:]],
    ]
    for f in forms:
        _same_lists(dp.model_inference_multi(f, _FakeGz(), BS=3, device="cpu"), exp)
        G = _FakeGzTable()
        _same_lists(dp.model_inference_multi(f, G, BS=3, device="cpu"), exp)
        assert G.tables == 1                # the identities' projections once per call, then gathered per batch


def _forced_worker(rank, world, port, q):
    from ghost_amd.inference import dp
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        G = _FakeGz()
        crops = torch.from_numpy(np.random.Generator(np.random.PCG64(3)).integers(0, 256, (11, 8, 8, 3),
                                                                              dtype=np.uint8))
        z = torch.full((1, 512), 5.0)
        out = {}
        for dst in (None, 0):
            pipe = dp.GatherPipeline(lambda c, o: G.swap_u8(c, z, out=o), (4, 8, 8, 3), "cpu", depth=2, dst=dst,
                                     force_collective=True)
            assert pipe.collective and pipe.gath[0] is not pipe.outs[0]
            t = [pipe.submit(crops[0:4]), pipe.submit(crops[4:8])]
            assert pipe.in_flight() == 2
            got = [pipe.result(t[0]).clone()]
            t.append(pipe.submit(crops[8:11], counts=[3]))       # reuses slot 0
            try:
                pipe.result(t[0])
                stale = False
            except RuntimeError:
                stale = True
            got += [pipe.result(t[1]).clone(), pipe.result(t[2]).clone()]
            pipe.drain()
            out[dst] = (torch.cat(got).numpy().copy(), stale, pipe.in_flight())
        idents, _ = _multi_case()
        multi = dp.model_inference_multi(idents, G, BS=3, device="cpu", force_collective=True)
        q.put((out, G.swap_u8(crops, z).numpy().copy(),
               [[f if isinstance(f, list) else f.copy() for f in fl] for fl in multi]))
    finally:
        dist.destroy_process_group()


def test_gather_pipeline_force_collective_one_rank_gloo():
    """VERDICT r04 item 1 (CPU half; the RCCL half is tests/test_gpu_pipeline.py): force_collective issues the
    gather / all-gather in a one-rank group — same bytes as the direct swap, a reused slot's ticket still raises,
    drain() leaves nothing in flight; model_inference_multi with it returns the expected lists."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_forced_worker, args=(0, 1, _free_port(), q))
    p.start()
    out, ref, multi = q.get(timeout=180)
    p.join(timeout=60)
    assert p.exitcode == 0
    for dst in (None, 0):
        got, stale, left = out[dst]
        assert np.array_equal(got, ref) and stale and left == 0
    _same_lists(multi, _multi_expect())


def test_force_collective_needs_a_group():
    from ghost_amd.inference import dp
    with pytest.raises(RuntimeError, match="process group"):
        dp.GatherPipeline(lambda c, o: None, (2, 8, 8, 3), "cpu", force_collective=True)


def _bench_cmd(*args):
    import sys
    return [sys.executable, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "bench.py"),
            *args]


def _clean_env(**extra):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "MASTER_PORT")}
    env.update(extra)
    return env


def test_bench_launcher_spawns_ranks_cpu():
    """``python bench.py --gpus 2`` with no outside launcher starts 2 ranks itself (child
    processes with RANK / WORLD_SIZE / MASTER_* set) and relays rank 0's one JSON line: n_gpus 2, the group's own
    size in rccl_world, both ranks' timed regions, value = all ranks' frames / the slower rank's time.  Here on
    gloo with the CPU stand-in swap (the GPU ranks run the same launcher, timed region and record)."""
    import json
    import subprocess
    r = subprocess.run(_bench_cmd("--gpus", "2", "--standin-cpu", "--steps", "3", "--warmup", "1", "--batch", "2"),
                       capture_output=True, text=True, env=_clean_env(), timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    recs = [json.loads(ln) for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(recs) == 1, r.stdout
    rec = recs[0]
    assert rec["n_gpus"] == 2 and rec["rccl_world"] == 2 and rec["config"]["parallelism"] == "dp2"
    assert rec["config"]["global_batch"] == 4 and rec["steps"] == 3 and rec["warmup"] == 1
    assert len(rec["per_rank_s"]) == 2
    el = max(rec["per_rank_s"])
    assert abs(rec["value"] - 2 * 2 * 3 / el) <= 0.02 * rec["value"] + 0.01


def test_bench_world_mismatch_exits_nonzero():
    """--gpus N under an outside launcher that started a different number of ranks: refuse (exit 2) before any
    device or group is touched."""
    import subprocess
    r = subprocess.run(_bench_cmd("--gpus", "2", "--standin-cpu", "--steps", "1", "--warmup", "0"),
                       capture_output=True, text=True, env=_clean_env(WORLD_SIZE="1", RANK="0", LOCAL_RANK="0"),
                       timeout=120)
    assert r.returncode == 2
    assert "WORLD_SIZE=1" in r.stderr and not r.stdout.strip()


def test_bench_single_process_default_is_one_rank_cpu():
    """No --gpus, no launcher: one rank, n_gpus 1, rccl_world 1 (the driver's default N = 1 run)."""
    import json
    import subprocess
    r = subprocess.run(_bench_cmd("--standin-cpu", "--steps", "2", "--warmup", "1", "--batch", "2"),
                       capture_output=True, text=True, env=_clean_env(), timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    rec = json.loads(r.stdout.strip().splitlines()[-1])
    assert rec["n_gpus"] == 1 and rec["rccl_world"] == 1 and len(rec["per_rank_s"]) == 1
