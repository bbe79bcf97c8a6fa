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
