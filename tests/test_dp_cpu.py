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
        got, prev = [], None
        for k, bt in enumerate(batches):
            slot = pipe.submit(bt)
            if prev is not None:      # batch k-1's gather, read while batch k's is in flight
                got.append(pipe.result(prev).clone())
            prev = slot
        got.append(pipe.result(prev).clone())
        pipe.drain()
        q.put((rank, [g.numpy() for g in got]))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("depth", [1, 2, 3])
def test_gather_pipeline_gloo(depth):
    """dp.GatherPipeline (bench.py's swap -> all-gather stream): batch k's gathered swaps, in rank
    order, on every rank, with batch k+1 submitted before batch k is read."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pipe_worker, args=(r, world, port, depth, q)) for r in range(world)]
    for p in procs:
        p.start()
    results = dict(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    B = 3
    for k in range(5):
        expect = torch.cat([fake_swap(torch.full((B, 4, 4, 3), 10 * k + r, dtype=torch.uint8)
                                      + torch.arange(B, dtype=torch.uint8).view(B, 1, 1, 1)) for r in range(world)])
        for r in range(world):
            if depth == 1 and k < 4:
                continue      # depth 1 reuses the slot: only the last batch is still readable
            assert np.array_equal(results[r][k], expect.numpy()), (r, k)


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
