"""Data-parallel frame sharding for the swap path, one process per GPU.

The reference runs every frame of an identity through G on one GPU in batches of BS
(utils/inference/core.py:57-88).  Frames are independent inside G (eval BatchNorm,
per-sample InstanceNorm), so the build shards them:

* rank r of W swaps the contiguous block of present crops ``[r*S, min(N, (r+1)*S))`` with
  ``S = ceil(N / W)`` (the last block padded to S so every rank contributes equal bytes);
* one all-gather over the process group (RCCL over xGMI on MI355X, gloo in the CPU tests)
  returns every rank's uint8 swaps — or, for the video mux, one gather to rank 0 only (the
  reference writes the video from one process, core.py:72-88; the other ranks then copy nothing
  to the host); because blocks are contiguous and gathered in rank order, trimming the padding
  restores frame order exactly;
* the ``present`` bookkeeping of core.py:79-88 then re-inserts ``[]`` for frames without
  a face, bit-exactly as the single-GPU path.

No collective other than that all-gather (or gather) is on the data path.
"""
from __future__ import annotations

from typing import Callable, List, NamedTuple, Optional, Sequence, Tuple

import numpy as np
import torch
import torch.distributed as dist

from .core import reinsert_present


def shard_bounds(n: int, world: int, rank: int):
    """[start, end) of rank's contiguous block and the padded per-rank size S = ceil(n / world)."""
    per = (n + world - 1) // world if n else 0
    start = min(n, rank * per)
    return start, min(n, start + per), per


def gather_frames(local: torch.Tensor, per: int, n: int, group=None, dst: Optional[int] = None):
    """Collect each rank's [<=per, ...] uint8 block (padded to per) and return the first n rows in frame
    order.  ``dst=None``: an all-gather, every rank returns the n rows.  ``dst=r``: a gather to rank r
    only (the video mux rank, core.py:72-88 writes the frames on one process), which returns the n rows
    there and ``None`` on every other rank."""
    world = dist.get_world_size(group)
    rank = dist.get_rank(group)
    pad = torch.zeros((per,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
    pad[:local.shape[0]] = local
    if dst is not None:
        out = (torch.empty((world * per,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
               if rank == dst else None)
        dist.gather(pad, list(out.chunk(world)) if out is not None else None, dst=_global_rank(group, dst),
                    group=group)
        return out[:n] if out is not None else None
    if dist.get_backend(group) == "nccl":
        out = torch.empty((world * per,) + tuple(local.shape[1:]), dtype=local.dtype, device=local.device)
        dist.all_gather_into_tensor(out, pad, group=group)
    else:
        parts = [torch.empty_like(pad) for _ in range(world)]
        dist.all_gather(parts, pad, group=group)
        out = torch.cat(parts, 0)
    return out[:n]


def _global_rank(group, r: int) -> int:
    return r if group is None else dist.get_global_rank(group, r)


def swap_frames_dp(crops: torch.Tensor, swap: Callable[[torch.Tensor], torch.Tensor], BS: int = 64,
                   group=None, dst: Optional[int] = None):
    """Shard N crops [N,256,256,3] (uint8, identical on every rank) over the group, swap this
    rank's block in batches of BS with ``swap`` (crops -> uint8 swaps), then collect: every rank
    returns the N swapped crops in frame order (``dst=None``, all-gather), or only rank ``dst`` does
    and the others return ``None`` (gather)."""
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    n = crops.shape[0]
    start, end, per = shard_bounds(n, world, rank)
    outs = [swap(crops[i:min(end, i + BS)]) for i in range(start, end, BS)]
    local = torch.cat(outs, 0) if outs else crops[:0].clone()
    return gather_frames(local, per, n, group, dst)


def model_inference_dp(resized_frs: np.ndarray, present: Sequence[int], source_embed: torch.Tensor, G,
                       BS: int = 64, device=None, group=None, collect: str = "rank0") -> Optional[List]:
    """core.py:57-88 for one identity, data-parallel over the group.  ``collect="rank0"`` (default): the
    swapped crops are gathered to rank 0 only, which copies them to the host and returns the per-frame
    list (swapped crop or ``[]``) for the video mux; every other rank returns ``None`` and copies nothing
    to the host.  ``collect="all"``: all-gather, every rank returns the list."""
    if collect not in ("rank0", "all"):
        raise ValueError(f"ghost_amd: collect must be 'rank0' or 'all', got {collect!r}")
    device = torch.device(device or "cuda")
    crops = torch.from_numpy(np.ascontiguousarray(resized_frs)).to(device)
    gathered = swap_frames_dp(crops, lambda c: G.swap_u8(c, source_embed), BS, group,
                              dst=0 if collect == "rank0" else None)
    if gathered is None:
        return None
    return reinsert_present(gathered.cpu().numpy(), present)


def _identity_crops(ident):
    """One identity of model_inference_multi -> (crops of its present frames in frame order (a list of host uint8
    arrays, one host [n,h,w,3] array, or a device tensor — resize_frames' output), present, source embedding, whether
    the crops still need resize_frames' 224 -> 256 resize)."""
    if len(ident) == 3:                       # (resized_frs, present, source_embed): resize_frames already ran
        resized, present, emb = ident
        if present is None:                   # (crop_frames, None, source_embed): the crop_frames form
            return _identity_crops((resized, emb))
        return resized, np.asarray(present), emb, False
    if len(ident) == 2:                       # (crop_frames, source_embed): crop_frames_and_get_transforms' lists
        crop_frames, emb = ident
        present = np.ones(len(crop_frames))
        keep = []
        for i, fr in enumerate(crop_frames):
            a = None if isinstance(fr, list) else np.asarray(fr)
            if a is None or a.ndim != 3 or a.size == 0:
                present[i] = 0
            else:
                keep.append(a)
        return keep, present, emb, True
    raise ValueError("ghost_amd: an identity is (crop_frames, source_embed) or (resized_frs, present, source_embed)")


def model_inference_multi(identities: Sequence, G, BS: int = 64, device=None, group=None, collect: str = "rank0",
                          output: str = "host", streams: int = 2, force_collective: bool = False):
    """The identity loop of model_inference (utils/inference/core.py:56-88) for every identity of a video at once,
    data-parallel over the group (BASELINE config 5: several source -> target identities in one video).

    ``identities``: per identity either ``(crop_frames, source_embed)`` — crop_frames_and_get_transforms' list for
    that identity, one 224x224 uint8 crop or ``[]`` per video frame; resize_frames (video_processing.py:174-188)
    runs here, its cv2.resize on the device — or ``(resized_frs, present, source_embed)`` after resize_frames.

    Every identity's present crops form one sequence in identity-major, frame order; rank r of W swaps the
    contiguous block ``shard_bounds(N, W, r)`` of it in batches of BS.  A batch may hold crops of several
    identities: each crop carries its identity's embedding row (per-sample z_id rows, ``swap_mixed_identities``).
    Batches run through a ``GatherPipeline`` (``streams`` batches in flight; each batch gathered to rank 0 —
    ``collect="rank0"``, the video mux rank — or to every rank with ``collect="all"``, while the next batch is
    swapped).  The receiving rank places every rank's rows at their sequence positions, copies them to pinned host
    memory batch by batch on a copy stream (``output="host"``), and returns ``final_frames_list`` as core.py:88
    builds it: per identity one entry per video frame, the swapped uint8 crop or ``[]``.  ``output="device"``
    returns the same lists holding device tensor views instead (no host copy).  Ranks that receive nothing return
    ``None``.  ``force_collective``: issue the per-batch gather even in a one-rank group (GatherPipeline), the N > 1
    data path on one GPU."""
    if collect not in ("rank0", "all"):
        raise ValueError(f"ghost_amd: collect must be 'rank0' or 'all', got {collect!r}")
    if output not in ("host", "device"):
        raise ValueError(f"ghost_amd: output must be 'host' or 'device', got {output!r}")
    device = torch.device(device or "cuda")
    gpu = device.type == "cuda"
    dist_on = dist.is_available() and dist.is_initialized()
    world = dist.get_world_size(group) if dist_on else 1
    rank = dist.get_rank(group) if dist_on else 0
    idents = [_identity_crops(i) for i in identities]
    counts = [len(c) for c, _, _, _ in idents]
    n = sum(counts)
    offs = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64)
    start, end, per = shard_bounds(n, world, rank)
    # the per-crop shape every rank agrees on (all ranks hold the host lists): 256x256 after resize_frames
    fshape = (256, 256, 3)
    for crops, _, _, needs in idents:
        if len(crops) and not needs:
            fshape = tuple(crops[0].shape) if torch.is_tensor(crops) else tuple(np.asarray(crops[0]).shape)
            break
    # this rank's crops (host -> device once, per identity part; crop_frames parts resized 224 -> 256 on the device,
    # video_processing.py:184) and their identity rows
    parts, ids = [], []
    for q, (crops, _, _, needs) in enumerate(idents):
        a, b = max(start, int(offs[q])), min(end, int(offs[q + 1]))
        if a >= b:
            continue
        part = crops[a - offs[q]:b - offs[q]]
        if torch.is_tensor(part):             # resize_frames' device crops (or a host tensor)
            dpart = part.to(device)
        else:
            host = torch.from_numpy(np.ascontiguousarray(np.stack(part) if isinstance(part, list) else np.asarray(part)))
            dpart = host.pin_memory().to(device, non_blocking=True) if gpu else host.to(device)
        if needs and tuple(dpart.shape[1:3]) != (256, 256):
            from .blend import resize_u8
            dpart = resize_u8(dpart, (256, 256))
        parts.append(dpart)
        ids.append(np.full(b - a, q, np.int64))
    embeds = torch.stack([torch.as_tensor(e).reshape(-1) for _, _, e, _ in idents]).to(device) if idents else None
    # the identities' projections once (AEI_Net.identity_table: every AADLayer's fc1/fc2 and up1 per source
    # embedding), each batch then gathers its samples' rows by identity index (swap_u8_indexed); a swap object
    # without the table API gets per-sample embedding rows instead
    indexed = hasattr(G, "identity_table") and hasattr(G, "swap_u8_indexed")
    table = None
    if parts:
        local = parts[0] if len(parts) == 1 else torch.cat(parts)
        if tuple(local.shape[1:]) != fshape:
            raise ValueError(f"ghost_amd: identities' crops differ in shape ({tuple(local.shape[1:])} vs {fshape})")
        try:
            pdt = next(G.parameters()).dtype
        except (AttributeError, StopIteration):
            pdt = None
        if pdt == torch.float16:
            embeds = embeds.half()                          # core.py:65-66 (a .half() module)
        ids_d = torch.from_numpy(np.concatenate(ids)).to(device)
        if indexed:
            table = G.identity_table(embeds)
            z_all = ids_d.to(torch.int32)                   # valid by construction: built from 0..len(idents)-1
        else:
            z_all = embeds.index_select(0, ids_d)
    else:
        local = torch.empty((0,) + fshape, dtype=torch.uint8, device=device)
        z_all = None
    nb = (per + BS - 1) // BS if per else 0
    B = max(1, min(BS, per))
    zb = [None]
    streams = max(1, streams) if gpu else 1
    if indexed:
        def swap(c, o):
            return G.swap_u8_indexed(c, table, zb[0], out=o)
    else:
        def swap(c, o):
            return G.swap_u8(c, zb[0], out=o)
    pipe = GatherPipeline(swap, (B,) + fshape, device, group=group,
                          depth=2 * streams, streams=streams, dst=0 if collect == "rank0" else None,
                          force_collective=force_collective)
    receiver = pipe.receiver
    out_all = torch.empty((n,) + fshape, dtype=torch.uint8, device=device) if receiver else None
    host_all = (torch.empty((n,) + fshape, dtype=torch.uint8, pin_memory=True)
                if receiver and output == "host" and gpu else None)
    if host_all is not None:
        from .streams import stream_set
        copy = stream_set(device).d2h
    else:
        copy = None
    cur = torch.cuda.current_stream(device) if gpu else None
    bounds = [shard_bounds(n, world, r)[:2] for r in range(world)]

    def place(k, ticket):
        g = pipe.result(ticket)                              # caller's stream waits for the batch
        if g is None:
            return
        row = 0
        for r, (s0, e0) in enumerate(bounds):
            a = s0 + k * B
            c = max(0, min(B, e0 - a))
            if c:
                out_all[a:a + c].copy_(g[row:row + c])
                if copy is not None:
                    ev = torch.cuda.Event()
                    ev.record(cur)
                    with torch.cuda.stream(copy):
                        copy.wait_event(ev)
                        host_all[a:a + c].copy_(out_all[a:a + c], non_blocking=True)
            row += c

    pending = []
    for k in range(nb):
        a = k * B
        c = max(0, min(B, (end - start) - a))
        kc = [max(0, min(B, e0 - s0 - a)) for s0, e0 in bounds]
        zb[0] = z_all[a:a + c] if c else None
        pending.append((k, pipe.submit(local[a:a + c], counts=kc)))
        if len(pending) > pipe.depth - 1:                   # consume a slot before it is reused
            place(*pending.pop(0))
    for kt in pending:
        place(*kt)
    pipe.drain()
    if not receiver:
        if gpu:
            torch.cuda.current_stream(device).synchronize()
        return None
    if copy is not None:
        copy.synchronize()
        out_all.record_stream(copy)
        rows = host_all.numpy()
    elif output == "host":
        rows = out_all.numpy()           # CPU tensors (gloo tests)
    else:
        rows = out_all
    return [reinsert_present(rows[offs[q]:offs[q + 1]], present) for q, (_, present, _, _) in enumerate(idents)]


def swap_mixed_identities(crops: torch.Tensor, identity_index: torch.Tensor, source_embeds: torch.Tensor, G,
                          out: Optional[torch.Tensor] = None, table=None) -> torch.Tensor:
    """Config 5 (several identities in one batch): each crop carries the index of its source identity.  With
    ``table`` (``G.identity_table(source_embeds)``, built once per video) the identity rows of every AADLayer are
    gathered per sample (``swap_u8_indexed``); without it the per-sample z_id rows are gathered on the device and
    projected inside the swap (fc1/fc2 per sample, AADLayer.py:28-29).  Same bytes either way (batches <= 64)."""
    if table is not None:
        return G.swap_u8_indexed(crops, table, identity_index, out=out)
    z = source_embeds.reshape(source_embeds.shape[0], -1).index_select(0, identity_index.to(source_embeds.device))
    return G.swap_u8(crops, z, out=out)


class Ticket(NamedTuple):
    """What ``GatherPipeline.submit`` hands back: the buffer slot, the slot's generation when this batch
    was written to it, and every rank's count of valid rows in it."""
    slot: int
    gen: int
    counts: Tuple[int, ...]


class GatherPipeline:
    """A stream of per-rank batches, each swapped on this GPU and then all-gathered to every rank,
    with the all-gather of batch k in flight (RCCL's own stream, over xGMI) while batch k+1 is
    swapped.  ``depth`` output/gather buffer pairs rotate; a slot's previous all-gather is waited on
    (stream-ordered for RCCL: ``Work.wait()`` makes the compute stream wait, the host does not block)
    before the swap overwrites it, so no batch's bytes change while a collective reads them.

    ``swap(crops, out)`` writes the uint8 swaps of ``crops`` into ``out`` (``AEI_Net.swap_u8``).
    ``submit(crops, counts)`` returns a ``Ticket``; ``result(ticket)`` is the gathered batch in rank
    order.  A slot is rewritten ``depth`` submits later: reading a ticket whose slot has been reused
    raises instead of returning another batch's bytes.  A short batch (fewer rows than
    ``batch_shape[0]``, e.g. the last one of a shard) needs ``counts``, the valid-row count of every rank
    for this submit (known to all ranks from ``shard_bounds``); ``result`` then returns only the valid
    rows, rank by rank.  Rows past a rank's count travel as padding and are dropped.

    ``streams`` > 1 keeps that many batches in flight on the GPU: submit k runs its swap (and issues its
    all-gather) on compute stream k % streams of the device's ``StreamSet`` (streams.py: 0 is the caller's current
    stream, 1 the set's side stream; a stream other than the caller's first waits for the caller's stream, where
    the crops were produced); consecutive batches are independent, so the low-resolution, latency-bound stages of
    one batch (encoder, 2x2..8x8 blocks) overlap the HBM- and MFMA-bound 64x64..256x256 stages of the other.
    ``result`` and ``drain`` make the caller's stream wait for the batch's stream.  ``depth`` is rounded up
    to a multiple of ``streams`` so a slot is always rewritten on the stream that last wrote it.
    """

    def __init__(self, swap: Callable, batch_shape, device, dtype=torch.uint8, group=None, depth: int = 2,
                 streams: int = 1, dst: Optional[int] = None, force_collective: bool = False):
        self.nstreams = max(1, int(streams))
        depth = max(1, depth)
        depth = (depth + self.nstreams - 1) // self.nstreams * self.nstreams
        self.swap, self.group, self.depth = swap, group, depth
        self.device = torch.device(device)
        # batch k runs on compute stream k % streams of the device's StreamSet: 0 = the caller's current stream,
        # 1 = the set's side stream (the process's stream count stays fixed however many pipelines it builds)
        if self.nstreams > 1:
            from .streams import stream_set
            ss = stream_set(self.device)
            self.streams = [ss.compute(i) for i in range(self.nstreams)]
        else:
            self.streams = [None]
        self.done = [None] * depth             # per slot: event after its swap + all-gather issue (streams > 1)
        dist_on = dist.is_available() and dist.is_initialized()
        self.world = dist.get_world_size(group) if dist_on else 1
        self.rank = dist.get_rank(group) if dist_on else 0
        # force_collective: issue the gather / all-gather even in a one-rank group, so the N > 1 data path (async
        # RCCL collective per slot, Work.wait() on a pipeline stream, slot reuse under a live work object) runs on a
        # single GPU exactly as it does on eight
        if force_collective and not dist_on:
            raise RuntimeError("GatherPipeline: force_collective needs an initialised process group")
        self.collective = self.world > 1 or bool(force_collective)
        self.nccl = self.collective and dist.get_backend(group) == "nccl"
        shape = tuple(batch_shape)
        self.rows = shape[0]
        self.outs = [torch.empty(shape, dtype=dtype, device=device) for _ in range(self.depth)]
        # dst: gather to that rank only (the video mux rank); the other ranks keep no gather buffers and
        # their ``result`` is None
        self.dst = dst
        self.receiver = dst is None or self.rank == dst
        self.gath = ([torch.empty((self.world * shape[0],) + shape[1:], dtype=dtype, device=device)
                      if self.receiver else None for _ in range(self.depth)] if self.collective else self.outs)
        self.pending: List[Optional[object]] = [None] * self.depth
        self.gen = [0] * self.depth
        self.k = 0

    def _wait(self, slot: int):
        w = self.pending[slot]
        if w is not None:
            w.wait()
            self.pending[slot] = None

    def submit(self, crops: torch.Tensor, counts: Optional[Sequence[int]] = None) -> Ticket:
        n = crops.shape[0]
        if n > self.rows:
            raise ValueError(f"GatherPipeline: batch of {n} rows exceeds the pipeline's {self.rows}")
        if counts is None:
            if n != self.rows:
                raise ValueError("GatherPipeline: a short batch needs counts (every rank's valid rows)")
            counts = (self.rows,) * self.world
        counts = tuple(int(c) for c in counts)
        if len(counts) != self.world or counts[self.rank] != n or any(c < 0 or c > self.rows for c in counts):
            raise ValueError(f"GatherPipeline: counts {counts} do not fit world {self.world}, rank {self.rank} "
                             f"with {n} rows of at most {self.rows}")
        slot = self.k % self.depth
        st = self.streams[self.k % self.nstreams]
        if st is not None and st == torch.cuda.current_stream(self.device):
            st = None                               # the caller runs on the side stream itself
        if st is not None:
            st.wait_stream(torch.cuda.current_stream(self.device))   # the crops are ready on the caller's stream
            crops.record_stream(st)
        with torch.cuda.stream(st) if st is not None else _nullctx():
            self._wait(slot)                      # the collective still reading this slot's buffer
            if n:
                self.swap(crops, self.outs[slot][:n])
            if self.collective and self.dst is not None:
                g = self.gath[slot]
                self.pending[slot] = dist.gather(self.outs[slot], list(g.chunk(self.world)) if g is not None else None,
                                                 dst=_global_rank(self.group, self.dst), group=self.group,
                                                 async_op=True)
            elif self.collective:
                if self.nccl:
                    self.pending[slot] = dist.all_gather_into_tensor(self.gath[slot], self.outs[slot],
                                                                     group=self.group, async_op=True)
                else:
                    self.pending[slot] = dist.all_gather(list(self.gath[slot].chunk(self.world)), self.outs[slot],
                                                         group=self.group, async_op=True)
            if self.nstreams > 1:
                ev = torch.cuda.Event()
                ev.record(st if st is not None else torch.cuda.current_stream(self.device))
                self.done[slot] = ev
        self.gen[slot] += 1
        self.k += 1
        return Ticket(slot, self.gen[slot], counts)

    def result(self, ticket: Ticket) -> torch.Tensor:
        if not isinstance(ticket, Ticket):
            raise TypeError("GatherPipeline.result takes the Ticket that submit returned")
        if self.gen[ticket.slot] != ticket.gen:
            raise RuntimeError(f"GatherPipeline: the batch of this ticket was overwritten ({self.gen[ticket.slot] - ticket.gen}"
                               f" later submit(s) reused slot {ticket.slot}; depth {self.depth})")
        self._wait(ticket.slot)
        if self.done[ticket.slot] is not None:
            torch.cuda.current_stream(self.device).wait_event(self.done[ticket.slot])
        g = self.gath[ticket.slot]
        if g is None:         # gather to another rank
            return None
        if all(c == self.rows for c in ticket.counts):
            return g
        return torch.cat([g[r * self.rows:r * self.rows + c] for r, c in enumerate(ticket.counts)])

    def in_flight(self) -> int:
        """Collectives issued and not yet waited on (0 after ``drain``)."""
        return sum(w is not None for w in self.pending)

    def drain(self):
        for s in range(self.depth):
            self._wait(s)
            if self.done[s] is not None:
                torch.cuda.current_stream(self.device).wait_event(self.done[s])


class _nullctx:
    def __enter__(self):
        return None

    def __exit__(self, *exc):
        return False
