"""The HIP streams of the swap path, one fixed set per device for the whole process.

An MI355X process gets GPU_MAX_HW_QUEUES = 4 hardware queues per priority (HIP's default, the box's setting); a
stream created past that shares a queue with an earlier one, and work on two streams that share a queue runs in
submission order — a D2H copy enqueued behind the other batch's kernels waits for them.  Which streams pair up
depends only on creation order (tools/queue_probe.py on the box: with the caller's default stream plus six pool
streams, pool streams 0-2 each had a queue of their own and 3, 4, 5 shared with 2, 1, 0).  Round 4's bench created
new streams in every leg and pipeline, so the D2H-inclusive and video legs moved by -15 % / +11 % depending on
which leg had run before them.

So every pipeline of this package takes its streams from one ``StreamSet`` per device, created in one go on first
use: the caller's stream (batch k of a two-batch pipeline), ``side`` (batch k + 1), ``d2h`` (device -> host copies)
and ``h2d`` (host -> device copies) — four streams for four queues.  The native library adds one more, its up-path
stream, created at the lowest priority (a queue pool of its own).
"""
from __future__ import annotations

import threading
from typing import Dict, List

import torch

_lock = threading.Lock()
_sets: Dict[int, "StreamSet"] = {}


class StreamSet:
    def __init__(self, device: torch.device):
        self.device = device
        self.side = torch.cuda.Stream(device)    # the second batch in flight (GatherPipeline streams = 2)
        self.d2h = torch.cuda.Stream(device)     # device -> host copies (per-batch .cpu(), blended frames)
        self.h2d = torch.cuda.Stream(device)     # host -> device copies (video frames)
        self._more: List[torch.cuda.Stream] = []

    def compute(self, i: int):
        """Compute stream i of a pipeline: 0 = None (the caller's current stream at submit time), 1 = ``side``,
        i >= 2 = further streams, created on first request (they share queues with the ones above)."""
        if i == 0:
            return None
        if i == 1:
            return self.side
        while len(self._more) < i - 1:
            self._more.append(torch.cuda.Stream(self.device))
        return self._more[i - 2]


def stream_set(device=None) -> StreamSet:
    """The process-wide stream set of ``device`` (default: the current CUDA device)."""
    dev = torch.device(device or "cuda")
    idx = dev.index if dev.index is not None else torch.cuda.current_device()
    with _lock:
        s = _sets.get(idx)
        if s is None:
            s = _sets[idx] = StreamSet(torch.device("cuda", idx))
        return s
