"""One swap of a fixed batch shape replayed as a HIP graph (BASELINE config 1: image-to-image at B = 1).

``AEI_Net.swap_u8`` issues the native plan's ~100 kernel launches from the host on every call (≈ 0.3-0.4 ms
of host time at B = 1, comparable to the GPU time of the whole forward).  For a caller that swaps batches of
one shape over and over — one target image after another (inference.py's image mode), or frame batches of a
video — ``GraphedSwap`` captures that launch sequence once (``torch.cuda.graph``: hipStreamBeginCapture on a
side stream; the plan's second, up-path stream joins the capture through the events it already records) and
replays it with one ``hipGraphLaunch``.  The inputs are copied into the graph's own device buffers first and
the result is read from its output buffer, so the replay runs the same kernels on the same weights: the
output bytes are identical to ``swap_u8``'s (tests/test_gpu_pipeline.py).

``two_streams`` (default 0): the plan option the capture runs with (set for the warm-up and capture, restored
afterwards).  With 0 the graph is one chain of kernels; with 1 (the eager default) the encoder's up path is a second
branch the replay runs beside the down path.  The replay issues the nodes back to back, so the two branches' small
B = 1 kernels overlap and contend far more than in an eager call (a rocprofv3 trace of the same calls,
tools/graph_trace.py: the graphed kernels' sum 15.9 ms against 11.1 eager for 705 fp32 launches), and on some boxes
the branch form replayed far slower than eager (round 4, before the plan ran batches of fewer than 8 frames on one
stream: bf16 2.86 ms graphed with two branches, 1.72 as one chain, 1.62 eager).  Since then the plan itself runs a batch
of B < 8 on one stream, so at B = 1 both settings capture the same single chain; the branch form exists from B = 8 on
(tests/test_gpu_pipeline.py covers it at B = 8).  One chain tracked eager on every box measured, so it is the default.

The graph holds the module's packed weights and workspace as they were at capture, and the ``GraphedSwap``
keeps that runtime (its packed weight tensors, native handle and workspace) alive for as long as it lives.  A
replay after the module was re-packed (``load_state_dict``, ``.to`` / ``.half``, an in-place parameter change,
a replaced parameter — anything ``PackedModule`` invalidates on) raises instead of running the stale plan:
build a new ``GraphedSwap`` then.
"""
from __future__ import annotations

from typing import Optional

import torch


class GraphedSwap:
    def __init__(self, G, B: int, device, z_rows: int = 1, z_dtype: Optional[torch.dtype] = None,
                 two_streams: Optional[int] = 0):
        dev = torch.device(device)
        if z_rows not in (1, B):
            raise ValueError("ghost_amd: z_rows must be 1 or B")
        self.G, self.B, self.device = G, B, dev
        zt = z_dtype or next(G.parameters()).dtype
        self.crops = torch.zeros(B, 256, 256, 3, dtype=torch.uint8, device=dev)
        self.z = torch.zeros(z_rows, G.c_id, dtype=zt, device=dev)
        self.out = torch.empty(B, 256, 256, 3, dtype=torch.uint8, device=dev)
        side = torch.cuda.Stream(dev)
        cur = torch.cuda.current_stream(dev)
        side.wait_stream(cur)
        with torch.cuda.stream(side):           # warm-up outside the capture: packs the weights, creates the
            G.swap_u8(self.crops, self.z, out=self.out)   # native handle (its options), streams/events, workspace
        saved = G.get_option("two_streams")
        if two_streams is not None:
            G.set_option("two_streams", int(two_streams))
        try:
            with torch.cuda.stream(side):
                for _ in range(2):
                    G.swap_u8(self.crops, self.z, out=self.out)
            cur.wait_stream(side)
            torch.cuda.synchronize(dev)
            self.graph = torch.cuda.CUDAGraph()
            # a capture stream of its own: the module's workspace cache is keyed by stream, so the captured
            # workspace (allocated in the graph's private pool) is never handed to an eager call or to another
            # GraphedSwap
            self._capture_stream = torch.cuda.Stream(dev)
            with torch.cuda.graph(self.graph, stream=self._capture_stream):
                G.swap_u8(self.crops, self.z, out=self.out)
            torch.cuda.synchronize(dev)
            # the workspace the captured kernels write (allocated in the graph's private pool): held here, so neither
            # the module's LRU cache nor an option change (which clears that cache) can release it under the graph
            self._ws = list(G._rt.ws.ws.values())
        finally:
            if G.get_option("two_streams") != saved:
                G.set_option("two_streams", saved)
        # the captured kernels read the packed weights of this runtime (and its handle / workspace): hold it
        self._rt = G._rt

    def __call__(self, crops_u8: torch.Tensor, z_id: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """swap_u8(crops_u8, z_id): inputs copied into the graph's buffers, one graph launch on the current
        stream; returns ``out`` (copied) or the graph's own output buffer (overwritten by the next call)."""
        if tuple(crops_u8.shape) != tuple(self.crops.shape) or crops_u8.dtype != torch.uint8:
            raise RuntimeError(f"ghost_amd: GraphedSwap was captured for uint8 {tuple(self.crops.shape)}, got "
                               f"{crops_u8.dtype} {tuple(crops_u8.shape)}")
        z = z_id.reshape(z_id.shape[0], -1)
        if tuple(z.shape) != tuple(self.z.shape):
            raise RuntimeError(f"ghost_amd: GraphedSwap was captured for z_id {tuple(self.z.shape)}, got "
                               f"{tuple(z_id.shape)}")
        if not self.G._pack_current(self._rt):
            raise RuntimeError("ghost_amd: the module was re-packed (load_state_dict / .to / .half / a parameter "
                               "change) after this GraphedSwap was captured; its graph would replay the old weights. "
                               "Capture a new GraphedSwap.")
        self.crops.copy_(crops_u8, non_blocking=True)
        self.z.copy_(z, non_blocking=True)
        self.graph.replay()
        if out is None:
            return self.out
        out.copy_(self.out, non_blocking=True)
        return out
