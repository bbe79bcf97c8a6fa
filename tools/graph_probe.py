"""Eager launches vs HIP-graph replay of the bench step (same process, same buffers):
python tools/graph_probe.py [--steps K].  Measured (r01, B = 64 unet/2): eager 7.43 ms/step, graph replay 7.48 —
the launch queue already runs the ~110 kernels back to back, so bench.py launches eagerly."""
import argparse
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ghost_amd.network import AEI_Net  # noqa: E402
from oracle.aei_ref import make_weights, param_specs  # noqa: E402  (synthetic weights; test infrastructure)

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=20)
a = ap.parse_args()
dev = torch.device("cuda:0")
G = AEI_Net("unet", num_blocks=2, c_id=512, compute_dtype=torch.bfloat16).eval()
G.load_state_dict(make_weights(param_specs("unet", 2)))
G = G.to(dev)
B = 64
rng = np.random.Generator(np.random.PCG64(1000))
crops = torch.from_numpy(rng.integers(0, 256, size=(B, 256, 256, 3), dtype=np.uint8)).to(dev)
z = torch.randn(1, 512, device=dev)
out = torch.empty(B, 256, 256, 3, dtype=torch.uint8, device=dev)
for _ in range(3):
    G.swap_u8(crops, z, out=out)
torch.cuda.synchronize()
ref = out.clone()


def timed(fn, k):
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(k):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / k * 1e3


eager = timed(lambda: G.swap_u8(crops, z, out=out), a.steps)
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g, stream=s):
    G.swap_u8(crops, z, out=out)
torch.cuda.synchronize()
out.zero_()
g.replay()
torch.cuda.synchronize()
same = bool(torch.equal(out, ref))
graph = timed(g.replay, a.steps)
eager2 = timed(lambda: G.swap_u8(crops, z, out=out), a.steps)
print(f"eager {eager:.3f} ms/step, graph {graph:.3f} ms/step, eager again {eager2:.3f}; graph output identical: {same}",
      flush=True)
