"""Drive the ArcFace (iresnet100) embedding path for profiling: python tools/run_arc.py [N] [iters] [bf16|fp32]."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ghost_amd.arcface import iresnet100  # noqa: E402
from oracle.arcface_ref import make_weights, param_specs  # noqa: E402

N = int(sys.argv[1]) if len(sys.argv) > 1 else 64
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 5
dt = torch.bfloat16 if (sys.argv[3] if len(sys.argv) > 3 else "bf16") == "bf16" else torch.float32
net = iresnet100(compute_dtype=dt).eval()
net.load_state_dict(make_weights(param_specs()))
net = net.cuda()
crops = torch.from_numpy(np.random.Generator(np.random.PCG64(5)).integers(0, 256, (N, 224, 224, 3),
                                                                       dtype=np.uint8)).cuda()
for _ in range(2):
    net.embed_u8(crops)
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(iters):
    net.embed_u8(crops)
e.record()
torch.cuda.synchronize()
ms = s.elapsed_time(e) / iters
print(f"iresnet100 {dt} N={N}: {ms:.3f} ms/batch, {N / ms * 1e3:.1f} embeddings/s, "
      f"{24.18e9 * N / ms / 1e9:.1f} TFLOP/s", flush=True)
