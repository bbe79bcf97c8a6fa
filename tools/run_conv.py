"""Run one generator conv shape repeatedly (for PMC passes): python tools/run_conv.py H Cin Cout [iters]."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ghost_amd import _lib  # noqa: E402
from ghost_amd.network.pack import pack_conv  # noqa: E402

H, ci, co = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3])
iters = int(sys.argv[4]) if len(sys.argv) > 4 else 5
B, dt, dev = 64, torch.bfloat16, torch.device("cuda:0")
lib = _lib.load()
x = torch.randn(B, H, H, ci, device=dev).to(dt)
w = pack_conv(torch.randn(co, ci, 3, 3, device=dev) * 0.05, dt)
y = torch.empty(B, H, H, co, dtype=dt, device=dev)
ws = torch.empty(64 << 20, dtype=torch.uint8, device=dev)
st = torch.cuda.current_stream().cuda_stream
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for it in range(iters + 1):
    if it == 1:
        s.record()
    _lib.check(lib.ghost_conv2d_nhwc(_lib.gdtype(dt), x.data_ptr(), B, H, H, ci, ci, w.data_ptr(), co, w.shape[0],
                                     w.shape[1], 3, 3, 1, 1, None, None, 1.0, None, 0, 0, y.data_ptr(), co,
                                     ws.data_ptr(), ws.numel(), st))
e.record()
torch.cuda.synchronize()
us = s.elapsed_time(e) / iters * 1e3
print(f"conv3x3 B={B} {H}x{H} {ci}->{co}: {us:.1f} us, {2.0 * B * H * H * ci * co * 9 / us / 1e6:.1f} TF/s")
