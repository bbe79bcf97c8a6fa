"""Run one AAD kernel shape repeatedly (for PMC passes):
python tools/run_aad.py C Ca n L up [iters]   (B = 64, bf16, through ghost_aad_layers_v3_nhwc)."""
import ctypes as C
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ghost_amd import _lib  # noqa: E402

c, ca, n, L, up = (int(v) for v in sys.argv[1:6])
iters = int(sys.argv[6]) if len(sys.argv) > 6 else 5
B, dt, dev = 64, torch.bfloat16, torch.device("cuda:0")
lib = _lib.load()
hn = n // 2 if up else n
h = torch.randn(B, hn, hn, c, device=dev).to(dt)
za = torch.randn(B, n, n, ca, device=dev).to(dt)
keep, w3, b3, wh, bh, ids, outs = [], [], [], [], [], [], []
for _ in range(L):
    t = [torch.randn(c // 64 * 128, ca, device=dev).to(dt) * 0.05, torch.zeros(c // 64 * 128, device=dev),
         torch.randn(c, device=dev) * 0.05, torch.zeros(1, device=dev), torch.randn(B, 2 * c, device=dev),
         torch.empty(B, n, n, c, dtype=dt, device=dev)]
    keep += t
    for lst, v in zip((w3, b3, wh, bh, ids, outs), t):
        lst.append(v.data_ptr())
arr = lambda xs: (C.c_void_p * L)(*xs)  # noqa: E731
ldo = (C.c_int * L)(*([c] * L))
ws = torch.empty(512 << 20, dtype=torch.uint8, device=dev)
st = torch.cuda.current_stream().cuda_stream
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for it in range(iters + 1):
    if it == 1:
        s.record()
    _lib.check(lib.ghost_aad_layers_v3_nhwc(h.data_ptr(), c, up, za.data_ptr(), ca, B, n, n, c, ca, L, arr(w3), arr(b3),
                                            arr(wh), arr(bh), arr(ids), 2 * c, 0.0, arr(outs), ldo, ws.data_ptr(),
                                            ws.numel(), st))
e.record()
torch.cuda.synchronize()
print(f"aad C={c} Ca={ca} n={n} L={L} up={up}: {s.elapsed_time(e) / iters * 1e3:.1f} us (stats + kernel)")
