"""Split-K / BK sweep of the AAD gamma/beta GEMM (1x1 conv with the fused AADLayer epilogue) at the
low-resolution stages (C = 1024, Ca = 1024 / 2048; B = 64): python tools/tune_aad_gemm.py (GHOST_CONV_BK)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ghost_amd import _lib  # noqa: E402

DEV = torch.device("cuda:0")


def timeit(fn, iters):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3

lib = _lib.load()
B, dt = 64, torch.bfloat16
ws = torch.empty(1 << 30, dtype=torch.uint8, device=DEV)
st = torch.cuda.current_stream().cuda_stream
for n, C, Ca in [(8, 1024, 1024), (4, 1024, 2048), (2, 1024, 1024)]:
    h = torch.randn(B, n, n, C, device=DEV).to(dt)
    za = torch.randn(B, n, n, Ca, device=DEV).to(dt)
    Npad, Kpad = 2 * C, Ca
    gbw = (torch.randn(Npad, Kpad, device=DEV) * 0.03).to(dt)
    gbb = torch.zeros(Npad, device=DEV)
    wh = torch.randn(C, device=DEV) * 0.03
    bh = torch.zeros(1, device=DEV)
    idgb = torch.randn(B, 2 * C, device=DEV)
    out = torch.empty(B, n, n, C, dtype=dt, device=DEV)
    for s in (0, 1, 2, 4, 8):
        _lib.check(lib.ghost_set_split_k(s))
        run = lambda: _lib.check(lib.ghost_aad_layer_nhwc(  # noqa: E731
            _lib.gdtype(dt), h.data_ptr(), C, za.data_ptr(), Ca, B, n, n, C, Ca, gbw.data_ptr(), Npad, Kpad,
            gbb.data_ptr(), wh.data_ptr(), bh.data_ptr(), idgb.data_ptr(), 2 * C, 0.0, out.data_ptr(), C,
            ws.data_ptr(), ws.numel(), st))
        us = timeit(run, 20)
        fl = 2.0 * B * n * n * 2 * C * Ca
        print(f"bk={os.environ.get('GHOST_CONV_BK', 'auto')} aad {n}x{n} C={C} Ca={Ca} split={s} {us:8.1f} us "
              f"(stats+mask+gemm) {fl / us / 1e6:7.1f} TF/s", flush=True)
_lib.check(lib.ghost_set_split_k(0))
