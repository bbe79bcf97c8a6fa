"""Low-resolution GEMM probe: hipBLASLt (torch.matmul, bf16) on the im2col'd GEMM shapes of the generator's
2x2..8x8 stages and the encoder's conv5..7, beside this library's conv on the same shape:
    python tools/probe_gemm.py [lib|blas|both] [case-substring]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ghost_amd import _lib  # noqa: E402
from ghost_amd.network.pack import pack_conv  # noqa: E402

DEV = torch.device("cuda:0")
mode = sys.argv[1] if len(sys.argv) > 1 else "both"
only = sys.argv[2] if len(sys.argv) > 2 else ""


def timeit(fn, iters=20):
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


B, dt = 64, torch.bfloat16
ws = torch.empty(1 << 30, dtype=torch.uint8, device=DEV)
st = torch.cuda.current_stream().cuda_stream
lib = _lib.load()
cases = [("gen2 3x3 1024", 2, 1024, 1024, 3, 1, 1), ("gen4 3x3 1024", 4, 1024, 1024, 3, 1, 1),
         ("gen8 3x3 1024", 8, 1024, 1024, 3, 1, 1),
         ("gen8 1x1 1024->2048", 8, 1024, 2048, 1, 1, 0), ("gen4 1x1 2048->2048", 4, 2048, 2048, 1, 1, 0),
         ("gen2 1x1 1024->2048", 2, 1024, 2048, 1, 1, 0),
         ("enc conv5 16 256->512", 16, 256, 512, 4, 2, 1), ("enc conv6 8 512->1024", 8, 512, 1024, 4, 2, 1),
         ("enc conv7 4 1024->1024", 4, 1024, 1024, 4, 2, 1)]
for name, H, ci, co, k, stride, pad in cases:
    if only and only not in name:
        continue
    Ho = (H + 2 * pad - k) // stride + 1
    M, N, K = B * Ho * Ho, co, k * k * ci
    fl = 2.0 * M * N * K
    if mode in ("blas", "both"):
        a = torch.randn(M, K, device=DEV).to(dt)
        b = torch.randn(K, N, device=DEV).to(dt)
        us = timeit(lambda: torch.matmul(a, b))
        print(f"{name:24s} hipBLASLt M={M} N={N} K={K}: {us:8.1f} us {fl / us / 1e6:7.1f} TF/s", flush=True)
    if mode in ("lib", "both"):
        x = torch.randn(B, H, H, ci, device=DEV).to(dt)
        w = pack_conv(torch.randn(co, ci, k, k, device=DEV) * 0.05, dt)
        y = torch.empty(B, Ho, Ho, co, dtype=dt, device=DEV)

        def run():
            _lib.check(lib.ghost_conv2d_nhwc(_lib.gdtype(dt), x.data_ptr(), B, H, H, ci, ci, w.data_ptr(), co,
                                             w.shape[0], w.shape[1], k, k, stride, pad, None, None, 1.0, None, 0,
                                             0, y.data_ptr(), co, ws.data_ptr(), ws.numel(), st))
        us = timeit(run)
        print(f"{name:24s} ghost conv: {us:8.1f} us {fl / us / 1e6:7.1f} TF/s", flush=True)
