"""Micro-benchmarks of the individual gfx950 kernels at the generator's B=64 shapes.

    python tools/bench_ops.py [--only conv|aad|up|stats] [--iters 20]

Each case is timed with HIP events around `iters` back-to-back launches on one stream
(after 3 warm-ups) and reported as us/launch, TFLOP/s (convs) or algorithmic GB/s.
Used to A/B kernel variants quickly (cdna_hip_programming.md §5.4 rule 24: same process).
"""
from __future__ import annotations

import argparse
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
from ghost_amd import _lib  # noqa: E402
from ghost_amd.network.pack import pack_conv, pack_convT4x4, rup  # noqa: E402

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
    return s.elapsed_time(e) / iters * 1e3   # us


def conv_cases(lib, iters, dt=torch.bfloat16, only_pp=False):
    B = 64
    ws = torch.empty(512 << 20, dtype=torch.uint8, device=DEV)
    st = torch.cuda.current_stream().cuda_stream
    # (name, H, Cin, Cout, k, stride, pad)
    cases = [("gen256 64->64", 256, 64, 64, 3, 1, 1), ("gen256 cat128->3", 256, 128, 3, 3, 1, 1),
             ("gen128 128->128", 128, 128, 128, 3, 1, 1), ("gen128 cat256->64", 128, 256, 64, 3, 1, 1),
             ("gen64 256->256", 64, 256, 256, 3, 1, 1), ("gen64 cat512->128", 64, 512, 128, 3, 1, 1),
             ("gen32 512->512", 32, 512, 512, 3, 1, 1), ("gen32 cat1024->256", 32, 1024, 256, 3, 1, 1),
             ("gen16 1024->1024", 16, 1024, 1024, 3, 1, 1),
             ("gen8 1024->1024", 8, 1024, 1024, 3, 1, 1), ("gen4 1024->1024", 4, 1024, 1024, 3, 1, 1),
             ("enc conv2 32->64", 128, 32, 64, 4, 2, 1), ("enc conv1 3->32", 256, 3, 32, 4, 2, 1)]
    if only_pp:   # the persistent halo conv's shapes
        cases = [c for c in cases if c[1] >= 32 and c[4] == 3 and c[3] >= 64]
    for name, H, ci, co, k, s, p in cases:
        x = torch.randn(B, H, H, ci, device=DEV).to(dt)
        w = pack_conv(torch.randn(co, ci, k, k, device=DEV) * 0.05, dt)
        Ho = (H + 2 * p - k) // s + 1
        y = torch.empty(B, Ho, Ho, co, dtype=dt, device=DEV)

        def run():
            _lib.check(lib.ghost_conv2d_nhwc(_lib.gdtype(dt), x.data_ptr(), B, H, H, ci, ci, w.data_ptr(), co,
                                             w.shape[0], w.shape[1], k, k, s, p, None, None, 1.0, None, 0, 0,
                                             y.data_ptr(), co, ws.data_ptr(), ws.numel(), st))
        us = timeit(run, iters)
        fl = 2.0 * B * Ho * Ho * co * ci * k * k
        by = (x.numel() + y.numel()) * x.element_size()
        print(f"conv  {name:22s} {us:9.1f} us  {fl / us / 1e6:7.1f} TF/s  {by / us / 1e3:7.1f} GB/s(io)", flush=True)


def arc_cases(lib, iters, dt=torch.bfloat16):
    """ArcFace (iresnet100 at B=64) conv shapes through ghost_conv2d_nhwc."""
    B = 64
    ws = torch.empty(512 << 20, dtype=torch.uint8, device=DEV)
    st = torch.cuda.current_stream().cuda_stream
    for name, H, ci, co, k, s, p in [("arc112 64->64", 112, 64, 64, 3, 1, 1), ("arc56 64->64", 56, 64, 64, 3, 1, 1),
                                     ("arc28 128->128", 28, 128, 128, 3, 1, 1),
                                     ("arc14 256->256", 14, 256, 256, 3, 1, 1),
                                     ("arc7 512->512", 7, 512, 512, 3, 1, 1),
                                     ("arc28s2 128->256", 28, 128, 256, 3, 2, 1),
                                     ("gen32 512->512", 32, 512, 512, 3, 1, 1),
                                     ("gen16 1024->1024", 16, 1024, 1024, 3, 1, 1)]:
        x = torch.randn(B, H, H, ci, device=DEV).to(dt)
        w = pack_conv(torch.randn(co, ci, k, k, device=DEV) * 0.05, dt)
        Ho = (H + 2 * p - k) // s + 1
        y = torch.empty(B, Ho, Ho, co, dtype=dt, device=DEV)

        def run():
            _lib.check(lib.ghost_conv2d_nhwc(_lib.gdtype(dt), x.data_ptr(), B, H, H, ci, ci, w.data_ptr(), co,
                                             w.shape[0], w.shape[1], k, k, s, p, None, None, 1.0, None, 0, 0,
                                             y.data_ptr(), co, ws.data_ptr(), ws.numel(), st))
        us = timeit(run, iters)
        fl = 2.0 * B * Ho * Ho * co * ci * k * k
        print(f"conv  {name:22s} M={B * Ho * Ho:7d} N={co:4d} K={ci * k * k:5d} {us:9.1f} us  "
              f"{fl / us / 1e6:7.1f} TF/s", flush=True)


def enc_cases(lib, iters, dt=torch.bfloat16):
    """Every encoder contraction of unet at B = 64: Conv4x4/s2 (conv1..7) and ConvT4x4/s2 (deconv1..6)."""
    B = 64
    ws = torch.empty(1 << 30, dtype=torch.uint8, device=DEV)
    st = torch.cuda.current_stream().cuda_stream
    down = [(3, 32), (32, 64), (64, 128), (128, 256), (256, 512), (512, 1024), (1024, 1024)]
    H = 256
    tot = 0.0
    for i, (ci, co) in enumerate(down, 1):
        ldx = 4 if ci == 3 else ci      # the runtime's network input has a zero fourth channel
        x = torch.randn(B, H, H, ldx, device=DEV).to(dt)
        w = pack_conv(torch.randn(co, ci, 4, 4, device=DEV) * 0.05, dt)
        y = torch.empty(B, H // 2, H // 2, co, dtype=dt, device=DEV)

        def run():
            _lib.check(lib.ghost_conv2d_nhwc(_lib.gdtype(dt), x.data_ptr(), B, H, H, ci, ldx, w.data_ptr(), co,
                                             w.shape[0], w.shape[1], 4, 4, 2, 1, None, None, 0.1, None, 0, 0,
                                             y.data_ptr(), co, ws.data_ptr(), ws.numel(), st))
        us = timeit(run, iters)
        tot += us
        fl = 2.0 * B * (H // 2) ** 2 * co * ci * 16
        print(f"enc   conv{i} {ci:4d}->{co:4d} @{H // 2:3d} {us:9.1f} us  {fl / us / 1e6:7.1f} TF/s", flush=True)
        H //= 2
    up = [(1024, 1024, 2), (2048, 512, 4), (1024, 256, 8), (512, 128, 16), (256, 64, 32), (128, 32, 64)]
    for i, (ci, co, H) in enumerate(up, 1):
        x = torch.randn(B, H, H, ci, device=DEV).to(dt)
        w = pack_convT4x4(torch.randn(ci, co, 4, 4, device=DEV) * 0.05, dt)
        y = torch.empty(B, 2 * H, 2 * H, 2 * co, dtype=dt, device=DEV)

        def run():
            _lib.check(lib.ghost_conv_transpose4x4s2_nhwc(_lib.gdtype(dt), x.data_ptr(), B, H, H, ci, ci, w.data_ptr(),
                                                          co, w.shape[1], w.shape[2], None, None, 0.1, None, 0,
                                                          y.data_ptr(), 2 * co, ws.data_ptr(), ws.numel(), st))
        us = timeit(run, iters)
        tot += us
        fl = 2.0 * B * (2 * H) ** 2 * co * ci * 4
        print(f"enc   deconv{i} {ci:4d}->{co:4d} @{2 * H:3d} {us:9.1f} us  {fl / us / 1e6:7.1f} TF/s", flush=True)
    print(f"enc   total {tot:9.1f} us", flush=True)


def aad_cases(lib, iters, dt=torch.bfloat16):
    B = 64
    st = torch.cuda.current_stream().cuda_stream
    ws = torch.empty(512 << 20, dtype=torch.uint8, device=DEV)
    for C, Ca, n in [(64, 64, 256), (128, 128, 128), (256, 256, 64), (512, 512, 32), (1024, 512, 16)]:
        h = torch.randn(B, n, n, C, device=DEV).to(dt)
        za = torch.randn(B, n, n, Ca, device=DEV).to(dt)
        out = torch.empty_like(h)
        gbw = torch.randn(rup(2 * C, 128), rup(Ca, 32), device=DEV).to(dt) * 0.05
        gbb = torch.zeros(rup(2 * C, 128), device=DEV)
        wh = torch.randn(C, device=DEV) * 0.05
        bh = torch.zeros(1, device=DEV)
        idgb = torch.randn(B, 2 * C, device=DEV)

        def run():
            _lib.check(lib.ghost_aad_layer_nhwc(_lib.gdtype(dt), h.data_ptr(), C, za.data_ptr(), Ca, B, n, n, C, Ca,
                                                gbw.data_ptr(), gbw.shape[0], gbw.shape[1], gbb.data_ptr(),
                                                wh.data_ptr(), bh.data_ptr(), idgb.data_ptr(), 2 * C, 0.0,
                                                out.data_ptr(), C, ws.data_ptr(), ws.numel(), st))
        us = timeit(run, iters)
        by = (h.numel() * 2 + za.numel()) * h.element_size()
        print(f"aad   C={C:4d} Ca={Ca:4d} n={n:3d} (stats+mask/fused) {us:9.1f} us  {by / us / 1e3:7.1f} GB/s(alg)",
              flush=True)


def aad_v3_cases(lib, iters):
    """Register-epilogue AAD kernels through ghost_aad_layers_v3_nhwc (stats + kernel)."""
    import ctypes as C
    B, dt = 64, torch.bfloat16
    st = torch.cuda.current_stream().cuda_stream
    ws = torch.empty(512 << 20, dtype=torch.uint8, device=DEV)
    # up: 1 = h_in through the x2 upsample
    for c, ca, n, L, up in [(64, 64, 256, 2, 1), (64, 64, 256, 2, 0), (64, 64, 256, 1, 0),
                            (128, 64, 128, 1, 0), (128, 64, 128, 2, 0), (128, 64, 128, 2, 1),
                            (256, 128, 64, 1, 0), (512, 256, 32, 1, 0), (1024, 512 // 2, 16, 1, 0)]:
        hn = n // 2 if up & 1 else n
        zn = n
        h = torch.randn(B, hn, hn, c, device=DEV).to(dt)
        za = torch.randn(B, zn, zn, ca, device=DEV).to(dt)
        keep, w3, b3, wh, bh, ids, outs = [], [], [], [], [], [], []
        for _ in range(L):
            t = [torch.randn(c // 64 * 128, ca, device=DEV).to(dt) * 0.05, torch.zeros(c // 64 * 128, device=DEV),
                 torch.randn(c, device=DEV) * 0.05, torch.zeros(1, device=DEV), torch.randn(B, 2 * c, device=DEV),
                 torch.empty(B, n, n, c, dtype=dt, device=DEV)]
            keep += t
            for lst, v in zip((w3, b3, wh, bh, ids, outs), t):
                lst.append(v.data_ptr())
        arr = lambda xs: (C.c_void_p * L)(*xs)  # noqa: E731
        ldo = (C.c_int * L)(*([c] * L))

        def run():
            _lib.check(lib.ghost_aad_layers_v3_nhwc(h.data_ptr(), c, up, za.data_ptr(), ca, B, n, n, c, ca, L,
                                                    arr(w3), arr(b3), arr(wh), arr(bh), arr(ids), 2 * c, 0.0,
                                                    arr(outs), ldo, ws.data_ptr(), ws.numel(), st))
        us = timeit(run, iters)
        alg = B * n * n * L * (2 * c + ca) * 2    # SURVEY formula: per layer |h_in| + |z_attr| + |out|
        print(f"aadv3 C={c:4d} Ca={ca:4d} n={n:3d} L={L} up={up} (stats+kernel) {us:9.1f} us  "
              f"{alg / us / 1e3:7.1f} GB/s(alg)", flush=True)


def up_cases(lib, iters, dt=torch.bfloat16):
    B = 64
    st = torch.cuda.current_stream().cuda_stream
    for C, n in [(64, 128), (128, 64)]:
        x = torch.randn(B, n, n, C, device=DEV).to(dt)
        y = torch.empty(B, 2 * n, 2 * n, C, dtype=dt, device=DEV)
        us = timeit(lambda: _lib.check(lib.ghost_upsample2x_nhwc(_lib.gdtype(dt), x.data_ptr(), C, y.data_ptr(), C,
                                                                 B, n, n, C, st)), iters)
        by = (x.numel() + y.numel()) * x.element_size()
        print(f"up2x  C={C} {n}->{2 * n} {us:9.1f} us  {by / us / 1e3:7.1f} GB/s", flush=True)


def stats_cases(lib, iters, dt=torch.bfloat16):
    B = 64
    st = torch.cuda.current_stream().cuda_stream
    ws = torch.empty(256 << 20, dtype=torch.uint8, device=DEV)
    for C, n in [(64, 256), (128, 128), (512, 32), (1024, 16)]:
        x = torch.randn(B, n, n, C, device=DEV).to(dt)
        stat = torch.empty(B, C, 2, device=DEV)
        us = timeit(lambda: _lib.check(lib.ghost_instnorm_stats_nhwc(_lib.gdtype(dt), x.data_ptr(), B, n * n, C, C,
                                                                     stat.data_ptr(), ws.data_ptr(), ws.numel(), st)),
                    iters)
        print(f"stats C={C} n={n} {us:9.1f} us  {x.numel() * x.element_size() / us / 1e3:7.1f} GB/s", flush=True)
    for C, n in [(64, 128), (128, 64)]:   # statistics of the x2 upsample of an n x n source
        x = torch.randn(B, n, n, C, device=DEV).to(dt)
        stat = torch.empty(B, C, 2, device=DEV)
        us = timeit(lambda: _lib.check(lib.ghost_instnorm_stats_up2x_nhwc(_lib.gdtype(dt), x.data_ptr(), B, n, n, C, C,
                                                                          stat.data_ptr(), ws.data_ptr(), ws.numel(),
                                                                          st)), iters)
        print(f"stats_up2x C={C} {n}->{2 * n} {us:9.1f} us  {x.numel() * x.element_size() / us / 1e3:7.1f} GB/s(src)",
              flush=True)


def ceiling_cases(iters, dt=torch.bfloat16):
    """Library ceilings on the same work: hipBLASLt GEMM of the im2col shape and MIOpen conv."""
    import torch.nn.functional as F
    B = 64
    for name, H, ci, co in [("gen256 64->64", 256, 64, 64), ("gen128 128->128", 128, 128, 128),
                            ("gen64 256->256", 64, 256, 256), ("gen64 cat512->128", 64, 512, 128),
                            ("gen32 512->512", 32, 512, 512)]:
        M, N, K = B * H * H, co, ci * 9
        a = torch.randn(M, K, device=DEV).to(dt)
        b = torch.randn(K, N, device=DEV).to(dt)
        us = timeit(lambda: torch.matmul(a, b), iters)
        fl = 2.0 * M * N * K
        print(f"blas  {name:22s} M={M} N={N} K={K} {us:9.1f} us  {fl / us / 1e6:7.1f} TF/s", flush=True)
        del a, b
        x = torch.randn(B, ci, H, H, device=DEV).to(dt).contiguous(memory_format=torch.channels_last)
        w = (torch.randn(co, ci, 3, 3, device=DEV) * 0.05).to(dt).contiguous(memory_format=torch.channels_last)
        try:
            us = timeit(lambda: F.conv2d(x, w, padding=1), iters)
            print(f"miopen {name:21s} {us:9.1f} us  {fl / us / 1e6:7.1f} TF/s", flush=True)
        except RuntimeError as e:   # noqa: BLE001
            print(f"miopen {name}: {e}")
        del x, w
    for n in (8192,):
        a = torch.randn(n, n, device=DEV).to(dt)
        b = torch.randn(n, n, device=DEV).to(dt)
        us = timeit(lambda: torch.matmul(a, b), iters)
        print(f"blas  square {n} {us:9.1f} us  {2.0 * n ** 3 / us / 1e6:7.1f} TF/s", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="")
    ap.add_argument("--iters", type=int, default=20)
    a = ap.parse_args()
    lib = _lib.load()
    print("env:", {k: v for k, v in os.environ.items() if k.startswith("GHOST_")})
    if a.only == "ceil":
        ceiling_cases(a.iters)
    if a.only in ("", "conv", "pp"):
        conv_cases(lib, a.iters, only_pp=a.only == "pp")
    if a.only in ("", "arc"):
        arc_cases(lib, a.iters)
    if a.only in ("", "enc"):
        enc_cases(lib, a.iters)
    if a.only in ("", "aad"):
        aad_cases(lib, a.iters)
    if a.only in ("", "aad", "aadv3"):
        aad_v3_cases(lib, a.iters)
    if a.only in ("", "up"):
        up_cases(lib, a.iters)
    if a.only in ("", "stats"):
        stats_cases(lib, a.iters)


if __name__ == "__main__":
    main()
