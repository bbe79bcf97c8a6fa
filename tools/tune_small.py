"""Tile / split-K sweep for the generator's low-resolution convs and the encoder's strided convs (B = 64).
Tiles come from GHOST_CONV_TILE / GHOST_CONV_BK (read once per process); splits via ghost_set_split_k:
    bash tools/tune_small.sh   (one process per tile configuration)"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ghost_amd import _lib  # noqa: E402
from ghost_amd.network.pack import pack_conv, pack_convT4x4  # noqa: E402

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
tag = f"tile={os.environ.get('GHOST_CONV_TILE', 'auto')} bk={os.environ.get('GHOST_CONV_BK', 'auto')}"
# (name, H, Cin, Cout, k, stride, pad, transposed)
cases = [("gen8 3x3 1024", 8, 1024, 1024, 3, 1, 1, False), ("gen4 3x3 1024", 4, 1024, 1024, 3, 1, 1, False),
         ("enc conv2 128 32->64", 128, 32, 64, 4, 2, 1, False), ("enc conv3 64 64->128", 64, 64, 128, 4, 2, 1, False),
         ("enc conv4 32 128->256", 32, 128, 256, 4, 2, 1, False),
         ("enc conv5 16 256->512", 16, 256, 512, 4, 2, 1, False),
         ("enc deconv2 4 2048->512", 4, 2048, 512, 4, 2, 1, True),
         ("enc deconv3 8 1024->256", 8, 1024, 256, 4, 2, 1, True)]
for name, H, ci, co, k, stride, pad, tr in cases:
    x = torch.randn(B, H, H, ci, device=DEV).to(dt)
    if tr:
        w = pack_convT4x4(torch.randn(ci, co, 4, 4, device=DEV) * 0.05, dt)
        Ho = 2 * H
    else:
        w = pack_conv(torch.randn(co, ci, k, k, device=DEV) * 0.05, dt)
        Ho = (H + 2 * pad - k) // stride + 1
    y = torch.empty(B, Ho, Ho, co, dtype=dt, device=DEV)
    fl = 2.0 * B * Ho * Ho * co * ci * (4 if tr else k * k)
    for s in (0, 1, 2, 4, 8):
        _lib.check(lib.ghost_set_split_k(s))
        if tr:
            def run():
                _lib.check(lib.ghost_conv_transpose4x4s2_nhwc(_lib.gdtype(dt), x.data_ptr(), B, H, H, ci, ci,
                                                              w.data_ptr(), co, w.shape[1], w.shape[2], None, None,
                                                              1.0, None, 0, y.data_ptr(), co, ws.data_ptr(),
                                                              ws.numel(), st))
        else:
            def run():
                _lib.check(lib.ghost_conv2d_nhwc(_lib.gdtype(dt), x.data_ptr(), B, H, H, ci, ci, w.data_ptr(), co,
                                                 w.shape[0], w.shape[1], k, k, stride, pad, None, None, 1.0, None, 0,
                                                 0, y.data_ptr(), co, ws.data_ptr(), ws.numel(), st))
        try:
            us = timeit(run, 20)
        except RuntimeError as e:
            print(f"{tag} {name} split={s}: {str(e)[:80]}", flush=True)
            continue
        print(f"{tag} {name:26s} split={s} {us:8.1f} us {fl / us / 1e6:7.1f} TF/s", flush=True)
_lib.check(lib.ghost_set_split_k(0))
