"""Probe: do the low-resolution deep-K GEMMs (AADBlk1-3 convs and AAD GEMMs, encoder conv5-7) lose time to
power-of-two row strides (activation pixel stride 2 KB, weight row stride Kpad * 2 B)?  Times each shape with
the runtime's layout and with padded strides (ldx + 32 channels; Kpad + 32 zero columns, which the K loop
then reads as one extra all-zero channel block of the padded pixel), B = 64 bf16:
    python tools/lowres_probe.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ghost_amd import _lib  # noqa: E402
from ghost_amd.network.pack import pack_conv  # noqa: E402

DEV = torch.device("cuda:0")


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


lib = _lib.load()
B, dt = 64, torch.bfloat16
ws = torch.empty(1 << 30, dtype=torch.uint8, device=DEV)
st = torch.cuda.current_stream().cuda_stream
# (name, H, Cin, Cout, k, stride, pad)
cases = [("gen2 3x3 1024", 2, 1024, 1024, 3, 1, 1), ("gen4 3x3 1024", 4, 1024, 1024, 3, 1, 1),
         ("gen8 1x1 1024->2048", 8, 1024, 2048, 1, 1, 0), ("gen4 1x1 2048->2048", 4, 2048, 2048, 1, 1, 0),
         ("enc conv5 16 256->512", 16, 256, 512, 4, 2, 1), ("enc conv6 8 512->1024", 8, 512, 1024, 4, 2, 1),
         ("enc conv7 4 1024->1024", 4, 1024, 1024, 4, 2, 1)]
for name, H, ci, co, k, stride, pad in cases:
    Ho = (H + 2 * pad - k) // stride + 1
    fl = 2.0 * B * Ho * Ho * co * ci * k * k
    w0 = pack_conv(torch.randn(co, ci, k, k, device=DEV) * 0.05, dt)
    y = torch.empty(B, Ho, Ho, co, dtype=dt, device=DEV)
    ref = None
    for xpad, kpad in ((0, 0), (32, 0), (0, 32), (32, 32), (64, 64)):
        if kpad and not xpad and ci % 32 == 0:
            xpad_eff = 32   # the extra K block reads channels [ci, ci + 32) of the pixel: they must exist
        else:
            xpad_eff = xpad
        ldx = ci + xpad_eff
        xf = torch.zeros(B, H, H, ldx, device=DEV, dtype=dt)
        torch.manual_seed(0)
        xf[..., :ci] = torch.randn(B, H, H, ci, device=DEV).to(dt)
        w = torch.zeros(w0.shape[0], w0.shape[1] + kpad, dtype=dt, device=DEV)
        w[:, :w0.shape[1]] = w0

        def run():
            _lib.check(lib.ghost_conv2d_nhwc(_lib.gdtype(dt), xf.data_ptr(), B, H, H, ci, ldx, w.data_ptr(), co,
                                             w.shape[0], w.shape[1], k, k, stride, pad, None, None, 1.0, None, 0,
                                             0, y.data_ptr(), co, ws.data_ptr(), ws.numel(), st))
        try:
            us = timeit(run)
        except RuntimeError as e:
            print(f"{name:24s} ldx={ldx} Kpad={w.shape[1]}: {str(e)[:60]}", flush=True)
            continue
        if ref is None:
            ref = y.float().clone()
        err = float((y.float() - ref).abs().max())
        print(f"{name:24s} ldx={ldx:5d} Kpad={w.shape[1]:6d} {us:8.1f} us {fl / us / 1e6:7.1f} TF/s  (max|d| vs first {err:.1e})",
              flush=True)
