"""Probe: two batches in flight on two HIP streams created with hipExtStreamCreateWithCUMask (each stream
restricted to a subset of the 256 CUs), against unrestricted streams.  python tools/cumask_probe.py"""
import ctypes
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ghost_amd.network import AEI_Net  # noqa: E402
from oracle import aei_ref  # noqa: E402

dev = torch.device("cuda:0")
hip = ctypes.CDLL("libamdhip64.so")
ncu = torch.cuda.get_device_properties(0).multi_processor_count
print("CUs:", ncu, flush=True)


def masked_stream(bits):
    words = (ncu + 31) // 32
    arr = (ctypes.c_uint32 * words)()
    for b in bits:
        arr[b // 32] |= 1 << (b % 32)
    s = ctypes.c_void_p()
    rc = hip.hipExtStreamCreateWithCUMask(ctypes.byref(s), ctypes.c_uint32(words), arr)
    assert rc == 0, rc
    return torch.cuda.ExternalStream(s.value, device=dev)


B = 64
G = AEI_Net("unet", num_blocks=2, c_id=512, compute_dtype=torch.bfloat16).eval()
G.load_state_dict(aei_ref.make_weights(aei_ref.param_specs("unet", 2)))
G = G.to(dev)
crops = torch.from_numpy(np.random.Generator(np.random.PCG64(3)).integers(0, 256, (B, 256, 256, 3), dtype=np.uint8)).to(dev)
z = torch.randn(1, 512, device=dev)
outs = [torch.empty(B, 256, 256, 3, dtype=torch.uint8, device=dev) for _ in range(4)]


def run(streams, n):
    main = torch.cuda.current_stream(dev)
    for s in streams:
        s.wait_stream(main)
    for k in range(n):
        s = streams[k % len(streams)]
        with torch.cuda.stream(s):
            G.swap_u8(crops, z, out=outs[k % len(streams)])
    for s in streams:
        main.wait_stream(s)


def bench(name, streams, steps=20):
    run(streams, 4)
    torch.cuda.synchronize()
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0.record()
    run(streams, steps)
    t1.record()
    torch.cuda.synchronize()
    ms = t0.elapsed_time(t1) / steps
    print(f"{name:40s} {ms:.3f} ms/batch {B / ms * 1e3:8.0f} frames/s", flush=True)


full = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
half_lo = list(range(ncu // 2))
half_hi = list(range(ncu // 2, ncu))
even = list(range(0, ncu, 2))
odd = list(range(1, ncu, 2))
cfgs = [("unmasked x2", full),
        ("halves (bits 0-127 / 128-255)", [masked_stream(half_lo), masked_stream(half_hi)]),
        ("interleaved (even / odd bits)", [masked_stream(even), masked_stream(odd)]),
        ("overlap 3/4 each", [masked_stream(range(0, 3 * ncu // 4)), masked_stream(range(ncu // 4, ncu))]),
        ("one stream", [torch.cuda.Stream(dev)])]
for name, st in cfgs + cfgs[:2]:
    bench(name, st)
