"""Probe: throughput of consecutive swap_u8 batches issued on one stream vs alternating between two HIP streams
(two batches in flight; each stream its own output buffer, the runtime's workspace comes per stream from torch's
caching allocator).  python tools/pipe_probe.py [steps]"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ghost_amd.network import AEI_Net  # noqa: E402
from oracle import aei_ref  # noqa: E402

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
dev = torch.device("cuda:0")
B = 64
G = AEI_Net("unet", num_blocks=2, c_id=512, compute_dtype=torch.bfloat16).eval()
G.load_state_dict(aei_ref.make_weights(aei_ref.param_specs("unet", 2)))
G = G.to(dev)
crops = torch.from_numpy(np.random.Generator(np.random.PCG64(3)).integers(0, 256, (B, 256, 256, 3), dtype=np.uint8)).to(dev)
z = torch.randn(1, 512, device=dev)
z = z / z.norm()
streams = [torch.cuda.current_stream(dev), torch.cuda.Stream(dev), torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
outs = [torch.empty(B, 256, 256, 3, dtype=torch.uint8, device=dev) for _ in streams]


def run(nstreams, n):
    main = torch.cuda.current_stream(dev)
    ev = torch.cuda.Event()
    ev.record(main)
    for s in streams[1:nstreams]:
        s.wait_event(ev)
    for k in range(n):
        s = streams[k % nstreams]
        with torch.cuda.stream(s):
            G.swap_u8(crops, z, out=outs[k % nstreams])
    for s in streams[1:nstreams]:
        e = torch.cuda.Event()
        e.record(s)
        main.wait_event(e)


for opt in (1, 0):
    G.set_option("two_streams", opt)
    for ns in (1, 2, 3, 1, 2):
        run(ns, 4)
        torch.cuda.synchronize()
        t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        t0.record()
        run(ns, steps)
        t1.record()
        torch.cuda.synchronize()
        ms = t0.elapsed_time(t1) / steps
        print(f"two_streams={opt} caller streams={ns}: {ms:.3f} ms/batch, {B / ms * 1e3:.0f} frames/s", flush=True)
# the alternating-stream outputs equal the single-stream output
run(1, 1); torch.cuda.synchronize(); ref = outs[0].clone()
run(2, 2); torch.cuda.synchronize()
print("outputs identical:", bool(torch.equal(outs[0], ref)), bool(torch.equal(outs[1], ref)))
