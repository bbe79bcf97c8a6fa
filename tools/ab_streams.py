"""Same-process A/B of the two-stream plan (GHOST_AEI_OPT_TWO_STREAMS): B = 64 unet/2 bf16 swaps,
alternating one-stream / two-stream rounds, HIP-event timed; also checks the two outputs are identical."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ghost_amd.network import AEI_Net  # noqa: E402
from oracle import aei_ref  # noqa: E402

dev = torch.device("cuda:0")
bb, nb = (sys.argv[1], int(sys.argv[2])) if len(sys.argv) > 2 else ("unet", 2)
G = AEI_Net(bb, num_blocks=nb, c_id=512, compute_dtype=torch.bfloat16).eval()
G.load_state_dict(aei_ref.make_weights(aei_ref.param_specs(bb, nb)))
G = G.to(dev)
B = 64
crops = torch.from_numpy(aei_ref.make_u8_crops(B, 3)).to(dev)
z = torch.randn(1, 512, device=dev)
outs = {}
for mode in (0, 1):
    G.set_option("two_streams", mode)
    outs[mode] = G.swap_u8(crops, z).clone()
torch.cuda.synchronize()
print("identical:", bool(torch.equal(outs[0], outs[1])), flush=True)
times = {0: [], 1: []}
out = torch.empty_like(outs[0])
for rnd in range(6):
    for mode in (0, 1):
        G.set_option("two_streams", mode)
        for _ in range(3):
            G.swap_u8(crops, z, out=out)
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda.synchronize()
        s.record()
        for _ in range(10):
            G.swap_u8(crops, z, out=out)
        e.record()
        torch.cuda.synchronize()
        times[mode].append(s.elapsed_time(e) / 10)
for mode in (0, 1):
    t = sorted(times[mode])
    print(f"{bb}/{nb} two_streams={mode}: median {t[len(t) // 2]:.3f} ms/step  min {t[0]:.3f}  "
          f"({B / t[len(t) // 2] * 1e3:.0f} frames/s)", flush=True)
