"""GraphedSwap (one chain) against eager swap_u8 for fuse_reduce 0 / 1 at a batch size:
python tools/graph_fuse_check.py [B] [two_streams] — prints, per setting, the fraction of output bytes that differ."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import aei_ref  # noqa: E402  (synthetic weights and inputs: test infrastructure)


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    ts = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    from ghost_amd.inference import GraphedSwap
    from ghost_amd.network import AEI_Net
    dev = torch.device("cuda:0")
    G = AEI_Net("unet", num_blocks=2, c_id=512, compute_dtype=torch.bfloat16).eval()
    G.load_state_dict(aei_ref.make_weights(aei_ref.param_specs("unet", 2)))
    G = G.to(dev)
    for fuse in (0, 1):
        G.set_option("fuse_reduce", fuse)
        g = GraphedSwap(G, B, dev, two_streams=ts)
        for seed in (3, 4, 5):
            crops = torch.from_numpy(aei_ref.make_u8_crops(B, seed)).to(dev)
            z = torch.randn(1, 512, generator=torch.Generator().manual_seed(seed)).to(dev)
            got = g(crops, z).clone()
            ref = G.swap_u8(crops, z)
            torch.cuda.synchronize()
            diff = (got != ref).float().mean().item()
            rows = [(got[i] != ref[i]).float().mean().item() for i in range(B)]
            print(f"B={B} ts={ts} fuse_reduce={fuse} seed={seed}: differing bytes {diff:.4f} per row "
                  f"{[round(r, 3) for r in rows]}", flush=True)
        del g


if __name__ == "__main__":
    main()
