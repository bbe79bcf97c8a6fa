"""B = 1 latency of swap_u8 (bf16 / fp32) for same-box A/B of plan knobs: python tools/lat_ab.py [n]."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    dev = torch.device("cuda", 0)
    bench.stream_set(dev)
    crop = torch.from_numpy(np.random.Generator(np.random.PCG64(21)).integers(0, 256, (1, 256, 256, 3),
                                                                           dtype=np.uint8)).to(dev)
    z = bench.identity_rows(1, dev)
    out = {"env": {k: v for k, v in os.environ.items() if k.startswith("GHOST_")}}
    for name, dt in (("bf16", torch.bfloat16), ("fp32", torch.float32)):
        G = bench.make_model("unet", 2, dt, dev)
        y = torch.empty(1, 256, 256, 3, dtype=torch.uint8, device=dev)
        for _ in range(10):
            G.swap_u8(crop, z, out=y)
        torch.cuda.synchronize()
        lat = []
        for _ in range(n):
            t0 = time.perf_counter()
            G.swap_u8(crop, z, out=y)
            torch.cuda.synchronize()
            lat.append(time.perf_counter() - t0)
        out[name] = round(float(np.median(lat)) * 1e3, 3)
        del G
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
