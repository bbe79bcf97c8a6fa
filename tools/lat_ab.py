"""B = 1 latency of swap_u8 (bf16 / fp32) for same-box A/B: python tools/lat_ab.py [n] [option=v0,v1 ...].

Without option arguments: the plan as configured (env knobs of a tuning build apply).  With option arguments
(AEI_Net.set_option names, e.g. fuse_reduce=0,1): every value is timed eager and graphed in the same process,
interleaved over three rounds, one JSON line per (dtype, option value)."""
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def timed(fn, n):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    lat = []
    for _ in range(n):
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        lat.append(time.perf_counter() - t0)
    return float(np.median(lat)) * 1e3


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 50
    opts = [a.split("=") for a in sys.argv[2:]]
    dev = torch.device("cuda", 0)
    bench.stream_set(dev)
    crop = torch.from_numpy(np.random.Generator(np.random.PCG64(21)).integers(0, 256, (1, 256, 256, 3),
                                                                           dtype=np.uint8)).to(dev)
    z = bench.identity_rows(1, dev)
    if not opts:
        out = {"env": {k: v for k, v in os.environ.items() if k.startswith("GHOST_")}}
        from ghost_amd.inference import GraphedSwap
        for name, dt in (("bf16", torch.bfloat16), ("fp32", torch.float32)):
            G = bench.make_model("unet", 2, dt, dev)
            y = torch.empty(1, 256, 256, 3, dtype=torch.uint8, device=dev)
            out[name] = round(timed(lambda: G.swap_u8(crop, z, out=y), n), 3)
            gs = GraphedSwap(G, 1, dev)
            out[name + "_graphed"] = round(timed(lambda: gs(crop, z, out=y), n), 3)
            del gs, G
        print(json.dumps(out), flush=True)
        return
    from ghost_amd.inference import GraphedSwap
    for name, dt in (("bf16", torch.bfloat16), ("fp32", torch.float32)):
        G = bench.make_model("unet", 2, dt, dev)
        y = torch.empty(1, 256, 256, 3, dtype=torch.uint8, device=dev)
        res = {}
        for rnd in range(3):
            for opt, vals in opts:
                for v in vals.split(","):
                    G.set_option(opt, int(v))
                    e = timed(lambda: G.swap_u8(crop, z, out=y), n)
                    gs = GraphedSwap(G, 1, dev)
                    g = timed(lambda: gs(crop, z, out=y), n)
                    del gs
                    res.setdefault((opt, v), []).append((e, g))
        for (opt, v), r in res.items():
            print(json.dumps({"dtype": name, opt: int(v), "eager_ms": [round(a, 3) for a, _ in r],
                              "graphed_ms": [round(b, 3) for _, b in r]}), flush=True)
        del G


if __name__ == "__main__":
    main()
