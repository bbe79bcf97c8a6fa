"""Which part of bench.py's config5_multi leg slows the legs that run after it.

Measures the D2H-inclusive config-2 rate (bench.d2h_leg) after each step of what config5_multi does, one at a time:
build a second (linknet/3) model, swap with it once, run model_inference_multi with device output, then with host
output (pinned host memory), then drop the model.

    python tools/leg_probe.py
"""
import gc
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from ghost_amd.inference.streams import stream_set  # noqa: E402


def main():
    dev = torch.device("cuda", 0)
    stream_set(dev)
    G = bench.make_model("unet", 2, torch.bfloat16, dev)
    B = 64
    crops = torch.from_numpy(np.random.Generator(np.random.PCG64(1000)).integers(0, 256, size=(B, 256, 256, 3),
                                                                              dtype=np.uint8)).to(dev)
    zs = bench.identity_rows(1, dev)
    table = G.identity_table(zs)
    idx = torch.zeros(B, dtype=torch.int32, device=dev)

    def swap(c, o):
        return G.swap_u8_indexed(c, table, idx, out=o)

    def d2h(tag):
        r = bench.d2h_leg(swap, crops, 20, 2)
        print(json.dumps({"after": tag, "d2h": r["windows_frames_per_s"]}), flush=True)

    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("--order", default="d2h,model,swap5,c5dev,d2h,c5host,d2h,drop,d2h",
                    help="comma list of d2h / model / swap5 / c5dev / c5host / drop / gc / bench5 (bench.config5_multi_leg)")
    a = ap.parse_args()
    from ghost_amd.inference.dp import model_inference_multi
    G5 = None
    rng = np.random.Generator(np.random.PCG64(55))
    pool = rng.integers(0, 256, size=(48, 224, 224, 3), dtype=np.uint8)
    present = rng.random((4, 240)) > 0.1
    embeds = bench.identity_rows(4, torch.device("cpu"))
    idents = [([pool[(q * 7 + i) % 48] if present[q, i] else [] for i in range(240)], embeds[q:q + 1])
              for q in range(4)]
    done = []
    ss = stream_set(dev)
    named = {"cur": torch.cuda.current_stream(dev), "side": ss.side, "d2h": ss.d2h, "h2d": ss.h2d}

    def qcheck(tag):
        """'X' when work on the second stream waited for a 30 ms spin on the first (a shared hardware queue)."""
        import time
        small = torch.zeros(16, device=dev)
        out = {}
        for x in named:
            for y in named:
                if x >= y:
                    continue
                torch.cuda.synchronize()
                with torch.cuda.stream(named[x]):
                    torch.cuda._sleep(70_000_000)
                with torch.cuda.stream(named[y]):
                    small.add_(1)
                    ev = torch.cuda.Event()
                    ev.record(named[y])
                t1 = time.perf_counter()
                ok = False
                while time.perf_counter() - t1 < 0.010:
                    if ev.query():
                        ok = True
                        break
                out[f"{x}/{y}"] = "." if ok else "X"
                torch.cuda.synchronize()
        print(json.dumps({"after": tag, "queues": out}), flush=True)

    def up_of(model, name):
        import ctypes as C
        ptr = C.c_void_p()
        model._rt.lib.ghost_aei_up_stream(model._rt.h, 0, C.byref(ptr))
        if ptr.value:
            named[name] = torch.cuda.ExternalStream(ptr.value, device=dev)

    for step in a.order.split(","):
        if step == "upG":
            up_of(G, "upG")
            continue
        if step == "upG5":
            up_of(G5, "upG5")
            continue
        if step == "d2h":
            d2h("+".join(done) or "start")
            continue
        if step == "q":
            qcheck("+".join(done) or "start")
            continue
        if step == "model":
            G5 = bench.make_model("linknet", 3, torch.bfloat16, dev)
        elif step == "swap5":
            c5 = torch.from_numpy(np.random.Generator(np.random.PCG64(5)).integers(0, 256, size=(64, 256, 256, 3),
                                                                                dtype=np.uint8)).to(dev)
            G5.swap_u8(c5, zs)
        elif step in ("c5dev", "c5host"):
            for _ in range(4):
                r = model_inference_multi(idents, G5, BS=64, device=dev, collect="rank0",
                                          output="device" if step == "c5dev" else "host")
                del r
        elif step == "drop":
            del G5
            G5 = None
            torch.cuda.empty_cache()
        elif step == "gc":
            gc.collect()
        elif step == "bench5":
            bench.config5_multi_leg(dev, 1, 240)
        elif step == "pipe":                 # bench.py's headline loop: 25 batches through GatherPipeline(streams=2)
            from ghost_amd.inference.dp import GatherPipeline
            pipe = GatherPipeline(swap, (B, 256, 256, 3), dev, depth=2, streams=2)
            for _ in range(25):
                pipe.submit(crops)
            pipe.drain()
        elif step == "pipe1":                # its one-batch-at-a-time profile pass
            from ghost_amd.inference.dp import GatherPipeline
            p1 = GatherPipeline(swap, (B, 256, 256, 3), dev, depth=2, streams=1)
            for _ in range(20):
                p1.submit(crops)
            p1.drain()
        torch.cuda.synchronize()
        done.append(step)


if __name__ == "__main__":
    main()
