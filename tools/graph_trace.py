"""Eager vs GraphedSwap at B = 1 (BASELINE config 1) for one dtype, laid out for a rocprofv3 kernel trace:
    rocprofv3 --kernel-trace -d DIR -o run -- python3 tools/graph_trace.py fp32
    python3 tools/graph_trace.py --analyze DIR/run_results.db
Phase 1: 5 eager swap_u8 calls, synchronised after each; a 50 ms pause; phase 2: 5 graph replays, synchronised
after each.  --analyze splits the trace at the pause and prints, per phase, the per-call span (first kernel start
to last kernel end), the kernel time summed, and the kernels whose duration differs most between the phases
(fp32 replays ran 2x slower than eager)."""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(dt_name):
    import numpy as np
    import torch
    from ghost_amd.inference import GraphedSwap
    from ghost_amd.network import AEI_Net
    from oracle.aei_ref import make_weights, param_specs   # synthetic weights (test infrastructure)
    dt = {"fp32": torch.float32, "bf16": torch.bfloat16}[dt_name]
    dev = torch.device("cuda:0")
    G = AEI_Net("unet", num_blocks=2, c_id=512, compute_dtype=dt).eval()
    G.load_state_dict(make_weights(param_specs("unet", 2)))
    G = G.to(dev)
    crop = torch.from_numpy(np.random.Generator(np.random.PCG64(21)).integers(0, 256, (1, 256, 256, 3),
                                                                           dtype=np.uint8)).to(dev)
    z = torch.randn(1, 512, generator=torch.Generator().manual_seed(2)).to(dev)
    y = torch.empty(1, 256, 256, 3, dtype=torch.uint8, device=dev)
    gs = GraphedSwap(G, 1, dev)
    for _ in range(3):
        G.swap_u8(crop, z, out=y)
        gs(crop, z, out=y)
    torch.cuda.synchronize()
    time.sleep(0.05)
    te = []
    for _ in range(5):
        t0 = time.perf_counter()
        G.swap_u8(crop, z, out=y)
        torch.cuda.synchronize()
        te.append(time.perf_counter() - t0)
    time.sleep(0.05)
    tg = []
    for _ in range(5):
        t0 = time.perf_counter()
        gs(crop, z, out=y)
        torch.cuda.synchronize()
        tg.append(time.perf_counter() - t0)
    print(f"{dt_name}: eager {np.median(te) * 1e3:.3f} ms, graphed {np.median(tg) * 1e3:.3f} ms (wall, median of 5)",
          flush=True)


def analyze(db):
    import collections
    import re
    import sqlite3
    rows = sqlite3.connect(db).execute(
        "select d.start, d.end, s.kernel_name from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s "
        "on d.kernel_id = s.id order by d.start").fetchall()
    # phases: split at gaps > 20 ms; calls: split at gaps > 200 us
    groups, cur = [], [rows[0]]
    for r in rows[1:]:
        if r[0] - cur[-1][1] > 20e6:
            groups.append(cur)
            cur = []
        cur.append(r)
    groups.append(cur)
    phases = groups[-2:]
    for name, ph in zip(("eager", "graphed"), phases):
        calls, c = [], [ph[0]]
        for r in ph[1:]:
            if r[0] - c[-1][1] > 200e3:
                calls.append(c)
                c = []
            c.append(r)
        calls.append(c)
        spans = [(cl[-1][1] - cl[0][0]) / 1e3 for cl in calls]
        ksum = [sum(r[1] - r[0] for r in cl) / 1e3 for cl in calls]
        print(f"{name}: {len(calls)} calls, kernels per call {[len(cl) for cl in calls]}, span us {[round(x) for x in spans]}, "
              f"kernel-sum us {[round(x) for x in ksum]}")
    per = []
    for ph in phases:
        d = collections.defaultdict(list)
        for st, en, nm in ph:
            d[re.sub(r"\(.*", "", nm)[:90]].append((en - st) / 1e3)
        per.append(d)
    diffs = []
    for k in per[0]:
        if k in per[1]:
            a, b = sum(per[0][k]) / len(per[0][k]), sum(per[1][k]) / len(per[1][k])
            diffs.append((b - a, a, b, len(per[0][k]), k))
    diffs.sort(reverse=True)
    for row in (diffs[:15] + [None] + diffs[-15:] if len(diffs) > 30 else diffs):
        if row is None:
            print("  ...")
            continue
        dd, a, b, n, k = row
        print(f"  {dd:+8.1f} us  eager {a:8.1f} graphed {b:8.1f}  x{n}  {k}")
    # gaps between consecutive kernels inside a call
    for name, ph in zip(("eager", "graphed"), phases):
        gaps = [(ph[i + 1][0] - ph[i][1]) / 1e3 for i in range(len(ph) - 1) if ph[i + 1][0] - ph[i][1] < 200e3]
        print(f"{name}: inter-kernel gaps inside calls: sum {sum(gaps):.0f} us over {len(gaps)}, max {max(gaps):.1f}")


if __name__ == "__main__":
    if sys.argv[1] == "--analyze":
        analyze(sys.argv[2])
    else:
        run(sys.argv[1])
