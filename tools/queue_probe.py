"""Which HIP streams of this process share a hardware queue (the D2H / video legs regressed
when another leg ran first and created more streams than the box's GPU_MAX_HW_QUEUES = 4).

For every ordered pair (i, j) of the streams below: a ~30 ms spin kernel on stream i, then on stream j a tiny kernel
(or a 1 MB D2H copy into pinned memory) and an event; the host polls the event for 10 ms.  If it completes while
i still spins, i and j run on different queues ('.'); if not, j's work sat behind i's ('X').

    python tools/queue_probe.py [--extra N]     # N extra pool streams beyond the bench's own
"""
import argparse
import time

import torch


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--extra", type=int, default=6)
    ap.add_argument("--set", action="store_true", help="create ghost_amd's StreamSet first (side, d2h, h2d)")
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    torch.cuda.init()
    names = ["cur"]
    streams = [torch.cuda.current_stream(dev)]
    if a.set:
        import os
        import sys
        sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        from ghost_amd.inference.streams import stream_set
        ss = stream_set(dev)
        names += ["side", "d2h", "h2d"]
        streams += [ss.side, ss.d2h, ss.h2d]
    for i in range(a.extra):
        names.append(f"pool{i}")
        streams.append(torch.cuda.Stream(dev))
    hp = torch.cuda.Stream(dev, priority=-1)
    names.append("hiprio")
    streams.append(hp)
    small = torch.zeros(16, device=dev)
    dsrc = torch.zeros(1 << 20, dtype=torch.uint8, device=dev)
    host = torch.empty(1 << 20, dtype=torch.uint8, pin_memory=True)
    torch.cuda._sleep(1000)
    torch.cuda.synchronize()
    # calibrate the spin: cycles for ~30 ms
    t0 = time.perf_counter()
    torch.cuda._sleep(10_000_000)
    torch.cuda.synchronize()
    per = (time.perf_counter() - t0) / 10_000_000
    cyc = int(0.030 / per)
    print(f"spin: {per * 1e9:.3f} ns/cycle -> {cyc} cycles for 30 ms", flush=True)
    for kind in ("kernel", "d2h"):
        print(f"\n{kind}: row = spinning stream, column = probed stream ('X' = blocked behind the spin)")
        print("          " + " ".join(f"{n:>7}" for n in names))
        for i, si in enumerate(streams):
            row = []
            for j, sj in enumerate(streams):
                if i == j:
                    row.append("      -")
                    continue
                torch.cuda.synchronize()
                with torch.cuda.stream(si):
                    torch.cuda._sleep(cyc)
                with torch.cuda.stream(sj):
                    if kind == "kernel":
                        small.add_(1)
                    else:
                        host.copy_(dsrc, non_blocking=True)
                    ev = torch.cuda.Event()
                    ev.record(sj)
                t1 = time.perf_counter()
                done = False
                while time.perf_counter() - t1 < 0.010:
                    if ev.query():
                        done = True
                        break
                row.append("      ." if done else "      X")
                torch.cuda.synchronize()
            print(f"{names[i]:>9} " + " ".join(row), flush=True)


if __name__ == "__main__":
    main()
