"""Per-(kernel, grid) table from a rocprofv3 kernel trace, optionally joined with PMC passes.

    python tools/kernel_table.py TRACE_CSV|RESULTS_DB [PMC_CSV ...] [--top 30] [--stats-csv OUT]

TRACE may be a rocprofv3 kernel-trace CSV or the run's rocpd SQLite database (*.db, the
default output format of rocprofv3 7.x); --stats-csv writes the per-kernel summary
(name, calls, total/avg/min/max ns, percent) like rocprofv3 --stats.

Durations are averaged per (kernel name, grid size); PMC counters are averaged per
dispatch with the same key.  Derived: MFMA busy fraction = SQ_VALU_MFMA_BUSY_CYCLES /
(GRBM_GUI_ACTIVE * CUs ... ) is left to the reader; the raw means are printed.
"""
from __future__ import annotations

import argparse
import collections
import csv
import re


def short(name: str) -> str:
    m = re.match(r"_ZN5ghost\d+(\w+?)I(.*)EEvNS_8ConvArgsE", name)
    if m:
        return f"{m.group(1)}<{m.group(2)}>"
    m = re.match(r"_ZN5ghost\d+(\w+?)I", name)
    return m.group(1) if m else name[:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("pmc", nargs="*")
    ap.add_argument("--top", type=int, default=40)
    ap.add_argument("--stats-csv")
    a = ap.parse_args()
    dur = collections.defaultdict(list)
    if a.trace.endswith(".db"):
        import sqlite3
        db = sqlite3.connect(a.trace)
        q = ("select s.kernel_name, d.grid_size_x * d.grid_size_y * d.grid_size_z, d.end - d.start "
             "from rocpd_kernel_dispatch d join rocpd_info_kernel_symbol s on d.kernel_id = s.id")
        for name, grid, ns in db.execute(q):
            dur[(name, int(grid))].append(ns / 1e3)
    else:
        for r in csv.DictReader(open(a.trace)):
            key = (r["Kernel_Name"], int(r["Grid_Size_X"]) * int(r.get("Grid_Size_Y", 1)) * int(r.get("Grid_Size_Z", 1))
                   if "Grid_Size_X" in r else int(r["Grid_Size"]))
            dur[key].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    if a.stats_csv:
        by_name = collections.defaultdict(list)
        for (name, _g), ds in dur.items():
            by_name[name] += ds
        tot = sum(sum(v) for v in by_name.values())
        with open(a.stats_csv, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs"])
            for name, ds in sorted(by_name.items(), key=lambda kv: -sum(kv[1])):
                w.writerow([name, len(ds), round(sum(ds) * 1e3), round(sum(ds) / len(ds) * 1e3),
                            round(sum(ds) / tot * 100, 3), round(min(ds) * 1e3), round(max(ds) * 1e3)])
    pmc = collections.defaultdict(lambda: collections.defaultdict(list))
    for path in a.pmc:
        for r in csv.DictReader(open(path)):
            pmc[(r["Kernel_Name"], int(r["Grid_Size"]))][r["Counter_Name"]].append(float(r["Counter_Value"]))
    total = sum(sum(v) for v in dur.values())
    rows = sorted(dur.items(), key=lambda kv: -sum(kv[1]))
    for (name, grid), ds in rows[:a.top]:
        extra = ""
        if (name, grid) in pmc:
            extra = " ".join(f"{k}={sum(v) / len(v):.3g}" for k, v in sorted(pmc[(name, grid)].items()))
        print(f"{sum(ds) / total * 100:5.1f}% {len(ds):4d}x {sum(ds) / len(ds):9.1f}us grid={grid:<10} {short(name)[:70]} {extra}")


if __name__ == "__main__":
    main()
