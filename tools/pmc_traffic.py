"""Summarise rocprofv3 PMC passes into per-kernel HBM traffic.

    python tools/pmc_traffic.py FETCH_CSV WRITE_CSV [--out profiles/rNN_traffic.json]

FETCH_CSV / WRITE_CSV are the ``*_counter_collection.csv`` files of two separate
``rocprofv3 --pmc FETCH_SIZE`` and ``--pmc WRITE_SIZE`` runs of the same command
(they cannot share a pass on gfx950: MI355X_MICROARCH.md §rocprofv3 PMC slots).
Correction per MI355X_MICROARCH.md §HBM: FETCH_SIZE (KB) reports half the bytes of a
wide coalesced stream on gfx950, so read bytes = 2 * FETCH_SIZE * 1024; write bytes =
WRITE_SIZE * 1024.  Output: per kernel name and grid size, mean bytes per dispatch.
"""
from __future__ import annotations

import argparse
import collections
import csv
import json


def load(path, counter):
    acc = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        acc[(r["Kernel_Name"], int(r["Grid_Size"]))].append(float(r["Counter_Value"]))
    return acc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch")
    ap.add_argument("write")
    ap.add_argument("--out")
    ap.add_argument("--source", default="rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes")
    a = ap.parse_args()
    f = load(a.fetch, "FETCH_SIZE")
    w = load(a.write, "WRITE_SIZE")
    rows = []
    for key in sorted(set(f) | set(w)):
        fv, wv = f.get(key, []), w.get(key, [])
        rd = 2.0 * 1024 * sum(fv) / len(fv) if fv else None
        wr = 1024 * sum(wv) / len(wv) if wv else None
        rows.append({"kernel": key[0], "grid": key[1], "dispatches": max(len(fv), len(wv)),
                     "read_bytes": rd, "write_bytes": wr,
                     "hbm_bytes": (rd or 0) + (wr or 0) if rd is not None and wr is not None else None})
    rows.sort(key=lambda r: -(r["hbm_bytes"] or 0) * r["dispatches"])
    for r in rows[:25]:
        print(f"{r['dispatches']:4d} x grid {r['grid']:>10}  read {r['read_bytes'] or 0:14.0f}  "
              f"write {r['write_bytes'] or 0:14.0f}  {r['kernel'][:90]}")
    if a.out:
        json.dump({"correction": "read = 2*FETCH_SIZE*1024 (gfx950 half-count), write = WRITE_SIZE*1024",
                   "source": a.source, "kernels": rows}, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
