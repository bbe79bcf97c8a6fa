"""Per-kernel MFMA / VALU utilisation from rocprofv3 --pmc passes (tools/pmc_mfma.sh).

    python tools/pmc_mfma.py --gen P1.csv P2.csv --arc P3.csv P4.csv --out profiles/r04_mfma.json

Counters (MI355X_MICROARCH.md: SQ_WAVE_CYCLES / SQ_WAIT_* / SQ_ACTIVE_INST_* count quad-cycles,
SQ_VALU_MFMA_BUSY_CYCLES counts cycles; GRBM_GUI_ACTIVE is summed over the 8 XCDs):
* clock cycles of a dispatch  = GRBM_GUI_ACTIVE / 8
* mfma_busy                   = SQ_VALU_MFMA_BUSY_CYCLES / (clock cycles * 1024 SIMDs)  -- the fraction of SIMD
                                cycles the matrix core was busy during the dispatch (the rocprof MFMA-util metric)
* mfma_cycles_per_inst        = SQ_VALU_MFMA_BUSY_CYCLES / SQ_INSTS_MFMA (16 for v_mfma_f32_16x16x32_bf16 if the busy
                                counter sums SIMD cycles: the calibration of the line above)
* valu_per_mfma               = SQ_INSTS_VALU / SQ_INSTS_MFMA (issue pressure beside the matrix work)
* wait_frac / active_frac     = SQ_WAIT_ANY / SQ_WAVE_CYCLES, SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES
* eff_clock_ghz               = clock cycles / dispatch duration (when the csv carries timestamps)
Rows: mean per dispatch of each (kernel, grid); ``totals``: the sums over every dispatch of a program.
"""
from __future__ import annotations

import argparse
import collections
import csv
import json
import re

N_SIMD = 256 * 4
N_XCD = 8


def load(paths):
    """(kernel, grid) -> counter -> [values per dispatch]; also durations per (kernel, grid)."""
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    dur = collections.defaultdict(dict)
    for p in paths:
        for r in csv.DictReader(open(p)):
            key = (r["Kernel_Name"], int(r["Grid_Size"]))
            acc[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
            s, e = r.get("Start_Timestamp"), r.get("End_Timestamp")
            if s and e:
                dur[key][(p, r.get("Dispatch_Id"))] = (float(e) - float(s))
    return acc, dur


def short(name):
    name = re.sub(r"^void ", "", name)
    name = re.sub(r"\(.*$", "", name)
    return name.replace("ghost::", "")[:110]


def rows_of(acc, dur):
    rows = []
    tot = collections.Counter()
    for key, cs in acc.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        n = max(len(v) for v in cs.values())
        for c, v in cs.items():
            tot[c] += sum(v)
        clk = m.get("GRBM_GUI_ACTIVE", 0) / N_XCD
        r = {"kernel": short(key[0]), "grid": key[1], "dispatches": n}
        if clk:
            r["clock_cycles"] = round(clk)
        if "SQ_VALU_MFMA_BUSY_CYCLES" in m and clk:
            r["mfma_busy"] = round(m["SQ_VALU_MFMA_BUSY_CYCLES"] / (clk * N_SIMD), 4)
        if m.get("SQ_INSTS_MFMA"):
            r["mfma_insts"] = m["SQ_INSTS_MFMA"]
            if "SQ_VALU_MFMA_BUSY_CYCLES" in m:
                r["mfma_cycles_per_inst"] = round(m["SQ_VALU_MFMA_BUSY_CYCLES"] / m["SQ_INSTS_MFMA"], 2)
            if "SQ_INSTS_VALU" in m:
                r["valu_per_mfma"] = round(m["SQ_INSTS_VALU"] / m["SQ_INSTS_MFMA"], 2)
        for c in ("SQ_INSTS_VALU", "SQ_INSTS_LDS", "SQ_INSTS_SALU", "SQ_WAVES"):
            if c in m:
                r[c.lower()[3:]] = m[c]
        wc = m.get("SQ_WAVE_CYCLES")
        for c, nm in (("SQ_WAIT_ANY", "wait_frac"), ("SQ_WAIT_INST_ANY", "wait_inst_frac"),
                      ("SQ_ACTIVE_INST_ANY", "active_frac"), ("SQ_ACTIVE_INST_VALU", "active_valu_frac"),
                      ("SQ_ACTIVE_INST_LDS", "active_lds_frac"), ("SQ_INST_CYCLES_VMEM", "vmem_cycles_frac")):
            if c in m and wc:
                r[nm] = round(m[c] / wc, 4)
        if "SQ_BUSY_CYCLES" in m and clk:
            r["sq_busy_per_clock"] = round(m["SQ_BUSY_CYCLES"] / clk, 3)
        if dur.get(key):
            d = sum(dur[key].values()) / len(dur[key])
            r["avg_ns"] = round(d)
            if clk:
                r["eff_clock_ghz"] = round(clk / d, 3)
        rows.append(r)
    rows.sort(key=lambda r: -(r.get("clock_cycles", 0) * r["dispatches"]))
    totals = {}
    clk = tot.get("GRBM_GUI_ACTIVE", 0) / N_XCD
    if clk:
        totals["clock_cycles"] = round(clk)
        if tot.get("SQ_VALU_MFMA_BUSY_CYCLES"):
            totals["mfma_busy"] = round(tot["SQ_VALU_MFMA_BUSY_CYCLES"] / (clk * N_SIMD), 4)
    if tot.get("SQ_INSTS_MFMA"):
        totals["valu_per_mfma"] = round(tot.get("SQ_INSTS_VALU", 0) / tot["SQ_INSTS_MFMA"], 2)
        totals["mfma_cycles_per_inst"] = round(tot.get("SQ_VALU_MFMA_BUSY_CYCLES", 0) / tot["SQ_INSTS_MFMA"], 2)
    return rows, totals


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gen", nargs="+", required=True)
    ap.add_argument("--arc", nargs="*", default=[])
    ap.add_argument("--out")
    ap.add_argument("--source", default="rocprofv3 --pmc")
    a = ap.parse_args()
    res = {"source": a.source,
           "definitions": {"mfma_busy": "SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE/8 * 1024 SIMDs)",
                           "mfma_cycles_per_inst": "SQ_VALU_MFMA_BUSY_CYCLES / SQ_INSTS_MFMA",
                           "valu_per_mfma": "SQ_INSTS_VALU / SQ_INSTS_MFMA",
                           "wait_frac": "SQ_WAIT_ANY / SQ_WAVE_CYCLES (both quad-cycles)",
                           "active_frac": "SQ_ACTIVE_INST_ANY / SQ_WAVE_CYCLES"}}
    for nm, paths in (("generator", a.gen), ("arcface", a.arc)):
        if not paths:
            continue
        rows, totals = rows_of(*load(paths))
        res[nm] = {"totals": totals, "kernels": rows}
        print(f"== {nm}: totals {totals}")
        for r in rows[:30]:
            print(f"{r['dispatches']:4d} x {r.get('clock_cycles', 0):9d} cyc  mfma {r.get('mfma_busy', '-')!s:7s} "
                  f"cyc/inst {r.get('mfma_cycles_per_inst', '-')!s:6s} valu/mfma {r.get('valu_per_mfma', '-')!s:7s} "
                  f"wait {r.get('wait_frac', '-')!s:6s}  {r['kernel'][:80]}")
    if a.out:
        json.dump(res, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
