"""Kernel sequence of the last bench step from a rocprofv3 database:
python tools/step_trace.py gpurun_out/<dir>/run_results.db  (a step starts at crops_kernel)."""
import re
import sqlite3
import sys

con = sqlite3.connect(sys.argv[1])
cur = con.cursor()
rows = cur.execute("select d.start, d.end, d.grid_size_x, d.workgroup_size_x, s.kernel_name from rocpd_kernel_dispatch d "
                   "join rocpd_info_kernel_symbol s on d.kernel_id = s.id order by d.start").fetchall()
starts = [i for i, r in enumerate(rows) if "crops_kernel" in r[4]]
if len(starts) >= 2:
    rows = rows[starts[-2]:starts[-1]]
elif starts:
    rows = rows[starts[-1]:]
tot = 0.0
for st, en, g, wg, name in rows:
    us = (en - st) / 1e3
    tot += us
    short = re.sub(r"\(.*", "", name.replace("void ghost::", "").replace("ghost::", ""))[:70]
    print(f"{us:8.1f} us  grid={g:<9d} wg={wg:<4d} {short}")
span = (rows[-1][1] - rows[0][0]) / 1e3 if rows else 0.0
print(f"sum {tot:.1f} us over {len(rows)} kernels, span {span:.1f} us")
