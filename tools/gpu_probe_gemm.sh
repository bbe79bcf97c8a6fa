set -e
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
R=/tmp/pg; rm -rf $R; mkdir -p $R
timeout -k 10 200 python3 tools/probe_gemm.py both > gpurun_out/probe_gemm.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum --output-format csv -d $R/a -o run -- python3 tools/probe_gemm.py lib > $R/a.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INST_CYCLES_VMEM SQ_WAVES --output-format csv -d $R/b -o run -- python3 tools/probe_gemm.py lib > $R/b.log 2>&1
python3 - $R >> gpurun_out/probe_gemm.log <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(list)
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "ghost" in r["Kernel_Name"]:
            acc[(r["Kernel_Name"][:70], r["Grid_Size"], r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, g, c), v in sorted(acc.items()):
    print(f"{c:26s} {sum(v)/len(v):16.0f} n={len(v):3d} grid={g} {k}")
PY
