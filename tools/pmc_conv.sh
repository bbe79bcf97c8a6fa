# PMC breakdown of the persistent halo conv: bash tools/pmc_conv.sh H CIN COUT (outputs gpurun_out/pmc_conv_H.txt)
set -e
export TMPDIR=/tmp
H=$1; CI=$2; CO=$3
R=/tmp/pmcconv_$H; rm -rf $R; mkdir -p $R gpurun_out
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS --output-format csv -d $R/a -o run -- python3 tools/run_conv.py $H $CI $CO 3 > $R/a.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAVES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC --output-format csv -d $R/b -o run -- python3 tools/run_conv.py $H $CI $CO 3 > $R/b.log 2>&1 || true
python3 - "$R" "$H" <<'PY' > gpurun_out/pmc_conv_$2.txt 2>&1
import csv, glob, sys, collections
R, H = sys.argv[1], sys.argv[2]
acc = collections.defaultdict(list)
for f in glob.glob(R + "/*/run_counter_collection.csv") + glob.glob(R + "/*/*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "halo" in r["Kernel_Name"] or "conv" in r["Kernel_Name"]:
            acc[(r["Kernel_Name"][:80], r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(acc.items()):
    print(f"{c:28s} {sum(v)/len(v):16.0f}  n={len(v)}  {k}")
PY
tail -3 $R/a.log >> gpurun_out/pmc_conv_$H.txt
