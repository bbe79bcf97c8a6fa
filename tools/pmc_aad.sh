# PMC breakdown of one AAD kernel shape: bash tools/pmc_aad.sh C Ca n L up (outputs gpurun_out/pmc_aad_<n>_<L>_<up>.txt)
set -e
export TMPDIR=/tmp
C=$1; CA=$2; N=$3; L=$4; UP=$5; TAG=${N}_${L}_${UP}
R=/tmp/pmcaad_$TAG; rm -rf $R; mkdir -p $R gpurun_out
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS --output-format csv -d $R/a -o run -- python3 tools/run_aad.py $C $CA $N $L $UP 3 > $R/a.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_SALU SQ_BUSY_CYCLES SQ_WAVES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_WAIT_INST_LDS SQ_ACTIVE_INST_MISC --output-format csv -d $R/b -o run -- python3 tools/run_aad.py $C $CA $N $L $UP 3 > $R/b.log 2>&1 || true
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR --output-format csv -d $R/c -o run -- python3 tools/run_aad.py $C $CA $N $L $UP 3 > $R/c.log 2>&1 || true
python3 - "$R" <<'PY' > gpurun_out/pmc_aad_$TAG.txt 2>&1
import csv, glob, sys, collections
R = sys.argv[1]
acc = collections.defaultdict(list)
for f in glob.glob(R + "/*/run_counter_collection.csv") + glob.glob(R + "/*/*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "aad" in r["Kernel_Name"]:
            acc[(r["Kernel_Name"][:60], r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(acc.items()):
    print(f"{c:28s} {sum(v)/len(v):16.0f}  n={len(v)}  {k}")
PY
tail -2 $R/a.log >> gpurun_out/pmc_aad_$TAG.txt
