# Same-box A/B of one AAD shape under PMC (tuning build: GHOST_KNOB variants):
#   bash tools/pmc_ab.sh "C Ca n L up" NAME1:ENV=V,ENV=V NAME2:ENV=V ...
# per variant: run time (tools/run_aad.py), FETCH_SIZE / WRITE_SIZE (separate passes, gfx950 FETCH x2) and SQ
# counters -> gpurun_out/pmc_ab.txt
set -e
export TMPDIR=/tmp PYTHONUNBUFFERED=1 GHOST_TUNING=1
SHAPE=$1; shift
OUT=gpurun_out/pmc_ab.txt
mkdir -p gpurun_out; : > $OUT
for v in "$@"; do
  name=${v%%:*}; envs=${v#*:}
  R=/tmp/pmcab_$name; rm -rf $R; mkdir -p $R
  ENVS=$(echo "$envs" | tr ',' ' ')
  echo "== $name ($envs)" >> $OUT
  env $ENVS timeout -k 10 120 python3 tools/run_aad.py $SHAPE 10 >> $OUT 2>&1
  env $ENVS timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/f -o run -- python3 tools/run_aad.py $SHAPE 3 > $R/f.log 2>&1
  env $ENVS timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/w -o run -- python3 tools/run_aad.py $SHAPE 3 > $R/w.log 2>&1
  env $ENVS timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU --output-format csv -d $R/q -o run -- python3 tools/run_aad.py $SHAPE 3 > $R/q.log 2>&1
  python3 - "$R" >> $OUT 2>&1 <<'PY'
import csv, glob, sys, collections
R = sys.argv[1]
acc = collections.defaultdict(list)
for f in glob.glob(R + "/*/run_counter_collection.csv") + glob.glob(R + "/*/*/run_counter_collection.csv"):
    for r in csv.DictReader(open(f)):
        if "aad_v" in r["Kernel_Name"]:
            acc[(r["Kernel_Name"].split("(")[0][-40:], r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(acc.items()):
    m = sum(v) / len(v)
    extra = f"  -> {2 * m * 1024 / 1e6:.1f} MB read" if c == "FETCH_SIZE" else (f"  -> {m * 1024 / 1e6:.1f} MB written" if c == "WRITE_SIZE" else "")
    print(f"  {c:24s} {m:16.0f}  n={len(v)}  {k}{extra}")
PY
done
