# same-box A/B: aad_v4 XCD-contiguous block order (working tree) vs the saved library, kernel time + PMC fetch
set -e
export TMPDIR=/tmp PYTHONUNBUFFERED=1
mkdir -p gpurun_out
R=/tmp/v4xcd; rm -rf $R; mkdir -p $R
for lib in libghost_amd_ab.so libghost_amd.so libghost_amd_ab.so libghost_amd.so; do
  echo "== $lib" >> gpurun_out/v4xcd.log
  GHOST_LIB_FILE=$lib timeout -k 10 60 python3 tools/run_aad.py 64 64 256 2 1 20 >> gpurun_out/v4xcd.log 2>&1
done
for lib in libghost_amd_ab.so libghost_amd.so; do
  GHOST_LIB_FILE=$lib timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/f_$lib -o run -- python3 tools/run_aad.py 64 64 256 2 1 3 > $R/f_$lib.log 2>&1
  python3 - $R/f_$lib $lib >> gpurun_out/v4xcd.log <<'PY'
import csv, glob, sys
v = [float(r["Counter_Value"]) for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)
     for r in csv.DictReader(open(f)) if "aad_v4" in r["Kernel_Name"]]
print(sys.argv[2], "aad_v4 FETCH bytes x2 per launch (MB):", [round(2 * x * 1024 / 1e6, 1) for x in v])
PY
done
for lib in libghost_amd_ab.so libghost_amd.so libghost_amd_ab.so libghost_amd.so; do
  GHOST_LIB_FILE=$lib timeout -k 10 300 python3 bench.py --legs '' --cpu-batches '' > $R/b.log 2>&1
  python3 -c "import json,sys; d=json.loads([l for l in open('$R/b.log') if l.startswith('{')][-1]); print('$lib', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])" >> gpurun_out/v4xcd.log
done
