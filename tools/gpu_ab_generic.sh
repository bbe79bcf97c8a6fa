# same-box A/B of the working tree's library against ghost_amd/libghost_amd_ab.so:
#   bash tools/gpu_ab_generic.sh "<pytest -k expr>" "<bench_ops --only>" [bench reps]
set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
K=$1; OPS=$2; N=${3:-2}
rm -f gpurun_out/ab.log
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ -k "$K" > gpurun_out/ab_tests.log 2>&1
tail -3 gpurun_out/ab_tests.log >> gpurun_out/ab.log
for lib in libghost_amd_ab.so libghost_amd.so; do
  echo "== ops $lib" >> gpurun_out/ab.log
  GHOST_LIB_FILE=$lib timeout -k 10 200 python tools/bench_ops.py --only $OPS >> gpurun_out/ab.log 2>&1
done
for i in $(seq $N); do
for lib in libghost_amd_ab.so libghost_amd.so; do
  GHOST_LIB_FILE=$lib timeout -k 10 300 python bench.py --legs '' --cpu-batches '' > /tmp/b.log 2>&1
  python3 -c "import json; d=json.loads([l for l in open('/tmp/b.log') if l.startswith('{')][-1]); print('bench $lib', d['value'], d['ms_per_step'], d['kernel_ms_per_step'])" >> gpurun_out/ab.log
done
done
