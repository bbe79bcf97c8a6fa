# same-box A/B of one environment knob: bash tools/gpu_ab.sh VAR "v1 v2 ..." [bench_ops --only arg]
set -e
export PYTHONUNBUFFERED=1
var=$1; vals=$2; only=${3:-aadv3}
for v in $vals; do
  env $var=$v timeout -k 10 200 python tools/bench_ops.py --only $only > gpurun_out/ab_ops_$v.log 2>&1
done
for v in $vals; do
  env $var=$v timeout -k 10 300 python bench.py > gpurun_out/ab_bench_$v.log 2>&1
done
