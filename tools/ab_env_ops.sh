# Same-box A/B of tuning-build env settings on per-op times: bash tools/ab_env_ops.sh OPS "SPEC1;SPEC2;..."
# (OPS: a tools/bench_ops.py --only value; SPEC: env assignments, '' = defaults), two passes in alternating order.
export PYTHONUNBUFFERED=1 TMPDIR=/tmp GHOST_TUNING=1
mkdir -p gpurun_out
IFS=';' read -ra specs <<< "$2"
for pass in 1 2; do
  for v in "${specs[@]}"; do
    echo "== pass $pass [$v]" >> gpurun_out/ab_env_ops.txt
    eval env $v timeout -k 10 200 python -u tools/bench_ops.py --only $1 --iters 20 >> gpurun_out/ab_env_ops.txt 2>&1 || exit $?
  done
done
