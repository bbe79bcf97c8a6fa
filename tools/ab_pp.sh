# Same-box A/B of the persistent 3x3 conv's experiment variants (tuning build): per-op times at the generator's
# shapes for each GHOST_HALO_DBG value, two passes in alternating order.   bash tools/ab_pp.sh "0 256 512 768"
export PYTHONUNBUFFERED=1 TMPDIR=/tmp GHOST_TUNING=1
mkdir -p gpurun_out
for pass in 1 2; do
  for v in $1; do
    echo "== pass $pass GHOST_HALO_DBG=$v" >> gpurun_out/ab_pp.txt
    GHOST_HALO_DBG=$v timeout -k 10 200 python -u tools/bench_ops.py --only pp --iters 20 >> gpurun_out/ab_pp.txt 2>&1 || exit $?
  done
done
