# A/B: non-temporal stores in the z_attr8 upsample (GHOST_UP_NT=1, default) vs plain stores (0), same box;
# plus the ArcFace leg at 128 faces per launch
set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out; rm -f gpurun_out/upnt.log
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "upsample or swap_u8" > gpurun_out/upnt_tests.log 2>&1
for v in 1 0; do
  rm -rf /tmp/n_$v
  GHOST_TUNING=1 GHOST_UP_NT=$v timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/n_$v -o run -- python3 bench.py --steps 3 --warmup 2 --legs "" --cpu-batches "" --no-profile --streams 1 --opt two_streams=0 > /tmp/n_$v.log 2>&1
  echo "== up_nt=$v" >> gpurun_out/upnt.log
  python3 tools/step_trace.py /tmp/n_$v/run_results.db | grep -E "upsample2x_rows_kernelIDF16bLi2ELb1|upsample2x_rows_kernelIDF16bLi2ELb0|aad_v4|sum" >> gpurun_out/upnt.log
done
for v in 1 0 1 0; do
  echo "== bench up_nt=$v" >> gpurun_out/upnt.log
  GHOST_TUNING=1 GHOST_UP_NT=$v timeout -k 10 300 python bench.py --legs "" --cpu-batches "" --no-profile | grep '^{' | cut -c1-200 >> gpurun_out/upnt.log
done
echo "== arcface B=128" >> gpurun_out/upnt.log
timeout -k 10 300 python bench.py --legs arcface --arc-batch 128 --cpu-batches "" --no-profile --steps 5 > /tmp/arc128.log 2>&1
grep '^{' /tmp/arc128.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['legs']['arcface'])" >> gpurun_out/upnt.log
