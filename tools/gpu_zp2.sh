set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out; rm -f gpurun_out/zp2.log
for zp in 0 1 2; do
  rm -rf /tmp/zt$zp
  timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/zt$zp -o run -- python3 bench.py --steps 3 --warmup 2 --legs "" --cpu-batches "" --no-profile --streams 1 --opt tap_partials=$zp > /tmp/zt$zp.log 2>&1
  echo "== zp=$zp" >> gpurun_out/zp2.log
  python3 tools/step_trace.py /tmp/zt$zp/run_results.db | tail -12 >> gpurun_out/zp2.log
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_bf16_parity.py tests/test_gpu_parity.py -k "bf16 or swap_u8" > gpurun_out/zp2_tests.log 2>&1 || true
tail -3 gpurun_out/zp2_tests.log >> gpurun_out/zp2.log
