# tap-partials AAD kernels at two workgroups per CU: GPU suite, then one-stream traces (tap partials 0 / 2), then the bench
set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out; rm -f gpurun_out/zp3.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1
for zp in 2 0; do
  rm -rf /tmp/zt$zp
  timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/zt$zp -o run -- python3 bench.py --steps 3 --warmup 2 --legs "" --cpu-batches "" --no-profile --streams 1 --opt tap_partials=$zp > /tmp/zt$zp.log 2>&1
  echo "== zp=$zp" >> gpurun_out/zp3.log
  python3 tools/step_trace.py /tmp/zt$zp/run_results.db | tail -12 >> gpurun_out/zp3.log
done
timeout -k 10 300 python bench.py --legs "" --cpu-batches "" > gpurun_out/bench_quick.log 2>&1
