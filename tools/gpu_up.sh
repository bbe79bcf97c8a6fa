set -e
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "upsample or fp32_matches or swap_u8" > gpurun_out/up_tests.log 2>&1
for v in 1 2 4; do
  GHOST_LIB_FILE=libghost_amd_tuning.so GHOST_UP_ROWS=$v timeout -k 10 100 python tools/bench_ops.py --only up --iters 20 > gpurun_out/up_ops_$v.log 2>&1
done
timeout -k 10 200 python bench.py --legs "" --cpu-batches "" > gpurun_out/up_bench.log 2>&1
