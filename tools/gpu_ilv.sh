set -e
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_bf16_parity.py -x -q --timeout 120 --timeout-method thread -k "conv or bf16 or fp32_matches" > gpurun_out/ilv_tests.log 2>&1
for v in 0 1; do
  GHOST_LIB_FILE=libghost_amd_tuning.so GHOST_HALO_ILV=$v timeout -k 10 200 python tools/bench_ops.py --only conv --iters 20 > gpurun_out/ilv_ops_$v.log 2>&1
done
GHOST_LIB_FILE=libghost_amd_ab.so timeout -k 10 200 python tools/bench_ops.py --only conv --iters 20 > gpurun_out/ilv_ops_old.log 2>&1
for lib in libghost_amd_ab.so libghost_amd.so libghost_amd_ab.so libghost_amd.so; do
  GHOST_LIB_FILE=$lib timeout -k 10 300 python bench.py --legs '' --cpu-batches '' --no-profile >> gpurun_out/ilv_bench_$lib.log 2>&1
done
