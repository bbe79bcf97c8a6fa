# same-box A/B of the working tree's library against a saved one (ghost_amd/libghost_amd_ab.so):
#   bash tools/gpu_libab.sh "<pytest -k expr>" "<bench_ops --only>"
set -e
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
K=${1:-aad}; OPS=${2:-aadv3}
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_bf16_parity.py -k "$K" > gpurun_out/ab_tests.log 2>&1
for lib in libghost_amd_ab.so libghost_amd.so; do
  GHOST_LIB_FILE=$lib timeout -k 10 200 python tools/bench_ops.py --only $OPS > gpurun_out/ab_ops_$lib.log 2>&1
done
for lib in libghost_amd_ab.so libghost_amd.so libghost_amd_ab.so libghost_amd.so; do
  GHOST_LIB_FILE=$lib timeout -k 10 300 python bench.py --legs '' --cpu-batches '' >> gpurun_out/ab_bench_$lib.log 2>&1
done
