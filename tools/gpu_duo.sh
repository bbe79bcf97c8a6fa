# conv_duo A/B: GPU suite on the shipping library (duo on), conv micro-bench duo off/on (tuning
# build), quick bench
set -e
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -k "conv" > gpurun_out/duo_convtests.log 2>&1
for v in 0 1; do
  GHOST_LIB_FILE=libghost_amd_tuning.so GHOST_CONV_DUO=$v timeout -k 10 200 python tools/bench_ops.py --only conv --iters 20 > gpurun_out/duo_ops_$v.log 2>&1
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/duo_gputests.log 2>&1
timeout -k 10 200 python bench.py --legs "" --cpu-batches "" > gpurun_out/duo_bench.log 2>&1
