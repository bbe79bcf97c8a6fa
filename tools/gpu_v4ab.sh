# v4 A/B on one box: the packed-fp32 kernel vs the round-2 one (tuning build), then the shipping build
set -e
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py tests/test_bf16_parity.py -k "aad_layers_v3 or full_batch64 or bf16 or golden" > gpurun_out/v4_tests.log 2>&1
for v in 0 1 0 1; do
  GHOST_TUNING=1 GHOST_AAD_V4_OLD=$v timeout -k 10 300 python bench.py --legs '' --cpu-batches '' >> gpurun_out/v4_bench_$v.log 2>&1
done
