# round-2 diagnostics: new pipeline tests, persistent-conv debug variants (tuning build), conv PMC
set -e
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pipeline_tests.log 2>&1
for d in 0 6 8 16 22 24 30 2 4; do
  GHOST_LIB_FILE=libghost_amd_tuning.so GHOST_HALO_DBG=$d timeout -k 10 120 python tools/bench_ops.py --only pp --iters 20 > gpurun_out/ppdbg_$d.log 2>&1
done
bash tools/pmc_conv.sh 64 256 256
bash tools/pmc_conv.sh 32 512 512
