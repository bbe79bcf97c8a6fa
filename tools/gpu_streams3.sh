set -e
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py -x -q --timeout 120 --timeout-method thread > gpurun_out/streams3_tests.log 2>&1
timeout -k 10 200 python tools/ab_streams.py unet 2 > gpurun_out/streams3_ab.log 2>&1
