set -e
export PYTHONUNBUFFERED=1
timeout -k 10 120 python tools/tune_small.py > gpurun_out/tune_small.log 2>&1
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "conv or deconv or encoder or unet or arc" > gpurun_out/t_tune2.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1
