set -e
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "aad_layers_v3 or unet or linknet" > gpurun_out/t_wide4.log 2>&1
timeout -k 10 200 python tools/bench_ops.py --only aadv3 > gpurun_out/aad_w4.log 2>&1
GHOST_AAD_WIDE4=0 timeout -k 10 200 python tools/bench_ops.py --only aadv3 > gpurun_out/aad_w0.log 2>&1
GHOST_AAD_WIDE4=0 timeout -k 10 300 python bench.py > gpurun_out/bench_w0.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/bench_w4.log 2>&1
