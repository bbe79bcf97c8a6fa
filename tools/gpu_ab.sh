set -e
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "aad_layers_v3 or unet or linknet or resnet" > gpurun_out/t_mask.log 2>&1
timeout -k 10 200 python tools/bench_ops.py --only aadv3 > gpurun_out/aad_m1.log 2>&1
GHOST_MASK_REG=0 timeout -k 10 200 python tools/bench_ops.py --only aadv3 > gpurun_out/aad_m0.log 2>&1
GHOST_MASK_REG=0 timeout -k 10 300 python bench.py > gpurun_out/bench_m0.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/bench_m1.log 2>&1
