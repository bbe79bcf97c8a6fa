set -e
export PYTHONUNBUFFERED=1
timeout -k 10 200 python tools/bench_ops.py --only conv > gpurun_out/conv_c256.log 2>&1
GHOST_HALO_PP_MAXCIN=1024 timeout -k 10 200 python tools/bench_ops.py --only conv > gpurun_out/conv_c1024.log 2>&1
GHOST_HALO_PP_MAXCIN=1024 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "conv or unet" > gpurun_out/t_ppcin.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/bench_c256.log 2>&1
GHOST_HALO_PP_MAXCIN=1024 timeout -k 10 300 python bench.py > gpurun_out/bench_c1024.log 2>&1
