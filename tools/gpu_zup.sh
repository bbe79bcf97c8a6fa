set -e
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "aad_layers_v3 or virtual_zattr8 or through_upsample or fused_tail" > gpurun_out/t_zup.log 2>&1
timeout -k 10 200 python tools/bench_ops.py --only aadv3 > gpurun_out/aad_zup.log 2>&1
GHOST_AAD_Z4=0 timeout -k 10 200 python tools/bench_ops.py --only aadv3 > gpurun_out/aad_zup8.log 2>&1
GHOST_FUSE_ZUP=0 timeout -k 10 300 python bench.py > gpurun_out/bench_z0.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/bench_z1.log 2>&1
