set -e
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "instnorm or through_upsample or aad_layers_v3 or virtual" > gpurun_out/t_stats.log 2>&1
timeout -k 10 200 python tools/bench_ops.py --only stats > gpurun_out/stats.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1
