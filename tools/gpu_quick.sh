# usage: bash tools/gpu_quick.sh  — GPU suite + pp conv micro-bench + 1-GPU bench (each step time-limited)
set -e
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1
timeout -k 10 180 python tools/bench_ops.py --only pp --iters 20 > gpurun_out/ops_pp.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1
