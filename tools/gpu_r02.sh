# round-2 GPU session helper: bash tools/gpu_r02.sh <what...>  (each step time-limited, stops at the first failure)
set -e
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
for w in "$@"; do
  case $w in
    tests) timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1 ;;
    bisect) timeout -k 10 300 python tools/bf16_bisect.py --backbone unet --num-blocks 2 --fp16 --json gpurun_out/bisect_unet2.json > gpurun_out/bisect_unet2.log 2>&1
            timeout -k 10 300 python tools/bf16_bisect.py --backbone linknet --num-blocks 3 --fp16 --json gpurun_out/bisect_linknet3.json > gpurun_out/bisect_linknet3.log 2>&1 ;;
    bench) timeout -k 10 300 python bench.py > gpurun_out/bench.log 2>&1 ;;
    arc) timeout -k 10 300 python bench.py --legs arcface --cpu-batches "" --steps 10 > gpurun_out/bench_arc.log 2>&1 ;;
    quick) timeout -k 10 200 python bench.py --legs "" --cpu-batches "" > gpurun_out/bench_quick.log 2>&1 ;;
    trace) export TMPDIR=/tmp; R=/tmp/ghost_trace; rm -rf $R; mkdir -p $R
           timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R -o run -- python3 bench.py --steps 5 --warmup 2 --legs "" --cpu-batches "" > gpurun_out/trace_bench.log 2>&1
           python3 tools/kernel_table.py $R/run_results.db --top 70 --stats-csv gpurun_out/trace_kernel_stats.csv > gpurun_out/trace_kernel_table.txt 2>&1 || true
           python3 tools/step_trace.py $R/run_results.db > gpurun_out/trace_step.txt 2>&1 || true ;;
    *) echo "unknown step $w"; exit 2 ;;
  esac
done
