# One launcher for GPU-box work (run through gpurun from the repo root):
#
#   bash tools/gpu.sh STEP [STEP ...]
#
# Steps run in order, each under its own time limit; the first failing step ends the script.
#   tests          pytest -m gpu (one process, per-test timeout)          -> gpurun_out/gputests.log
#   tests:EXPR     the same, -k EXPR                                       -> gpurun_out/gputests.log
#   smoke          __graft_entry__.smoke()                                 -> gpurun_out/smoke.log
#   bench          python bench.py (default legs + CPU baseline)           -> gpurun_out/bench.log
#   quick          bench.py without legs / CPU baseline                    -> gpurun_out/quick.log
#   quick1         the same with one batch in flight (--streams 1)         -> gpurun_out/quick1.log
#   trace          one-stream kernel trace, per-step kernel sequence       -> gpurun_out/step_trace.txt
#   ops:NAME       tools/bench_ops.py --only NAME                          -> gpurun_out/ops_NAME.log
#   profile        the round's committed profile set (tools/profile_round.sh, ROUND=rNN)
#   ab:LIB         bench.py quick with GHOST_LIB_FILE=LIB (same-box A/B)   -> gpurun_out/ab_LIB.log
# Extra bench.py arguments for quick/quick1/ab: BENCH_ARGS="--opt tap_partials=1".
set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
Q='--legs "" --cpu-batches ""'
for step in "$@"; do
  echo "[gpu.sh] $step $(date +%T)"
  case "$step" in
    tests) timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1 ;;
    tests:*) timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -k "${step#tests:}" > gpurun_out/gputests.log 2>&1 ;;
    smoke) timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 ;;
    bench) timeout -k 10 600 python -u bench.py > gpurun_out/bench.log 2>&1 ;;
    quick) eval timeout -k 10 300 python -u bench.py $Q $BENCH_ARGS > gpurun_out/quick.log 2>&1 ;;
    quick1) eval timeout -k 10 300 python -u bench.py $Q --streams 1 $BENCH_ARGS > gpurun_out/quick1.log 2>&1 ;;
    trace)
      rm -rf /tmp/gt
      eval timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/gt -o run -- python3 bench.py --steps 3 --warmup 2 $Q --no-profile --streams 1 $BENCH_ARGS > gpurun_out/trace.log 2>&1
      python3 tools/step_trace.py /tmp/gt/run_results.db > gpurun_out/step_trace.txt ;;
    ops:*) timeout -k 10 300 python -u tools/bench_ops.py --only "${step#ops:}" > "gpurun_out/ops_${step#ops:}.log" 2>&1 ;;
    profile) bash tools/profile_round.sh ;;
    ab:*) eval GHOST_LIB_FILE="${step#ab:}" timeout -k 10 300 python -u bench.py $Q $BENCH_ARGS > "gpurun_out/ab_${step#ab:}.log" 2>&1 ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "[gpu.sh] done $(date +%T)"
