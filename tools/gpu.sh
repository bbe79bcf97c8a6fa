# One launcher for GPU-box work (run through gpurun from the repo root):
#
#   bash tools/gpu.sh STEP [STEP ...]
#
# Steps run in order, each under its own time limit.  A test step that only reports failed tests goes on to the
# next step; any other failure (a timeout, an abort, a fault) ends the script there.
#   tests          pytest -m gpu (one process, per-test timeout)          -> gpurun_out/gputests.log
#   tests:EXPR     the same, -k EXPR                                       -> gpurun_out/gputests.log
#   smoke          __graft_entry__.smoke()                                 -> gpurun_out/smoke.log
#   bench          python bench.py (default legs + CPU baseline)           -> gpurun_out/bench.log
#   quick          bench.py without legs / CPU baseline                    -> gpurun_out/quick.log
#   quick1         the same with one batch in flight (--streams 1)         -> gpurun_out/quick1.log
#   trace          one-stream kernel trace, per-step kernel sequence       -> gpurun_out/step_trace.txt
#   trace1         the same at B = 1                                       -> gpurun_out/step_trace_b1.txt
#   ops:NAME       tools/bench_ops.py --only NAME                          -> gpurun_out/ops_NAME.log
#   profile        the round's committed profile set (tools/profile_round.sh, ROUND=rNN)
#   ab:LIB         bench.py quick with GHOST_LIB_FILE=LIB (same-box A/B)   -> gpurun_out/ab_LIB.log
#   knobs:SPECS    bench.py quick through the tuning build, one run per spec and --streams 1 / 2; SPECS is
#                  ';'-separated env settings, e.g. "GHOST_V5_IPW=1;GHOST_V5_IPW=2;GHOST_AAD_V5=0"
#                                                                          -> gpurun_out/ab_knobs.txt
#   envab:SPECS    bench.py quick (40 steps) once per ';'-separated env setting (shipping build) -> gpurun_out/ab_env.txt
#   streams:LIST   bench.py quick at --streams N for N in the ','-list     -> gpurun_out/ab_streams.txt
#   arc:LIST       tools/run_arc.py N for N in the ','-list (ArcFace)      -> gpurun_out/arc_batch.txt
#   arctrace:N     kernel trace of tools/run_arc.py N (ArcFace)            -> gpurun_out/arc_kt_N.txt
#   gtrace:DT      kernel trace of eager vs GraphedSwap at B = 1 (DT fp32/bf16) -> gpurun_out/gtrace_DT.txt
#   mfma           MFMA / VALU PMC passes (tools/pmc_mfma.sh, ROUND=rNN)   -> gpurun_out/rNN_mfma.json
#   qprobeset      the same with ghost_amd's StreamSet created first       -> gpurun_out/queue_probe_set.txt
#   qprobe         which streams share a hardware queue (tools/queue_probe.py) -> gpurun_out/queue_probe.txt
#   legs:LIST      bench.py with --legs LIST (':'-separated), no CPU baseline -> gpurun_out/legs_LIST.log
# Extra bench.py arguments for quick/quick1/ab/knobs/streams: BENCH_ARGS="--opt tap_partials=1".
# knobs needs the tuning library on the box (GHOST_TUNING=1 python -m ghost_amd.build; list the shipping
# library in .gpurunignore for that call if the push should carry only one of them).
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
Q='--legs "" --cpu-batches ""'
ok() { rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "[gpu.sh] stop: rc=$rc"; exit $rc; }; }
must() { rc=$1; [ $rc -eq 0 ] || { echo "[gpu.sh] stop: rc=$rc"; exit $rc; }; }
last() { python3 -c "import json,sys;d=json.loads(open('$1').read().strip().split('\n')[-1]);r=d.get('roofline',{});print(sys.argv[1],d['value'],d['ms_per_step'],'live',r.get('live_clock_us'),'iso',r.get('isolated',{}).get('avg_launch_us'))" "$2"; }
for step in "$@"; do
  echo "[gpu.sh] $step $(date +%T)"
  case "$step" in
    tests) timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail 6 --timeout 150 --timeout-method thread > gpurun_out/gputests.log 2>&1; ok $? ;;
    tests:*) timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 150 --timeout-method thread -k "${step#tests:}" > gpurun_out/gputests.log 2>&1; ok $? ;;
    smoke) timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; must $? ;;
    bench) timeout -k 10 600 python -u bench.py > gpurun_out/bench.log 2>&1; must $? ;;
    quick) eval timeout -k 10 300 python -u bench.py $Q $BENCH_ARGS > gpurun_out/quick.log 2>&1; must $? ;;
    quick1) eval timeout -k 10 300 python -u bench.py $Q --streams 1 $BENCH_ARGS > gpurun_out/quick1.log 2>&1; must $? ;;
    trace1)
      rm -rf /tmp/gt1
      eval timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/gt1 -o run -- python3 bench.py --batch 1 --steps 5 --warmup 3 $Q --no-profile --streams 1 $BENCH_ARGS > gpurun_out/trace1.log 2>&1; must $?
      python3 tools/step_trace.py /tmp/gt1/run_results.db > gpurun_out/step_trace_b1.txt ;;
    trace)
      rm -rf /tmp/gt
      eval timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/gt -o run -- python3 bench.py --steps 3 --warmup 2 $Q --no-profile --streams 1 $BENCH_ARGS > gpurun_out/trace.log 2>&1; must $?
      python3 tools/step_trace.py /tmp/gt/run_results.db > gpurun_out/step_trace.txt ;;
    ops:*) timeout -k 10 300 python -u tools/bench_ops.py --only "${step#ops:}" > "gpurun_out/ops_${step#ops:}.log" 2>&1; must $? ;;
    profile) bash tools/profile_round.sh; must $? ;;
    ab:*) eval GHOST_LIB_FILE="${step#ab:}" timeout -k 10 300 python -u bench.py $Q $BENCH_ARGS > "gpurun_out/ab_${step#ab:}.log" 2>&1; must $? ;;
    knobs:*)
      IFS=';' read -ra specs <<< "${step#knobs:}"
      for v in "${specs[@]}"; do
        for st in 1 2; do
          eval env GHOST_TUNING=1 $v timeout -k 10 200 python -u bench.py $Q --streams $st $BENCH_ARGS > /tmp/o.log 2>&1
          rc=$?; [ $rc -eq 0 ] || cp /tmp/o.log gpurun_out/knobs_fail.log; must $rc
          last /tmp/o.log "$v streams=$st" >> gpurun_out/ab_knobs.txt
        done
      done ;;
    envab:*)
      IFS=';' read -ra specs <<< "${step#envab:}"
      for v in "${specs[@]}"; do
        eval env $v timeout -k 10 200 python -u bench.py $Q --steps 40 $BENCH_ARGS > /tmp/o.log 2>&1
        rc=$?; [ $rc -eq 0 ] || cp /tmp/o.log gpurun_out/envab_fail.log; must $rc
        last /tmp/o.log "$v" >> gpurun_out/ab_env.txt
      done ;;
    streams:*)
      IFS=',' read -ra ns <<< "${step#streams:}"
      for st in "${ns[@]}"; do
        eval timeout -k 10 200 python -u bench.py $Q --streams $st --steps 40 $BENCH_ARGS > /tmp/o.log 2>&1
        rc=$?; [ $rc -eq 0 ] || cp /tmp/o.log gpurun_out/streams_fail.log; must $rc
        last /tmp/o.log "streams=$st" >> gpurun_out/ab_streams.txt
      done ;;
    arc:*)
      IFS=',' read -ra ns <<< "${step#arc:}"
      for n in "${ns[@]}"; do timeout -k 10 200 python -u tools/run_arc.py $n 8 >> gpurun_out/arc_batch.txt 2>&1; must $?; done ;;
    arctrace:*)
      n="${step#arctrace:}"
      rm -rf /tmp/at
      timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/at -o run -- python3 tools/run_arc.py $n 5 > "gpurun_out/arc_tr_$n.log" 2>&1; must $?
      python3 tools/kernel_table.py /tmp/at/run_results.db --top 24 > "gpurun_out/arc_kt_$n.txt" 2>&1 ;;
    gtrace:*)
      dt="${step#gtrace:}"
      rm -rf /tmp/gtr
      timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/gtr -o run -- python3 tools/graph_trace.py $dt > "gpurun_out/gtrace_$dt.txt" 2>&1; must $?
      python3 tools/graph_trace.py --analyze /tmp/gtr/run_results.db >> "gpurun_out/gtrace_$dt.txt" 2>&1 ;;
    mfma) bash tools/pmc_mfma.sh; must $? ;;
    qprobe) timeout -k 10 120 python -u tools/queue_probe.py > gpurun_out/queue_probe.txt 2>&1; must $? ;;
    qprobeset) timeout -k 10 120 python -u tools/queue_probe.py --set --extra 3 > gpurun_out/queue_probe_set.txt 2>&1; must $? ;;
    legs:*)
      l="${step#legs:}"
      eval timeout -k 10 400 python -u bench.py --cpu-batches '""' --legs "${l//:/,}" $BENCH_ARGS > "gpurun_out/legs_${l//:/_}.log" 2>&1; must $? ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "[gpu.sh] done $(date +%T)"
