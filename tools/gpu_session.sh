#!/bin/bash
# Run a sequence of GPU steps on the gpurun box; every step has its own time limit and
# the session stops at the first crash-type exit (fault/abort/segv/timeout/kill).
# Ordinary failures (e.g. pytest exit 1) are recorded and the next step runs.
# usage: tools/gpu_session.sh "name|seconds|command" ...
mkdir -p gpurun_out
export TMPDIR=/tmp
status=0
for spec in "$@"; do
  name="${spec%%|*}"; rest="${spec#*|}"; secs="${rest%%|*}"; cmd="${rest#*|}"
  echo "=== [$name] (limit ${secs}s): $cmd"
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc in $(( $(date +%s) - start ))s"
  tail -n 25 "gpurun_out/$name.log"
  case $rc in
    0) ;;
    1|2|5) status=1 ;;                       # test failures / usage: keep going
    *) echo "=== crash-type exit $rc: stopping session"; exit $rc ;;
  esac
done
exit $status
