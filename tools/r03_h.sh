# round-3 final pass: GPU suite, smoke, then the round's profile set (bench line last, against the same run's
# summaries)
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
ok() { rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "stop: rc=$rc"; exit $rc; }; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail 6 --timeout 150 --timeout-method thread > gpurun_out/gputests.log 2>&1; ok $?
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; ok $?
ROUND=r03 bash tools/profile_round.sh; ok $?
echo done
