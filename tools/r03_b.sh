# round-3: GPU suite, ArcFace kernel trace (B=128), the round's profile set
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
ok() { rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "stop: rc=$rc"; exit $rc; }; }
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail 6 --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1; ok $?
rm -rf /tmp/at
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/at -o run -- python3 tools/run_arc.py 128 5 > gpurun_out/arc_trace.log 2>&1; ok $?
python3 tools/kernel_table.py /tmp/at/run_results.db --top 40 > gpurun_out/arc_kernel_table.txt 2>&1
echo done
