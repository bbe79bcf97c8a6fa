# round-3: 3x3/s2 patch kernel (ArcFace) — op tests, ArcFace tests, timing; conv plan listing (tuning build)
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
ok() { rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "stop: rc=$rc"; exit $rc; }; }
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_arcface.py -m gpu -v --timeout 150 --timeout-method thread -k "ex_epilogues or arcface or embed or stage or match" > gpurun_out/tests_f.log 2>&1; ok $?
timeout -k 10 200 python -u tools/run_arc.py 128 10 > gpurun_out/arc_f.log 2>&1; ok $?
timeout -k 10 200 python -u tools/run_arc.py 64 10 >> gpurun_out/arc_f.log 2>&1; ok $?
GHOST_TUNING=1 GHOST_CONV_TRACE=1 timeout -k 10 200 python -u tools/run_arc.py 128 1 > gpurun_out/arc_plan.log 2>&1; ok $?
rm -rf /tmp/at
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/at -o run -- python3 tools/run_arc.py 128 5 > gpurun_out/arc_tr_f.log 2>&1; ok $?
python3 tools/kernel_table.py /tmp/at/run_results.db --top 24 > gpurun_out/arc_kt_f.txt 2>&1
timeout -k 10 300 python -u bench.py --legs arcface --cpu-batches= > gpurun_out/quick_f.log 2>&1; ok $?
echo done
