# round-3 first pass: fp16 block probe, full GPU suite (test failures do not stop the script; faults do), quick bench
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
ok() { rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "stop: rc=$rc"; exit $rc; }; }
timeout -k 10 300 python -u tools/fp16_probe.py --st fp16 --block 7 > gpurun_out/probe16.log 2>&1; ok $?
timeout -k 10 300 python -u tools/fp16_probe.py --st bf16 --block 7 > gpurun_out/probe_bf.log 2>&1; ok $?
timeout -k 10 900 python -u -m pytest tests -m gpu -v --maxfail 6 --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1; ok $?
timeout -k 10 300 python -u bench.py --legs fp16,arcface,latency --cpu-batches "" > gpurun_out/quick.log 2>&1; ok $?
echo done
