# GPU suite, a one-stream trace of the AADBlk7/8 statistics + tail, then the committed round-2 profile set
set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1
rm -rf /tmp/zt
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/zt -o run -- python3 bench.py --steps 3 --warmup 2 --legs "" --cpu-batches "" --no-profile --streams 1 > /tmp/zt.log 2>&1
python3 tools/step_trace.py /tmp/zt/run_results.db > gpurun_out/step1.txt
bash tools/profile_r02.sh
