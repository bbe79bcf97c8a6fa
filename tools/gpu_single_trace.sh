# single-stream kernel trace of one bench step (the two-stream plan off) + isolated encoder convs
set -e
export TMPDIR=/tmp PYTHONUNBUFFERED=1
R=/tmp/ghost_st; rm -rf $R; mkdir -p $R gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace -d $R/trace -o run -- python3 bench.py --steps 3 --warmup 2 --legs "" --cpu-batches "" --no-profile --opt two_streams=0 > gpurun_out/st_prof.log 2>&1
python3 tools/step_trace.py $R/trace/run_results.db > gpurun_out/r02_step_trace_1stream.txt 2>&1
timeout -k 10 200 python3 tools/bench_ops.py --only enc > gpurun_out/enc_ops.log 2>&1
