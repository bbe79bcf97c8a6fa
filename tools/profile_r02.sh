# Round-2 committed measurements (run on the GPU box; summaries are copied into profiles/ afterwards):
# the full bench line (default: two batches in flight), a kernel trace + rocprofv3 --stats of the same
# timed-region configuration (--no-profile: no untimed one-batch pass mixed into the averages), a one-stream
# kernel trace for the per-step kernel sequence, and two separate PMC passes (FETCH_SIZE, WRITE_SIZE) for
# per-kernel HBM traffic.  Raw profiler output stays in /tmp.
set -e
export TMPDIR=/tmp PYTHONUNBUFFERED=1
R=/tmp/ghost_prof
rm -rf $R && mkdir -p $R gpurun_out
timeout -k 10 400 python3 bench.py > gpurun_out/r02_bench.log 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/trace -o run -- python3 bench.py --steps 5 --warmup 2 --legs "" --cpu-batches "" --no-profile > gpurun_out/r02_prof.log 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace -d $R/trace1 -o run -- python3 bench.py --steps 3 --warmup 2 --legs "" --cpu-batches "" --no-profile --streams 1 > gpurun_out/r02_prof1.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/fetch -o run -- python3 bench.py --steps 2 --warmup 1 --no-profile --legs "" --cpu-batches "" --streams 1 > gpurun_out/r02_pmcf.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/write -o run -- python3 bench.py --steps 2 --warmup 1 --no-profile --legs "" --cpu-batches "" --streams 1 > gpurun_out/r02_pmcw.log 2>&1
set +e
find $R -maxdepth 3 > gpurun_out/r02_prof_files.txt
cp $R/trace/run_kernel_stats.csv gpurun_out/r02_rocprof_kernel_stats.csv 2>/dev/null || find $R/trace -name "*kernel_stats*" -exec cp {} gpurun_out/r02_rocprof_kernel_stats.csv \;
python3 tools/kernel_table.py $R/trace/run_results.db --top 80 --stats-csv gpurun_out/r02_kernel_stats.csv > gpurun_out/r02_kernel_table.txt 2>&1
python3 tools/pmc_traffic.py $R/fetch/run_counter_collection.csv $R/write/run_counter_collection.csv --out gpurun_out/r02_traffic.json --source "r02: rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE (separate passes, csv), python3 bench.py --steps 2 --warmup 1 --no-profile --legs '' --cpu-batches '' --streams 1 (B=64 unet/2 bf16)" > gpurun_out/r02_traffic.log 2>&1
python3 tools/step_trace.py $R/trace1/run_results.db > gpurun_out/r02_step_trace.txt 2>&1
exit 0
