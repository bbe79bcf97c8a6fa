# The round's committed measurements (run on the GPU box; the summaries are copied into profiles/ after):
# the bench line, a kernel trace + stats, and the two PMC passes for per-kernel HBM traffic.  The raw
# profiler output stays in /tmp on the box (it exceeds gpurun's 64 MiB copy-back); summaries go to gpurun_out/.
set -e
export TMPDIR=/tmp PYTHONUNBUFFERED=1
R=/tmp/ghost_prof
rm -rf $R && mkdir -p $R gpurun_out
timeout -k 10 300 python3 bench.py > gpurun_out/r01_bench.log 2>&1
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/trace -o run -- python3 bench.py --steps 5 --warmup 2 > gpurun_out/prof_r01.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/fetch -o run -- python3 bench.py --steps 2 --warmup 1 --no-profile > gpurun_out/pmcf.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/write -o run -- python3 bench.py --steps 2 --warmup 1 --no-profile > gpurun_out/pmcw.log 2>&1
find $R -maxdepth 3 > gpurun_out/r01_prof_files.txt
set +e
python3 tools/kernel_table.py $R/trace/run_results.db --top 70 --stats-csv gpurun_out/r01_kernel_stats.csv > gpurun_out/r01_kernel_table.txt 2>&1
python3 tools/pmc_traffic.py $R/fetch/run_counter_collection.csv $R/write/run_counter_collection.csv --out gpurun_out/r01_traffic.json > gpurun_out/r01_traffic.log 2>&1
python3 tools/step_trace.py $R/trace/run_results.db > gpurun_out/r01_step_trace.txt 2>&1
ls -la $R/*/ >> gpurun_out/r01_prof_files.txt 2>&1
exit 0
