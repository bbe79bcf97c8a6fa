# The round's committed measurements (run on the GPU box: bash tools/gpu.sh profile, ROUND=rNN); the summaries
# land in gpurun_out/ and are copied into profiles/ afterwards.  Raw profiler output stays in /tmp (it exceeds
# gpurun's 64 MiB copy-back).
#   ${ROUND}_kernel_stats.csv        rocprofv3 --kernel-trace of bench.py's timed configuration (two batches in
#                                    flight, profiling on: the roofline kernel's in-kernel clock runs as in the
#                                    bench line); per-kernel calls / average ns (tools/kernel_table.py --stats-csv)
#   ${ROUND}_kernel_table.txt        the same trace per (kernel, grid)
#   ${ROUND}_kernel_stats_1stream.csv  the same with one batch at a time (--streams 1): the roofline's isolated row
#   ${ROUND}_step_trace.txt          one step's kernel sequence (one stream)
#   ${ROUND}_traffic.json            per-kernel HBM bytes: separate --pmc FETCH_SIZE / WRITE_SIZE passes (gfx950
#                                    FETCH x2 correction, tools/pmc_traffic.py), one batch at a time
#   ${ROUND}_bench.log               the full bench line (two batches in flight, legs, CPU baseline), run LAST
#                                    with the summaries above already in this box's profiles/, so its
#                                    roofline.rocprof / traffic / rocprof_agreement cite this same run's files
set -e
export TMPDIR=/tmp PYTHONUNBUFFERED=1
ROUND=${ROUND:-r04}
R=/tmp/ghost_prof
Q='--legs "" --cpu-batches ""'
rm -rf $R && mkdir -p $R gpurun_out
eval timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/trace -o run -- python3 bench.py --steps 10 --warmup 3 $Q > gpurun_out/${ROUND}_prof.log 2>&1
eval timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/trace1 -o run -- python3 bench.py --steps 10 --warmup 3 $Q --streams 1 > gpurun_out/${ROUND}_prof1.log 2>&1
eval timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/fetch -o run -- python3 bench.py --steps 2 --warmup 1 --no-profile $Q --streams 1 > gpurun_out/${ROUND}_pmcf.log 2>&1
eval timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/write -o run -- python3 bench.py --steps 2 --warmup 1 --no-profile $Q --streams 1 > gpurun_out/${ROUND}_pmcw.log 2>&1
find $R -maxdepth 3 > gpurun_out/${ROUND}_prof_files.txt
python3 tools/kernel_table.py $R/trace/run_results.db --top 80 --stats-csv gpurun_out/${ROUND}_kernel_stats.csv > gpurun_out/${ROUND}_kernel_table.txt
python3 tools/kernel_table.py $R/trace1/run_results.db --top 0 --stats-csv gpurun_out/${ROUND}_kernel_stats_1stream.csv > /dev/null
python3 tools/pmc_traffic.py $R/fetch/run_counter_collection.csv $R/write/run_counter_collection.csv --out gpurun_out/${ROUND}_traffic.json --source "${ROUND}: rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE (separate passes, csv), python3 bench.py --steps 2 --warmup 1 --no-profile --legs '' --cpu-batches '' --streams 1 (B=64 unet/2 bf16)" > gpurun_out/${ROUND}_traffic.log 2>&1
python3 tools/step_trace.py $R/trace1/run_results.db > gpurun_out/${ROUND}_step_trace.txt 2>&1
cp gpurun_out/${ROUND}_kernel_stats.csv gpurun_out/${ROUND}_kernel_stats_1stream.csv gpurun_out/${ROUND}_traffic.json profiles/
timeout -k 10 600 python3 bench.py > gpurun_out/${ROUND}_bench.log 2>&1
