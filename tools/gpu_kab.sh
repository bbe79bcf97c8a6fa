# per-kernel A/B of the tree's library against libghost_amd_ab.so: rocprofv3 kernel stats of a short bench each
# usage: bash tools/gpu_kab.sh "<pytest -k expr>"
set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_bf16_parity.py -x -q --timeout 120 --timeout-method thread -k "$1" > gpurun_out/kab_tests.log 2>&1
for lib in libghost_amd_ab.so libghost_amd.so; do
  R=/tmp/kab_$lib; rm -rf $R
  GHOST_LIB_FILE=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R -o run -- python3 bench.py --steps 10 --warmup 3 --legs "" --cpu-batches "" --no-profile > gpurun_out/kab_bench_$lib.log 2>&1
  python3 tools/kernel_table.py $R/run_results.db --top 60 > gpurun_out/kab_table_$lib.txt 2>&1 || true
done
