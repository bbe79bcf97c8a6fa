# A/B: 16-byte epilogue stores in the 256x256 persistent conv (tree library) vs the saved HEAD build
# (libghost_amd_ab.so), same box: parity tests, one-stream traces, bench lines
set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out; rm -f gpurun_out/w16.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1
for lib in libghost_amd.so libghost_amd_ab.so; do
  rm -rf /tmp/w_$lib
  GHOST_LIB_FILE=$lib timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/w_$lib -o run -- python3 bench.py --steps 3 --warmup 2 --legs "" --cpu-batches "" --no-profile --streams 1 --opt two_streams=0 > /tmp/w_$lib.log 2>&1
  echo "== $lib" >> gpurun_out/w16.log
  python3 tools/step_trace.py /tmp/w_$lib/run_results.db | grep -E "conv3x3_halo_pp|aad_v4|sum" >> gpurun_out/w16.log
done
for lib in libghost_amd.so libghost_amd_ab.so libghost_amd.so libghost_amd_ab.so; do
  echo "== bench $lib" >> gpurun_out/w16.log
  GHOST_LIB_FILE=$lib timeout -k 10 300 python bench.py --legs "" --cpu-batches "" --no-profile | grep '^{' | cut -c1-200 >> gpurun_out/w16.log
done
