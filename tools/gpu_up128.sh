# A/B: AADBlk7's block-input pair sampling upsample2x(AADBlk6 output) in its dual kernel (GHOST_FUSE_UP128=1)
# vs the materialised upsample (0), same box: GPU suite, one-stream traces, quick bench lines
set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out; rm -f gpurun_out/up128.log
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputests.log 2>&1
for v in 1 0; do
  rm -rf /tmp/u_$v
  GHOST_TUNING=1 GHOST_FUSE_UP128=$v timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/u_$v -o run -- python3 bench.py --steps 3 --warmup 2 --legs "" --cpu-batches "" --no-profile --streams 1 --opt two_streams=0 > /tmp/u_$v.log 2>&1
  echo "== up128=$v" >> gpurun_out/up128.log
  python3 tools/step_trace.py /tmp/u_$v/run_results.db | grep -E "aad_v3_wide_kernelILi128|upsample2x|in_stats_up|sum" >> gpurun_out/up128.log
done
for v in 1 0 1 0; do
  echo "== bench up128=$v" >> gpurun_out/up128.log
  GHOST_TUNING=1 GHOST_FUSE_UP128=$v timeout -k 10 300 python bench.py --legs "" --cpu-batches "" --no-profile | grep '^{' | cut -c1-200 >> gpurun_out/up128.log
done
