# round-3 A/B through the tuning build (GHOST_KNOB switches read the environment; defaults = the shipping
# library's).  Pushed with the tuning library only (.gpurunignore swapped for this call).
export PYTHONUNBUFFERED=1 TMPDIR=/tmp GHOST_TUNING=1
mkdir -p gpurun_out
ok() { rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "stop: rc=$rc"; exit $rc; }; }
Q='--legs "" --cpu-batches ""'
timeout -k 10 600 python -u -m pytest tests -m gpu -v --timeout 120 --timeout-method thread -k "permutation or half_module or graphed" > gpurun_out/tests_c.log 2>&1; ok $?
GHOST_HALO_RING=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_bf16_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "ring or conv2d_op or forward or decoder_block" > gpurun_out/ring.log 2>&1; ok $?
GHOST_HALO_PAIR=1 timeout -k 10 400 python -u -m pytest tests/test_arcface.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/pair.log 2>&1; ok $?
timeout -k 10 200 python -u tools/run_arc.py 128 10 > gpurun_out/arc_base.log 2>&1; ok $?
GHOST_HALO_PAIR=1 timeout -k 10 200 python -u tools/run_arc.py 128 10 > gpurun_out/arc_pair.log 2>&1; ok $?
timeout -k 10 200 python -u tools/run_arc.py 64 10 >> gpurun_out/arc_base.log 2>&1; ok $?
GHOST_HALO_PAIR=1 timeout -k 10 200 python -u tools/run_arc.py 64 10 >> gpurun_out/arc_pair.log 2>&1; ok $?
for r in 0 1 0 1; do
  eval GHOST_HALO_RING=$r timeout -k 10 300 python -u bench.py $Q --streams 1 > gpurun_out/ring$r.json 2>&1; ok $?
  python3 -c "import json;d=json.loads(open('gpurun_out/ring$r.json').read().strip().split('\n')[-1]);print('ring=$r',d['value'],d['kernel_ms_per_step'])" >> gpurun_out/ab_ring.txt
done
eval timeout -k 10 300 python -u bench.py --legs arcface,latency --cpu-batches "" > gpurun_out/legs_c.log 2>&1; ok $?
echo done
