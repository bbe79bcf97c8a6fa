# round-3 A/B of the v5 AAD kernel's knobs (tuning build; .gpurunignore swapped so only the tuning library
# travels): work items per workgroup, XCD-contiguous order, the compiler-opaque DMA pipeline; one batch at a
# time and two in flight
export PYTHONUNBUFFERED=1 TMPDIR=/tmp GHOST_TUNING=1
mkdir -p gpurun_out
ok() { rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "stop: rc=$rc"; exit $rc; }; }
timeout -k 10 300 python -u -m pytest tests/test_arcface.py -m gpu -q --timeout 150 --timeout-method thread -k "above_one or u8" > gpurun_out/tests_g.log 2>&1; ok $?
timeout -k 10 200 python -u tools/run_arc.py 128 10 > gpurun_out/arc_g.log 2>&1; ok $?
for v in "GHOST_V5_IPW=1" "GHOST_V5_IPW=2" "GHOST_V5_XCD=0" "GHOST_V5_ASM=0" "GHOST_AAD_V5=0" "GHOST_V5_IPW=1"; do
  for st in 1 2; do
    env $v timeout -k 10 200 python -u bench.py --legs= --cpu-batches= --streams $st > /tmp/o.log 2>&1; ok $?
    python3 -c "import json;d=json.loads(open('/tmp/o.log').read().strip().split('\n')[-1]);r=d['roofline'];print('$v streams=$st',d['value'],r['kernel'][:40],'live',r['live_clock_us'],'iso',r['isolated']['avg_launch_us'])" >> gpurun_out/ab_v5.txt
  done
done
echo done
