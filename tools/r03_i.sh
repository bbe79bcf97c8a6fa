# batches in flight A/B on the shipping library (same box): --streams 2 (default) vs 3 vs 4
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
ok() { rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "stop: rc=$rc"; exit $rc; }; }
for st in 2 3 4 2 3; do
  timeout -k 10 200 python -u bench.py --legs= --cpu-batches= --streams $st --steps 40 > /tmp/o.log 2>&1; ok $?
  python3 -c "import json;d=json.loads(open('/tmp/o.log').read().strip().split('\n')[-1]);print('streams=$st',d['value'],d['ms_per_step'])" >> gpurun_out/ab_streams3.txt
done
echo done
