# bench A/B of AAD kernel knobs (tuning build): bash tools/ab_v5.sh "ENV=V ENV=V" "ENV=V" ...
set -e
export PYTHONUNBUFFERED=1 GHOST_TUNING=1
for v in "$@"; do
  echo "== $v" >> gpurun_out/ab_v5.txt
  for st in 1 2; do
    env $v timeout -k 10 200 python -u bench.py --legs "" --cpu-batches "" --streams $st > /tmp/o.log 2>&1
    python3 -c "import json;d=json.loads(open('/tmp/o.log').read().strip().split('\n')[-1]);r=d['roofline'];print('streams=$st',d['value'],r['kernel'][:32],'timed',r['avg_launch_us'],'iso',r['isolated']['avg_launch_us'])" >> gpurun_out/ab_v5.txt
  done
done
