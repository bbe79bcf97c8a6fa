set -e
export PYTHONUNBUFFERED=1 GHOST_TUNING=1
for v in "GHOST_AAD_V5=0" "GHOST_AAD_V5=1" "GHOST_AAD_V5=1 GHOST_V5_XCD=0"; do
  echo "== $v" >> gpurun_out/ab_v5.txt
  env $v timeout -k 10 200 python -u bench.py --legs "" --cpu-batches "" --streams 1 > /tmp/o.log 2>&1
  python3 -c "import json;d=json.loads(open('/tmp/o.log').read().strip().split('\n')[-1]);r=d['roofline'];print(d['value'],r['kernel'][:32],r['avg_launch_us'],r['isolated']['avg_launch_us'])" >> gpurun_out/ab_v5.txt
  env $v timeout -k 10 200 python -u bench.py --legs "" --cpu-batches "" > /tmp/o.log 2>&1
  python3 -c "import json;d=json.loads(open('/tmp/o.log').read().strip().split('\n')[-1]);r=d['roofline'];print(d['value'],r['kernel'][:32],r['avg_launch_us'],r['isolated']['avg_launch_us'])" >> gpurun_out/ab_v5.txt
done
