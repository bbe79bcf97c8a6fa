export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
for args in "--legs config5_multi,d2h --no-profile" "--legs config5_multi,d2h" "--legs d2h" "--legs config5_multi,d2h --steps 40"; do
  timeout -k 10 300 python -u bench.py --cpu-batches "" $args > /tmp/o.log 2>&1 || { cp /tmp/o.log gpurun_out/c5_fail.log; exit 1; }
  python3 -c "import json,sys;d=json.loads(open('/tmp/o.log').read().strip().split('\n')[-1]);L=d['legs'];print(sys.argv[1], d['value'], L['d2h']['windows_frames_per_s'], L.get('config5_multi',{}).get('host'))" "$args" >> gpurun_out/c5_ab.txt
done
