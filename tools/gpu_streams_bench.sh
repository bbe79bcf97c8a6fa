set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out; rm -f gpurun_out/sb.log
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_pipeline.py > gpurun_out/sb_tests.log 2>&1
tail -2 gpurun_out/sb_tests.log >> gpurun_out/sb.log
for ns in 1 2 3 1 2 3; do
  timeout -k 10 300 python bench.py --legs '' --cpu-batches '' --streams $ns > /tmp/b.log 2>&1
  python3 -c "import json; d=json.loads([l for l in open('/tmp/b.log') if l.startswith('{')][-1]); r=d['roofline']; print('streams=$ns', d['value'], d['ms_per_step'], r['avg_launch_us'], r['frac'], d['kernel_ms_per_step'])" >> gpurun_out/sb.log
done
