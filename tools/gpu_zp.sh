set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out; rm -f gpurun_out/zp.log
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_bf16_parity.py tests/test_gpu_pipeline.py tests/test_gpu_parity.py -k "bf16 or swap_u8 or forward or pipeline or two_stream or config5 or aad" > gpurun_out/zp_tests.log 2>&1 || true
tail -15 gpurun_out/zp_tests.log >> gpurun_out/zp.log
for zp in 0 1 2 0 1 2; do
  timeout -k 10 300 python bench.py --legs '' --cpu-batches '' --opt tap_partials=$zp > /tmp/b.log 2>&1
  python3 -c "import json; d=json.loads([l for l in open('/tmp/b.log') if l.startswith('{')][-1]); r=d['roofline']; print('zp=$zp', d['value'], d['ms_per_step'], r['isolated'], d['kernel_ms_per_step'])" >> gpurun_out/zp.log
done
