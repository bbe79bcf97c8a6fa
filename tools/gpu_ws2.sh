set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp GHOST_TUNING=1
mkdir -p gpurun_out; rm -f gpurun_out/ws2.log
GHOST_CONV_AAD_GLDS=1 GHOST_CONV_DEEP=4 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "conv or aad or forward_fp32 or bf16_close" > gpurun_out/ws2_tests.log 2>&1
tail -2 gpurun_out/ws2_tests.log >> gpurun_out/ws2.log
for cfg in "0 8" "1 8" "0 6" "0 4" "1 4" "0 8" "1 8"; do
  set -- $cfg
  GHOST_CONV_AAD_GLDS=$1 GHOST_CONV_DEEP=$2 timeout -k 10 300 python bench.py --legs '' --cpu-batches '' > /tmp/b.log 2>&1
  python3 -c "import json; d=json.loads([l for l in open('/tmp/b.log') if l.startswith('{')][-1]); print('bench AAD_GLDS=$1 DEEP=$2', d['value'], d['ms_per_step'], d['kernel_ms_per_step'])" >> gpurun_out/ws2.log
done
