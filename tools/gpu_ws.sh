set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp GHOST_TUNING=1
mkdir -p gpurun_out; rm -f gpurun_out/ws.log
GHOST_CONV_WS=1 timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "conv or aad_layer_module or forward_fp32 or bf16_close" > gpurun_out/ws_tests.log 2>&1
tail -2 gpurun_out/ws_tests.log >> gpurun_out/ws.log
for cfg in "0 3" "1 3" "1 4" "0 4"; do
  set -- $cfg
  echo "== WS=$1 STAGES=$2" >> gpurun_out/ws.log
  GHOST_CONV_WS=$1 GHOST_CONV_STAGES=$2 timeout -k 10 200 python tools/probe_gemm.py lib >> gpurun_out/ws.log 2>&1
  GHOST_CONV_WS=$1 GHOST_CONV_STAGES=$2 timeout -k 10 200 python tools/bench_ops.py --only enc >> gpurun_out/ws.log 2>&1
done
for ws in 0 1 0 1; do
  GHOST_CONV_WS=$ws timeout -k 10 300 python bench.py --legs '' --cpu-batches '' > /tmp/b.log 2>&1
  python3 -c "import json; d=json.loads([l for l in open('/tmp/b.log') if l.startswith('{')][-1]); print('bench WS=$ws', d['value'], d['ms_per_step'], d['kernel_ms_per_step'])" >> gpurun_out/ws.log
done
