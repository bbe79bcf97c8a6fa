set -e
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
timeout -k 10 200 python tools/ab_streams.py unet 2 > gpurun_out/streams_ab.log 2>&1
timeout -k 10 200 python tools/ab_streams.py linknet 3 >> gpurun_out/streams_ab.log 2>&1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/streams_gputests.log 2>&1
timeout -k 10 200 python bench.py --legs "" --cpu-batches "" > gpurun_out/streams_bench.log 2>&1
