set -e
export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
for v in 0 1; do
  GHOST_LIB_FILE=libghost_amd_tuning.so GHOST_UP_STREAM_LOWPRIO=$v timeout -k 10 200 python tools/ab_streams.py unet 2 > gpurun_out/streams2_ab_$v.log 2>&1
done
