# decomposition of a persistent halo conv's time (tuning build, GHOST_HALO_DBG variants): bash tools/conv_dbg.sh H CIN COUT [VARIANTS]
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
for v in ${4:-0 2 4 6 8 16 22 24 30}; do
  echo "dbg=$v $(GHOST_TUNING=1 GHOST_HALO_DBG=$v timeout -k 10 120 python -u tools/run_conv.py $1 $2 $3 20 2>&1 | tail -1)" >> gpurun_out/conv_dbg.txt || exit 1
done
