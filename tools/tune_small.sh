# tile x split-K sweep of the low-resolution convs: one process per GHOST_CONV_TILE / GHOST_CONV_BK setting
set -e
for cfg in "auto auto" "128x128 64" "128x128 32" "64x128 32" "128x64 32" "256x64 32" "64x64 64"; do
  set -- $cfg
  if [ "$1" = auto ]; then unset GHOST_CONV_TILE; else export GHOST_CONV_TILE=$1; fi
  if [ "$2" = auto ]; then unset GHOST_CONV_BK; else export GHOST_CONV_BK=$2; fi
  timeout -k 10 120 python tools/tune_small.py >> gpurun_out/tune_small.log 2>&1
done
