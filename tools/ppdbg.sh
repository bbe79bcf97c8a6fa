# pp conv experiment variants (GHOST_HALO_DBG bits: 2 no halo DMA, 4 no weight DMA, 8 no MFMA, 16 no stores,
# 32 single fragment register set, 64 s_setprio(1) around the MFMAs)
set -e
for d in 0 32 64 96 18 50 82 114 22 54 86 118; do
  GHOST_HALO_DBG=$d timeout -k 10 120 python tools/bench_ops.py --only pp --iters 20 > gpurun_out/ppdbg_$d.log 2>&1
done
