set -e
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
echo "[ab1] ring test $(date +%T)"
GHOST_HALO_RING=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "ring or conv2d_op" > gpurun_out/ring.log 2>&1
echo "[ab1] pair arcface tests $(date +%T)"
GHOST_HALO_PAIR=1 timeout -k 10 400 python -u -m pytest tests/test_arcface.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/pair.log 2>&1
echo "[ab1] bench ring=0 $(date +%T)"
timeout -k 10 300 python -u bench.py --legs fp16,arcface --cpu-batches "" > gpurun_out/ab_base.log 2>&1
echo "[ab1] bench ring=1 pair=1 $(date +%T)"
GHOST_HALO_RING=1 GHOST_HALO_PAIR=1 timeout -k 10 300 python -u bench.py --legs fp16,arcface --cpu-batches "" > gpurun_out/ab_new.log 2>&1
echo "[ab1] done $(date +%T)"
