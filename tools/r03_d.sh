# ArcFace per-kernel traces with and without the two-sample halo window (tuning build, GHOST_HALO_PAIR)
export PYTHONUNBUFFERED=1 TMPDIR=/tmp GHOST_TUNING=1
mkdir -p gpurun_out
ok() { rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "stop: rc=$rc"; exit $rc; }; }
for n in 64 128; do
  for p in 0 1; do
    rm -rf /tmp/at
    GHOST_HALO_PAIR=$p timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/at -o run -- python3 tools/run_arc.py $n 5 > gpurun_out/arc_tr_${n}_$p.log 2>&1; ok $?
    python3 tools/kernel_table.py /tmp/at/run_results.db --top 16 > gpurun_out/arc_kt_${n}_$p.txt 2>&1
  done
done
timeout -k 10 300 python -u bench.py --legs arcface,latency --cpu-batches= > gpurun_out/legs_d.log 2>&1; ok $?
GHOST_HALO_PAIR=1 timeout -k 10 300 python -u bench.py --legs arcface --cpu-batches= > gpurun_out/legs_d_pair.log 2>&1; ok $?
echo done
