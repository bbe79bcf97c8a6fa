# ArcFace embeddings per launch: B = 128 / 256 / 512 (shipping library)
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
ok() { rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "stop: rc=$rc"; exit $rc; }; }
for n in 128 256 512 256; do
  timeout -k 10 200 python -u tools/run_arc.py $n 8 >> gpurun_out/arc_batch.txt 2>&1; ok $?
done
rm -rf /tmp/at
timeout -k 10 300 rocprofv3 --kernel-trace -d /tmp/at -o run -- python3 tools/run_arc.py 256 4 > gpurun_out/arc_tr_256.log 2>&1; ok $?
python3 tools/kernel_table.py /tmp/at/run_results.db --top 24 > gpurun_out/arc_kt_256.txt 2>&1
echo done
