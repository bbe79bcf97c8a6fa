# Kernel-trace summary of tools/bench_ops.py --only OPS under each env spec (';'-separated, e.g.
# "GHOST_V5_FLAGS=3;GHOST_V5_FLAGS=7"): bash tools/kt_ops.sh OPS SPECS [NAME_REGEX]  -> gpurun_out/kt_ops.txt
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
ops=$1
filt=${3:-aad|stats}
IFS=';' read -ra specs <<< "$2"
for v in "${specs[@]}"; do
  rm -rf /tmp/kt
  eval env $v timeout -k 10 240 rocprofv3 --kernel-trace --stats -d /tmp/kt -o run -- python3 tools/bench_ops.py --only "$ops" --iters 10 > /tmp/kt.log 2>&1 || { cp /tmp/kt.log gpurun_out/kt_fail.log; exit 1; }
  echo "== $v" >> gpurun_out/kt_ops.txt
  python3 tools/kernel_table.py /tmp/kt/run_results.db --top 0 --stats-csv /tmp/kt.csv > /dev/null || exit 1
  f=/tmp/kt.csv
  python3 -c "
import csv,sys,re
rows=list(csv.DictReader(open('$f')))
for r in rows:
    n=r['Name']
    if re.search('$filt', n): print('%10.1f us  %5s calls  %s' % (float(r['AverageNs'])/1e3, r['Calls'], n[:110]))
" >> gpurun_out/kt_ops.txt
done
