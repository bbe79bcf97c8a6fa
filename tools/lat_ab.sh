# same-box A/B of B = 1 latency under env settings (tuning build): bash tools/lat_ab.sh "SPEC1;SPEC2;..."
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
IFS=';' read -ra specs <<< "$1"
for rep in 1 2; do
  for v in "${specs[@]}"; do
    eval env GHOST_TUNING=1 $v timeout -k 10 200 python -u tools/lat_ab.py >> gpurun_out/lat_ab.txt 2>&1 || exit 1
  done
done
