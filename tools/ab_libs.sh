# Same-box A/B of saved library builds on one op class: bash tools/ab_libs.sh OPS LIB [LIB ...]
# (tools/bench_ops.py --only OPS through GHOST_LIB_FILE=LIB, twice per library, interleaved)
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
mkdir -p gpurun_out
ops=$1; shift
for rep in 1 2; do
  for lib in "$@"; do
    echo "== $lib rep $rep" >> gpurun_out/ab_libs.txt
    GHOST_LIB_FILE=$lib timeout -k 10 200 python -u tools/bench_ops.py --only "$ops" >> gpurun_out/ab_libs.txt 2>&1 || exit $?
  done
done
