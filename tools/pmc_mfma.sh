# MFMA / VALU utilisation per kernel: separate rocprofv3 --pmc passes over the bench's one-stream
# configuration (B=64 unet/2 bf16) and the ArcFace leg (tools/run_arc.py), summarised by tools/pmc_mfma.py into
# gpurun_out/${ROUND}_mfma.json (copied to profiles/ afterwards).  Each pass stays within one run's counter slots
# (<= 8 SQ_, 2 GRBM_), the program after `--`, each under its own kill timeout.
set -e
export TMPDIR=/tmp PYTHONUNBUFFERED=1
ROUND=${ROUND:-r04}
R=/tmp/ghost_mfma
rm -rf $R && mkdir -p $R gpurun_out
B='python3 bench.py --steps 2 --warmup 1 --no-profile --legs "" --cpu-batches "" --streams 1'
A='python3 tools/run_arc.py 256 2'
P1='SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS GRBM_GUI_ACTIVE GRBM_COUNT'
P2='SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_SALU SQ_WAVES SQ_INST_CYCLES_VMEM'
i=0
for prog in "$B" "$A"; do
  for pass in "$P1" "$P2"; do
    i=$((i+1))
    eval timeout -s KILL 240 rocprofv3 --pmc $pass --output-format csv -d $R/p$i -o run -- $prog > gpurun_out/${ROUND}_mfma_p$i.log 2>&1
  done
done
python3 tools/pmc_mfma.py --gen "$R/p1/run_counter_collection.csv" "$R/p2/run_counter_collection.csv" \
  --arc "$R/p3/run_counter_collection.csv" "$R/p4/run_counter_collection.csv" --out gpurun_out/${ROUND}_mfma.json \
  --source "${ROUND}: rocprofv3 --pmc (2 passes each) over '$B' and '$A'" > gpurun_out/${ROUND}_mfma.txt
