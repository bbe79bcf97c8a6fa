export PYTHONUNBUFFERED=1
mkdir -p gpurun_out
for o in "pipe,upG,q,model,swap5,upG5,q,drop,d2h,q" "model,swap5,upG5,drop,pipe,upG,q,d2h"; do
  timeout -k 10 300 python -u tools/leg_probe.py --order "$o" >> gpurun_out/c5_probe4.txt 2>&1 || exit 1
done
