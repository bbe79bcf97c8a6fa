export GHOST_TUNING=1 GHOST_CONV_TRACE=1
timeout -k 10 120 python3 bench.py --steps 1 --warmup 0 --legs "" --cpu-batches "" --no-profile --streams 1 --opt two_streams=0 > gpurun_out/conv_trace.log 2>&1
