#!/bin/bash
# r5 session 5: north-star config 4 at its stated 20/5 shape with the r5 kernels (Llama-3-70B bf16 at
# TP=1 on one MI355X, multi-step agent with the plot tool bound, 64 conversations).
set -u
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 1100 python3 -u bench.py --model llama3-70b --tool-steps 3 --convs 64 --steps 20 --warmup 5 \
  > gpurun_out/r5_config4_70b_tp1_20x5.json 2> gpurun_out/r5_config4_70b_tp1_20x5.err
rc=$?
tail -3 gpurun_out/r5_config4_70b_tp1_20x5.err
exit $rc
