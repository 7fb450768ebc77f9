#!/bin/bash
# r5 session 39: config 4 (Llama-3-70B TP=1, --tool-steps 3, 64 convs) short run at the final HEAD
# (6 timed steps, 2 warmup), unprofiled.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 1000 python3 -u bench.py --model llama3-70b --tool-steps 3 --convs 64 --steps 6 --warmup 2 \
    > gpurun_out/r5_s39_config4_6x2.json 2> gpurun_out/r5_s39_config4_6x2.err
