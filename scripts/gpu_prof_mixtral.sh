#!/bin/bash
# rocprofv3 kernel statistics of the Mixtral-8x7B fp8 bench (config 5) at HEAD; trace kept on the box.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 480 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/profmx -o run -- \
    python3 bench.py --steps 20 --warmup 5 --model mixtral-8x7b --dtype fp8 > gpurun_out/profmx.log 2>&1
rc=$?
find /tmp/profmx -name '*kernel_stats.csv' -exec cp {} gpurun_out/profmx_kernel_stats.csv \;
tail -2 gpurun_out/profmx.log
exit $rc
