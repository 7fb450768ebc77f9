#!/bin/bash
# rocprofv3 kernel statistics of the driver bench; the per-dispatch trace is deleted on the box
# (it exceeds the 64 MiB copy-back), only the stats CSV comes home.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 420 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof8 -o run -- \
    python3 bench.py --steps 20 --warmup 5 > gpurun_out/prof8.log 2>&1
rc=$?
find /tmp/prof8 -name '*kernel_stats.csv' -exec cp {} gpurun_out/prof8_kernel_stats.csv \;
tail -3 gpurun_out/prof8.log
exit $rc
