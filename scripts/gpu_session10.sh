#!/bin/bash
# GPU session 10: per-dispatch kernel times of the stream-K probe, new vs pre-stream-K library.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
export PYTHONPATH=$PWD
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d /tmp/skn -o run -- python3 scripts/sk_probe.py > gpurun_out/skn.log 2>&1 || exit 1
find /tmp/skn -name '*kernel_trace.csv' -exec cp {} gpurun_out/sk_new_trace.csv \;
PENNY_KERNEL_LIB=$PWD/ab/libpenny_old.so timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d /tmp/sko -o run -- python3 scripts/sk_probe.py > gpurun_out/sko.log 2>&1 || exit 1
find /tmp/sko -name '*kernel_trace.csv' -exec cp {} gpurun_out/sk_old_trace.csv \;
