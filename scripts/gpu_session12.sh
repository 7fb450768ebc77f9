#!/bin/bash
# GPU session 12: effective clock of the tile GEMM by occupied CUs (GRBM_GUI_ACTIVE per dispatch).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
export PYTHONPATH=$PWD
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE GRBM_COUNT --kernel-trace --output-format csv -d /tmp/clk -o run -- python3 scripts/clock_probe.py > gpurun_out/clk.log 2>&1
rc=$?
find /tmp/clk -name '*counter_collection.csv' -exec cp {} gpurun_out/clk_counters.csv \;
find /tmp/clk -name '*kernel_trace.csv' -exec cp {} gpurun_out/clk_trace.csv \;
tail -3 gpurun_out/clk.log
exit $rc
