#!/bin/bash
# r5 session 47 (final HEAD): the whole GPU suite + smoke(), then the driver bench once.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
stop_if_bad() { case "$1" in 124|134|137|139) echo "stopping after rc=$1"; exit "$1";; esac; }
timeout -k 10 900 python3 -u -m pytest -q --timeout 600 --timeout-method thread -m gpu tests/ \
    > gpurun_out/r5_s47_gpu_suite.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r5_s47_gpu_suite.txt; stop_if_bad $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5_s47_smoke.txt 2>&1
rc=$?; stop_if_bad $rc
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 > gpurun_out/r5_s47_bench.json 2> gpurun_out/r5_s47_bench.err
