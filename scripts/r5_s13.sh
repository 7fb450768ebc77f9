#!/bin/bash
# r5 session 13: split-K gate|up (slabs + reduce-SiLU) -- GPU tests, then the gate|up shapes
# (70B TP=8 shard, 70B TP=1 row-major, 8B above 160 rows) against hipBLASLt + silu_mul and the fused kernel.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
stop_if_bad() { case "$1" in 124|134|137|139) echo "stopping after rc=$1"; exit "$1";; esac; }
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread \
    tests/test_kernels_gpu.py -k "gateup" > gpurun_out/r5_s13_gpu_tests.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r5_s13_gpu_tests.txt; stop_if_bad $rc
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u -m financial_chatbot_llm_amd.bench.kernels --only gateup_shapes > gpurun_out/r5_s13_gateup_shapes.jsonl 2> gpurun_out/r5_s13_gateup_shapes.err
