#!/bin/bash
# r5 session 16: prefill attention with a 4-deep K/V ring (variant 7 = variant 5 with NBUF 4: three blocks
# in flight instead of two) -- numerics tests, then the workload mixed-step A/B.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
stop_if_bad() { case "$1" in 124|134|137|139) echo "stopping after rc=$1"; exit "$1";; esac; }
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread \
    tests/test_kernels_gpu.py -k "prefill" > gpurun_out/r5_s16_gpu_tests.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r5_s16_gpu_tests.txt; stop_if_bad $rc
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u -m financial_chatbot_llm_amd.bench.kernels --only prefill_mixed > gpurun_out/r5_s16_prefill_mixed.jsonl 2> gpurun_out/r5_s16_prefill_mixed.err
