#!/bin/bash
# r5 session 26: decode split-K kernels with 256-row token chunks (M > 256) -- GPU tests, then the
# chunked vs production / hipBLASLt / tile-kernel A/B at small prefill steps of narrow shapes.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
stop_if_bad() { case "$1" in 124|134|137|139) echo "stopping after rc=$1"; exit "$1";; esac; }
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_kernels_gpu.py -k "splitk or gateup" > gpurun_out/r5_s26_gpu_tests.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r5_s26_gpu_tests.txt; stop_if_bad $rc
[ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python3 -u -m financial_chatbot_llm_amd.bench.kernels --only chunked_prefill > gpurun_out/r5_s26_chunked.jsonl 2> gpurun_out/r5_s26_chunked.err
