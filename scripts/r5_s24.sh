#!/bin/bash
# r5 session 24: decode GEMM streams with paired BK=64 stages -- bit-identity GPU tests, then the
# single vs paired A/B at the 70B TP=1 / TP=8 and 8B decode shapes.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
stop_if_bad() { case "$1" in 124|134|137|139) echo "stopping after rc=$1"; exit "$1";; esac; }
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_kernels_gpu.py -k "splitk or gateup" > gpurun_out/r5_s24_gpu_tests.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r5_s24_gpu_tests.txt; stop_if_bad $rc
[ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python3 -u -m financial_chatbot_llm_amd.bench.kernels --only rm_pair > gpurun_out/r5_s24_rm_pair.jsonl 2> gpurun_out/r5_s24_rm_pair.err
