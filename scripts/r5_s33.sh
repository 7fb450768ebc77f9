#!/bin/bash
# r5 session 33: 256-row split-K workgroups (nf = 16) -- split-K / gate|up GPU tests, then nf 16 vs
# the tables at M = 32-128.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
stop_if_bad() { case "$1" in 124|134|137|139) echo "stopping after rc=$1"; exit "$1";; esac; }
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_kernels_gpu.py -k "splitk or gateup" > gpurun_out/r5_s33_gpu_tests.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r5_s33_gpu_tests.txt; stop_if_bad $rc
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u -m financial_chatbot_llm_amd.bench.kernels --only nf16 > gpurun_out/r5_s33_nf16.jsonl 2> gpurun_out/r5_s33_nf16.err
