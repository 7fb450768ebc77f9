#!/bin/bash
# r5 session 45: the prefill tile kernel on fragment-tiled weights -- GEMM GPU tests (bit-equality with
# the row-major form), then tiled vs row-major timing on the 8B / 70B TP=1 prefill shapes.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
stop_if_bad() { case "$1" in 124|134|137|139) echo "stopping after rc=$1"; exit "$1";; esac; }
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_kernels_gpu.py -k "gemm or qkv_rope" > gpurun_out/r5_s45_gpu_tests.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r5_s45_gpu_tests.txt; stop_if_bad $rc
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u -m financial_chatbot_llm_amd.bench.kernels --only gemm_tiled_w > gpurun_out/r5_s45_tiled_w.jsonl 2> gpurun_out/r5_s45_tiled_w.err
