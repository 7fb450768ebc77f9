#!/bin/bash
# r5 session 31: the tile GEMM's L2 token-tile grouping swept (GM 1-16) on the 8B prefill projections,
# plus the new K4 / chunk GPU tests.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
stop_if_bad() { case "$1" in 124|134|137|139) echo "stopping after rc=$1"; exit "$1";; esac; }
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_kernels_gpu.py -k "splitk or gateup or gemm or chunk or shard" > gpurun_out/r5_s31_gpu_tests.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r5_s31_gpu_tests.txt; stop_if_bad $rc
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python3 -u -m financial_chatbot_llm_amd.bench.kernels --only gemm_group > gpurun_out/r5_s31_gemm_group.jsonl 2> gpurun_out/r5_s31_gemm_group.err
