#!/bin/bash
# r5 session 19: prefill attention out-of-loop tweaks (16-B output stores via permlane16 pairs, static
# priority of the younger wave half) -- numerics tests, then the in-process A/B against variant 9
# (variant 5 with the old 8-B store tail and no priority) on the workload's mixed steps.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
stop_if_bad() { case "$1" in 124|134|137|139) echo "stopping after rc=$1"; exit "$1";; esac; }
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread \
    tests/test_kernels_gpu.py -k "prefill" > gpurun_out/r5_s19_gpu_tests.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r5_s19_gpu_tests.txt; stop_if_bad $rc
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u -m financial_chatbot_llm_amd.bench.kernels --only prefill_mixed > gpurun_out/r5_s19_prefill_mixed.jsonl 2> gpurun_out/r5_s19_prefill_mixed.err
