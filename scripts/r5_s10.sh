#!/bin/bash
# r5 session 10: lean decode with the in-kernel (ticketed) merge -- GPU tests, the lean A/B kernel
# bench (fused vs separate merge, alone and concurrent with a prefill), then the driver bench.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
stop_if_bad() { case "$1" in 124|134|137|139) echo "stopping after rc=$1"; exit "$1";; esac; }
timeout -k 10 700 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread \
    tests/test_kernels_gpu.py tests/test_engine_gpu.py -k "decode or engine or graph" \
    > gpurun_out/r5_s10_gpu_tests.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r5_s10_gpu_tests.txt; stop_if_bad $rc
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u -m financial_chatbot_llm_amd.bench.kernels --only decode_lean > gpurun_out/r5_s10_decode_lean_fused.jsonl 2> gpurun_out/r5_s10_decode_lean_fused.err
rc=$?; stop_if_bad $rc
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 > gpurun_out/r5_s10_bench.json 2> gpurun_out/r5_s10_bench.err
rc=$?; stop_if_bad $rc
export PENNY_DECODE_LEAN_FUSED=0
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 > gpurun_out/r5_s10_bench_sepmerge.json 2> gpurun_out/r5_s10_bench_sepmerge.err
