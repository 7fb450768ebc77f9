#!/bin/bash
# r5 session 28: lean decode with non-temporal loads for the blocks one row reads (the host marks the
# shared prefix) -- decode / engine GPU tests, the kernel A/B, then the driver bench on / off.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
stop_if_bad() { case "$1" in 124|134|137|139) echo "stopping after rc=$1"; exit "$1";; esac; }
timeout -k 10 700 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_kernels_gpu.py tests/test_engine_gpu.py -k "decode or engine or graph" > gpurun_out/r5_s28_gpu_tests.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r5_s28_gpu_tests.txt; stop_if_bad $rc
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u -m financial_chatbot_llm_amd.bench.kernels --only decode_lean > gpurun_out/r5_s28_decode_lean.jsonl 2> gpurun_out/r5_s28_decode_lean.err
rc=$?; stop_if_bad $rc
PENNY_DECODE_LEAN_FLAGS=1 timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 > gpurun_out/r5_s28_bench_ntm.json 2> gpurun_out/r5_s28_bench_ntm.err
rc=$?; stop_if_bad $rc
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 > gpurun_out/r5_s28_bench_default.json 2> gpurun_out/r5_s28_bench_default.err
