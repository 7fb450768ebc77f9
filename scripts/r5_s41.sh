#!/bin/bash
# r5 session 41: the lean decode merge, 1 vs 4 heads per workgroup (A/B) -- decode / engine GPU tests, then the
# decode_lean bench under rocprofv3 kernel stats (merge kernel time per call).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
stop_if_bad() { case "$1" in 124|134|137|139) echo "stopping after rc=$1"; exit "$1";; esac; }
timeout -k 10 700 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_kernels_gpu.py tests/test_engine_gpu.py -k "decode or engine or graph" > gpurun_out/r5_s41_gpu_tests.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r5_s41_gpu_tests.txt; stop_if_bad $rc
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof41 -o run -- \
    python3 -m financial_chatbot_llm_amd.bench.kernels --only decode_lean > gpurun_out/r5_s41_decode_lean.jsonl 2> gpurun_out/r5_s41_decode_lean.err
rc=$?; [ $rc -eq 0 ] || exit $rc
st=$(find /tmp/prof41 -name '*kernel_stats.csv' | head -1)
cp "$st" gpurun_out/r5_s41_kernel_stats.csv
