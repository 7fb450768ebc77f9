#!/bin/bash
# r5 session 6: GPU tests touched by the cascade removal (decode attention kernels, engine, world-8),
# then the driver bench under rocprofv3 --kernel-trace with the idle-gap attribution (profsum gaps).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
stop_if_bad() { case "$1" in 124|134|137|139) echo "stopping after rc=$1"; exit "$1";; esac; }
timeout -k 10 700 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread \
    tests/test_kernels_gpu.py -k "decode" tests/test_engine_gpu.py tests/test_world8_gpu.py tests/test_custom_ar_gpu.py \
    > gpurun_out/r5_s6_gpu_tests.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r5_s6_gpu_tests.txt; stop_if_bad $rc
[ $rc -eq 0 ] || exit $rc
timeout -k 10 480 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof -o run -- \
    python3 bench.py --steps 20 --warmup 5 > gpurun_out/r5_s6_prof_bench.json 2> gpurun_out/r5_s6_prof_bench.err
rc=$?; stop_if_bad $rc
st=$(find /tmp/prof -name '*kernel_stats.csv' | head -1); tr=$(find /tmp/prof -name '*kernel_trace.csv' | head -1)
cp "$st" gpurun_out/r5_s6_prof_kernel_stats.csv
python3 -m financial_chatbot_llm_amd.bench.profsum "$st" --trace "$tr" --title "r5 driver bench 20x5, cascade removed, idle-gap attribution" > gpurun_out/r5_s6_prof_kernel_stats.md 2>&1
rm -rf /tmp/prof
