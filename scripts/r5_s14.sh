#!/bin/bash
# r5 session 14: final-HEAD kernel breakdown of the driver config (rocprofv3 --kernel-trace --stats, with
# the engine's roctx ranges for the idle-gap attribution), then the driver bench unprofiled.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
stop_if_bad() { case "$1" in 124|134|137|139) echo "stopping after rc=$1"; exit "$1";; esac; }
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_world8_gpu.py tests/test_tp_gpu.py tests/test_kernels_gpu.py -k "world8 or tp or gateup or splitk" \
    > gpurun_out/r5_s14_gpu_tests.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r5_s14_gpu_tests.txt; stop_if_bad $rc
[ $rc -eq 0 ] || exit $rc
export PENNY_MARKERS=1
timeout -k 10 480 rocprofv3 --kernel-trace --marker-trace --stats --output-format csv -d /tmp/prof -o run -- \
    python3 bench.py --steps 20 --warmup 5 > gpurun_out/r5_s14_prof_bench.json 2> gpurun_out/r5_s14_prof_bench.err
rc=$?; stop_if_bad $rc
unset PENNY_MARKERS
st=$(find /tmp/prof -name '*kernel_stats.csv' | head -1); tr=$(find /tmp/prof -name '*kernel_trace.csv' | head -1)
mk=$(find /tmp/prof -name '*marker_api_trace.csv' | head -1)
cp "$st" gpurun_out/r5_s14_prof_kernel_stats.csv
python3 -m financial_chatbot_llm_amd.bench.profsum "$st" --trace "$tr" --markers "$mk" --title "r5 final HEAD: driver bench 20x5 kernel breakdown" > gpurun_out/r5_s14_prof_kernel_stats.md 2>&1
rm -rf /tmp/prof
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 > gpurun_out/r5_s14_bench.json 2> gpurun_out/r5_s14_bench.err
