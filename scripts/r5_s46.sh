#!/bin/bash
# r5 session 46: gate|up weights kept only fragment-tiled (70B TP=1) -- the tiled-only engine test + the
# engine / kernel GPU subsets, then config 4's short run with the setting on and off.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
stop_if_bad() { case "$1" in 124|134|137|139) echo "stopping after rc=$1"; exit "$1";; esac; }
timeout -k 10 700 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_engine_gpu.py tests/test_kernels_gpu.py -k "tiled or engine or graph or gateup or gemm" > gpurun_out/r5_s46_gpu_tests.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r5_s46_gpu_tests.txt; stop_if_bad $rc
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python3 -u bench.py --model llama3-70b --tool-steps 3 --convs 64 --steps 6 --warmup 2 \
    > gpurun_out/r5_s46_config4_tiled.json 2> gpurun_out/r5_s46_config4_tiled.err
rc=$?; stop_if_bad $rc
PENNY_TILED_ONLY=0 timeout -k 10 500 python3 -u bench.py --model llama3-70b --tool-steps 3 --convs 64 --steps 6 --warmup 2 \
    > gpurun_out/r5_s46_config4_rowmajor.json 2> gpurun_out/r5_s46_config4_rowmajor.err
