#!/bin/bash
# r5 session 25: paired-stage decode GEMM table -- kernel + engine GPU tests, then the driver bench
# with the table (default) and with pairing off (A/B, same box).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
stop_if_bad() { case "$1" in 124|134|137|139) echo "stopping after rc=$1"; exit "$1";; esac; }
timeout -k 10 700 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_kernels_gpu.py tests/test_engine_gpu.py tests/test_world8_gpu.py > gpurun_out/r5_s25_gpu_tests.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r5_s25_gpu_tests.txt; stop_if_bad $rc
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 > gpurun_out/r5_s25_bench_paired.json 2> gpurun_out/r5_s25_bench_paired.err
rc=$?; stop_if_bad $rc
PENNY_PAIR_STAGES=0 timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 > gpurun_out/r5_s25_bench_single.json 2> gpurun_out/r5_s25_bench_single.err
