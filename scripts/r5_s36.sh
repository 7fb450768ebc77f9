#!/bin/bash
# r5 session 36: q prescaled at its one rounding in the fused QKV epilogue (PENNY_PRESCALE_Q) --
# prefill / fused-QKV GPU tests, the engine GPU tests with the mode on, then the driver bench on / off.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
stop_if_bad() { case "$1" in 124|134|137|139) echo "stopping after rc=$1"; exit "$1";; esac; }
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_kernels_gpu.py -k "prefill or qkv_rope" > gpurun_out/r5_s36_gpu_tests.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r5_s36_gpu_tests.txt; stop_if_bad $rc
[ $rc -eq 0 ] || exit $rc
PENNY_PRESCALE_Q=1 timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread \
    tests/test_engine_gpu.py tests/test_world8_gpu.py > gpurun_out/r5_s36_engine_tests_qpre.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r5_s36_engine_tests_qpre.txt; stop_if_bad $rc
[ $rc -eq 0 ] || exit $rc
PENNY_PRESCALE_Q=1 timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 > gpurun_out/r5_s36_bench_qpre.json 2> gpurun_out/r5_s36_bench_qpre.err
rc=$?; stop_if_bad $rc
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 > gpurun_out/r5_s36_bench_base.json 2> gpurun_out/r5_s36_bench_base.err
