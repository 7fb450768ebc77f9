#!/bin/bash
# r5 session 21: the two GPU tests fixed after the late-HEAD suite (world-8 results as bytes, the
# custom-AR self-test assertion up to 4 ranks on one GPU) plus the decode-dispatch tests.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 900 python3 -u -m pytest -q --timeout 600 --timeout-method thread \
    tests/test_world8_gpu.py tests/test_custom_ar_gpu.py tests/test_engine_gpu.py > gpurun_out/r5_s21_gpu_tests.txt 2>&1
echo "pytest rc=$?" >> gpurun_out/r5_s21_gpu_tests.txt
