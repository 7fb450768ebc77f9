#!/bin/bash
# r5 session 32: the secondary configurations at HEAD s29+ (paired stages, non-temporal lean decode) -- Mixtral-8x7B fp8 (20/5), BASELINE config 2
# (--no-tools, 20/5) and the no-flag default bench.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
stop_if_bad() { case "$1" in 124|134|137|139) echo "stopping after rc=$1"; exit "$1";; esac; }
timeout -k 10 540 python3 -u bench.py --steps 20 --warmup 5 --model mixtral-8x7b --dtype fp8 > gpurun_out/r5_s32_mixtral.json 2> gpurun_out/r5_s32_mixtral.err
rc=$?; stop_if_bad $rc
timeout -k 10 300 python3 -u bench.py --steps 20 --warmup 5 --no-tools > gpurun_out/r5_s32_notools.json 2> gpurun_out/r5_s32_notools.err
rc=$?; stop_if_bad $rc
timeout -k 10 300 python3 -u bench.py > gpurun_out/r5_s32_default.json 2> gpurun_out/r5_s32_default.err
