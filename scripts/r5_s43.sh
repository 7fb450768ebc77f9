#!/bin/bash
# r5 session 43: step-row quantisation from any chunk (PENNY_QUANTISE_ANY 1 / 0, alternating, two runs
# each) on the driver bench.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
stop_if_bad() { case "$1" in 124|134|137|139) echo "stopping after rc=$1"; exit "$1";; esac; }
for i in 1 2; do
  for A in 1 0; do
    PENNY_QUANTISE_ANY=$A timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 \
        > gpurun_out/r5_s43_bench_any${A}_run${i}.json 2> gpurun_out/r5_s43_bench_any${A}_run${i}.err
    rc=$?; stop_if_bad $rc
  done
done
