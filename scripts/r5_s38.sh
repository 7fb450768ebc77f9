#!/bin/bash
# r5 session 38: same-box A/B of the prescaled q (PENNY_PRESCALE_Q 0 / 1, alternating, two runs each).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
stop_if_bad() { case "$1" in 124|134|137|139) echo "stopping after rc=$1"; exit "$1";; esac; }
for i in 1 2; do
  for Q in 0 1; do
    PENNY_PRESCALE_Q=$Q timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 \
        > gpurun_out/r5_s38_bench_q${Q}_run${i}.json 2> gpurun_out/r5_s38_bench_q${Q}_run${i}.err
    rc=$?; stop_if_bad $rc
  done
done
