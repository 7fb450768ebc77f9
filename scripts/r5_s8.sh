#!/bin/bash
# r5 session 8: host-side cost of the engine thread (cProfile, PENNY_PYPROFILE) over the driver
# bench, and the serving thread's share -- where the launch-bound eager steps spend host time.
set -u
mkdir -p gpurun_out/pyprof
export TMPDIR=/tmp PYTHONUNBUFFERED=1
stop_if_bad() { case "$1" in 124|134|137|139) echo "stopping after rc=$1"; exit "$1";; esac; }
export PENNY_PYPROFILE=gpurun_out/pyprof
timeout -k 10 480 python3 -u bench.py --steps 20 --warmup 5 > gpurun_out/r5_s8_pyprof_bench.json 2> gpurun_out/r5_s8_pyprof_bench.err
rc=$?; stop_if_bad $rc
unset PENNY_PYPROFILE
python3 - > gpurun_out/r5_s8_pyprof_top.txt 2>&1 <<'PY'
import pstats
p = pstats.Stats("gpurun_out/pyprof/engine_r0.prof")
p.sort_stats("tottime").print_stats(45)
p.sort_stats("cumulative").print_stats(60)
PY
