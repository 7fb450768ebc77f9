#!/bin/bash
# r5 session 9: host-overhead trims (raw current stream, reused fork/join events, cached env knob):
# engine + attention GPU tests, the driver bench unprofiled, then the engine thread under cProfile.
set -u
mkdir -p gpurun_out/pyprof9
export TMPDIR=/tmp PYTHONUNBUFFERED=1
stop_if_bad() { case "$1" in 124|134|137|139) echo "stopping after rc=$1"; exit "$1";; esac; }
timeout -k 10 700 python3 -u -m pytest -x -q --timeout 240 --timeout-method thread \
    tests/test_engine_gpu.py tests/test_kernels_gpu.py -k "engine or decode or mixed or overlap or graph" \
    > gpurun_out/r5_s9_gpu_tests.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r5_s9_gpu_tests.txt; stop_if_bad $rc
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 > gpurun_out/r5_s9_bench.json 2> gpurun_out/r5_s9_bench.err
rc=$?; stop_if_bad $rc
export PENNY_PYPROFILE=gpurun_out/pyprof9
timeout -k 10 480 python3 -u bench.py --steps 20 --warmup 5 > gpurun_out/r5_s9_pyprof_bench.json 2> gpurun_out/r5_s9_pyprof_bench.err
rc=$?; stop_if_bad $rc
unset PENNY_PYPROFILE
python3 - > gpurun_out/r5_s9_pyprof_top.txt 2>&1 <<'PY'
import pstats
p = pstats.Stats("gpurun_out/pyprof9/engine_r0.prof")
p.sort_stats("tottime").print_stats(30)
p.sort_stats("cumulative").print_stats(40)
PY
rm -f gpurun_out/pyprof9/*.prof
