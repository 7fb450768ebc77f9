#!/bin/bash
# r5 session 29 (HEAD after paired stages + non-temporal lean decode): the whole GPU suite + smoke(), the driver-config kernel breakdown under
# rocprofv3 (with the engine's roctx ranges), then the driver bench unprofiled.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
stop_if_bad() { case "$1" in 124|134|137|139) echo "stopping after rc=$1"; exit "$1";; esac; }
timeout -k 10 900 python3 -u -m pytest -q --timeout 600 --timeout-method thread -m gpu tests/ \
    > gpurun_out/r5_s29_gpu_suite.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r5_s29_gpu_suite.txt; stop_if_bad $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5_s29_smoke.txt 2>&1
rc=$?; stop_if_bad $rc
export PENNY_MARKERS=1
timeout -k 10 480 rocprofv3 --kernel-trace --marker-trace --stats --output-format csv -d /tmp/prof -o run -- \
    python3 bench.py --steps 20 --warmup 5 > gpurun_out/r5_s29_prof_bench.json 2> gpurun_out/r5_s29_prof_bench.err
rc=$?; stop_if_bad $rc
unset PENNY_MARKERS
st=$(find /tmp/prof -name '*kernel_stats.csv' | head -1); tr=$(find /tmp/prof -name '*kernel_trace.csv' | head -1)
mk=$(find /tmp/prof -name '*marker_api_trace.csv' | head -1)
python3 -m financial_chatbot_llm_amd.bench.profsum "$st" --trace "$tr" --markers "$mk" --title "r5 HEAD s29: driver bench 20x5 kernel breakdown" > gpurun_out/r5_s29_prof_kernel_stats.md 2>&1
rm -rf /tmp/prof
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 > gpurun_out/r5_s29_bench.json 2> gpurun_out/r5_s29_bench.err
