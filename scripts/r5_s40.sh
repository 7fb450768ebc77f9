#!/bin/bash
# r5 session 40: final-HEAD driver-config kernel breakdown under rocprofv3 (with the engine's roctx
# ranges), prescaled q on.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
export PENNY_MARKERS=1
timeout -k 10 480 rocprofv3 --kernel-trace --marker-trace --stats --output-format csv -d /tmp/prof -o run -- \
    python3 bench.py --steps 20 --warmup 5 > gpurun_out/r5_s40_prof_bench.json 2> gpurun_out/r5_s40_prof_bench.err
rc=$?; [ $rc -eq 0 ] || exit $rc
st=$(find /tmp/prof -name '*kernel_stats.csv' | head -1); tr=$(find /tmp/prof -name '*kernel_trace.csv' | head -1)
mk=$(find /tmp/prof -name '*marker_api_trace.csv' | head -1)
python3 -m financial_chatbot_llm_amd.bench.profsum "$st" --trace "$tr" --markers "$mk" --title "r5 final HEAD (s40): driver bench 20x5 kernel breakdown" > gpurun_out/r5_s40_prof_kernel_stats.md 2>&1
rm -rf /tmp/prof
