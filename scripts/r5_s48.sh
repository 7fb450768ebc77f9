#!/bin/bash
# r5 session 48: config 4 (70B TP=1, --tool-steps 3) short run under rocprofv3 kernel stats at the
# final HEAD (tiled-only gate|up).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 800 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof48 -o run -- \
    python3 bench.py --model llama3-70b --tool-steps 3 --convs 64 --steps 6 --warmup 2 \
    > gpurun_out/r5_s48_config4_prof.json 2> gpurun_out/r5_s48_config4_prof.err
rc=$?; [ $rc -eq 0 ] || exit $rc
st=$(find /tmp/prof48 -name '*kernel_stats.csv' | head -1); tr=$(find /tmp/prof48 -name '*kernel_trace.csv' | head -1)
python3 -m financial_chatbot_llm_amd.bench.profsum "$st" --trace "$tr" --title "r5 final HEAD: Llama-3-70B TP=1, --tool-steps 3, 64 convs, 6/2, under rocprofv3" > gpurun_out/r5_s48_config4_kernel_stats.md 2>&1
rm -rf /tmp/prof48
