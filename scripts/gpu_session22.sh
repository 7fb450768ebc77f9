#!/bin/bash
# GPU session 22: config 4 (Llama-3-70B, multi-step agent) at TP=1 on one GPU, short run at the final HEAD.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 1000 python -u bench.py --model llama3-70b --tool-steps 3 --convs 64 --steps 5 --warmup 2 > gpurun_out/b_70b.log 2>&1 || exit 1
tail -1 gpurun_out/b_70b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['p50_ttft_ms'], d['p99_ttft_ms'], d['turn_errors'])"
