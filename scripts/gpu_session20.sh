#!/bin/bash
# GPU session 20: Mixtral-8x7B fp8 (config 5) at the final HEAD (attention projections now on the tile kernel).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 480 python -u bench.py --steps 20 --warmup 5 --model mixtral-8x7b --dtype fp8 > gpurun_out/b_mx_final.log 2>&1 || exit 1
tail -1 gpurun_out/b_mx_final.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['p50_ttft_ms'], d['p99_ttft_ms'])"
