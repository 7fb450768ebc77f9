#!/bin/bash
# GPU session 18: lean split-KV prefill on/off at the driver config (final HEAD).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 env PENNY_PREFILL_LEAN=0 python -u bench.py --steps 20 --warmup 5 > gpurun_out/b_nolean.log 2>&1 || exit 1
tail -1 gpurun_out/b_nolean.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('lean off', d['value'], d['p50_ttft_ms'], d['p99_ttft_ms'])"
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/b_lean.log 2>&1 || exit 1
tail -1 gpurun_out/b_lean.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('lean on', d['value'], d['p50_ttft_ms'], d['p99_ttft_ms'])"
