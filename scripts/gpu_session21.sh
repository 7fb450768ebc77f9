#!/bin/bash
# GPU session 21: the no-flag default bench and config 2 (no tools) at the final HEAD.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u bench.py > gpurun_out/b_noflag.log 2>&1 || exit 1
tail -1 gpurun_out/b_noflag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('noflag', d['value'], d['p50_ttft_ms'], d['p99_ttft_ms'])"
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --no-tools > gpurun_out/b_notools.log 2>&1 || exit 1
tail -1 gpurun_out/b_notools.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('notools', d['value'], d['p50_ttft_ms'], d['p99_ttft_ms'])"
