#!/bin/bash
# GPU session 17: per-step token budget re-sweep at HEAD (all prefill GEMMs on the tile kernel).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
for b in 6144 3584; do
  timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 --max-batched-tokens $b > gpurun_out/b_mbt$b.log 2>&1 || exit 1
  tail -1 gpurun_out/b_mbt$b.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print($b, d['value'], d['p50_ttft_ms'], d['p99_ttft_ms'])"
done
