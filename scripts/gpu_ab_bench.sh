#!/bin/bash
# Interleaved A/B of the driver's bench config (python bench.py --steps 20 --warmup 5) over env
# variants given as arguments, e.g.:  bash scripts/gpu_ab_bench.sh "PENNY_PREFILL_PP=0" "PENNY_PREFILL_PP=1"
# Each variant runs once per round; ROUNDS (default 1) rounds.  Results: gpurun_out/ab_<i>_<r>.json
set -u
mkdir -p gpurun_out
ROUNDS=${ROUNDS:-1}
STEPS=${STEPS:-20}
WARM=${WARM:-5}
for r in $(seq 1 "$ROUNDS"); do
  i=0
  for v in "$@"; do
    i=$((i + 1))
    echo "[$(date +%T)] round $r variant $i: $v" | tee -a gpurun_out/ab.log
    env $v timeout -k 10 400 python -u bench.py --steps "$STEPS" --warmup "$WARM" \
        > "gpurun_out/ab_${i}_${r}.json" 2> "gpurun_out/ab_${i}_${r}.err"
    rc=$?
    echo "[$(date +%T)] rc=$rc $(tail -1 gpurun_out/ab_${i}_${r}.json | python3 -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["p50_ttft_ms"], d["p99_ttft_ms"])' 2>/dev/null)" | tee -a gpurun_out/ab.log
    [ $rc -eq 0 ] || exit $rc
  done
done
