#!/bin/bash
# GPU session 7: TTFT-tail admission anatomy (short_wait) at HEAD and the short-first A/B.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  echo "[$(date +%T)] $name" | tee -a gpurun_out/session7.log
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" | tee -a gpurun_out/session7.log
  tail -1 "gpurun_out/$name.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['engine_rank0']; print(d['value'], d['p50_ttft_ms'], d['p99_ttft_ms'], e.get('short_wait'))"
  return $rc
}
step b7_anat 360 python -u bench.py --steps 20 --warmup 5 || exit 1
step b7_sfirst 360 env PENNY_SHORT_FIRST=1 python -u bench.py --steps 20 --warmup 5 || exit 1
