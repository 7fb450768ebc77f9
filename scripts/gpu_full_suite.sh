#!/bin/bash
# The round-end tiers at HEAD: the whole GPU test suite (one process), smoke(), then the driver bench.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  echo "[$(date +%T)] $name" | tee -a gpurun_out/full.log
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" | tee -a gpurun_out/full.log
  tail -3 "gpurun_out/$name.log"
  return $rc
}
step f_gpu 900 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread || exit 1
step f_smoke 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit 1
step f_bench 400 python -u bench.py --steps 20 --warmup 5 || exit 1
