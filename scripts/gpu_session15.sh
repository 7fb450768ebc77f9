#!/bin/bash
# GPU session 15: O projection on the tile kernel at every prefill size -- decoder-level policy
# tests, then the driver bench.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  echo "[$(date +%T)] $name" | tee -a gpurun_out/session15.log
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" | tee -a gpurun_out/session15.log
  tail -2 "gpurun_out/$name.log" | cut -c1-400
  return $rc
}
step t_pol 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_prefill_policy_gpu.py tests/test_prefill_policy.py || exit 1
step b_qpol 400 python -u bench.py --steps 20 --warmup 5 || exit 1
