#!/bin/bash
# GPU session 13: software-pipelined prefill attention (variant 5) -- numerics vs fp32 and the
# mixed-step A/B against variant 4.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  echo "[$(date +%T)] $name" | tee -a gpurun_out/session13.log
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" | tee -a gpurun_out/session13.log
  tail -3 "gpurun_out/$name.log"
  return $rc
}
step t_pf4 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "prefill_attention" || exit 1
step b_pf4 300 python -u -m financial_chatbot_llm_amd.bench.kernels --only prefill_mixed --out gpurun_out/prefill_mixed_pf4.jsonl || exit 1
