#!/bin/bash
# GPU session 8: stream-K tail of the tile GEMM -- numerics vs whole tiles / fp32, the per-shape
# prefill policy sweep against hipBLASLt, then the TTFT admission anatomy A/B.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  echo "[$(date +%T)] $name" | tee -a gpurun_out/session8.log
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" | tee -a gpurun_out/session8.log
  tail -3 "gpurun_out/$name.log"
  return $rc
}
step t_sk 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "prefill_gemm or qkv or rope" || exit 1
step b_pol 400 python -u -m financial_chatbot_llm_amd.bench.kernels --only prefill_policy_quick --out gpurun_out/prefill_policy_sk.jsonl || exit 1
