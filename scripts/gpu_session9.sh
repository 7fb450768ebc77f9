#!/bin/bash
# GPU session 9: stream-K tail A/B -- new kernel vs the pre-stream-K library (ab/libpenny_old.so)
# vs whole tiles only, on the prefill policy shapes.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  echo "[$(date +%T)] $name" | tee -a gpurun_out/session9.log
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" | tee -a gpurun_out/session9.log
  return $rc
}
step p_new 300 python -u -m financial_chatbot_llm_amd.bench.kernels --only prefill_policy_quick --out gpurun_out/pol_new.jsonl || exit 1
step p_old 300 env PENNY_KERNEL_LIB=$PWD/ab/libpenny_old.so python -u -m financial_chatbot_llm_amd.bench.kernels --only prefill_policy_quick --out gpurun_out/pol_old.jsonl || exit 1
step p_dp 300 env PENNY_GEMM_TAIL=0 python -u -m financial_chatbot_llm_amd.bench.kernels --only prefill_policy_quick --out gpurun_out/pol_dp.jsonl || exit 1
