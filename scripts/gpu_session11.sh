#!/bin/bash
# GPU session 11: stream-K tail after the combine-load fix -- numerics, then policy sweep new vs
# the pre-stream-K library.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  echo "[$(date +%T)] $name" | tee -a gpurun_out/session11.log
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" | tee -a gpurun_out/session11.log
  tail -2 "gpurun_out/$name.log"
  return $rc
}
step t_sk 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_kernels_gpu.py -k "prefill_gemm or qkv or rope" || exit 1
step p_new 300 env PENNY_GEMM_SK=1 python -u -m financial_chatbot_llm_amd.bench.kernels --only prefill_policy_quick --out gpurun_out/pol_new.jsonl || exit 1
step p_dp 300 env PENNY_GEMM_SK=0 python -u -m financial_chatbot_llm_amd.bench.kernels --only prefill_policy_quick --out gpurun_out/pol_dp.jsonl || exit 1
step p_old 300 env PENNY_KERNEL_LIB=$PWD/ab/libpenny_old.so python -u -m financial_chatbot_llm_amd.bench.kernels --only prefill_policy_quick --out gpurun_out/pol_old.jsonl || exit 1
