#!/bin/bash
# GPU session: new kernels' numerics + timing.  PART=1: kernel tests + microbenches;
# PART=2: world-8 TP rehearsal + TP decode overlap microbench.
# Every GPU step has its own time limit; the script stops at the first failure.
set -u
mkdir -p gpurun_out
PART=${PART:-1}
step() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  echo "[$(date +%T)] $name" | tee -a gpurun_out/session.log
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" | tee -a gpurun_out/session.log
  tail -4 "gpurun_out/$name.log"
  return $rc
}
if [ "$PART" = 1 ]; then
  step t_attn 420 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
       -k "prefill_attention or fused_lm_head or sampler or agreement or production or route_quant or moe_prefill or moe_grouped or vw" || exit 1
  step b_attn 300 python -u -m financial_chatbot_llm_amd.bench.kernels --only prefill_mixed --out gpurun_out/prefill_mixed.jsonl || exit 1
  step b_vw 300 python -u -m financial_chatbot_llm_amd.bench.kernels --only vw --out gpurun_out/vw.jsonl || exit 1
  step b_moe 300 python -u -m financial_chatbot_llm_amd.bench.kernels --only moe_prefill --out gpurun_out/moe_prefill.jsonl || exit 1
else
  step t_world8 700 python -u -m pytest -x -q --timeout 600 --timeout-method thread tests/test_world8_gpu.py -k tp8 || exit 1
  step b_tpov 400 python -u -m financial_chatbot_llm_amd.bench.tp_decode_overlap --world 8 --layers 4 --batch 64 --ctx 1024 --out gpurun_out/tp_decode_overlap.jsonl || exit 1
fi
