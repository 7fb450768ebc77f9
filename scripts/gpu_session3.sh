#!/bin/bash
# GPU session 3: MFMA-busy PMC of the tile GEMMs (bf16 + fp8 MoE after the phase fix), the MoE
# tile A/B (balanced vs plain read schedule), the driver bench at HEAD.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  echo "[$(date +%T)] $name" | tee -a gpurun_out/session3.log
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" | tee -a gpurun_out/session3.log
  tail -3 "gpurun_out/$name.log"
  return $rc
}
step t_pf 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "prefill_attention or moe_prefill_fp8 or moe_grouped or route_quant" || exit 1
step t_mx 200 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "mfma_scale_operand or mx_gemm or mx_handoff"
step b_pf 300 python -u -m financial_chatbot_llm_amd.bench.kernels --only prefill_mixed --out gpurun_out/prefill_mixed_v2.jsonl || exit 1
step pmc_tiles 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAVES GRBM_GUI_ACTIVE \
     --kernel-trace --output-format csv -d gpurun_out/pmc_tiles -o run -- \
     python3 -m financial_chatbot_llm_amd.bench.kernels --only gemm_lds_probe || exit 1
step moe_plain 240 env PENNY_MOE_TILE_SCHED=plain python -u -m financial_chatbot_llm_amd.bench.kernels --only moe_prefill \
     --out gpurun_out/moe_prefill_plain.jsonl || exit 1
step moe_mx 240 env PENNY_MOE_MX=1 python -u -m financial_chatbot_llm_amd.bench.kernels --only moe_prefill \
     --out gpurun_out/moe_prefill_mx.jsonl || exit 1
step bench8b 420 python -u bench.py --steps 20 --warmup 5 || exit 1
