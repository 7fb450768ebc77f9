#!/bin/bash
# GPU session 6: row-parallel lean prefill merge -- numerics, mixed-step A/B (incl. single-decide
# steps where the split fires), per-kernel times of the merge, then the driver bench.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  echo "[$(date +%T)] $name" | tee -a gpurun_out/session6.log
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" | tee -a gpurun_out/session6.log
  tail -3 "gpurun_out/$name.log"
  return $rc
}
step t_lean 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "lean or prefill" || exit 1
step b_mixed 300 python -u -m financial_chatbot_llm_amd.bench.kernels --only prefill_mixed --out gpurun_out/prefill_mixed_merge.jsonl || exit 1
step p_mixed 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pm -o run -- \
     python3 -m financial_chatbot_llm_amd.bench.kernels --only prefill_mixed || exit 1
find /tmp/pm -name '*kernel_stats.csv' -exec cp {} gpurun_out/prefill_mixed_kernel_stats.csv \;
step b8_merge 360 python -u bench.py --steps 20 --warmup 5 || exit 1
