#!/bin/bash
# GPU session 16: finer lean split-KV balance targets for prefill attention (mixed-step A/B).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m financial_chatbot_llm_amd.bench.kernels --only prefill_mixed --out gpurun_out/prefill_mixed_fine.jsonl > gpurun_out/b_fine.log 2>&1 || exit 1
python3 -c "
import json
for l in open('gpurun_out/prefill_mixed_fine.jsonl'):
    d=json.loads(l); print(d['step'], d['pf2_sb_us'], d['pf2_sb_lean_us'], d['pf2_sb_lean_x2_us'], d['pf2_sb_lean_x4_us'], d['pf2_sb_lean_x4_maxdiff_vs_pf2'])"
