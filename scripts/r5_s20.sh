#!/bin/bash
# r5 session 20: the Llama-3-8B decode projections (QKV / O / down split-K slabs) re-swept over (S, nf) at
# HEAD, M = 32..256, weights streamed from HBM.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
timeout -k 10 500 python3 -u -m financial_chatbot_llm_amd.bench.kernels --only decode_8b > gpurun_out/r5_s20_decode_8b.jsonl 2> gpurun_out/r5_s20_decode_8b.err
