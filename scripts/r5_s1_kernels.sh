#!/bin/bash
# r5 session 1: numerics of the new split-K epilogues (bf16 out, streaming LM-head sampler, nf=2
# gate|up), then the shard-shape and streaming LM-head benches.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 300 --timeout-method thread \
  -k "stream or bf16_gemm or nf2 or lm_head or splitk or gateup" > gpurun_out/r5_s1_tests.txt 2>&1 || exit $?
timeout -k 10 400 python -u -m financial_chatbot_llm_amd.bench.kernels --only lm_head_stream,lm_head_stream_shard \
  --out gpurun_out/r5_lm_head_stream.jsonl > gpurun_out/r5_lm_head_stream.log 2>&1 || exit $?
timeout -k 10 600 python -u -m financial_chatbot_llm_amd.bench.kernels --only shard_shapes \
  --out gpurun_out/r5_shard_shapes.jsonl > gpurun_out/r5_shard_shapes.log 2>&1 || exit $?
