#!/bin/bash
# r5 session 2: GPU tests of the decode/TP paths (incl. the custom-AR init self-test at world 8 on one
# GPU), re-measure with the 16-deep ring for narrow configs, then the driver bench.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_custom_ar_gpu.py tests/test_world8_gpu.py \
  tests/test_tp_gpu.py tests/test_engine_gpu.py -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r5_s2_tests.txt 2>&1 || exit $?
timeout -k 10 300 python -u -m financial_chatbot_llm_amd.bench.kernels --only lm_head_stream,lm_head_stream_shard \
  --out gpurun_out/r5_lm_head_stream_v2.jsonl > gpurun_out/r5_lm_head_stream_v2.log 2>&1 || exit $?
timeout -k 10 300 python -u -m financial_chatbot_llm_amd.bench.kernels --only shard_shapes_tp8 \
  --out gpurun_out/r5_shard_shapes_tp8_v2.jsonl > gpurun_out/r5_shard_shapes_tp8_v2.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r5_s2_bench.json 2> gpurun_out/r5_s2_bench.err || exit $?
