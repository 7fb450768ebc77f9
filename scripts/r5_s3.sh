#!/bin/bash
# r5 session 3: GPU suite subset (kernels incl. the FOLD prefill variant 5 + its forced-rescale test,
# engine, TP world-8, custom AR), prefill-attention A/B on the workload's mixed steps, one PMC pass of
# the prefill kernels, the re-measured narrow-ring decode GEMMs and LM head, then the driver bench.
set -o pipefail
mkdir -p gpurun_out
export PYTHONUNBUFFERED=1 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests/test_kernels_gpu.py tests/test_custom_ar_gpu.py tests/test_world8_gpu.py \
  tests/test_tp_gpu.py tests/test_engine_gpu.py -x -v --timeout 300 --timeout-method thread \
  > gpurun_out/r5_s3_tests.txt 2>&1 || exit $?
timeout -k 10 300 python -u -m financial_chatbot_llm_amd.bench.kernels --only prefill_mixed \
  --out gpurun_out/r5_prefill_fold_ab.jsonl > gpurun_out/r5_prefill_fold_ab.log 2>&1 || exit $?
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA GRBM_GUI_ACTIVE \
  --kernel-trace --output-format csv -d /tmp/pa -o run -- python3 -m financial_chatbot_llm_amd.bench.kernels --only prefill_mixed \
  > gpurun_out/r5_pa_pmc.log 2>&1 || exit $?
find /tmp/pa -name '*counter_collection.csv' -exec cp {} gpurun_out/r5_pa_counters.csv \;
python -m financial_chatbot_llm_amd.bench.pmc_mfma gpurun_out/r5_pa_counters.csv --match prefill --md > gpurun_out/r5_pa_pmc.md 2>&1
timeout -k 10 300 python -u -m financial_chatbot_llm_amd.bench.kernels --only lm_head_stream,lm_head_stream_shard,shard_shapes_tp8 \
  --out gpurun_out/r5_decode_v2.jsonl > gpurun_out/r5_decode_v2.log 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r5_s3_bench.json 2> gpurun_out/r5_s3_bench.err || exit $?
