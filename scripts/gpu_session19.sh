#!/bin/bash
# GPU session 19: MFMA-busy of the prefill attention kernel (variant 4) on the workload's mixed steps.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVES SQ_INSTS_VALU SQ_INSTS_MFMA GRBM_GUI_ACTIVE --kernel-trace --output-format csv -d /tmp/pa -o run -- python3 -m financial_chatbot_llm_amd.bench.kernels --only prefill_mixed > gpurun_out/pa_pmc.log 2>&1
rc=$?
find /tmp/pa -name '*counter_collection.csv' -exec cp {} gpurun_out/pa_counters.csv \;
tail -2 gpurun_out/pa_pmc.log | cut -c1-200
exit $rc
