#!/bin/bash
# r5 session 17: prefill attention as two 4-wave workgroups per CU (variant 8) vs the 8-wave kernel.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
stop_if_bad() { case "$1" in 124|134|137|139) echo "stopping after rc=$1"; exit "$1";; esac; }
timeout -k 10 300 python3 -u -m financial_chatbot_llm_amd.bench.kernels --only prefill_nw4 > gpurun_out/r5_s17_prefill_nw4.jsonl 2> gpurun_out/r5_s17_prefill_nw4.err
