#!/bin/bash
# r5 session 11: the whole GPU suite at HEAD (after the fused-merge revert and the host trims), then the
# Llama-3-70B prefill projection policy measured with each GEMM's consumer (incl. the residual epilogue).
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
stop_if_bad() { case "$1" in 124|134|137|139) echo "stopping after rc=$1"; exit "$1";; esac; }
timeout -k 10 900 python3 -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/ \
    > gpurun_out/r5_s11_gpu_suite.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r5_s11_gpu_suite.txt; stop_if_bad $rc
timeout -k 10 400 python3 -u -m financial_chatbot_llm_amd.bench.kernels --only prefill_policy_70b > gpurun_out/r5_s11_prefill_policy_70b.jsonl 2> gpurun_out/r5_s11_prefill_policy_70b.err
