#!/bin/bash
# r5 session 4: tile-GEMM stall anatomy by PMC (measure the limiter first), the
# final-HEAD kernel breakdown + GPU-busy union of the driver config under rocprofv3, then the driver
# bench unprofiled.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
stop_if_bad() { case "$1" in 124|134|137|139) echo "stopping after rc=$1"; exit "$1";; esac; }
timeout -s KILL 60 rocprofv3 -L > gpurun_out/r5_counters_list.txt 2>&1; stop_if_bad $?
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE"
P2="SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_INSTS_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P --kernel-trace --output-format csv -d /tmp/gp$i -o run -- \
    python3 -m financial_chatbot_llm_amd.bench.kernels --only gemm_lds_probe > gpurun_out/r5_gemm_pmc$i.log 2>&1
  rc=$?; stop_if_bad $rc
  find /tmp/gp$i -name '*counter_collection.csv' -exec cp {} gpurun_out/r5_gemm_pmc$i.csv \;
done
timeout -k 10 480 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof -o run -- \
    python3 bench.py --steps 20 --warmup 5 > gpurun_out/r5_prof_bench.json 2> gpurun_out/r5_prof_bench.err
rc=$?; stop_if_bad $rc
st=$(find /tmp/prof -name '*kernel_stats.csv' | head -1); tr=$(find /tmp/prof -name '*kernel_trace.csv' | head -1)
cp "$st" gpurun_out/r5_prof_kernel_stats.csv
python3 -m financial_chatbot_llm_amd.bench.profsum "$st" --trace "$tr" --title "r5 driver bench 20x5 at HEAD (prefill attention variant 5, streaming LM head)" > gpurun_out/r5_prof_kernel_stats.md 2>&1
rm -rf /tmp/prof
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 > gpurun_out/r5_s4_bench.json 2> gpurun_out/r5_s4_bench.err
stop_if_bad $?
