#!/bin/bash
# GPU session 14: decode lean reduce with speculative partial loads -- numerics, then kernel stats
# of the decode_lean microbench with the new and the previous library.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
export PYTHONPATH=$PWD
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "decode or cascade" > gpurun_out/t_red.log 2>&1 || { tail -5 gpurun_out/t_red.log; exit 1; }
tail -1 gpurun_out/t_red.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/rn -o run -- python3 -m financial_chatbot_llm_amd.bench.kernels --only decode_lean > gpurun_out/red_new.log 2>&1 || exit 1
find /tmp/rn -name '*kernel_stats.csv' -exec cp {} gpurun_out/red_new_stats.csv \;
PENNY_KERNEL_LIB=$PWD/ab/libpenny_old.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/ro -o run -- python3 -m financial_chatbot_llm_amd.bench.kernels --only decode_lean > gpurun_out/red_old.log 2>&1 || exit 1
find /tmp/ro -name '*kernel_stats.csv' -exec cp {} gpurun_out/red_old_stats.csv \;
grep -h "decode_lean_reduce" gpurun_out/red_new_stats.csv gpurun_out/red_old_stats.csv | cut -c1-200
