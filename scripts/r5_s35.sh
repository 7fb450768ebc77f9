#!/bin/bash
# r5 session 35: HBM bytes fetched by the lean decode kernel under each cache policy (rocprofv3
# FETCH_SIZE, one process per policy), B = 128 and B = 64 workload batches.
set -u
mkdir -p gpurun_out/r5_s35
export TMPDIR=/tmp PYTHONUNBUFFERED=1
for B in 128 64; do
  for F in 0 1; do
    PENNY_DECODE_LEAN_FLAGS=$F timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv \
        -d /tmp/pmc_${B}_${F} -o run -- python3 -m financial_chatbot_llm_amd.bench.lean_nt_pmc --b $B \
        > gpurun_out/r5_s35/run_${B}_${F}.json 2> gpurun_out/r5_s35/run_${B}_${F}.err || exit $?
    f=$(find /tmp/pmc_${B}_${F} -name '*counter_collection.csv' | head -1)
    cp "$f" gpurun_out/r5_s35/counters_${B}_${F}.csv
  done
done
