#!/bin/bash
# GPU session 5: the driver bench at HEAD (prefill attention variant 4), its rocprofv3 kernel
# breakdown, the TTFT-tail reservation A/B, and Mixtral fp8 (config 5) with the MX hand-off.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
step() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  echo "[$(date +%T)] $name" | tee -a gpurun_out/session5.log
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" | tee -a gpurun_out/session5.log
  tail -2 "gpurun_out/$name.log"
  return $rc
}
step b8_head 360 python -u bench.py --steps 20 --warmup 5 || exit 1
step b8_res512 360 env PENNY_SHORT_RESERVE=512 python -u bench.py --steps 20 --warmup 5 || exit 1
step b_mixtral_mx 420 env PENNY_MOE_MX=${MOE_MX:-1} python -u bench.py --steps 20 --warmup 5 --model mixtral-8x7b --dtype fp8 || exit 1
step prof8 420 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof8 -o run -- \
     python3 bench.py --steps 20 --warmup 5 || exit 1
