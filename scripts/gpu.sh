#!/bin/bash
# One parameterised driver for every GPU session (replaces the per-session scripts of r1-r5).
# Run through gpurun; each step has its own time limit, steps chain with && semantics (the first
# failing step ends the call), output goes to gpurun_out/<tag>_<step>.log.
#
#   scripts/gpu.sh TAG step [step ...]
#
# steps (arguments after ':' are split on ','):
#   suite                   whole GPU test suite, one process
#   smoke                   __graft_entry__.smoke()
#   test:EXPR               pytest -m gpu -k EXPR
#   bench[:ARGS]            bench.py (driver config unless ARGS), JSON to gpurun_out/TAG_bench.json
#                           (the n-th bench step of a call: TAG_bench<n>.json)
#   prof[:ARGS]             bench.py under rocprofv3 --kernel-trace --stats -> TAG_prof_kernel_stats.md
#   kbench:ONLY             bench.kernels --only ONLY -> TAG_kbench.jsonl
#   kprof:ONLY              bench.kernels --only ONLY under rocprofv3 --kernel-trace --stats -> TAG_kprof_*
#   pmc:ONLY:C1+C2+...      bench.kernels --only ONLY under rocprofv3 --pmc (one pass) -> TAG_pmc.md
#   py:MODULE[,ARGS]        python -m MODULE ARGS
#   env:K=V[,K=V]           export for the following steps (e.g. env:PENNY_DIST_BACKEND=gloo,PENNY_KV_FRACTION=0.4
#                           then bench:--gpus,2 rehearses dp2 on one GPU: bench.py spawns its own ranks)
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
TAG=$1; shift

run() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  echo "[$(date +%T)] $TAG $name: $*"
  timeout -k 10 "$t" "$@" > "gpurun_out/${TAG}_${name}.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $TAG $name rc=$rc"
  tail -4 "gpurun_out/${TAG}_${name}.log"
  return $rc
}

for spec in "$@"; do
  kind=${spec%%:*}; rest=""; [ "$kind" != "$spec" ] && rest=${spec#*:}
  args=(${rest//,/ })
  case $kind in
    suite) run suite 1000 python -u -m pytest tests/ -x -q -m gpu --timeout 300 --timeout-method thread || exit $? ;;
    smoke) run smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit $? ;;
    test) run "test_${rest//[^a-zA-Z0-9]/_}" 600 python -u -m pytest tests/ -x -v -m gpu -k "$rest" --timeout 300 \
            --timeout-method thread || exit $? ;;
    bench) [ ${#args[@]} -eq 0 ] && args=(--steps 20 --warmup 5)
           NB=$(( ${NB:-0} + 1 )); bn=bench; [ "$NB" -gt 1 ] && bn=bench$NB    # A/B: bench, bench2, ...
           run $bn 900 python -u bench.py "${args[@]}" --json-out "gpurun_out/${TAG}_${bn}.json" || exit $? ;;
    prof) [ ${#args[@]} -eq 0 ] && args=(--steps 20 --warmup 5)
          rm -rf /tmp/prof_$TAG
          run prof 900 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof_$TAG -o run -- \
              python3 bench.py "${args[@]}" --json-out "gpurun_out/${TAG}_prof_bench.json" || exit $?
          st=$(find /tmp/prof_$TAG -name '*kernel_stats.csv' | head -1)
          tr=$(find /tmp/prof_$TAG -name '*kernel_trace.csv' | head -1)
          python3 -m financial_chatbot_llm_amd.bench.profsum "$st" --trace "$tr" --title "$TAG: bench ${args[*]}" \
              > "gpurun_out/${TAG}_prof_kernel_stats.md" 2>&1
          # PROF_KEEP=<regex>: keep the trace rows (grid sizes, timestamps) of the matching kernels
          [ -n "${PROF_KEEP:-}" ] && grep -E "Kernel_Name|${PROF_KEEP}" "$tr" > "gpurun_out/${TAG}_prof_kept_trace.csv"
          rm -rf /tmp/prof_$TAG ;;
    kbench) run "kbench_${rest//[^a-zA-Z0-9]/_}" 600 python -u -m financial_chatbot_llm_amd.bench.kernels --only "$rest" \
              --out "gpurun_out/${TAG}_kbench_${rest//[^a-zA-Z0-9]/_}.jsonl" || exit $? ;;
    kprof) rm -rf /tmp/kprof_$TAG
           run "kprof_${rest//[^a-zA-Z0-9]/_}" 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/kprof_$TAG \
               -o run -- python3 -m financial_chatbot_llm_amd.bench.kernels --only "$rest" || exit $?
           st=$(find /tmp/kprof_$TAG -name '*kernel_stats.csv' | head -1)
           tr=$(find /tmp/kprof_$TAG -name '*kernel_trace.csv' | head -1)
           cp "$tr" "gpurun_out/${TAG}_kprof_trace.csv"
           python3 -m financial_chatbot_llm_amd.bench.profsum "$st" --trace "$tr" --title "$TAG: kernels $rest" \
               > "gpurun_out/${TAG}_kprof_kernel_stats.md" 2>&1
           rm -rf /tmp/kprof_$TAG ;;
    pmc) only=${rest%%:*}; ctrs=${rest#*:}; ctrs=${ctrs//+/ }
         rm -rf /tmp/pmc_$TAG
         run "pmc_${only//[^a-zA-Z0-9]/_}" 240 rocprofv3 --pmc $ctrs --kernel-trace --output-format csv -d /tmp/pmc_$TAG \
             -o run -- python3 -m financial_chatbot_llm_amd.bench.kernels --only "$only" || exit $?
         ctr=$(find /tmp/pmc_$TAG -name '*counter_collection.csv' | head -1)
         cp "$ctr" "gpurun_out/${TAG}_pmc_counters.csv"
         python3 -m financial_chatbot_llm_amd.bench.pmc_mfma "gpurun_out/${TAG}_pmc_counters.csv" --md \
             > "gpurun_out/${TAG}_pmc.md" 2>&1
         rm -rf /tmp/pmc_$TAG ;;
    env) for kv in "${args[@]}"; do export "$kv"; done ;;
    py) run "py_${args[0]##*.}" 900 python -u -m "${args[@]}" || exit $? ;;
    *) echo "unknown step $spec"; exit 2 ;;
  esac
done
