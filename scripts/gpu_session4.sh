#!/bin/bash
# GPU session 4: the 8-rank-on-one-GPU TP rehearsals -- world-8 tests (dual-chain decode graphs,
# vocab-parallel sampling), the TP decode all-reduce exposure microbench, and the config-4 bench
# (llama3-70b TP=8, step ring + pipelined followers) for the leader/follower timing breakdown.
set -u
mkdir -p gpurun_out
step() {  # name, timeout, command...
  local name=$1 t=$2; shift 2
  echo "[$(date +%T)] $name" | tee -a gpurun_out/session4.log
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "[$(date +%T)] $name rc=$rc" | tee -a gpurun_out/session4.log
  tail -3 "gpurun_out/$name.log"
  return $rc
}
step t_world8 600 python -u -m pytest -x -q --timeout 500 --timeout-method thread tests/test_world8_gpu.py -k tp8 || exit 1
step b_tpov 300 python -u -m financial_chatbot_llm_amd.bench.tp_decode_overlap --world 8 --layers 4 --batch 64 --ctx 1024 \
     --out gpurun_out/tp_decode_overlap.jsonl || exit 1
step b_tp8 420 env PENNY_DIST_BACKEND=gloo PENNY_KV_FRACTION=0.02 python -m torch.distributed.run --nnodes 1 \
     --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 8 --tp 8 --model llama3-70b \
     --tool-steps 3 --convs 4 --steps 1 --warmup 1 --respond-tokens 16 --max-batched-tokens 256 --corpus 100000 \
     --users 100 || exit 1
