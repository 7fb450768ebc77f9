#!/usr/bin/env bash
# Launch the serving stack on one node: PENNY_NPROC ranks (one per GPU) via torchrun.
#   PENNY_NPROC=8 PENNY_TP=1 -> 8 x Llama-3-8B DP replicas (north-star configs 2/3)
#   PENNY_NPROC=8 PENNY_TP=8 PENNY_MODEL=llama3-70b TOOL_STEPS=3 -> one 70B TP=8 group (config 4)
#   PENNY_NPROC=8 PENNY_TP=1 PENNY_MODEL=mixtral-8x7b PENNY_DTYPE=fp8 -> 8 fp8 MoE replicas (config 5)
# Env (see financial_chatbot_llm_amd/config.py): KAFKA_SERVER / KAFKA_USERNAME / KAFKA_PASSWORD,
# MONGODB_URI, PORT (replica r serves PORT + r), LOG_LEVEL, PENNY_* engine knobs (the xGMI one-shot
# all-reduce is on by default under TP; PENNY_CUSTOM_AR=0 forces RCCL), PENNY_CORPUS_PATH (a collection
# snapshot directory or JSONL/Parquet transactions to ingest), PENNY_EMBED_WEIGHTS / PENNY_EMBED_VOCAB
# (bge safetensors + vocab.txt), PENNY_TOOLS=0 (legacy no-tools chat, llm_service.py).
set -euo pipefail
NPROC="${PENNY_NPROC:-1}"
TP="${PENNY_TP:-1}"
exec torchrun --nnodes=1 --nproc-per-node "$NPROC" --master-addr 127.0.0.1 --master-port "${MASTER_PORT:-29500}" \
  -m financial_chatbot_llm_amd.serving.launch --tp "$TP" --model "${PENNY_MODEL:-llama3-8b}" \
  --tool-steps "${TOOL_STEPS:-1}" --port "${PORT:-8000}" --corpus "${PENNY_CORPUS_SIZE:-0}" \
  --corpus-path "${PENNY_CORPUS_PATH:-}"
