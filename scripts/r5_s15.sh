#!/bin/bash
# r5 session 15: config 4's TP=8 process model rehearsed on ONE MI355X (8 ranks time-sharing the card,
# real 70B shard shapes: split-K gate|up, bf16-out O/down shards, streaming shard LM head, custom-AR
# self-test at init), then Llama-3-70B TP=1 under rocprofv3 (6/2, 64 convs) for the kernel breakdown.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
stop_if_bad() { case "$1" in 124|134|137|139) echo "stopping after rc=$1"; exit "$1";; esac; }
PENNY_DIST_BACKEND=gloo PENNY_KV_FRACTION=0.02 timeout -k 10 420 python3 -m torch.distributed.run --nnodes 1 \
     --nproc-per-node 8 --master-addr 127.0.0.1 --master-port 29517 bench.py --gpus 8 --tp 8 --model llama3-70b \
     --tool-steps 3 --convs 4 --steps 1 --warmup 1 --respond-tokens 16 --max-batched-tokens 256 --corpus 100000 \
     --users 100 > gpurun_out/r5_s15_tp8_rehearsal.json 2> gpurun_out/r5_s15_tp8_rehearsal.err
rc=$?; stop_if_bad $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/prof70 -o run -- \
    python3 bench.py --model llama3-70b --tool-steps 3 --convs 64 --steps 6 --warmup 2 \
    > gpurun_out/r5_s15_70b_prof.json 2> gpurun_out/r5_s15_70b_prof.err
rc=$?; stop_if_bad $rc
st=$(find /tmp/prof70 -name '*kernel_stats.csv' | head -1); tr=$(find /tmp/prof70 -name '*kernel_trace.csv' | head -1)
python3 -m financial_chatbot_llm_amd.bench.profsum "$st" --trace "$tr" --title "r5 HEAD: Llama-3-70B TP=1, --tool-steps 3, 64 convs, 6/2, under rocprofv3" > gpurun_out/r5_s15_70b_kernel_stats.md 2>&1
rm -rf /tmp/prof70
