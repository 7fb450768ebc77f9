#!/bin/bash
# dp2 rehearsal of the driver's multi-GPU bench on ONE GPU: two ranks over gloo sharing the card
# (RCCL refuses two ranks on one device), each with half the KV pool.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 env PENNY_DIST_BACKEND=gloo PENNY_KV_FRACTION=0.4 python -m torch.distributed.run --nnodes 1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 \
    > gpurun_out/dp2.log 2>&1
rc=$?
grep '^{' gpurun_out/dp2.log | tail -1 | cut -c1-600
exit $rc
