#!/bin/bash
# r5 session 44 (final HEAD: + step-row quantisation from any chunk): the whole GPU suite + smoke(), the driver bench twice
# (run-to-run spread), then the dp2 rehearsal of the driver's multi-GPU launch on one GPU.
set -u
mkdir -p gpurun_out
export TMPDIR=/tmp PYTHONUNBUFFERED=1
stop_if_bad() { case "$1" in 124|134|137|139) echo "stopping after rc=$1"; exit "$1";; esac; }
timeout -k 10 900 python3 -u -m pytest -q --timeout 600 --timeout-method thread -m gpu tests/ \
    > gpurun_out/r5_s44_gpu_suite.txt 2>&1
rc=$?; echo "pytest rc=$rc" >> gpurun_out/r5_s44_gpu_suite.txt; stop_if_bad $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5_s44_smoke.txt 2>&1
rc=$?; stop_if_bad $rc
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 > gpurun_out/r5_s44_bench1.json 2> gpurun_out/r5_s44_bench1.err
rc=$?; stop_if_bad $rc
timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 > gpurun_out/r5_s44_bench2.json 2> gpurun_out/r5_s44_bench2.err
rc=$?; stop_if_bad $rc
PENNY_DIST_BACKEND=gloo PENNY_KV_FRACTION=0.4 timeout -k 10 600 python3 -m torch.distributed.run --nnodes 1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 5 --warmup 2 \
    > gpurun_out/r5_s44_dp2.json 2> gpurun_out/r5_s44_dp2.err
