"""C4 (TP step broadcast) latency microbench on CPU: gloo vs the shared-memory ring.

    python -m financial_chatbot_llm_amd.bench.c4_latency --world 8 --msgs 300

World-size ``--world`` processes form one gloo TP group (ranks on one host, as a TP group on an
MI355X node is).  The leader publishes ``--msgs`` packed step payloads per size -- 4 KB (a decode
step's ids / positions / slots / block tables at B = 128), 64 KB and 512 KB (prefill steps) --
pacing them ``--gap-ms`` apart like the engine's step cadence, and every follower stamps the
arrival (CLOCK_MONOTONIC, comparable across processes).  Latency of a message = the LAST
follower's arrival - the leader's send start; p50 / p99 / max per channel and size, one JSON line
each (the leader's ``broadcast_step`` path: gloo = header + payload broadcasts, ring =
``parallel.step_ring.StepChannel``).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import time

import numpy as np


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, args, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), OMP_NUM_THREADS="1")
    import torch
    import torch.distributed as dist
    torch.set_num_threads(1)
    from financial_chatbot_llm_amd.parallel.dist import init_distributed, shutdown, state
    from financial_chatbot_llm_amd.parallel.step_ring import StepChannel
    init_distributed(tp_size=world, backend="gloo", device_type="cpu")
    s = state()
    group = s.tp_cpu_group if s.tp_cpu_group is not None else s.tp_group
    leader = s.tp_leader_rank
    followers = [r for r in range(world) if r != leader]
    ch = StepChannel(group, leader, rank == leader, followers.index(rank) if rank != leader else 0, len(followers),
                     nslots=8, slot_bytes=1 << 20)

    def gloo_send(p):
        head = torch.tensor([p.size], dtype=torch.int64)
        dist.broadcast(head, src=leader, group=group)
        dist.broadcast(torch.from_numpy(p), src=leader, group=group)

    def gloo_recv():
        head = torch.zeros(1, dtype=torch.int64)
        dist.broadcast(head, src=leader, group=group)
        buf = torch.empty(int(head[0]), dtype=torch.uint8)
        dist.broadcast(buf, src=leader, group=group)
        return buf.numpy()

    out = []
    for size in (4 << 10, 64 << 10, 512 << 10):
        payload = np.random.default_rng(size).integers(0, 256, size, dtype=np.uint8)
        for chan in ("gloo", "ring"):
            stamps = np.zeros(args.msgs, np.int64)
            dist.barrier(group=group)
            for i in range(args.msgs):
                if rank == leader:
                    time.sleep(args.gap_ms * 1e-3)
                    stamps[i] = time.monotonic_ns()
                    gloo_send(payload) if chan == "gloo" else ch.send(payload)
                else:
                    got = gloo_recv() if chan == "gloo" else ch.recv()
                    stamps[i] = time.monotonic_ns()
                    assert got.size == size
            t = torch.from_numpy(stamps)
            parts = [torch.empty_like(t) for _ in range(world)]
            dist.all_gather(parts, t, group=group)
            if rank == leader:
                arr = torch.stack(parts).numpy()
                lat = (np.delete(arr, leader, 0).max(0) - arr[leader]) / 1e3      # us
                out.append({"op": "c4_latency", "channel": chan, "world": world, "bytes": size, "msgs": args.msgs,
                            "p50_us": round(float(np.percentile(lat, 50)), 1),
                            "p99_us": round(float(np.percentile(lat, 99)), 1),
                            "max_us": round(float(lat.max()), 1)})
    if rank == leader:
        ch.send(None)
    else:
        assert ch.recv() is None
    q.put(out)
    shutdown()


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--msgs", type=int, default=300)
    ap.add_argument("--gap-ms", type=float, default=2.0)
    args = ap.parse_args(argv)
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, args.world, port, args, q)) for r in range(args.world)]
    for p in procs:
        p.start()
    rows = []
    for _ in range(args.world):
        rows += q.get(timeout=900)
    for p in procs:
        p.join(timeout=60)
    for r in rows:
        print(json.dumps(r), flush=True)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
