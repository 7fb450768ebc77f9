"""TP decode all-reduce exposure microbench.

``world`` ranks (default 8, all on cuda:0 on a one-GPU box -- the custom xGMI all-reduce runs over
IPC-mapped peer buffers exactly as across GPUs) each hold the Llama-3-70B TP=8 shard of ``layers``
decoder layers and replay hipGraph-captured decode steps of B rows (ctx tokens each) four ways:

* ``single``       one chain, every row-parallel all-reduce inline (``DecoderModel.forward``)
* ``dual``         two micro-batch chains on two streams, own custom-AR channel each
                   (``forward_decode_dual``): one chain's all-reduce hides under the other's compute
* ``*_noar``       the same graphs with ``comm.tp_all_reduce`` replaced by the identity -- the
                   compute-only floor

AR-exposed time per layer = (mode - mode_noar) / layers.  Per mode each rank times ``iters`` graph
replays between a gloo barrier + device sync; the slowest rank is reported.  On one GPU the 8 ranks
time-share the CUs, so a rank's all-reduce also waits for the other ranks' compute: the absolute
numbers are an upper bound for the 8-GPU node; the single-vs-dual difference is what the overlap
buys.  Rank 0 prints one JSON line per mode.

    python -m financial_chatbot_llm_amd.bench.tp_decode_overlap --world 8 --layers 4 --batch 64
"""
from __future__ import annotations

import argparse
import dataclasses
import json
import os
import socket
import sys
import time


def _free_port() -> int:
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank: int, world: int, port: int, args, q) -> None:
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    try:
        import torch
        import torch.distributed as dist

        from financial_chatbot_llm_amd.models.common import AttentionMetadata, KVCache
        from financial_chatbot_llm_amd.models.configs import get_model_config
        from financial_chatbot_llm_amd.models.llama import LlamaModel
        from financial_chatbot_llm_amd.ops.attention import KV_BS, DecodeWorkspace
        from financial_chatbot_llm_amd.parallel import comm
        from financial_chatbot_llm_amd.parallel.dist import init_distributed, shutdown, state

        torch.cuda.set_device(0 if args.one_gpu else rank)
        dev = torch.device("cuda", torch.cuda.current_device())
        init_distributed(tp_size=world, backend="gloo", device_type="cuda")
        comm.enable_custom_all_reduce()
        comm.enable_second_channel()
        base = get_model_config(args.model)
        cfg = dataclasses.replace(base, name=base.name + f"-{args.layers}l", num_layers=args.layers)
        m = LlamaModel(cfg, device=dev, tp_rank=rank, tp_size=world).init_random(seed=7, std=0.02)
        B, ctx = args.batch, args.ctx
        nbs = -(-ctx // KV_BS)
        kv = KVCache(cfg.num_layers, B * nbs + 1, m.hkv, m.D, device=dev)
        bt = (torch.arange(B * nbs, dtype=torch.int32, device=dev).view(B, nbs) + 1).contiguous()
        ctx_lens = torch.full((B,), ctx, dtype=torch.int32, device=dev)
        pos = ctx_lens - 1
        slots = (bt[:, -1] * KV_BS + (ctx - 1) % KV_BS).to(torch.int32)
        ids = torch.randint(100, 30000, (B,), dtype=torch.int32, device=dev)
        ws1 = DecodeWorkspace.create(B, m.hq, m.D, ctx + 64, dev)
        ws2 = DecodeWorkspace.create(B, m.hq, m.D, ctx + 64, dev)
        k = B // 2

        def run_single():
            meta = AttentionMetadata(slots=slots, num_prefill_tokens=0, num_decode=B, ctx_lens_d=ctx_lens,
                                     block_tables_d=bt, decode_ws=ws1)
            return m.forward(ids, pos, meta, kv)

        def run_dual():
            metas = [AttentionMetadata(slots=slots[a:b], num_prefill_tokens=0, num_decode=b - a,
                                       ctx_lens_d=ctx_lens[a:b], block_tables_d=bt[a:b], decode_ws=ws)
                     for (a, b), ws in (((0, k), ws1), ((k, B), ws2))]
            return m.forward_decode_dual(ids, pos, metas, k, kv)

        real_ar = comm.tp_all_reduce
        pool = torch.cuda.graph_pool_handle()
        graphs = {}
        with torch.no_grad():
            for noar in (False, True):
                comm.tp_all_reduce = (lambda x: x) if noar else real_ar
                for name, fn in (("single", run_single), ("dual", run_dual)):
                    fn()
                    torch.cuda.synchronize()
                    g = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g, pool=pool):
                        fn()
                    graphs[name + ("_noar" if noar else "")] = g
            comm.tp_all_reduce = real_ar
        grp = state().tp_cpu_group if hasattr(state(), "tp_cpu_group") else None
        res = {}
        for name in ("single", "dual", "single_noar", "dual_noar", "single", "dual"):
            g = graphs[name]
            for _ in range(args.warmup):
                g.replay()
            torch.cuda.synchronize()
            dist.barrier(group=grp)
            t0 = time.perf_counter()
            for _ in range(args.iters):
                g.replay()
            torch.cuda.synchronize()
            dt = (time.perf_counter() - t0) / args.iters * 1e3
            res[name] = min(res.get(name, 1e30), dt)     # each AR mode timed twice, best of two
        q.put((rank, "OK", res))
        shutdown()
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, "ERR", traceback.format_exc()))


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--model", default="llama3-70b")
    ap.add_argument("--layers", type=int, default=4)
    ap.add_argument("--batch", type=int, default=64)
    ap.add_argument("--ctx", type=int, default=1024)
    ap.add_argument("--iters", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--one-gpu", action="store_true", default=True,
                    help="all ranks on cuda:0 (the one-GPU rehearsal; default)")
    ap.add_argument("--out", default=None, help="append the JSON lines to this file")
    args = ap.parse_args(argv)
    import torch.multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, args.world, port, args, q)) for r in range(args.world)]
    for p in procs:
        p.start()
    res = {}
    try:
        for _ in range(args.world):
            r, status, payload = q.get(timeout=900)
            res[r] = (status, payload)
    finally:
        for p in procs:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    bad = [(r, p) for r, (s, p) in res.items() if s != "OK"]
    if bad:
        print(bad[0][1], file=sys.stderr)
        return 1
    worst = {k: max(p[k] for _, p in res.values()) for k in res[0][1]}
    L = args.layers
    rows = []
    for mode in ("single", "dual"):
        rows.append({"bench": "tp_decode_overlap", "mode": mode, "world": args.world, "model": args.model,
                     "layers": L, "batch": args.batch, "ctx": args.ctx, "ms_per_step": round(worst[mode], 3),
                     "ms_per_step_noar": round(worst[mode + "_noar"], 3),
                     "ar_exposed_us_per_layer": round((worst[mode] - worst[mode + "_noar"]) / L * 1e3, 1),
                     "one_gpu_timeshared": bool(args.one_gpu)})
    for r in rows:
        print(json.dumps(r))
    if args.out:
        with open(args.out, "a") as f:
            for r in rows:
                f.write(json.dumps(r) + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
