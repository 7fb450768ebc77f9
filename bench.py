#!/usr/bin/env python3
"""Headline benchmark: chat turns/sec + p50 TTFT, Llama-3-8B RAG agent on 1/2/4/8 MI355X.

Metric/config from BASELINE.json.  Each GPU runs one engine replica (data parallel, one process
per GPU over torch.distributed/RCCL, launched by torchrun) serving its own closed-loop population
of ``--convs`` synthetic conversations through the FULL serving path (Kafka-fake ingest ->
agent decide [Llama-3-8B] -> retrieval [bge-base-en + 1M-vector filtered top-k] -> streamed
respond [Llama-3-8B] -> Kafka-fake egress + Mongo-fake save).  Weights are random-init bf16 of
the real architectures; data are synthetic (no network).

One step = one wave of ``--convs`` concurrent turns per GPU (weak scaling: per-GPU work fixed).
``value`` = whole-job completed turns / max-over-ranks wall time of the K timed waves.

    python bench.py --gpus 1 --steps 3 --warmup 1
    python bench.py --gpus 8 --steps 3 --warmup 1      # spawns its own 8 ranks (torch.distributed.run child)
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 bench.py --gpus 8 --steps 3 --warmup 1

``--gpus N`` must equal the launcher's WORLD_SIZE (non-zero exit otherwise).
"""
from __future__ import annotations

import argparse
import asyncio
import json
import os
import statistics
import sys
import time

METRIC = "chat turns/sec + p50 TTFT, Llama-3-8B RAG agent at 1/2/4/8 MI355X"


MODEL_LABELS = {"llama3-8b": "Llama-3-8B", "llama3.1-8b": "Llama-3.1-8B", "llama3-70b": "Llama-3-70B",
                "mixtral-8x7b": "Mixtral-8x7B"}


def log(msg: str) -> None:
    print(f"[bench r{os.environ.get('RANK', '0')} {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--tp", type=int, default=1,
                    help="tensor-parallel degree per replica (config 4: --model llama3-70b --tp 8 --tool-steps 3); "
                         "WORLD_SIZE / tp replicas, each TP leader serves --convs conversations, the other ranks "
                         "replay its steps")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--convs", type=int, default=128, help="concurrent conversations per GPU")
    ap.add_argument("--respond-tokens", type=int, default=128)
    ap.add_argument("--model", default="llama3-8b")
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp8"],
                    help="fp8: Mixtral experts as e4m3 on the fp8 MFMA path (attention/dense stay bf16)")
    ap.add_argument("--embed-model", default="bge-base-en")
    ap.add_argument("--corpus", type=int, default=1_000_000)
    ap.add_argument("--users", type=int, default=10_000)
    ap.add_argument("--max-model-len", type=int, default=8192)
    ap.add_argument("--max-batched-tokens", type=int, default=None,
                    help="per-step token budget; default 4096 for dense models (beats 3072-16384 by 2-4 %% "
                         "turns/s, profiles/r1_sweep_max_batched_tokens.txt), 16384 for MoE (bigger chunks give "
                         "every expert more rows: 20.8 vs 19.1 turns/s, profiles/r1_bench_mixtral8x7b_fp8_v12.txt)")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--tool-steps", type=int, default=1,
                    help=">1: multi-step agent with the plot tool bound (north-star config 4)")
    ap.add_argument("--no-tools", action="store_true",
                    help="BASELINE config 2: single-turn chat without tools (legacy llm_service.py chain); "
                         "no decide step, no retrieval")
    ap.add_argument("--decide-always-limit", action="store_true",
                    help="scripted decide always sends num_transactions=20 (round-2 workload); default follows "
                         "the reference few-shot: time-window queries send no limit (10000 -> token clamp)")
    ap.add_argument("--no-jump-forward", action="store_true",
                    help="decode grammar-forced tool-call tokens one step each (A/B of jump-forward decoding)")
    ap.add_argument("--arrival", default="closed", choices=["closed", "wave"],
                    help="closed: each conversation sends its next turn when its last completes (default); "
                         "wave: all conversations send in lock-step waves")
    ap.add_argument("--engine", default="thread", choices=["process", "thread"],
                    help="thread: in-process AsyncEngine (default); process: the engine step loop runs in a "
                         "child process (engine core) so its host work never shares the serving GIL.  Measured "
                         "equal turns/s here (the GPU is already never idle between steps, "
                         "PENNY_STEP_GPU_TIMING=1), ~60 ms higher p50 TTFT from the IPC hop")
    ap.add_argument("--device", default="cuda", choices=["cuda", "cpu"],
                    help="cpu: contract tests of the bench itself with tiny models (gloo for >1 rank)")
    ap.add_argument("--tp-shard-estimate", type=int, default=0, metavar="N",
                    help="estimate a TP=N replica on ONE GPU (VERDICT r5 item 6): the engine runs rank 0's shard "
                         "(1/N of heads, FFN, vocab) with its collectives stubbed to identity, and the JSON adds "
                         "the step's all-reduce volume priced at stated xGMI rates -- a projection, never a "
                         "multi-GPU measurement")
    ap.add_argument("--json-out", default="")
    return ap.parse_args(argv)


async def run(args, ps):
    import torch

    from financial_chatbot_llm_amd.bench.workload import RagWorkload, decide_script
    from financial_chatbot_llm_amd.config import EngineConfig
    from financial_chatbot_llm_amd.engine.async_engine import AsyncEngine
    from financial_chatbot_llm_amd.engine.backend import EngineLLM
    from financial_chatbot_llm_amd.parallel.dist import barrier as world_barrier

    def barrier() -> None:
        """Timing barrier of the replicas: the TP leaders only (followers sit in their step loop)."""
        if args.tp == 1:
            world_barrier()
        elif ps.dp_group is not None:
            import torch.distributed as dist
            if ps.backend == "nccl":
                dist.barrier(group=ps.dp_group, device_ids=[torch.cuda.current_device()])
            else:
                dist.barrier(group=ps.dp_group)
    from financial_chatbot_llm_amd.retrieval import BgeEmbedder, DeviceVectorStore, RetrievalService

    on_gpu = args.device == "cuda"
    dev = torch.device("cuda", torch.cuda.current_device()) if on_gpu else torch.device("cpu")
    sizes = tuple(s for s in (1, 2, 4, 8, 16, 24, 32, 48, 64, 96, 128, 192, 256) if s <= max(2 * args.convs, 1))
    ecfg = EngineConfig(model=args.model, max_num_seqs=max(sizes), max_num_batched_tokens=args.max_batched_tokens,
                        max_model_len=args.max_model_len, use_cuda_graph=not args.no_graph,
                        graph_batch_sizes=sizes, seed=0, device=args.device, dtype=args.dtype, tp_size=args.tp,
                        shard_of_tp=args.tp_shard_estimate,
                        # PENNY_KV_FRACTION: several ranks sharing one GPU (gloo rehearsal of dpN) split its HBM
                        kv_mem_fraction=float(os.environ.get("PENNY_KV_FRACTION", EngineConfig.kv_mem_fraction)),
                        sched_aging_s=float(os.environ.get("PENNY_SCHED_AGING_S", EngineConfig.sched_aging_s)),
                        step_time_target_ms=float(os.environ.get("PENNY_STEP_TIME_TARGET_MS",
                                                                 EngineConfig.step_time_target_ms)),
                        sched_burst_tokens=int(os.environ.get("PENNY_BURST_TOKENS", EngineConfig.sched_burst_tokens)),
                        sched_burst_age_s=float(os.environ.get("PENNY_BURST_AGE_S", EngineConfig.sched_burst_age_s)),
                        sched_sjf_tokens=int(os.environ.get("PENNY_SJF_TOKENS", EngineConfig.sched_sjf_tokens)),
                        sched_sjf_step_cap=int(os.environ.get("PENNY_SJF_STEP_CAP", EngineConfig.sched_sjf_step_cap)),
                        sched_short_reserve_tokens=int(os.environ.get("PENNY_SHORT_RESERVE",
                                                                      EngineConfig.sched_short_reserve_tokens)),
                        sched_short_first=os.environ.get("PENNY_SHORT_FIRST",
                                                         str(int(EngineConfig.sched_short_first))) == "1")
    if args.tp > 1 and not ps.is_tp_leader:
        # TP follower: the same engine shard, warmed up (graph capture) in lockstep with its leader,
        # then replays every step the leader broadcasts until the leader's engine shuts down
        import resource
        from financial_chatbot_llm_amd.engine.llm_engine import LLMEngine
        from financial_chatbot_llm_amd.parallel import comm
        eng = LLMEngine(ecfg)
        eng.warmup()
        ru0, t0 = resource.getrusage(resource.RUSAGE_SELF), time.perf_counter()
        eng.follower_loop()
        ru1, el = resource.getrusage(resource.RUSAGE_SELF), time.perf_counter() - t0
        cpu_s = (ru1.ru_utime - ru0.ru_utime) + (ru1.ru_stime - ru0.ru_stime)
        st = eng.stats()
        return {"follower": True, "host": {"rank": ps.rank, "follower": True, "cpu_s": round(cpu_s, 2),
                                           "cpu_util": round(cpu_s / max(el, 1e-9), 2),
                                           "gpu_step_s": st.get("gpu_step_s", 0.0),
                                           "gpu_idle_between_steps_s": st.get("gpu_idle_between_steps_s", 0.0),
                                           "custom_all_reduce": dict(comm.AR_STATUS)}}

    def sync() -> None:
        if on_gpu:
            torch.cuda.synchronize()
    t0 = time.perf_counter()
    embedder = BgeEmbedder(args.embed_model, device=str(dev), seed=ps.rank)
    store = DeviceVectorStore(embedder.dim, device=str(dev))
    store.load_synthetic(args.corpus, args.users, seed=ps.rank)
    retrieval = RetrievalService(embedder, store)
    log(f"retrieval ready ({args.corpus} vectors) in {time.perf_counter() - t0:.1f}s")

    if args.tp > 1:     # leader of a TP group: its followers warm up (capture graphs) alongside it
        from financial_chatbot_llm_amd.engine.llm_engine import LLMEngine
        core = LLMEngine(ecfg)
        core.warmup()
        engine = AsyncEngine(engine=core, warmup=False)
    elif args.engine == "process":   # engine core in its own interpreter: no GIL shared with serving
        from financial_chatbot_llm_amd.engine.process_engine import ProcessAsyncEngine
        engine = ProcessAsyncEngine(ecfg, device_index=torch.cuda.current_device() if on_gpu else None)
    else:
        engine = AsyncEngine(ecfg)
    log(f"engine ready in {time.perf_counter() - t0:.1f}s")
    llm = EngineLLM(engine, max_model_len=args.max_model_len, decide_script=decide_script,
                    respond_ignore_eos=True, respond_tokens=args.respond_tokens,
                    jump_forward=not args.no_jump_forward)
    wl = RagWorkload(llm, retrieval, args.convs, args.users, args.respond_tokens, rank=ps.rank,
                     max_tool_steps=args.tool_steps, tools=not args.no_tools)
    wl.progress = log
    wl.kafka.setup_consumer()
    consumer = asyncio.create_task(wl.worker.consume_messages())

    # a "step" = every conversation completes one more turn (W untimed, then K timed)
    if args.warmup:
        if args.arrival == "closed":
            r = await wl.run_closed_loop(args.warmup)
        else:
            for _ in range(args.warmup):
                r = await wl.run_wave()
        log(f"warmup ({args.warmup} turns/conv): {r.seconds:.2f}s turns={r.turns} errors={r.errors}")

    sync()
    barrier()
    tok0 = {p: dict(v) for p, v in llm.token_stats.items()}
    for lat in llm.latency.values():      # engine latency anatomy of the timed turns only
        for v in lat.values():
            v.clear()
    stats0 = engine.stats()
    prof = None
    if os.environ.get("PENNY_PYPROFILE"):   # host-side cProfile of the serving event loop
        import cProfile
        prof = cProfile.Profile()
        prof.enable()
    import resource
    ru0 = resource.getrusage(resource.RUSAGE_SELF)
    ruc0 = resource.getrusage(resource.RUSAGE_CHILDREN)
    t_start = time.perf_counter()
    results = []
    if args.arrival == "closed":
        r = await wl.run_closed_loop(args.steps)
        results.append(r)
        log(f"{args.steps} turns/conv closed-loop: {r.seconds:.2f}s turns={r.turns} errors={r.errors} "
            f"retrievals={r.retrievals} ttft_p50={1e3 * statistics.median(r.ttfts) if r.ttfts else float('nan'):.0f}ms")
    else:
        for k in range(args.steps):
            r = await wl.run_wave()
            results.append(r)
            log(f"wave {k}: {r.seconds:.2f}s turns={r.turns} errors={r.errors} retrievals={r.retrievals} "
                f"ttft_p50={1e3 * statistics.median(r.ttfts) if r.ttfts else float('nan'):.0f}ms")
    sync()
    barrier()
    elapsed = time.perf_counter() - t_start
    ru1 = resource.getrusage(resource.RUSAGE_SELF)
    ruc1 = resource.getrusage(resource.RUSAGE_CHILDREN)
    cpu_s = (ru1.ru_utime - ru0.ru_utime) + (ru1.ru_stime - ru0.ru_stime)
    cpu_child_s = (ruc1.ru_utime - ruc0.ru_utime) + (ruc1.ru_stime - ruc0.ru_stime)
    if prof is not None:
        prof.disable()
        os.makedirs(os.environ["PENNY_PYPROFILE"], exist_ok=True)
        prof.dump_stats(os.path.join(os.environ["PENNY_PYPROFILE"], f"loop_r{ps.rank}.prof"))
    wl.worker.stop()
    await consumer
    stats = engine.stats()
    engine.shutdown()
    turns = sum(r.turns for r in results)
    # prompt-token accounting of the timed turns (account for every prefill token)
    tokens = {}
    for p, v in llm.token_stats.items():
        d = {k: v[k] - tok0.get(p, {}).get(k, 0) for k in v}
        tokens[p] = {"calls": d["calls"], "prompt_per_turn": round(d["prompt"] / max(turns, 1), 1),
                     "prefilled_per_turn": round(d["prefilled"] / max(turns, 1), 1),
                     "cached_fraction": round(1 - d["prefilled"] / max(d["prompt"], 1), 3)}
    tokens["prefilled_per_turn"] = round(sum(t["prefilled_per_turn"] for t in tokens.values()), 1)
    tokens["kv_evictions"] = stats.get("kv_evictions", 0) - stats0.get("kv_evictions", 0)
    tokens["preemptions"] = stats.get("preemptions", 0) - stats0.get("preemptions", 0)
    stages = {k: [v for r in results for v in r.stages.get(k, [])] for k in ("decide", "retrieval", "respond_first_token")}

    def pct(v, q):
        v = sorted(v)
        return round(1e3 * v[min(len(v) - 1, int(q * len(v)))], 1) if v else None
    latency = {p: {k: {"p50": pct(v, 0.5), "p99": pct(v, 0.99)} for k, v in lat.items()}
               for p, lat in llm.latency.items()}
    # the host budget of this rank (N engine processes share one host in the dpN
    # run) and where the GPU's non-busy time went: device step time vs wall, idle between steps
    from financial_chatbot_llm_amd.parallel import comm
    nturns = max(sum(r.turns for r in results), 1)
    gpu_step = stats.get("gpu_step_s", 0.0) - stats0.get("gpu_step_s", 0.0)
    host = {"rank": ps.rank, "cpu_s": round(cpu_s, 2), "cpu_s_per_turn": round(cpu_s / nturns, 4),
            "cpu_s_children": round(cpu_child_s, 2), "cpu_util": round(cpu_s / max(elapsed, 1e-9), 2),
            "gpu_step_s": round(gpu_step, 2), "gpu_busy_frac": round(gpu_step / max(elapsed, 1e-9), 3),
            "gpu_idle_between_steps_s": round(stats.get("gpu_idle_between_steps_s", 0.0)
                                              - stats0.get("gpu_idle_between_steps_s", 0.0), 3),
            "max_rss_gib": round(ru1.ru_maxrss / 2**20, 2),      # host memory high-water mark (ru_maxrss is KiB)
            "custom_all_reduce": dict(comm.AR_STATUS) if args.tp > 1 else None}
    steps_timed = {k: stats.get(k, 0) - stats0.get(k, 0) for k in ("steps", "graph_steps", "tokens")}
    return {"elapsed": elapsed, "turns": sum(r.turns for r in results), "errors": sum(r.errors for r in results),
            "host": host, "steps_timed": steps_timed,
            "prefill_timed": {k: stats.get("prefill_" + k2, 0) - stats0.get("prefill_" + k2, 0)
                              for k, k2 in (("steps", "steps"), ("tokens", "step_tokens"))},
            "ttfts": [t for r in results for t in r.ttfts], "retrievals": sum(r.retrievals for r in results),
            "stages": stages, "engine": stats, "tokens": tokens, "latency": latency,
            "plots_ok": sum(r.plots_ok for r in results), "plots_failed": sum(r.plots_failed for r in results)}


def _share_host_cpus() -> None:
    """One process per GPU on a shared host: without an OMP_NUM_THREADS from the launcher, give each
    local rank an equal share of the CPUs for its intra-op thread pools (torch / OpenMP default to
    every core, so 8 ranks would each start one thread per core).  PENNY_PIN_CPUS=1 also pins each
    rank to its own contiguous CPU slice."""
    lws = int(os.environ.get("LOCAL_WORLD_SIZE", "1"))
    if lws <= 1:
        return
    lr = int(os.environ.get("LOCAL_RANK", "0"))
    cpus = sorted(os.sched_getaffinity(0))
    per = max(1, len(cpus) // lws)
    if os.environ.get("PENNY_PIN_CPUS") == "1" and per >= 2:
        os.sched_setaffinity(0, cpus[lr * per:(lr + 1) * per])
    if "OMP_NUM_THREADS" not in os.environ:     # torchrun sets it (to 1) unless the caller did
        os.environ["OMP_NUM_THREADS"] = str(min(per, 16))
        import torch
        torch.set_num_threads(min(per, 16))


def _launch_ranks(args, argv) -> int:
    """``bench.py --gpus N`` started without a launcher: run N local ranks (one per GPU) under
    ``torch.distributed.run`` as a CHILD process -- never exec, and nothing here has touched the GPU
    (``import torch`` / ``device_count`` do not initialise it) -- forward its output and exit code.
    The reference's scale-out is likewise N worker processes (gunicorn.conf.py:8-9)."""
    import socket
    import subprocess
    if args.device == "cuda" and not os.environ.get("PENNY_DIST_BACKEND"):
        import torch
        ndev = torch.cuda.device_count()
        if ndev < args.gpus:
            log(f"error: --gpus {args.gpus} but only {ndev} visible GPU(s); set PENNY_DIST_BACKEND=gloo to "
                "rehearse several ranks on one GPU")
            return 2
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    argv = list(sys.argv[1:] if argv is None else argv)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(args.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__), *argv]
    env = dict(os.environ, PENNY_BENCH_SPAWNED="1")
    log(f"launching {args.gpus} ranks: {' '.join(cmd[1:])}")
    return subprocess.run(cmd, env=env).returncode


# xGMI pricing of the stubbed collectives (tp_shard_projection): stated assumptions, not measurements
XGMI_LINK_GBPS = 153.0          # one xGMI link, per direction (MI355X: 7 links per GPU)
ONESHOT_LAT_US = 5.0            # custom one-shot all-reduce: flag round trip + in-graph launch boundary
RCCL_LAT_US = 15.0              # RCCL ring all-reduce launch + latency (prefill-size messages)
RCCL_BUSBW_GBPS = (300.0, 150.0)   # RCCL all-reduce bus bandwidth on 8 xGMI-meshed GPUs: optimistic, pessimistic


def tp_shard_projection(args, res, tmax: float, turns: int) -> dict:
    """Per-rank TP=N step estimate: the measured compute-only run of rank 0's shard plus the
    all-reduce time its collectives would take -- 1 (vocab-parallel embedding) + 2 per layer (O and
    down) of [T, hidden] bf16 per step: decode steps on the custom one-shot kernel (each rank reads
    its 7 peers' buffers over 7 links at once: bytes / link rate), prefill steps on RCCL's ring
    (2 (n-1)/n x bytes / bus bandwidth).  No overlap of the collectives with compute is assumed
    (the prefill micro-batch pipeline would hide part of it), so this bounds the TP=N group's rate
    from below for the given link rates."""
    from financial_chatbot_llm_amd.models.configs import get_model_config
    mc = get_model_config(args.model)
    n = args.tp_shard_estimate
    ars = 1 + 2 * mc.num_layers
    row_bytes = mc.hidden_size * 2
    st, pf = res["steps_timed"], res["prefill_timed"]
    dec_steps = max(st["steps"] - pf["steps"], 0)
    dec_tokens = max(st["tokens"] - pf["tokens"], 0)
    dec_s = ars * (dec_steps * ONESHOT_LAT_US * 1e-6 + dec_tokens * row_bytes / (XGMI_LINK_GBPS * 1e9))
    out = {"tp": n, "all_reduces_per_step": ars, "decode_steps": dec_steps, "decode_tokens": dec_tokens,
           "prefill_steps": pf["steps"], "prefill_tokens": pf["tokens"],
           "all_reduce_bytes": ars * st["tokens"] * row_bytes, "decode_comm_s": round(dec_s, 3),
           "compute_only_s": round(tmax, 3), "compute_only_turns_per_s": round(turns / tmax, 3),
           "assumptions": {"xgmi_link_GBps": XGMI_LINK_GBPS, "oneshot_latency_us": ONESHOT_LAT_US,
                           "rccl_latency_us": RCCL_LAT_US, "rccl_busbw_GBps": list(RCCL_BUSBW_GBPS),
                           "overlap": "none"}}
    for tag, bw in zip(("optimistic", "pessimistic"), RCCL_BUSBW_GBPS):
        pre_s = ars * (pf["steps"] * RCCL_LAT_US * 1e-6 + 2 * (n - 1) / n * pf["tokens"] * row_bytes / (bw * 1e9))
        total = tmax + dec_s + pre_s
        out[tag] = {"prefill_comm_s": round(pre_s, 3), "projected_s": round(total, 3),
                    "projected_turns_per_s_per_group": round(turns / total, 3)}
    return out


def main(argv=None) -> int:
    args = parse(argv)
    launched = "WORLD_SIZE" in os.environ
    if args.gpus < 1:
        log(f"error: --gpus {args.gpus}")
        return 2
    if not launched and args.gpus > 1:
        return _launch_ranks(args, argv)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        # a silent mismatch would print n_gpus for a different job than the one asked for
        log(f"error: --gpus {args.gpus} but the launcher started WORLD_SIZE {world} ranks")
        return 2
    if args.gpus % args.tp:
        log(f"error: --gpus {args.gpus} not divisible by --tp {args.tp}")
        return 2
    if args.max_batched_tokens is None:
        args.max_batched_tokens = 16384 if args.model.startswith("mixtral") else 4096
    os.environ.setdefault("LOG_LEVEL", "WARNING")
    if args.decide_always_limit:
        os.environ["PENNY_DECIDE_ALWAYS_LIMIT"] = "1"
    _share_host_cpus()
    import torch
    import torch.distributed as dist

    from financial_chatbot_llm_amd.parallel.dist import init_distributed
    ps = init_distributed(tp_size=args.tp, device_type=args.device)
    res = asyncio.run(run(args, ps))
    if ps.world_size > 1:
        # every rank joins (TP followers contribute None); the replicas' results are the leaders'
        every = [None] * ps.world_size
        dist.all_gather_object(every, res)
        allr = [r for r in every if r is not None and not r.get("follower")]
        hosts = [r["host"] for r in every if r is not None]
    else:
        allr = [res]
        hosts = [res["host"]]
    if ps.rank == 0:
        tmax = max(r["elapsed"] for r in allr)
        turns = sum(r["turns"] - r["errors"] for r in allr)    # completed turns: errored ones do not count
        ttfts = sorted(t for r in allr for t in r["ttfts"])
        p50 = statistics.median(ttfts) * 1e3 if ttfts else None
        p99 = ttfts[min(len(ttfts) - 1, int(0.99 * len(ttfts)))] * 1e3 if ttfts else None
        value = turns / tmax
        out = {
            "metric": METRIC, "value": round(value, 3), "unit": "turns/s", "n_gpus": ps.world_size,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(1e3 * tmax / max(args.steps, 1), 1),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "bf16" if args.dtype == "bf16" else "bf16 (fp8 e4m3 MoE experts)",
            "data": f"synthetic conversations + {args.corpus:,}-vector synthetic corpus per GPU; "
                    "random-init weights of the real architectures",
            "config": {"model": MODEL_LABELS.get(args.model, args.model), "embedder": args.embed_model, "global_batch": args.convs * ps.dp_size,
                       "convs_per_gpu": args.convs, "respond_tokens": args.respond_tokens,
                       "arrival": "closed-loop per conversation" if args.arrival == "closed" else "lock-step waves",
                       "tool_steps": 0 if args.no_tools else args.tool_steps,
                       "decide_decoding": "tool-call grammar, jump-forward" if not args.no_jump_forward else "token by token",
                       "decide_limits": ("num_transactions=20 on every call" if args.decide_always_limit else
                                         "reference few-shot: time windows send no limit (10000 -> token clamp)"),
                       "agent": "single-chain chat (no tools)" if args.no_tools else "tool-calling RAG agent",
                       "corpus_vectors": args.corpus, "seq_len": args.max_model_len,
                       "parallelism": f"dp{ps.dp_size}" if args.tp == 1 else f"dp{ps.dp_size}tp{args.tp}"},
            "p50_ttft_ms": None if p50 is None else round(p50, 1),
            "p99_ttft_ms": None if p99 is None else round(p99, 1),
            "turn_errors": sum(r["errors"] for r in allr),
            "retrieval_turns": sum(r["retrievals"] for r in allr),
            "plots": {"ok": sum(r["plots_ok"] for r in allr), "failed": sum(r["plots_failed"] for r in allr)},
            "ttft_p50_breakdown_ms": {k: round(1e3 * statistics.median(v), 1) if v else None
                                      for k, v in allr[0]["stages"].items()},
            "ttft_p90_ms": None if not ttfts else round(1e3 * ttfts[min(len(ttfts) - 1, int(0.9 * len(ttfts)))], 1),
            # per-stage p99 (each stage's own tail; they need not come from the same turns)
            "ttft_stage_p99_ms": {k: round(1e3 * sorted(v)[min(len(v) - 1, int(0.99 * len(v)))], 1) if v else None
                                  for k, v in allr[0]["stages"].items()},
            "prompt_tokens_rank0": allr[0]["tokens"],
            # per LLM call, engine side: queued before admission / admission -> first token / total
            "engine_call_latency_ms_rank0": allr[0]["latency"],
            "engine_rank0": allr[0]["engine"],
            "host": {"cpu_count": os.cpu_count(), "affinity_cpus": len(os.sched_getaffinity(0)),
                     "world_size": ps.world_size, "backend": ps.backend,
                     "local_world_size": int(os.environ.get("LOCAL_WORLD_SIZE", "1")),
                     "launcher": ("bench.py self-spawn (torch.distributed.run child)"
                                  if os.environ.get("PENNY_BENCH_SPAWNED") else
                                  "torch.distributed.run" if "WORLD_SIZE" in os.environ else "single process"),
                     "ranks": hosts},
        }
        if args.tp_shard_estimate > 1:
            out["tp_shard_estimate"] = tp_shard_projection(args, allr[0], tmax, turns)
            out["config"]["parallelism"] = f"tp{args.tp_shard_estimate} rank-0 shard on 1 GPU, collectives stubbed"
        line = json.dumps(out)
        print(line, flush=True)
        if args.json_out:
            with open(args.json_out, "w") as fh:
                fh.write(line + "\n")
    if ps.world_size > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
