"""Kernel microbenchmarks on the GPU (hipEvent timing, interleaved variants, median of rounds).

    python -m financial_chatbot_llm_amd.bench.kernels [--only decode,prefill,...]

Reports time and the roofline-relevant rate (GB/s for bandwidth-bound ops, TFLOP/s for MFMA
ones) on shapes taken from the Llama-3-8B RAG workload (B=64 decode, ~2k contexts with a shared
~1k-token system-prompt prefix).
"""
from __future__ import annotations

import argparse
import json
import math
import statistics
from typing import Callable, Dict, List

import numpy as np
import torch

from .. import ops
from ..ops.attention import KV_BS


def timeit(fn: Callable[[], None], iters: int = 20, rounds: int = 5) -> float:
    """Median over rounds of mean-per-iteration microseconds."""
    fn()
    torch.cuda.synchronize()
    res = []
    for _ in range(rounds):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        for _ in range(iters):
            fn()
        b.record()
        b.synchronize()
        res.append(a.elapsed_time(b) * 1e3 / iters)
    return statistics.median(res)


def _paged(B, ctx, shared, Hkv, D, dev, gen):
    """Block tables where the first `shared` tokens of every sequence are the SAME physical blocks."""
    nsh = shared // KV_BS
    nb = (ctx + KV_BS - 1) // KV_BS
    total = nsh + B * (nb - nsh) + 1
    tables = torch.zeros((B, nb), dtype=torch.int32)
    nxt = nsh
    for b in range(B):
        tables[b, :nsh] = torch.arange(nsh, dtype=torch.int32)
        tables[b, nsh:] = torch.arange(nxt, nxt + nb - nsh, dtype=torch.int32)
        nxt += nb - nsh
    kc = torch.randn((total, Hkv, KV_BS * D), generator=gen, device=dev).to(torch.bfloat16)
    vc = torch.randn((total, Hkv, KV_BS * D), generator=gen, device=dev).to(torch.bfloat16)
    return tables.to(dev), kc, vc, total


def bench_decode(dev) -> List[Dict]:
    out = []
    g = torch.Generator(device=dev).manual_seed(0)
    Hq, Hkv, D = 32, 8, 128
    for B, ctx, shared in [(64, 2048, 0), (64, 2048, 1024), (16, 2048, 1024), (64, 512, 0), (128, 4096, 1024),
                           (128, 2304, 1984), (128, 1536, 768), (64, 2304, 1984)]:
        tables, kc, vc, total = _paged(B, ctx, shared, Hkv, D, dev, g)
        q = torch.randn((B, Hq, D), generator=g, device=dev).to(torch.bfloat16)
        lens = torch.full((B,), ctx, dtype=torch.int32, device=dev)
        ws = ops.DecodeWorkspace.create(B, Hq, D, 8192, dev)
        o = torch.empty_like(q)
        us = timeit(lambda: ops.decode(q, lens, tables, kc, vc, 0.088, workspace=ws, out=o))
        uniq = (B * ctx - (B - 1) * shared) * Hkv * D * 2 * 2
        logical = B * ctx * Hkv * D * 2 * 2
        row = {"op": "decode_attn", "B": B, "ctx": ctx, "shared": shared, "us": round(us, 1),
               "GBps_unique": round(uniq / us / 1e3, 1), "GBps_logical": round(logical / us / 1e3, 1)}
        out.append(row)
    return out


def bench_decode_mixed(dev) -> List[Dict]:
    """Decode attention on the workload's decode batches: B rows with contexts spread over
    1.5k-6.5k tokens, the first 1k tokens (system prompt) shared by every row (prefix cache)."""
    out = []
    g = torch.Generator(device=dev).manual_seed(3)
    Hq, Hkv, D = 32, 8, 128
    for B in (64, 96, 128):
        rng = torch.Generator().manual_seed(B)
        ctxs = torch.randint(1500, 6500, (B,), generator=rng).tolist()
        shared = 1024
        nsh = shared // KV_BS
        W = max((c + KV_BS - 1) // KV_BS for c in ctxs)
        tables = torch.zeros((B, W), dtype=torch.int32)
        nxt = nsh
        for b, c in enumerate(ctxs):
            nb = (c + KV_BS - 1) // KV_BS
            tables[b, :nsh] = torch.arange(nsh, dtype=torch.int32)
            tables[b, nsh:nb] = torch.arange(nxt, nxt + nb - nsh, dtype=torch.int32)
            nxt += nb - nsh
        kc = torch.randn((nxt + 1, Hkv, KV_BS * D), generator=g, device=dev).to(torch.bfloat16)
        vc = torch.randn((nxt + 1, Hkv, KV_BS * D), generator=g, device=dev).to(torch.bfloat16)
        tables = tables.to(dev)
        q = torch.randn((B, Hq, D), generator=g, device=dev).to(torch.bfloat16)
        lens = torch.tensor(ctxs, dtype=torch.int32, device=dev)
        ws = ops.DecodeWorkspace.create(B, Hq, D, 8192, dev)
        o = torch.empty_like(q)
        us = timeit(lambda: ops.decode(q, lens, tables, kc, vc, 0.088, workspace=ws, out=o))
        uniq = (sum(ctxs) - (B - 1) * shared) * Hkv * D * 2 * 2
        out.append({"op": "decode_attn_mixed", "B": B, "ctx_mean": round(sum(ctxs) / B), "us": round(us, 1),
                    "GBps_unique": round(uniq / us / 1e3, 1)})
    return out


def bench_decode_lean(dev) -> List[Dict]:
    """Work-balanced (lean) vs partitioned split-K decode on workload-shaped batches, interleaved
    rounds.  GB/s counts unique KV bytes (the shared prefix once) and logical bytes (every row's full context)."""
    from ..ops import attention as A
    out = []
    g = torch.Generator(device=dev).manual_seed(3)
    Hq, Hkv, D = 32, 8, 128
    for B, lo, hi, shared in [(64, 1500, 6500, 1024), (128, 1500, 6500, 1024), (96, 2000, 8000, 2048),
                              (64, 2048, 2049, 0), (256, 1000, 3000, 768), (16, 1100, 8000, 1024)]:
        rng = torch.Generator().manual_seed(B + lo)
        ctxs = torch.randint(lo, hi, (B,), generator=rng).tolist()
        nsh = shared // KV_BS
        W = max((c + KV_BS - 1) // KV_BS for c in ctxs)
        tables = torch.zeros((B, W), dtype=torch.int32)
        nxt = nsh
        for b, c in enumerate(ctxs):
            nb = (c + KV_BS - 1) // KV_BS
            tables[b, :nsh] = torch.arange(nsh, dtype=torch.int32)
            tables[b, nsh:nb] = torch.arange(nxt, nxt + nb - nsh, dtype=torch.int32)
            nxt += nb - nsh
        kc = torch.randn((nxt + 1, Hkv, KV_BS * D), generator=g, device=dev).to(torch.bfloat16)
        vc = torch.randn((nxt + 1, Hkv, KV_BS * D), generator=g, device=dev).to(torch.bfloat16)
        tables_d = tables.to(dev)
        q = torch.randn((B, Hq, D), generator=g, device=dev).to(torch.bfloat16)
        lens = torch.tensor(ctxs, dtype=torch.int32, device=dev)
        ws = ops.DecodeWorkspace.create(B, Hq, D, 8192, dev)
        o = torch.empty_like(q)

        marked_d = torch.from_numpy(A.mark_shared_blocks(tables.numpy().copy(), np.asarray(ctxs))).to(dev)

        def mk(lean, flags=0, bt=tables_d):
            def f():
                A.DECODE_LEAN, A.LEAN_FLAGS = lean, flags
                ops.decode(q, lens, bt, kc, vc, 0.088, workspace=ws, out=o)
                A.LEAN_FLAGS = 0
            return f
        # lean_nt: every block non-temporal; lean_ntm: the shared-prefix blocks (marked in the table by
        # the host, as the engine does) on the default policy, the rest non-temporal
        fns = {"part": mk(False), "lean": mk(True), "lean_nt": mk(True, 1), "lean_ntm": mk(True, 1, marked_d),
               "lean_ntm_wmerge": mk(True, 3, marked_d)}
        ref = None
        errs = {}
        for k, f in fns.items():
            f()
            torch.cuda.synchronize()
            ref = o.float().clone() if ref is None else ref
            errs[k] = float((o.float() - ref).abs().max())
        ts = interleaved(fns, rounds=7, iters=20)
        # mixed-step shape: the decode rows' attention on a side stream concurrently with a prefill
        # attention (4 x 512 new tokens behind 2k context) on the main stream, as llama.py runs it
        ptab, pkc, pvc, _ = _paged(4, 2560, 0, Hkv, D, dev, g)
        pq = torch.randn((2048, Hq, D), generator=g, device=dev).to(torch.bfloat16)
        pcu = torch.arange(0, 2049, 512, dtype=torch.int32, device=dev)
        plens = torch.full((4,), 2560, dtype=torch.int32, device=dev)
        po = torch.empty_like(pq)
        side = torch.cuda.Stream()

        def pair(f):
            def g2():
                side.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(side):
                    f()
                ops.prefill(pq, pcu, plens, ptab, pkc, pvc, 0.088, True, 512, out=po)
                torch.cuda.current_stream().wait_stream(side)
            return g2
        tp = interleaved({"prefill_only": lambda: ops.prefill(pq, pcu, plens, ptab, pkc, pvc, 0.088, True, 512, out=po),
                          **{"with_" + k: pair(fns[k]) for k in fns}},
                         rounds=7, iters=20)
        A.DECODE_LEAN = True
        uniq = (sum(ctxs) - (B - 1) * shared) * Hkv * D * 2 * 2
        logical = sum(ctxs) * Hkv * D * 2 * 2
        row = {"op": "decode_lean_ab", "B": B, "ctx_range": [lo, hi], "ctx_mean": round(sum(ctxs) / B),
               "shared": shared, "MB_unique": round(uniq / 1e6, 1), "max_abs_diff": errs}
        for k, us in ts.items():
            row[k + "_us"] = round(us, 1)
            row[k + "_GBps_unique"] = round(uniq / us / 1e3, 1)
            row[k + "_GBps_logical"] = round(logical / us / 1e3, 1)
        row["concurrent_with_prefill_us"] = {k: round(v, 1) for k, v in tp.items()}
        print(json.dumps(row), flush=True)
        out.append(row)
    return out


def bench_prefill(dev) -> List[Dict]:
    out = []
    g = torch.Generator(device=dev).manual_seed(1)
    Hq, Hkv, D = 32, 8, 128
    for S, qlen, ctx in [(16, 512, 1536), (4, 2048, 2048), (1, 8192, 8192), (32, 256, 2048)]:
        tables, kc, vc, _ = _paged(S, ctx, 0, Hkv, D, dev, g)
        T = S * qlen
        q = torch.randn((T, Hq, D), generator=g, device=dev).to(torch.bfloat16)
        cu = torch.arange(0, T + 1, qlen, dtype=torch.int32, device=dev)
        lens = torch.full((S,), ctx, dtype=torch.int32, device=dev)
        o = torch.empty_like(q)
        us = timeit(lambda: ops.prefill(q, cu, lens, tables, kc, vc, 0.088, True, qlen, out=o), iters=5)
        # causal FLOPs: each query i attends to (ctx - qlen + i + 1) keys
        keys = S * (qlen * (ctx - qlen) + qlen * (qlen + 1) / 2)
        flops = 4 * keys * Hq * D
        out.append({"op": "prefill_attn", "S": S, "q_len": qlen, "ctx": ctx, "us": round(us, 1),
                    "TFLOPs": round(flops / us / 1e6, 1)})
    return out


# prefill-attention launches as the 20-turn RAG workload issues them: (q_len, ctx) per sequence of
# one mixed step -- respond chunks (~1.6-2k new tokens after a cached system prompt) next to decide
# prompts (~200 new tokens behind ~4.6k cached ones)
MIXED_STEPS = {
    "respond+8decides": [(1600, 3400)] + [(220, 4600)] * 8,
    "respond+16spec+4decides": [(1500, 3600)] + [(9, 5200)] * 16 + [(220, 4600)] * 4,
    "2respond": [(1800, 3000), (1900, 3900)],
    "16decides": [(200, 4800)] * 16,
    "respond-long": [(2400, 6400), (1600, 5200)],
    "first-turn": [(4096, 4096)],
    "1decide": [(220, 4600)],
    "2decides": [(230, 4700), (210, 4500)],
    "1respond-short": [(600, 4200)],
    # lean split-KV steps with more merges (16-20 split tiles)
    "4decides+16spec": [(220, 4600)] * 4 + [(9, 5200)] * 16,
    "respond-short+4decides": [(600, 3600)] + [(220, 4600)] * 4,
    # tiny chunks only (<= 32 tokens): speculative verify rows / known runs behind long contexts
    "16spec": [(9, 5200)] * 16,
    "4runs": [(2, 4600), (3, 3900), (2, 5100), (4, 4400)],
    "1run": [(2, 4600)],
}


def _paged_varlen(shape, Hkv, D, dev, gen):
    """Per-sequence contexts: (block tables [S, W], k/v caches)."""
    nbs = [(ctx + KV_BS - 1) // KV_BS for _, ctx in shape]
    W = max(nbs)
    tables = torch.zeros((len(shape), W), dtype=torch.int32)
    nxt = 0
    for i, nb in enumerate(nbs):
        tables[i, :nb] = torch.arange(nxt, nxt + nb, dtype=torch.int32)
        nxt += nb
    kc = torch.randn((nxt + 1, Hkv, KV_BS * D), generator=gen, device=dev).to(torch.bfloat16)
    vc = torch.randn((nxt + 1, Hkv, KV_BS * D), generator=gen, device=dev).to(torch.bfloat16)
    return tables.to(dev), kc, vc


def bench_prefill_mixed(dev) -> List[Dict]:
    """Prefill attention on the workload's real step shapes (varlen, prefix-cached contexts)."""
    out = []
    g = torch.Generator(device=dev).manual_seed(2)
    Hq, Hkv, D = 32, 8, 128
    for name, shape in MIXED_STEPS.items():
        tables, kc, vc = _paged_varlen(shape, Hkv, D, dev, g)
        qlens = [q for q, _ in shape]
        T = sum(qlens)
        q = torch.randn((T, Hq, D), generator=g, device=dev).to(torch.bfloat16)
        cu = torch.tensor([0] + list(torch.cumsum(torch.tensor(qlens), 0)), dtype=torch.int32, device=dev)
        lens = torch.tensor([c for _, c in shape], dtype=torch.int32, device=dev)
        o = torch.empty_like(q)
        wl = ops.attention.prefill_work_list(cu.cpu().numpy(), lens.cpu().numpy(), Hq // Hkv)
        wd = torch.from_numpy(wl).to(dev) if wl is not None else None
        ln = ops.attention.prefill_lean_list(cu.cpu().numpy(), lens.cpu().numpy(), Hq // Hkv, Hkv)
        ld = torch.from_numpy(ln).to(dev) if ln is not None else None
        lc = (int(ln[0, 1]), int(ln[0, 2]), int(ln[0, 3])) if ln is not None else None

        # production form: q prescaled by scale * log2(e) at the QKV epilogue's one rounding
        qp = (q.float() * (0.088 * 1.4426950408889634)).to(torch.bfloat16)

        def run(v):
            var, lean, qpre = v

            def f():
                ops.attention.prefill_variant(var)
                ops.prefill(qp if qpre else q, cu, lens, tables, kc, vc, 1 / 1.4426950408889634 if qpre else 0.088,
                            True, max(qlens), out=o, work=(ld if ld is not None else wd) if lean else wd,
                            lean=lc if lean else None, q_prescaled=qpre)
            return f
        variants = {"pf2_sb": (4, False, False), "pf2_fold": (5, False, False), "pf3": (7, False, False),
                    "pf2_fold_lean": (5, True, False), "pf3_lean": (7, True, False),
                    "pf2_prod": (5, True, True), "pf3_prod": (7, True, True),
                    "pf3_q": (7, False, True)}
        old = ops.attention.prefill_variant()
        outs = {}
        for k, v in variants.items():
            run(v)()
            outs[k] = o.clone()
        ts = interleaved({k: run(v) for k, v in variants.items()}, rounds=7, iters=5)
        ops.attention.prefill_variant(old)
        keys = sum(ql * (c - ql) + ql * (ql + 1) / 2 for ql, c in shape)
        flops = 4 * keys * Hq * D
        row = {"op": "prefill_attn_mixed", "step": name, "T": T,
               "lean_items": int(ln[0, 1]) if ln is not None else 0, "lean_splits": int(ln[0, 2]) if ln is not None else 0}
        for k in variants:
            row[f"{k}_us"] = round(ts[k], 1)
            row[f"{k}_TFLOPs"] = round(flops / ts[k] / 1e6, 1)
            row[f"{k}_maxdiff_vs_pf2_sb"] = round(float((outs[k].float() - outs["pf2_sb"].float()).abs().max()), 5)
        print(json.dumps(row), flush=True)
        out.append(row)
    return out


def bench_attn_overlap(dev) -> List[Dict]:
    """A mixed step's two attention kernels -- the prefill rows' (MFMA-bound, one 512-thread
    workgroup per CU) and the decode rows' (HBM-bound) -- serial on one stream vs concurrent on two
    (models/llama.py ATTN_OVERLAP): decode launched first (production through r6 s21), prefill
    launched first, and prefill first on a high-priority stream.  Interleaved rounds; each form
    ends joined on the current stream."""
    out = []
    g = torch.Generator(device=dev).manual_seed(5)
    Hq, Hkv, D = 32, 8, 128
    steps = {"respond+8decides|B96": (MIXED_STEPS["respond+8decides"], 96),
             "2respond|B112": (MIXED_STEPS["2respond"], 112),
             "respond-short+4decides|B100": (MIXED_STEPS["respond-short+4decides"], 100),
             "1decide|B120": (MIXED_STEPS["1decide"], 120)}
    main = torch.cuda.current_stream(dev)
    side = torch.cuda.Stream(device=dev)
    hi = torch.cuda.Stream(device=dev, priority=-1)
    for name, (shape, B) in steps.items():
        tables, kc, vc = _paged_varlen(shape, Hkv, D, dev, g)
        qlens = [q for q, _ in shape]
        T = sum(qlens)
        cu = torch.tensor([0] + list(torch.cumsum(torch.tensor(qlens), 0)), dtype=torch.int32, device=dev)
        lens = torch.tensor([c for _, c in shape], dtype=torch.int32, device=dev)
        qp = (torch.randn((T, Hq, D), generator=g, device=dev) * (0.088 * 1.4426950408889634)).to(torch.bfloat16)
        op = torch.empty_like(qp)
        plan = ops.attention.prefill_plan(cu.cpu().numpy(), lens.cpu().numpy(), Hq // Hkv, Hkv)
        pw = torch.from_numpy(plan).to(dev) if plan is not None else None
        lean = (int(plan[0, 1]), int(plan[0, 2]), int(plan[0, 3])) if plan is not None and plan.shape[1] == 6 else None
        # decode rows: their own contexts (1.5k-6.5k), separate cache
        rng = torch.Generator().manual_seed(B)
        ctxs = torch.randint(1500, 6500, (B,), generator=rng).tolist()
        W = max((c + KV_BS - 1) // KV_BS for c in ctxs)
        dt = torch.zeros((B, W), dtype=torch.int32)
        nxt = 0
        for b, c in enumerate(ctxs):
            nb = (c + KV_BS - 1) // KV_BS
            dt[b, :nb] = torch.arange(nxt, nxt + nb, dtype=torch.int32)
            nxt += nb
        dkc = torch.randn((nxt, Hkv, KV_BS * D), generator=g, device=dev).to(torch.bfloat16)
        dvc = torch.randn((nxt, Hkv, KV_BS * D), generator=g, device=dev).to(torch.bfloat16)
        dt, dl = dt.to(dev), torch.tensor(ctxs, dtype=torch.int32, device=dev)
        qd = torch.randn((B, Hq, D), generator=g, device=dev).to(torch.bfloat16)
        od = torch.empty_like(qd)
        ws = ops.DecodeWorkspace.create(B, Hq, D, 8192, dev)

        def pf():
            ops.prefill(qp, cu, lens, tables, kc, vc, 1 / 1.4426950408889634, True, max(qlens), out=op, work=pw,
                        lean=lean, q_prescaled=True)

        def dc(st=None):
            ops.decode(qd, dl, dt, dkc, dvc, 0.088, workspace=ws, out=od, stream=st)

        def serial():
            pf()
            dc()

        def fork(st):
            ev = torch.cuda.Event()
            ev.record(main)
            st.wait_event(ev)

        def join(st):
            ev = torch.cuda.Event()
            ev.record(st)
            main.wait_event(ev)

        def dfirst():
            fork(side)
            dc(side.cuda_stream)
            pf()
            join(side)

        def pfirst():
            fork(side)
            pf()
            dc(side.cuda_stream)
            join(side)

        def pfirst_hi():
            fork(hi)
            with torch.cuda.stream(hi):
                pf()
            dc()
            join(hi)

        fns = {"serial": serial, "dfirst": dfirst, "pfirst": pfirst, "pfirst_hi": pfirst_hi,
               "prefill_only": pf, "decode_only": dc}
        t = interleaved(fns, rounds=7, iters=5)
        row = {"op": "attn_overlap", "step": name, "T": T, "B": B, **{k: round(v, 1) for k, v in t.items()}}
        print(json.dumps(row), flush=True)
        out.append(row)
    return out


def bench_prefill_spec_split(dev) -> List[Dict]:
    """Mixed steps with speculative chunks (9 query tokens behind 5k-token contexts): one launch of
    the 8-wave kernel over every sequence (LPT work list; a spec chunk's 36 rows fill one 256-row
    tile) vs the long chunks on the 8-wave kernel + the spec chunks on the 4-wave 128-row kernel."""
    out = []
    g = torch.Generator(device=dev).manual_seed(3)
    Hq, Hkv, D = 32, 8, 128
    steps = {"respond+4decides+16spec": [(1500, 3600)] + [(220, 4600)] * 4 + [(9, 5200)] * 16,
             "2decides+32spec": [(220, 4600)] * 2 + [(9, 5200)] * 32,
             "respond+64spec": [(1500, 3600)] + [(9, 4800)] * 64}
    for name, shape in steps.items():
        tables, kc, vc = _paged_varlen(shape, Hkv, D, dev, g)
        qlens = [q for q, _ in shape]
        nb = sum(1 for q in qlens if q * (Hq // Hkv) > 128)
        T, T1 = sum(qlens), sum(qlens[:nb])
        q = torch.randn((T, Hq, D), generator=g, device=dev).to(torch.bfloat16)
        cu = torch.tensor([0] + list(torch.cumsum(torch.tensor(qlens), 0)), dtype=torch.int32, device=dev)
        lens = torch.tensor([c for _, c in shape], dtype=torch.int32, device=dev)
        o = torch.empty_like(q)
        wl = ops.attention.prefill_work_list(cu.cpu().numpy(), lens.cpu().numpy(), Hq // Hkv)
        wd = torch.from_numpy(wl).to(dev)
        cu1, lens1, tb1 = cu[:nb + 1], lens[:nb], tables[:nb]
        wl1 = ops.attention.prefill_work_list(cu1.cpu().numpy(), lens1.cpu().numpy(), Hq // Hkv)
        wd1 = torch.from_numpy(wl1).to(dev)
        cu2, lens2, tb2 = (cu[nb:] - T1).contiguous(), lens[nb:].contiguous(), tables[nb:].contiguous()
        q2, o2 = q[T1:], o[T1:]

        def split():
            ops.prefill(q[:T1], cu1, lens1, tb1, kc, vc, 0.088, True, max(qlens[:nb]), out=o[:T1], work=wd1)
            ops.prefill(q2, cu2, lens2, tb2, kc, vc, 0.088, True, max(qlens[nb:]), out=o2)
        ref = ops.prefill(q, cu, lens, tables, kc, vc, 0.088, True, max(qlens), work=wd).clone()
        split()
        err = float((o.float() - ref.float()).abs().max())
        ts = interleaved({"one": lambda: ops.prefill(q, cu, lens, tables, kc, vc, 0.088, True, max(qlens), out=o,
                                                     work=wd), "split": split}, rounds=7, iters=5)
        row = {"op": "prefill_spec_split", "step": name, "T": T, "one_launch_us": round(ts["one"], 1),
               "split_us": round(ts["split"], 1), "max_abs_diff": err}
        print(json.dumps(row), flush=True)
        out.append(row)
    return out


def bench_elementwise(dev) -> List[Dict]:
    out = []
    for T, H in [(64, 4096), (8192, 4096)]:
        x = torch.randn((T, H), device=dev).to(torch.bfloat16)
        r = torch.randn((T, H), device=dev).to(torch.bfloat16)
        w = torch.ones(H, device=dev, dtype=torch.bfloat16)
        us = timeit(lambda: ops.rms_norm(x, w, 1e-5, residual=r))
        out.append({"op": "add_rmsnorm", "T": T, "H": H, "us": round(us, 2), "GBps": round(4 * T * H * 2 / us / 1e3, 1)})
        gu = torch.randn((T, 2 * 14336), device=dev).to(torch.bfloat16)
        us = timeit(lambda: ops.silu_mul(gu))
        out.append({"op": "silu_mul", "T": T, "F": 14336, "us": round(us, 2), "GBps": round(3 * T * 14336 * 2 / us / 1e3, 1)})
        qkv = torch.randn((T, 48 * 128), device=dev).to(torch.bfloat16)
        cs = ops.rope_cos_sin(128, 8192, 5e5, device=dev)
        pos = torch.arange(T, dtype=torch.int32, device=dev)
        kc = torch.zeros(((T + 63) // 64 + 1, 8, 64 * 128), device=dev, dtype=torch.bfloat16)
        vc = torch.zeros(((T + 63) // 64 + 1, 8, 64 * 128), device=dev, dtype=torch.bfloat16)
        us = timeit(lambda: ops.rope_kv_write(qkv, pos, cs, pos, kc, vc, 32, 8, 128))
        out.append({"op": "rope_kv_write", "T": T, "us": round(us, 2), "GBps": round(2 * T * 48 * 128 * 2 / us / 1e3, 1)})
    # bge encoder LayerNorm (H = 768) at query-batch sizes: rows = queries x ~24 tokens
    for T in (24, 192, 768, 4096):
        x = torch.randn((T, 768), device=dev).to(torch.bfloat16)
        r = torch.randn((T, 768), device=dev).to(torch.bfloat16)
        gw = torch.ones(768, device=dev, dtype=torch.bfloat16)
        bw = torch.zeros(768, device=dev, dtype=torch.bfloat16)
        us = timeit(lambda: ops.layer_norm(x, gw, bw, 1e-12, residual=r), iters=50)
        out.append({"op": "layernorm_768", "T": T, "us": round(us, 2), "GBps": round(3 * T * 768 * 2 / us / 1e3, 1)})
    V = 128256
    for B in (64, 256):
        lg = torch.randn((B, V), device=dev).to(torch.bfloat16)
        t = torch.full((B,), 0.5, device=dev)
        s = torch.arange(B, device=dev, dtype=torch.int64)
        us = timeit(lambda: ops.sample(lg, t, s))
        out.append({"op": "sample", "B": B, "V": V, "us": round(us, 2), "GBps": round(B * V * 2 / us / 1e3, 1)})
    return out


def bench_topk(dev) -> List[Dict]:
    N, D = 1_000_000, 768
    corpus = torch.nn.functional.normalize(torch.randn((N, D), device=dev), dim=-1).to(torch.bfloat16)
    users = torch.randint(0, 10_000, (N,), device=dev, dtype=torch.int32)
    dates = torch.randint(0, 1 << 30, (N,), device=dev, dtype=torch.int64)
    out = []
    for nq in (1, 32, 64):
        q = torch.nn.functional.normalize(torch.randn((nq, D), device=dev), dim=-1).to(torch.bfloat16)
        qu = torch.randint(0, 10_000, (nq,), device=dev, dtype=torch.int32)
        qf = torch.zeros((nq,), device=dev, dtype=torch.int64)
        ks = torch.full((nq,), 20, device=dev, dtype=torch.int32)
        us = timeit(lambda: ops.filtered_topk(corpus, users, dates, q, qu, qf, ks, 20), iters=10)
        out.append({"op": "filtered_topk", "N": N, "nq": nq, "us": round(us, 1)})
    return out


def bench_gemm(dev) -> List[Dict]:
    """hipBLASLt (torch.nn.functional.linear) on the Llama-3-8B projection shapes."""
    out = []
    shapes = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336),
              "lm_head": (128256, 4096)}
    for M in (16, 64, 128, 4096):
        for name, (N, K) in shapes.items():
            w = torch.randn((N, K), device=dev).to(torch.bfloat16)
            x = torch.randn((M, K), device=dev).to(torch.bfloat16)
            us = timeit(lambda: torch.nn.functional.linear(x, w), iters=10)
            bytes_ = (N * K + M * K + M * N) * 2
            out.append({"op": "gemm", "name": name, "M": M, "N": N, "K": K, "us": round(us, 1),
                        "GBps": round(bytes_ / us / 1e3, 1), "TFLOPs": round(2 * M * N * K / us / 1e6, 1)})
    return out


def bench_gemm_prefill(dev) -> List[Dict]:
    """hipBLASLt at the prefill-step M values the 20-turn workload produces (mixed steps of
    ~500-4200 rows), random operands, default heuristic: where the 47 % GEMM share goes."""
    out = []
    shapes = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}
    ws = {n: torch.randn((N, K), device=dev).to(torch.bfloat16) * 0.02 for n, (N, K) in shapes.items()}
    for M in (512, 1024, 1536, 2048, 2400, 3000, 3584, 4096, 4224):
        tot_f, tot_us = 0.0, 0.0
        row = {"op": "gemm_prefill", "M": M}
        for name, (N, K) in shapes.items():
            x = torch.randn((M, K), device=dev).to(torch.bfloat16)
            us = timeit(lambda: torch.nn.functional.linear(x, ws[name]), iters=10)
            f = 2 * M * N * K
            row[name + "_TF"] = round(f / us / 1e6, 1)
            tot_f += f
            tot_us += us
        row["layer_TF"] = round(tot_f / tot_us / 1e6, 1)
        out.append(row)
    return out


def bench_lm_head(dev) -> List[Dict]:
    """LM head (vocab 128256) at the sampler counts of real steps: weight-streaming bound."""
    from ..ops import gemm
    gemm.load_gemm_tuning("llama3-8b")   # the library baseline runs the curated solutions, as in serving
    out = []
    V, K = 128256, 4096
    w = torch.randn((V, K), device=dev).to(torch.bfloat16) * 0.02
    for M in (1, 16, 37, 48, 64, 96, 100, 128, 160, 192, 217, 256):
        x = torch.randn((M, K), device=dev).to(torch.bfloat16)
        us = timeit(lambda: torch.nn.functional.linear(x, w), iters=10)
        row = {"op": "lm_head", "M": M, "hipblaslt_us": round(us, 1), "hipblaslt_TBps": round(V * K * 2 / us / 1e6, 2)}
        ref = torch.nn.functional.linear(x.float(), w.float())
        P = torch.empty((1, M, V), dtype=torch.float32, device=dev)
        for nf in (2, 4, 8):
            t = timeit(lambda: gemm.splitk_partials(x, w, V, 1, nf, out=P, rowmajor=True), iters=10)
            row[f"splitk_nf{nf}_us"] = round(t, 1)
            row[f"splitk_nf{nf}_err"] = float((P[0] - ref).abs().max())
        out.append(row)
    return out


def bench_lm_head_fused(dev) -> List[Dict]:
    """LM head + sampler per step (vocab 128256): hipBLASLt logits + the HIP sampler vs the fused
    tile-kernel LM head that samples in its epilogue (ops.lm_head_sample), temperature rows."""
    from .. import ops
    from ..ops import gemm
    gemm.load_gemm_tuning("llama3-8b")
    out = []
    V, K = 128256, 4096
    w = torch.randn((V, K), device=dev).to(torch.bfloat16) * 0.02
    for M in (1, 16, 32, 48, 64, 96, 128, 160, 192, 256):
        x = torch.randn((M, K), device=dev).to(torch.bfloat16)
        t = torch.full((M,), 0.7, device=dev)
        sd = torch.arange(M, dtype=torch.int64, device=dev) * 977
        lib = timeit(lambda: ops.sample(torch.nn.functional.linear(x, w), t, sd), iters=10)
        fused = timeit(lambda: ops.lm_head_sample(x, w, t, sd), iters=10)
        same = bool(torch.equal(ops.lm_head_sample(x, w, t, sd), ops.sample(gemm.prefill_gemm(x, w), t, sd)))
        out.append({"op": "lm_head_sample", "M": M, "lib_plus_sampler_us": round(lib, 1), "fused_us": round(fused, 1),
                    "speedup": round(lib / fused, 3), "fused_TBps": round(V * K * 2 / fused / 1e6, 2),
                    "fused_equals_tile_logits_then_sampler": same})
    return out


def bench_bge_query(dev) -> List[Dict]:
    """bge-base encoder latency on retrieval-size query batches (the per-turn critical path): the
    four projections on hipBLASLt (+ the GELU pass) vs the tile kernel with the bias / bias+GELU
    epilogues (PENNY_PREFILL_GEMM=0 / 1 / force)."""
    import os
    from ..models.bert import BertEncoder
    from ..models.configs import get_model_config
    enc = BertEncoder.build(get_model_config("bge-base-en"), device=dev)
    out = []
    for nq, L in ((1, 16), (8, 16), (24, 20), (64, 24), (128, 32)):
        ids = [[101] + [(1000 + 7 * q + 13 * j) % 30000 for j in range(L - 2)] + [102] for q in range(nq)]
        row = {"op": "bge_query", "queries": nq, "tokens": nq * L}
        fns = {}
        for mode in ("0", "1", "force"):
            def f(mode=mode):
                os.environ["PENNY_PREFILL_GEMM"] = mode
                enc.encode(ids)
            fns[f"mode_{mode}"] = f
        t = interleaved(fns, rounds=5, iters=5)
        os.environ.pop("PENNY_PREFILL_GEMM", None)
        row.update({k + "_us": round(v, 1) for k, v in t.items()})
        out.append(row)
        print(json.dumps(row), flush=True)
    return out


def bench_gemm_tail(dev, Ms=None) -> List[Dict]:
    """Tile GEMM with vs without the wave-quantisation tail (K-split tail tiles on idle CUs),
    interleaved A/B per (projection, M), each with its fused epilogue."""
    import os
    from ..ops import gemm
    shapes = {"qkv": (6144, 4096, None), "o": (4096, 4096, None), "gate_up": (28672, 4096, "silu"),
              "down": (4096, 14336, None)}
    rnd = lambda *s: ((torch.rand(s, device=dev) * 2 - 1) * 0.05).to(torch.bfloat16)  # noqa: E731
    ws = {n: rnd(N, K) for n, (N, K, _) in shapes.items()}
    out = []
    for M in Ms or [512, 1024, 1536, 2048, 2304, 2560, 3072, 3584]:
        row = {"op": "gemm_tail", "M": M}
        for n, (N, K, epi) in shapes.items():
            x = rnd(M, K)
            fns = {}
            for mode in ("0", "1"):
                def f(mode=mode, x=x, n=n, epi=epi):
                    os.environ["PENNY_GEMM_TAIL"] = mode
                    gemm.prefill_gemm(x, ws[n], epi)
                fns[mode] = f
            t = interleaved(fns, rounds=5, iters=5)
            os.environ.pop("PENNY_GEMM_TAIL", None)
            row[f"{n}_whole_us"] = round(t["0"], 1)
            row[f"{n}_tail_us"] = round(t["1"], 1)
        out.append(row)
        print(json.dumps(row), flush=True)
    return out


def bench_gemm_tune_sweep(dev) -> List[Dict]:
    """Prefill GEMMs at every M = 256k: hipBLASLt default heuristic vs a TunableOp-tuned solution
    (tuned here, written to ``PENNY_TUNE_OUT``): is a padded-M + tuned-solution policy worth it?"""
    import os
    out = []
    shapes = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}
    ws = {n: torch.randn((N, K), device=dev).to(torch.bfloat16) * 0.02 for n, (N, K) in shapes.items()}
    Ms = [256 * k for k in range(2, 17)]
    Ks = sorted({K for _, K in shapes.values()})
    # contiguous activations per K: TunableOp keys include the leading dimensions
    xs = {(M, K): torch.randn((M, K), device=dev).to(torch.bfloat16) for M in Ms for K in Ks}
    base = {}
    for M in Ms:
        for name, (N, K) in shapes.items():
            x = xs[(M, K)]
            base[(M, name)] = timeit(lambda: torch.nn.functional.linear(x, ws[name]), iters=10, rounds=3)
    tun = torch.cuda.tunable
    tun.enable(True)
    tun.tuning_enable(True)
    tun.set_max_tuning_duration(60)
    tun.set_max_tuning_iterations(40)
    tun.set_filename(os.environ.get("PENNY_TUNE_OUT", "tunableop_prefill.csv"))
    for M in Ms:
        for name, (N, K) in shapes.items():
            x = xs[(M, K)]
            torch.nn.functional.linear(x, ws[name])      # tunes this shape
    torch.cuda.synchronize()
    tun.tuning_enable(False)
    for M in Ms:
        row = {"op": "gemm_tune", "M": M}
        fb = ft = 0.0
        for name, (N, K) in shapes.items():
            x = xs[(M, K)]
            t = timeit(lambda: torch.nn.functional.linear(x, ws[name]), iters=10, rounds=3)
            f = 2 * M * N * K
            row[name] = [round(f / base[(M, name)] / 1e6), round(f / t / 1e6)]
            fb += base[(M, name)]
            ft += t
        tot = 2 * M * sum(N * K for N, K in shapes.values())
        row["layer_default_TF"] = round(tot / fb / 1e6, 1)
        row["layer_tuned_TF"] = round(tot / ft / 1e6, 1)
        out.append(row)
        print(json.dumps(row), flush=True)
    return out      # TunableOp flushes the tuned solutions to the file at exit


def bench_skinny(dev) -> List[Dict]:
    """Hand-written MFMA skinny GEMM vs hipBLASLt at decode batch sizes, every launch config."""
    from ..ops import gemm
    out = []
    shapes = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336),
              "lm_head": (128256, 4096)}
    for M in (16, 64):
        for name, (N, K) in shapes.items():
            w = torch.randn((N, K), device=dev).to(torch.bfloat16)
            x = torch.randn((M, K), device=dev).to(torch.bfloat16)
            bytes_ = (N * K + M * K + M * N) * 2
            base = timeit(lambda: torch.nn.functional.linear(x, w), iters=10)
            row = {"op": "skinny", "name": name, "M": M, "hipblaslt_us": round(base, 1),
                   "hipblaslt_GBps": round(bytes_ / base / 1e3, 1)}
            best = None
            saved = (gemm.TUNING.get((N, K)), gemm.SKINNY_MAX_M.get((N, K)))
            gemm.SKINNY_MAX_M[(N, K)] = 64
            wt = gemm.tile_weight(w)
            for cfg in [(2, 4), (2, 8), (4, 4), (1, 8), (1, 4)]:
                gemm.TUNING[(N, K)] = cfg
                if not gemm.skinny_ok(x, w, wt=wt):
                    continue
                us = timeit(lambda: gemm.linear(x, w, wt=wt), iters=10)
                row[f"cfg{cfg[0]}x{cfg[1]}_us"] = round(us, 1)
                if best is None or us < best[1]:
                    best = (cfg, us)
            gemm.TUNING.pop((N, K), None)
            gemm.SKINNY_MAX_M.pop((N, K), None)
            if saved[0] is not None:
                gemm.TUNING[(N, K)], gemm.SKINNY_MAX_M[(N, K)] = saved
            if best:
                row["best"] = list(best[0])
                row["best_GBps"] = round(bytes_ / best[1] / 1e3, 1)
            out.append(row)
    return out


SHAPES_8B = {"qkv": (6144, 4096), "o": (4096, 4096), "down": (4096, 14336)}
SHAPES_70B = {"qkv": (10240, 8192), "o": (8192, 8192), "down": (8192, 28672)}
SHAPES_70B_TP8 = {"qkv": (1280, 8192), "o": (8192, 1024), "down": (8192, 3584)}   # per-rank shards


def bench_splitk(dev, names=("qkv", "o", "down"), shapes=None) -> List[Dict]:
    """Mid-batch split-K GEMM (+ slab reduce) vs hipBLASLt on the Llama-3-8B decode projections.

    Weights rotate over enough copies (>= 768 MB) that every call streams W from HBM, not from
    the 256 MB Infinity Cache -- the situation of a 32-layer decode step."""
    from ..ops import gemm
    out = []
    shapes = shapes or SHAPES_8B
    for name, (N, K) in shapes.items():
        if name not in names:
            continue
        copies = max(2, (768 << 20) // (N * K * 2))
        ws = [torch.randn((N, K), device=dev).to(torch.bfloat16) for _ in range(copies)]
        wts = [gemm.tile_weight(w) for w in ws]
        it = [0]

        def nxt():
            it[0] = (it[0] + 1) % copies
            return it[0]

        for M in (16, 32, 48, 64, 96, 128, 192, 256):
            x = torch.randn((M, K), device=dev).to(torch.bfloat16)
            wbytes = N * K * 2
            base = timeit(lambda: torch.nn.functional.linear(x, ws[nxt()]), iters=copies * 2)
            row = {"op": "splitk", "name": name, "M": M, "hipblaslt_us": round(base, 1),
                   "hipblaslt_GBps": round(wbytes / base / 1e3, 1)}
            best = None
            for S in (1, 2, 4, 7, 8):
                for nf in (2, 4, 6, 8):
                    if K % (64 * S) or N % (16 * nf):
                        continue
                    P = torch.empty((S, M, N), dtype=torch.float32, device=dev)
                    us = timeit(lambda: gemm.splitk_partials(x, wts[nxt()], N, S, nf, out=P), iters=copies * 2)
                    y = torch.empty((M, N), dtype=torch.bfloat16, device=dev)
                    red = timeit(lambda: gemm.splitk_reduce(P, out=y), iters=20)
                    row[f"s{S}nf{nf}_us"] = round(us, 1)
                    row[f"s{S}nf{nf}_red_us"] = round(red, 1)
                    if best is None or us + red < best[1]:
                        best = ((S, nf), us + red, us)
            S_, nf_ = best[0]
            P = torch.empty((S_, M, N), dtype=torch.float32, device=dev)
            row["best_rowmajor_gemm_us"] = round(timeit(
                lambda: gemm.splitk_partials(x, ws[nxt()], N, S_, nf_, out=P, rowmajor=True), iters=copies * 2), 1)
            row["best"] = list(best[0])
            row["best_gemm_us"] = round(best[2], 1)
            row["best_total_us"] = round(best[1], 1)
            row["best_gemm_GBps"] = round(wbytes / best[2] / 1e3, 1)
            row["speedup_total"] = round(base / best[1], 2)
            out.append(row)
        del ws, wts
        torch.cuda.empty_cache()
    return out


def bench_gateup(dev, N: int = 28672, K: int = 4096) -> List[Dict]:
    """Fused gate|up + SiLU*up MFMA kernel vs hipBLASLt GEMM + silu_mul on the Llama-3-8B MLP
    (N = 2*14336, K = 4096), weights rotated so every call streams W from HBM."""
    from ..ops import activation, gemm
    if (N, K) == (28672, 4096):
        gemm.load_gemm_tuning("llama3-8b")   # the baseline runs the curated solutions, as in serving
    out = []
    copies = max(2, (768 << 20) // (N * K * 2))
    ws = [torch.randn((N, K), device=dev).to(torch.bfloat16) for _ in range(copies)]
    wts = [gemm.tile_weight(w) for w in ws]
    it = [0]

    def nxt():
        it[0] = (it[0] + 1) % copies
        return it[0]

    for M in (8, 16, 32, 48, 64, 96, 128, 192, 256):
        x = torch.randn((M, K), device=dev).to(torch.bfloat16)
        y = torch.empty((M, N // 2), dtype=torch.bfloat16, device=dev)
        base = timeit(lambda: activation.silu_mul(torch.nn.functional.linear(x, ws[nxt()]), interleave16=True),
                      iters=copies * 2)
        row = {"op": "gateup", "M": M, "hipblaslt_silu_us": round(base, 1)}
        best = None
        for nf in (4, 8):
            us = timeit(lambda: gemm.gateup_silu(x, wts[nxt()], N, nf, out=y), iters=copies * 2)
            row[f"nf{nf}_us"] = round(us, 1)
            rm = timeit(lambda: gemm.gateup_silu(x, ws[nxt()], N, nf, out=y, rowmajor=True), iters=copies * 2)
            row[f"rowmajor_nf{nf}_us"] = round(rm, 1)
            row[f"nf{nf}_GBps"] = round(N * K * 2 / us / 1e3, 1)
            if best is None or us < best[1]:
                best = (nf, us)
        row["best_nf"], row["speedup"] = best[0], round(base / best[1], 2)
        out.append(row)
    del ws, wts
    torch.cuda.empty_cache()
    return out


def bench_moe(dev) -> List[Dict]:
    """Mixtral-8x7B MoE layer (E=8, top-2, H=4096, F=14336): HIP fp8 pipeline vs bf16 per-expert
    hipBLASLt GEMMs (the eager bucketed path)."""
    from ..ops import activation, moe
    out = []
    E, H, F_, K = 8, 4096, 14336, 2
    g = torch.Generator(device=dev).manual_seed(0)
    w13 = (torch.randn((E, 2 * F_, H), device=dev, generator=g) * 0.02).to(torch.bfloat16)
    w2 = (torch.randn((E, H, F_), device=dev, generator=g) * 0.02).to(torch.bfloat16)
    q13, s13 = moe.quantize_fp8_rowwise(w13)
    q2, s2 = moe.quantize_fp8_rowwise(w2)
    t13, t2 = moe.tile_fp8_weight(q13), moe.tile_fp8_weight(q2)
    del q13, q2
    router = torch.randn((E, H), device=dev, generator=g).to(torch.bfloat16)
    ws = moe.MoEWorkspace(512, K, E, H, F_, dev)
    for T in (1, 16, 64, 256):
        h = torch.randn((T, H), device=dev, generator=g).to(torch.bfloat16)
        logits = (h @ router.t()).contiguous()
        us = timeit(lambda: moe.moe_decode_fp8(h, logits, t13, s13, t2, s2, K, ws), iters=10)
        active = int((ws.offsets[1:] > ws.offsets[:-1]).sum())
        wbytes = active * 3 * H * F_   # fp8 weights of the experts this batch touches

        def bf16_path():
            topw, topi = moe.topk_softmax(logits, K)
            _, offsets, tok_idx, tok_w = moe.route(topi, topw, E)
            offs = offsets.tolist()
            xs = h.index_select(0, tok_idx)
            ys = torch.empty_like(xs)
            for e in range(E):
                a, b = offs[e], offs[e + 1]
                if b > a:
                    ys[a:b] = torch.nn.functional.linear(
                        activation.silu_mul(torch.nn.functional.linear(xs[a:b], w13[e])), w2[e])
            o = torch.zeros_like(h)
            o.index_add_(0, tok_idx, (ys.float() * tok_w[:, None]).to(h.dtype))
        base = timeit(bf16_path, iters=5)
        out.append({"op": "moe", "T": T, "active_experts": active, "fp8_us": round(us, 1),
                    "fp8_GBps": round(wbytes / us / 1e3, 1), "bf16_hipblaslt_us": round(base, 1),
                    "bf16_GBps": round(2 * wbytes / base / 1e3, 1)})
    return out


def bench_moe_prefill(dev) -> List[Dict]:
    """Mixtral-8x7B MoE layer at prefill sizes: the device-only fp8 pipeline (device routing +
    grouped fp8 MFMA GEMMs, no host sync) vs per-expert hipBLASLt fp8 x fp8 GEMMs with a host
    round trip for the bucket sizes (the r1 prefill path)."""
    from ..ops import moe
    out = []
    E, H, F_, K = 8, 4096, 14336, 2
    g = torch.Generator(device=dev).manual_seed(0)
    w13 = (torch.randn((E, 2 * F_, H), device=dev, generator=g) * 0.02).to(torch.bfloat16)
    w13 = torch.stack([interleave16_rows(w13[e]) for e in range(E)])
    q13, s13 = moe.quantize_fp8_rowwise(w13)
    del w13
    w2 = (torch.randn((E, H, F_), device=dev, generator=g) * 0.02).to(torch.bfloat16)
    q2, s2 = moe.quantize_fp8_rowwise(w2)
    del w2
    t13, t2 = moe.tile_fp8_weight(q13), moe.tile_fp8_weight(q2)
    router = torch.randn((E, H), device=dev, generator=g).to(torch.bfloat16)
    for T in (512, 1024, 2048, 4096, 8192, 16384):
        h = torch.randn((T, H), device=dev, generator=g).to(torch.bfloat16)
        logits = (h @ router.t()).contiguous()
        def loop():
            topw, topi = moe.topk_softmax(logits, K)
            order, offsets, tok_idx, tok_w = moe.route(topi, topw, E)
            offs = offsets.tolist()
            xs = h.index_select(0, tok_idx)
            ys = torch.empty_like(xs)
            for e in range(E):
                a, b = offs[e], offs[e + 1]
                if b > a:
                    xq, xsc = moe.quant_rows_fp8(xs[a:b])
                    y13 = torch._scaled_mm(xq, q13[e].t(), scale_a=xsc[:, None], scale_b=s13[e][None, :],
                                           out_dtype=torch.bfloat16)
                    aq, asc = moe.silu_quant_rows_fp8(y13)
                    ys[a:b] = torch._scaled_mm(aq, q2[e].t(), scale_a=asc[:, None], scale_b=s2[e][None, :],
                                               out_dtype=torch.bfloat16)
            return moe.combine_weighted(ys, order, tok_w, T, K)
        ts = interleaved({"device": lambda: moe.moe_prefill_fp8(h, logits, t13, s13, t2, s2, K),
                          "tiles": lambda: moe.moe_prefill_fp8_tiles(h, logits, q13, s13, q2, s2, K),
                          "loop": loop}, rounds=5, iters=3)
        a = moe.moe_prefill_fp8(h, logits, t13, s13, t2, s2, K).float()
        c = moe.moe_prefill_fp8_tiles(h, logits, q13, s13, q2, s2, K).float()
        b = loop().float()
        flops = 2 * T * K * 3 * H * F_
        out.append({"op": "moe_prefill", "T": T, "device_fp8_us": round(ts["device"], 1),
                    "device_TFLOPs": round(flops / ts["device"] / 1e6, 1),
                    "tiles_fp8_us": round(ts["tiles"], 1), "tiles_TFLOPs": round(flops / ts["tiles"] / 1e6, 1),
                    "hipblaslt_fp8_loop_us": round(ts["loop"], 1), "loop_TFLOPs": round(flops / ts["loop"] / 1e6, 1),
                    "rel_diff_device": round(float((a - b).abs().max() / b.abs().max()), 4),
                    "rel_diff_tiles": round(float((c - b).abs().max() / b.abs().max()), 4)})
        print(json.dumps(out[-1]), flush=True)
    return out


def bench_gemm_hip(dev, Ms=None) -> List[Dict]:
    """Hand-written prefill GEMM (gemm_prefill.hip) vs hipBLASLt on the Llama-3-8B projections at
    the step sizes the scheduler emits, interleaved in one process on the same random operands.
    gate|up is timed with its SiLU epilogue against hipBLASLt + silu_mul; QKV / O / down also at
    split-K S = 2, 4 (f32 slabs, the form their RMSNorm / RoPE consumers read)."""
    from ..ops import gemm
    from ..ops.activation import silu_mul
    out = []
    shapes = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}
    ws = {n: (torch.rand((N, K), device=dev) * 2 - 1).to(torch.bfloat16) * 0.05 for n, (N, K) in shapes.items()}
    Ms = Ms or [256 * k for k in range(1, 17)]
    for M in Ms:
        row = {"op": "gemm_hip", "M": M}
        fl, t_lib, t_hip = 0.0, 0.0, 0.0
        for name, (N, K) in shapes.items():
            x = (torch.rand((M, K), device=dev) * 2 - 1).to(torch.bfloat16)
            w = ws[name]
            f = 2 * M * N * K
            if name == "gate_up":
                lib = timeit(lambda: silu_mul(torch.nn.functional.linear(x, w), interleave16=True), iters=10)
                hip = timeit(lambda: gemm.prefill_gemm(x, w, "silu"), iters=10)
                best = hip
            else:
                lib = timeit(lambda: torch.nn.functional.linear(x, w), iters=10)
                hip = timeit(lambda: gemm.prefill_gemm(x, w), iters=10)
                best = hip
                for S in (2, 4):
                    if K % (64 * S) == 0:
                        P = torch.empty((S, M, N), dtype=torch.float32, device=dev)
                        t = timeit(lambda: gemm.prefill_gemm(x, w, "slabs", S, out=P), iters=10)
                        row[f"{name}_S{S}_TF"] = round(f / t / 1e6, 1)
                        best = min(best, t)
            row[f"{name}_lib_TF"] = round(f / lib / 1e6, 1)
            row[f"{name}_hip_TF"] = round(f / hip / 1e6, 1)
            fl += f
            t_lib += lib
            t_hip += best
        row["layer_lib_TF"] = round(fl / t_lib / 1e6, 1)
        row["layer_hip_best_TF"] = round(fl / t_hip / 1e6, 1)
        print(json.dumps(row), flush=True)
        out.append(row)
    return out


def bench_prefill_policy(dev, Ms=None, model: str = "8b") -> List[Dict]:
    """Each Llama-3-8B (``model="70b"``: Llama-3-70B at TP=1) projection WITH its consumer, as the
    decoder layer runs it at a prefill step of M rows, under every available choice (microseconds;
    same random operands):
      qkv:     hipBLASLt + rope_kv_write | fused QKV+RoPE+KV-write tile kernel
      o, down: hipBLASLt + add&RMSNorm   | tile kernel bf16 + add&RMSNorm | split-K S slabs + slab RMSNorm
               | tile kernel adding the residual in place + RMSNorm (hipR)
      gate_up: hipBLASLt + silu_mul      | tile kernel with the SiLU epilogue
    -> the table ops/gemm.py PREFILL_POLICY is written from."""
    from ..ops import gemm
    from ..ops.activation import silu_mul
    from ..ops.attention import rope_cos_sin, rope_kv_write
    out = []
    H, F_, Hq, Hkv = (8192, 28672, 64, 8) if model == "70b" else (4096, 14336, 32, 8)
    NQ = (Hq + 2 * Hkv) * 128
    rnd = lambda *s: ((torch.rand(s, device=dev) * 2 - 1) * 0.05).to(torch.bfloat16)  # noqa: E731
    w = {"qkv": rnd(NQ, H), "o": rnd(H, Hq * 128), "gate_up": rnd(2 * F_, H), "down": rnd(H, F_)}
    nw = torch.ones(H, dtype=torch.bfloat16, device=dev)
    cs = rope_cos_sin(128, 8192, 500000.0, device=dev)
    Ms = Ms or [256 * k for k in range(1, 17)]
    nb = 4096 // 64 + 4
    kc = torch.zeros((nb, Hkv, 64 * 128), dtype=torch.bfloat16, device=dev)
    vc = torch.zeros_like(kc)
    for M in Ms:
        row = {"op": "prefill_policy", "model": model, "M": M}
        x = rnd(M, H)
        xf = rnd(M, F_)
        res = rnd(M, H)
        pos = torch.arange(M, dtype=torch.int32, device=dev)
        slots = torch.arange(M, dtype=torch.int32, device=dev)
        fns = {}
        fns["qkv_lib"] = lambda: rope_kv_write(torch.nn.functional.linear(x, w["qkv"]), pos, cs, slots, kc, vc,
                                               Hq, Hkv, 128)
        fns["qkv_fused"] = lambda: gemm.prefill_qkv_rope(x, w["qkv"], pos, cs, slots, kc, vc, Hq, Hkv)
        for S in (2, 4):   # split-K slabs summed by the RoPE / KV-write pass
            Pq = torch.empty((S, M, NQ), dtype=torch.float32, device=dev)
            fns[f"qkv_hipS{S}"] = (lambda S=S, Pq=Pq: rope_kv_write(gemm.Slabs(gemm.prefill_gemm(
                x, w["qkv"], "slabs", S, out=Pq)), pos, cs, slots, kc, vc, Hq, Hkv, 128))
        for name, a in (("o", x), ("down", xf)):
            K = a.shape[1]
            fns[f"{name}_lib"] = (lambda a=a, name=name: ops.rms_norm(torch.nn.functional.linear(a, w[name]), nw,
                                                                       1e-5, residual=res))
            fns[f"{name}_hip1"] = (lambda a=a, name=name: ops.rms_norm(gemm.prefill_gemm(a, w[name]), nw, 1e-5,
                                                                        residual=res))
            # residual added in the GEMM epilogue over the residual stream (in place), then a plain
            # RMSNorm: the decoder's fuse_residual path (ops.gemm.ResidualSum)
            fns[f"{name}_hipR"] = (lambda a=a, name=name: ops.rms_norm(gemm.ResidualSum(gemm.prefill_gemm(
                a, w[name], "residual", residual=res, out=res)), nw, 1e-5, residual=res))
            for S in (2, 4):
                if K % (64 * S) == 0:
                    P = torch.empty((S, M, H), dtype=torch.float32, device=dev)
                    fns[f"{name}_hipS{S}"] = (lambda a=a, name=name, S=S, P=P: ops.rms_norm(
                        gemm.Slabs(gemm.prefill_gemm(a, w[name], "slabs", S, out=P)), nw, 1e-5, residual=res))
        fns["gate_up_lib"] = lambda: silu_mul(torch.nn.functional.linear(x, w["gate_up"]), interleave16=True)
        fns["gate_up_hip1"] = lambda: gemm.prefill_gemm(x, w["gate_up"], "silu")
        t = interleaved(fns, rounds=5, iters=5)
        row.update({k: round(v, 1) for k, v in t.items()})
        lib = sum(v for k, v in t.items() if k.endswith("_lib"))
        best = {}
        for p in ("qkv", "o", "gate_up", "down"):
            k = min((k for k in t if k.rsplit("_", 1)[0] == p), key=lambda k: t[k])
            best[p] = k.rsplit("_", 1)[1]
        row["best"] = best
        row["layer_lib_us"] = round(lib, 1)
        row["layer_best_us"] = round(sum(t[f"{p}_{best[p]}"] for p in best), 1)
        print(json.dumps(row), flush=True)
        out.append(row)
    return out


def interleaved(fns: Dict[str, Callable[[], None]], rounds: int = 7, iters: int = 10) -> Dict[str, float]:
    """Median microseconds per call of each variant, timed in interleaved rounds (A B C A B C ...)
    so clock / thermal drift hits every variant alike (cdna_hip_programming.md §5.4 rule 24)."""
    for f in fns.values():
        f()
    torch.cuda.synchronize()
    res: Dict[str, List[float]] = {k: [] for k in fns}
    for _ in range(rounds):
        for k, f in fns.items():
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record()
            for _ in range(iters):
                f()
            b.record()
            b.synchronize()
            res[k].append(a.elapsed_time(b) * 1e3 / iters)
    return {k: statistics.median(v) for k, v in res.items()}


def bench_gemm_ablate(dev) -> List[Dict]:
    """Where the prefill tile kernel's cycles go: full kernel vs no LDS-DMA in the K loop vs no
    fragment reads, for one tile alone (one CU) and for a full chip (M = 4096, N = 4096)."""
    from ..ops import _native as Nn
    out = []
    for M, N_, K in [(256, 256, 32768), (4096, 4096, 4096), (4096, 28672, 4096), (2048, 6144, 4096),
                     (4096, 4096, 14336)]:
        x = ((torch.rand((M, K), device=dev) * 2 - 1) * 0.5).to(torch.bfloat16)
        w = ((torch.rand((N_, K), device=dev) * 2 - 1) * 0.05).to(torch.bfloat16)
        y = torch.empty((M, N_), dtype=torch.bfloat16, device=dev)
        row = {"op": "gemm_ablate", "M": M, "N": N_, "K": K}
        variants = ((0, "full"), (1, "no_glds"), (2, "no_dsread"), (3, "no_vmwait"), (10, "bal0"))

        def mk(ab):
            return lambda: Nn.call("penny_gemm_prefill_ablate", Nn.ptr(x), K, Nn.ptr(w), K, Nn.ptr(y), N_, M, N_, ab,
                                   Nn.stream())
        ts = interleaved({name: mk(ab) for ab, name in variants})
        for name, us in ts.items():
            row[name + "_us"] = round(us, 1)
            row[name + "_TF"] = round(2 * M * N_ * K / us / 1e6, 1)
        ref = x.float() @ w.float().t()
        for ab, name in ((0, "full"), (10, "bal0")):
            Nn.call("penny_gemm_prefill_ablate", Nn.ptr(x), K, Nn.ptr(w), K, Nn.ptr(y), N_, M, N_, ab, Nn.stream())
            row[name + "_err"] = round(float((y.float() - ref).abs().max() / ref.abs().max()), 4)
        print(json.dumps(row), flush=True)
        out.append(row)
    return out


def check_gemm_hip(dev) -> List[Dict]:
    """Numerics of gemm_prefill.hip against an f32 reference at odd M, every epilogue."""
    from ..ops import gemm
    out = []
    g = torch.Generator(device=dev).manual_seed(0)
    for M, N, K, epi, S in [(1, 256, 64, None, 1), (300, 512, 256, None, 1), (257, 768, 4096, "silu", 1),
                            (1000, 1024, 1024, "slabs", 4), (4096, 6144, 4096, None, 1), (513, 4096, 14336, "slabs", 2),
                            (777, 512, 512, "residual", 1)]:
        x = torch.randn((M, K), generator=g, device=dev).to(torch.bfloat16)
        w = (torch.randn((N, K), generator=g, device=dev) * 0.05).to(torch.bfloat16)
        r = torch.randn((M, N), generator=g, device=dev).to(torch.bfloat16) if epi == "residual" else None
        y = gemm.prefill_gemm(x, w, epi, S, residual=r)
        ref = x.float() @ w.float().t()
        if epi == "silu":
            from ..ops.activation import silu_mul
            ref = silu_mul(ref.to(torch.bfloat16), interleave16=True).float()
            got = y.float()
        elif epi == "slabs":
            got = y.sum(0)
        elif epi == "residual":
            ref = ref + r.float()
            got = y.float()
        else:
            got = y.float()
        err = float((got - ref).abs().max() / ref.abs().max())
        out.append({"op": "gemm_hip_check", "M": M, "N": N, "K": K, "epi": epi, "S": S, "rel_err": round(err, 5)})
        print(json.dumps(out[-1]), flush=True)
    # fused QKV + RoPE + KV write vs hipBLASLt + rope_kv_write
    from ..ops.attention import rope_cos_sin, rope_kv_write
    Hq, Hkv, K = 32, 8, 4096
    cs = rope_cos_sin(128, 8192, 500000.0, device=dev)
    for M in (300, 2048):
        x = torch.randn((M, K), generator=g, device=dev).to(torch.bfloat16)
        w = (torch.randn(((Hq + 2 * Hkv) * 128, K), generator=g, device=dev) * 0.02).to(torch.bfloat16)
        pos = torch.randint(0, 8000, (M,), generator=g, device=dev, dtype=torch.int32)
        nb = (M + 63) // 64 + 2
        perm = torch.randperm(nb * 64, generator=g, device=dev)[:M].to(torch.int32)
        slots = torch.where(torch.arange(M, device=dev) % 7 == 3, torch.full_like(perm, -1), perm)
        kc = [torch.zeros((nb, Hkv, 64 * 128), dtype=torch.bfloat16, device=dev) for _ in range(2)]
        vc = [torch.zeros((nb, Hkv, 64 * 128), dtype=torch.bfloat16, device=dev) for _ in range(2)]
        q0 = rope_kv_write(torch.nn.functional.linear(x, w), pos, cs, slots, kc[0], vc[0], Hq, Hkv, 128)
        q1 = gemm.prefill_qkv_rope(x, w, pos, cs, slots, kc[1], vc[1], Hq, Hkv)
        errs = [float((a.float() - b.float()).abs().max()) for a, b in ((q0, q1), (kc[0], kc[1]), (vc[0], vc[1]))]
        out.append({"op": "gemm_hip_check_qkv_rope", "M": M, "max_abs_err_q_k_v": [round(e, 4) for e in errs],
                    "scale": round(float(q0.float().abs().max()), 3)})
        print(json.dumps(out[-1]), flush=True)
    return out


def gemm_lds_probe(dev) -> List[Dict]:
    """A few launches of the bf16 tile GEMM (4096^3) and of the grouped fp8 MoE tile GEMMs, for
    rocprofv3 --pmc runs (LDS bank-conflict counters of the swizzled fragment reads)."""
    from ..ops import gemm, moe
    x = (torch.randn((4096, 4096), device=dev) * 0.5).to(torch.bfloat16)
    w = (torch.randn((4096, 4096), device=dev) * 0.05).to(torch.bfloat16)
    for _ in range(5):
        gemm.prefill_gemm(x, w, None, 1)
    E, H, F_ = 8, 4096, 14336
    w13q = torch.randint(0, 120, (E, 2 * F_, H), dtype=torch.uint8, device=dev)
    w2q = torch.randint(0, 120, (E, H, F_), dtype=torch.uint8, device=dev)
    s13 = torch.full((E, 2 * F_), 1e-3, device=dev)
    s2 = torch.full((E, H), 1e-3, device=dev)
    h = torch.randn((4096, H), device=dev).to(torch.bfloat16)
    logits = torch.randn((4096, E), device=dev).to(torch.bfloat16)
    for _ in range(3):
        moe.moe_prefill_fp8_tiles(h, logits, w13q, s13, w2q, s2, 2)
    torch.cuda.synchronize()
    return [{"op": "gemm_lds_probe", "done": True}]


# Every projection shape of the north-star config 4 (Llama-3-70B) that is not an 8B shape: the TP=8
# per-rank shards and the TP=1 weights.  kind: "col" = column-parallel
# output consumed by a row pass that reads split-K slabs (QKV -> RoPE/KV write), "row" = row-parallel
# output into the all-reduce (bf16), "gateup" = interleave16 gate|up with the fused SiLU*up.
SHARD_SHAPES = {
    "70b_tp8_qkv": (1280, 8192, "col"), "70b_tp8_o": (8192, 1024, "row"),
    "70b_tp8_gate_up": (7168, 8192, "gateup"), "70b_tp8_down": (8192, 3584, "row"),
    "70b_tp1_qkv": (10240, 8192, "col"), "70b_tp1_gate_up": (57344, 8192, "gateup"),
    "70b_tp1_o": (8192, 8192, "col"), "70b_tp1_down": (8192, 28672, "col"),
    "8b_gate_up": (28672, 4096, "gateup"),     # the 8B shape above the fused kernel's 160 rows
    # the 8B decode projections (TP=1: slabs read by the consumer), re-swept at HEAD
    "8b_qkv": (6144, 4096, "col"), "8b_o": (4096, 4096, "col"), "8b_down": (4096, 14336, "col"),
}


def bench_rm_pair(dev, names=("70b_tp8_o", "70b_tp8_down", "70b_tp8_qkv", "70b_tp8_gate_up", "70b_tp1_qkv", "70b_tp1_o",
                                "70b_tp1_down", "70b_tp1_gate_up", "8b_qkv", "8b_o", "8b_down", "8b_gate_up"),
                  Ms=(1, 8, 16, 32, 64, 96, 128, 192, 256)) -> List[Dict]:
    """Decode GEMM streams with BK=64 stages issued singly vs in pairs (gemm.PAIR_MODE / BKM = 2),
    per (S, nf) config, in the W layout the model streams at that shape (fragment-tiled where
    ``uses_tiled_weight``, else row-major), hipBLASLt as the reference; interleaved per M, weights
    rotated over >= 768 MB.  The paired stream must be bit-identical to the single one (same k order):
    checked per config."""
    from ..ops import gemm
    from ..ops.activation import silu_mul
    out = []
    rnd = lambda *s: ((torch.rand(s, device=dev) * 2 - 1) * 0.05).to(torch.bfloat16)  # noqa: E731

    def mode(f, m):
        def g():
            gemm.PAIR_MODE = m
            try:
                return f()
            finally:
                gemm.PAIR_MODE = "table"
        return g
    for name in names:
        N, K, kind = SHARD_SHAPES[name]
        rm = not gemm.uses_tiled_weight(N, K)
        copies = max(2, min(16, (768 << 20) // (N * K * 2)))
        ws = [rnd(N, K) for _ in range(copies)]
        w_lib = ws                      # hipBLASLt reads the row-major weights
        if not rm:
            ws = [gemm.tile_weight(w) for w in ws]
        it = [0]

        def nxt():
            it[0] = (it[0] + 1) % copies
            return it[0]
        for M in Ms:
            x = rnd(M, K)
            fns = {}
            if kind == "gateup":
                fns["lib"] = lambda: silu_mul(torch.nn.functional.linear(x, w_lib[nxt()]), interleave16=True)
                for nf in (4, 8):
                    fns[f"gu_nf{nf}"] = lambda nf=nf: gemm.gateup_silu(x, ws[nxt()], N, nf, rowmajor=rm)
                for S, nf in ((2, 2), (4, 2), (8, 2), (2, 4), (4, 4), (2, 8), (4, 8)):
                    if K % (128 * S) or N % (32 * nf):
                        continue
                    P = torch.empty((S, M, N), dtype=torch.float32, device=dev)
                    y = torch.empty((M, N // 2), dtype=torch.bfloat16, device=dev)
                    fns[f"guS{S}nf{nf}"] = (lambda S=S, nf=nf, P=P, y=y: gemm.gateup_splitk(
                        x, ws[nxt()], N, S, nf, rowmajor=rm, slabs=P, out=y))
            else:
                fns["lib"] = lambda: torch.nn.functional.linear(x, w_lib[nxt()])
                if kind == "row":
                    for nf in (2, 4, 8):
                        fns[f"bf16_nf{nf}"] = lambda nf=nf: gemm.splitk_bf16(x, ws[nxt()], N, nf, rowmajor=rm)
                for S in (1, 2, 4, 8):
                    for nf in (2, 4, 6, 8):
                        if K % (128 * S) or N % (16 * nf) or (N // (16 * nf)) * S < 128:
                            continue
                        P = torch.empty((S, M, N), dtype=torch.float32, device=dev)
                        if kind == "row":
                            y = torch.empty((M, N), dtype=torch.bfloat16, device=dev)
                            fns[f"S{S}nf{nf}+red"] = (lambda S=S, nf=nf, P=P, y=y: gemm.splitk_reduce(
                                gemm.splitk_partials(x, ws[nxt()], N, S, nf, out=P, rowmajor=rm), out=y))
                        else:
                            fns[f"S{S}nf{nf}"] = (lambda S=S, nf=nf, P=P: gemm.splitk_partials(
                                x, ws[nxt()], N, S, nf, out=P, rowmajor=rm))
            same = {}
            for k in [k for k in fns if k != "lib"]:
                f = fns[k]
                it[0] = copies - 1
                a = mode(f, "0")()
                it[0] = copies - 1
                b = mode(f, "1")()
                same[k] = bool(torch.equal(a, b))
                fns[k] = mode(f, "0")
                fns[k + "_p"] = mode(f, "1")
            t = interleaved(fns, rounds=5, iters=copies)
            single = min((k for k in t if k != "lib" and not k.endswith("_p")), key=lambda k: t[k])
            pair = min((k for k in t if k.endswith("_p")), key=lambda k: t[k])
            row = {"op": "rm_pair", "name": name, "N": N, "K": K, "kind": kind, "rowmajor": rm, "M": M,
                   **{k: round(v, 1) for k, v in t.items()}, "best_single": single, "best_pair": pair,
                   "pair_gain": round(t[single] / t[pair], 3), "pair_vs_lib": round(t["lib"] / t[pair], 3),
                   "pair_GBps": round(N * K * 2 / t[pair] / 1e3, 1), "bit_identical": all(same.values())}
            print(json.dumps(row), flush=True)
            out.append(row)
        del ws, w_lib
        torch.cuda.empty_cache()
    return out


def bench_chunked_prefill(dev, names=("70b_tp8_qkv", "70b_tp8_o", "70b_tp8_gate_up", "70b_tp8_down", "70b_tp1_qkv",
                                       "8b_qkv", "8b_o"),
                          Ms=(384, 512, 768, 1024, 1536, 2048)) -> List[Dict]:
    """Small prefill steps (M > 256) on the decode split-K kernels with 256-row token chunks side by
    side (grid y), vs the production path (``gemm.linear``: PREFILL_POLICY's library / tile-kernel
    choice), hipBLASLt and the tile kernel, interleaved per M.  W in the layout the model keeps at that
    shape.  "col" rows also report ``adj``: the time plus the consumer's extra slab read
    ((4S - 2) * M * N bytes at 5 TB/s) against a bf16 output."""
    from ..ops import gemm
    from ..ops.activation import silu_mul
    out = []
    rnd = lambda *s: ((torch.rand(s, device=dev) * 2 - 1) * 0.05).to(torch.bfloat16)  # noqa: E731
    for name in names:
        N, K, kind = SHARD_SHAPES[name]
        rm = not gemm.uses_tiled_weight(N, K)
        copies = max(2, min(16, (768 << 20) // (N * K * 2)))
        ws = [rnd(N, K) for _ in range(copies)]
        wts = [gemm.tile_weight(w) for w in ws] if not rm else ws
        it = [0]

        def nxt():
            it[0] = (it[0] + 1) % copies
            return it[0]
        for M in Ms:
            x = rnd(M, K)
            fns, extra = {}, {}
            if kind == "gateup":
                fns["lib"] = lambda: silu_mul(torch.nn.functional.linear(x, ws[nxt()]), interleave16=True)
                fns["prod"] = lambda: gemm.linear(x, ws[nxt()], epilogue="silu", wt=None if rm else wts[it[0]])
                fns["tile"] = lambda: gemm.prefill_gemm(x, ws[nxt()], "silu")
                for nf in (2, 4, 8):
                    fns[f"ch_gu_nf{nf}"] = lambda nf=nf: gemm.gateup_silu(x, wts[nxt()], N, nf, rowmajor=rm)
                for S, nf in ((2, 2), (2, 4), (4, 4), (2, 8)):
                    if K % (64 * S) or N % (32 * nf):
                        continue
                    P = torch.empty((S, M, N), dtype=torch.float32, device=dev)
                    y = torch.empty((M, N // 2), dtype=torch.bfloat16, device=dev)
                    fns[f"ch_guS{S}nf{nf}"] = (lambda S=S, nf=nf, P=P, y=y: gemm.gateup_splitk(
                        x, wts[nxt()], N, S, nf, rowmajor=rm, slabs=P, out=y))
            elif kind == "row":
                fns["lib"] = lambda: torch.nn.functional.linear(x, ws[nxt()])
                fns["prod"] = lambda: gemm.linear(x, ws[nxt()], wt=None if rm else wts[it[0]])
                fns["tile"] = lambda: gemm.prefill_gemm(x, ws[nxt()])
                for nf in (2, 4, 8):
                    fns[f"ch_bf16_nf{nf}"] = lambda nf=nf: gemm.splitk_bf16(x, wts[nxt()], N, nf, rowmajor=rm)
                for S, nf in ((2, 4), (4, 4), (2, 8)):
                    if K % (64 * S) or N % (16 * nf):
                        continue
                    P = torch.empty((S, M, N), dtype=torch.float32, device=dev)
                    y = torch.empty((M, N), dtype=torch.bfloat16, device=dev)
                    fns[f"ch_S{S}nf{nf}+red"] = (lambda S=S, nf=nf, P=P, y=y: gemm.splitk_reduce(
                        gemm.splitk_partials(x, wts[nxt()], N, S, nf, out=P, rowmajor=rm), out=y))
            else:
                fns["lib"] = lambda: torch.nn.functional.linear(x, ws[nxt()])
                fns["prod"] = lambda: gemm.linear(x, ws[nxt()], wt=None if rm else wts[it[0]], slabs=True)
                for S in (2, 4):
                    if K % (64 * S) == 0:
                        fns[f"tileS{S}"] = lambda S=S: gemm.prefill_gemm(x, ws[nxt()], "slabs", S)
                        extra[f"tileS{S}"] = (4 * S - 2) * M * N / 5e6
                for S in (1, 2, 4, 8):
                    for nf in (2, 4, 6, 8):
                        if K % (64 * S) or N % (16 * nf):
                            continue
                        P = torch.empty((S, M, N), dtype=torch.float32, device=dev)
                        fns[f"ch_S{S}nf{nf}"] = (lambda S=S, nf=nf, P=P: gemm.splitk_partials(
                            x, wts[nxt()], N, S, nf, out=P, rowmajor=rm))
                        extra[f"ch_S{S}nf{nf}"] = (4 * S - 2) * M * N / 5e6
            t = interleaved(fns, rounds=5, iters=copies)
            adj = {k: t[k] + extra.get(k, 0.0) for k in t}
            best = min((k for k in t if k.startswith("ch_")), key=lambda k: adj[k])
            row = {"op": "chunked_prefill", "name": name, "N": N, "K": K, "kind": kind, "rowmajor": rm, "M": M,
                   **{k: round(v, 1) for k, v in t.items()}, "best_chunked": best, "best_adj_us": round(adj[best], 1),
                   "prod_us": round(t["prod"], 1), "chunked_vs_prod": round(adj["prod"] / adj[best], 3),
                   "chunked_vs_lib": round(t["lib"] / adj[best], 3)}
            print(json.dumps(row), flush=True)
            out.append(row)
        del ws, wts
        torch.cuda.empty_cache()
    return out


def bench_gemm_group(dev, Ms=(1024, 2048, 2560, 3072, 4096), groups=(1, 2, 4, 8, 16)) -> List[Dict]:
    """The tile GEMM's L2 grouping (token tiles per group of each XCD's tile range; gemm_prefill.hip
    GM = 4) swept on the Llama-3-8B prefill projections with their production epilogues, interleaved
    per M."""
    from ..ops import gemm
    from ..ops import _native as Nn
    out = []
    rnd = lambda *s: ((torch.rand(s, device=dev) * 2 - 1) * 0.05).to(torch.bfloat16)  # noqa: E731
    shapes = {"gate_up": (28672, 4096, "silu"), "down": (4096, 14336, "residual"), "qkv": (6144, 4096, None),
              "o": (4096, 4096, "residual")}
    for name, (N, K, epi) in shapes.items():
        w = rnd(N, K)
        for M in Ms:
            x = rnd(M, K)
            r = rnd(M, N) if epi == "residual" else None

            def mk(g):
                def f():
                    Nn.call("penny_gemm_prefill_set_group", g)
                    gemm.prefill_gemm(x, w, epi, residual=r, out=r if epi == "residual" else None)
                    Nn.call("penny_gemm_prefill_set_group", 0)
                return f
            t = interleaved({f"gm{g}": mk(g) for g in groups}, rounds=5, iters=10)
            fl = 2 * M * N * K
            row = {"op": "gemm_group", "name": name, "M": M, "N": N, "K": K,
                   **{k: round(v, 1) for k, v in t.items()},
                   "best": min(t, key=t.get), "gm4_TF": round(fl / t["gm4"] / 1e6, 1)}
            print(json.dumps(row), flush=True)
            out.append(row)
    return out


def bench_gemm_tiled_w(dev, Ms=(512, 1024, 2048, 3072, 4096)) -> List[Dict]:
    """The prefill tile kernel on the fragment-tiled weight vs the row-major one (same epilogue),
    interleaved per M: could a shape keep only the decode kernels' tiled copy?"""
    from ..ops import gemm
    out = []
    rnd = lambda *s: ((torch.rand(s, device=dev) * 2 - 1) * 0.05).to(torch.bfloat16)  # noqa: E731
    shapes = {"8b_gate_up": (28672, 4096, "silu"), "8b_down": (4096, 14336, None), "8b_qkv": (6144, 4096, None),
              "70b_tp1_gate_up": (57344, 8192, "silu")}
    for name, (N, K, epi) in shapes.items():
        w = rnd(N, K)
        wt = gemm.tile_weight(w)
        for M in Ms:
            x = rnd(M, K)
            t = interleaved({"rowmajor": lambda: gemm.prefill_gemm(x, w, epi),
                             "tiled": lambda: gemm.prefill_gemm_tiled(x, wt, N, epi)}, rounds=5, iters=5)
            row = {"op": "gemm_tiled_w", "name": name, "M": M, **{k: round(v, 1) for k, v in t.items()},
                   "tiled_gain": round(t["rowmajor"] / t["tiled"], 3),
                   "tiled_TF": round(2 * M * N * K / t["tiled"] / 1e6, 1)}
            print(json.dumps(row), flush=True)
            out.append(row)
        del w, wt
        torch.cuda.empty_cache()
    return out


def bench_shard_shapes(dev, names=None, Ms=(1, 8, 16, 32, 64, 96, 128, 192, 256),
                       prefill_Ms=(384, 512, 768, 1024, 1536, 2048, 3072, 4096)) -> List[Dict]:
    """Decode and prefill kernels vs hipBLASLt at the 70B shard / TP=1 shapes, interleaved per M in
    one process (rule 24), weights rotated over >= 768 MB so every decode call streams HBM.

    decode (M <= 256): lib = F.linear (+ silu_mul); "row": bf16-output kernel nf x {row-major,
    tiled}, and split-K slabs + reduce; "col": split-K slabs (gemm-only time: the consumer reads
    them) per (S, nf); "gateup": fused gate|up kernel per nf.  prefill (M > 256): lib vs the tile
    kernel (bf16 / SiLU), split-K slabs S = 2, 4 (+ reduce for "row")."""
    from ..ops import gemm
    from ..ops.activation import silu_mul
    out = []
    rnd = lambda *s: ((torch.rand(s, device=dev) * 2 - 1) * 0.05).to(torch.bfloat16)  # noqa: E731
    for name, (N, K, kind) in SHARD_SHAPES.items():
        if names and name not in names:
            continue
        copies = max(2, min(16, (768 << 20) // (N * K * 2)))
        ws = [rnd(N, K) for _ in range(copies)]
        wts = [gemm.tile_weight(w) for w in ws]
        it = [0]

        def nxt():
            it[0] = (it[0] + 1) % copies
            return it[0]
        wbytes = N * K * 2
        for M in Ms:
            x = rnd(M, K)
            fns = {}
            if kind == "gateup":
                fns["lib"] = lambda: silu_mul(torch.nn.functional.linear(x, ws[nxt()]), interleave16=True)
                for nf in (2, 4, 8):
                    if N % (16 * nf) == 0:
                        fns[f"gu_nf{nf}_tiled"] = lambda nf=nf: gemm.gateup_silu(x, wts[nxt()], N, nf)
                        fns[f"gu_nf{nf}_rm"] = lambda nf=nf: gemm.gateup_silu(x, ws[nxt()], N, nf, rowmajor=True)
                # split-K slabs + the reduce-SiLU pass (gemm.gateup_splitk)
                for S in (2, 4, 8):
                    for nf in (2, 4, 8):
                        if K % (64 * S) or N % (32 * nf):
                            continue
                        P = torch.empty((S, M, N), dtype=torch.float32, device=dev)
                        y = torch.empty((M, N // 2), dtype=torch.bfloat16, device=dev)
                        fns[f"guS{S}nf{nf}_rm"] = (lambda S=S, nf=nf, P=P, y=y: gemm.gateup_splitk(
                            x, ws[nxt()], N, S, nf, rowmajor=True, slabs=P, out=y))
                        fns[f"guS{S}nf{nf}_tiled"] = (lambda S=S, nf=nf, P=P, y=y: gemm.gateup_splitk(
                            x, wts[nxt()], N, S, nf, slabs=P, out=y))
            else:
                fns["lib"] = lambda: torch.nn.functional.linear(x, ws[nxt()])
                if kind == "row":
                    for nf in (2, 4, 8):
                        if N % (16 * nf) == 0:
                            fns[f"bf16_nf{nf}_rm"] = lambda nf=nf: gemm.splitk_bf16(x, ws[nxt()], N, nf)
                            fns[f"bf16_nf{nf}_tiled"] = lambda nf=nf: gemm.splitk_bf16(x, wts[nxt()], N, nf,
                                                                                       rowmajor=False)
                for S in (2, 4, 8):
                    for nf in (2, 4, 8):
                        if K % (64 * S) or N % (16 * nf):
                            continue
                        P = torch.empty((S, M, N), dtype=torch.float32, device=dev)
                        y = torch.empty((M, N), dtype=torch.bfloat16, device=dev)
                        if kind == "row":   # the all-reduce needs the reduced bf16 output
                            fns[f"S{S}nf{nf}_rm+red"] = (lambda S=S, nf=nf, P=P, y=y: gemm.splitk_reduce(
                                gemm.splitk_partials(x, ws[nxt()], N, S, nf, out=P, rowmajor=True), out=y))
                        else:
                            fns[f"S{S}nf{nf}_rm"] = (lambda S=S, nf=nf, P=P: gemm.splitk_partials(
                                x, ws[nxt()], N, S, nf, out=P, rowmajor=True))
                            fns[f"S{S}nf{nf}_tiled"] = (lambda S=S, nf=nf, P=P: gemm.splitk_partials(
                                x, wts[nxt()], N, S, nf, out=P))
            t = interleaved(fns, rounds=5, iters=copies)
            best = min((k for k in t if k != "lib"), key=lambda k: t[k])
            row = {"op": "shard_shapes", "name": name, "N": N, "K": K, "kind": kind, "M": M,
                   **{k: round(v, 1) for k, v in t.items()}, "best": best, "best_us": round(t[best], 1),
                   "best_GBps": round(wbytes / t[best] / 1e3, 1), "speedup": round(t["lib"] / t[best], 2)}
            print(json.dumps(row), flush=True)
            out.append(row)
        del ws, wts
        torch.cuda.empty_cache()
        w = rnd(N, K)
        for M in prefill_Ms:
            x = rnd(M, K)
            fns = {}
            if kind == "gateup":
                fns["lib"] = lambda: silu_mul(torch.nn.functional.linear(x, w), interleave16=True)
                fns["hip"] = lambda: gemm.prefill_gemm(x, w, "silu")
            else:
                fns["lib"] = lambda: torch.nn.functional.linear(x, w)
                if N % 256 == 0:
                    fns["hip"] = lambda: gemm.prefill_gemm(x, w)
                    for S in (2, 4):
                        if K % (64 * S) == 0:
                            P = torch.empty((S, M, N), dtype=torch.float32, device=dev)
                            if kind == "row":
                                y = torch.empty((M, N), dtype=torch.bfloat16, device=dev)
                                fns[f"hipS{S}+red"] = (lambda S=S, P=P, y=y: gemm.splitk_reduce(
                                    gemm.prefill_gemm(x, w, "slabs", S, out=P), out=y))
                            else:
                                fns[f"hipS{S}"] = lambda S=S, P=P: gemm.prefill_gemm(x, w, "slabs", S, out=P)
            # the 128 x 128 tile kernel (gemm_mid.hip) with S K-slices, in the form each consumer takes
            for S in (1, 2, 3, 4, 8):
                if K % (64 * S) or N % 128:
                    continue
                for v in (0, 1, 2):
                    def mf(S=S, v=v):
                        gemm.mid_variant(v)
                        return gemm.mid_linear(x, w, S, "silu" if kind == "gateup" else None, slabs=kind == "col")
                    fns[f"mid{S}v{v}"] = mf
            t = interleaved(fns, rounds=5, iters=5)
            best = min((k for k in t if k != "lib"), key=lambda k: t[k]) if len(t) > 1 else "lib"
            row = {"op": "shard_shapes_prefill", "name": name, "N": N, "K": K, "kind": kind, "M": M,
                   **{k: round(v, 1) for k, v in t.items()}, "best": best,
                   "best_TF": round(2 * M * N * K / t[best] / 1e6, 1), "speedup": round(t["lib"] / t[best], 2)}
            print(json.dumps(row), flush=True)
            out.append(row)
        del w
        torch.cuda.empty_cache()
    return out


def bench_mid_decode(dev, Ms=(64, 96, 128, 192, 256)) -> List[Dict]:
    """The 8B decode projections at B = 64-256: the production decode path
    (``gemm.linear`` on the tiled weight: split-K slabs / fused gate|up) against the 128 x 128 tile
    kernel with S K-slices (row-major W), weights rotated over >= 768 MB so every call streams HBM.
    Reports TB/s of weight bytes."""
    from ..ops import gemm
    out = []
    rnd = lambda *s: ((torch.rand(s, device=dev) * 2 - 1) * 0.05).to(torch.bfloat16)  # noqa: E731
    shapes = {"8b_qkv": (6144, 4096, None), "8b_o": (4096, 4096, None), "8b_down": (4096, 14336, None),
              "8b_gate_up": (28672, 4096, "silu")}
    for name, (N, K, epi) in shapes.items():
        copies = max(2, min(16, (768 << 20) // (N * K * 2)))
        ws = [rnd(N, K) for _ in range(copies)]
        wts = [gemm.tile_weight(w) for w in ws]
        it = [0]

        def nxt():
            it[0] = (it[0] + 1) % copies
            return it[0]
        for M in Ms:
            x = rnd(M, K)
            fns = {"prod": lambda: gemm.linear(x, ws[it[0]], epilogue=epi, wt=wts[nxt()], slabs=epi is None)}
            for S in (1, 2, 4, 8):
                if K % (64 * S):
                    continue
                fns[f"mid{S}"] = lambda S=S: gemm.mid_linear(x, ws[nxt()], S, epi, slabs=epi is None)
            t = interleaved(fns, rounds=5, iters=copies)
            best = min((k for k in t if k != "prod"), key=lambda k: t[k])
            row = {"op": "mid_decode", "name": name, "N": N, "K": K, "M": M, **{k: round(v, 1) for k, v in t.items()},
                   "prod_TBps": round(N * K * 2 / t["prod"] / 1e6, 2), "best_mid": best,
                   "best_mid_TBps": round(N * K * 2 / t[best] / 1e6, 2)}
            print(json.dumps(row), flush=True)
            out.append(row)
        del ws, wts
        torch.cuda.empty_cache()
    return out


def bench_lm_head_stream(dev, V: int = 128256, K: int = 4096,
                         Ms=(1, 2, 4, 8, 16, 32, 48, 64, 96, 127)) -> List[Dict]:
    """LM head + sampler at decode sizes: hipBLASLt logits + the HIP sampler vs the 256x256 tile
    kernel with the sampler epilogue vs the weight-streaming split-K kernel (SK_SAMPLE) per
    (nf, row-major / tiled W, ring), W rotated so every call streams HBM.  ``same``: the streamed
    tokens equal ops.sample over the SK_BF16 logits of the same kernel shape (bitwise)."""
    from ..ops import gemm
    out = []
    copies = max(2, min(8, (2048 << 20) // (V * K * 2)))
    ws = [((torch.rand((V, K), device=dev) * 2 - 1) * 0.05).to(torch.bfloat16) for _ in range(copies)]
    wts = [gemm.tile_weight(w) for w in ws]
    it = [0]

    def nxt():
        it[0] = (it[0] + 1) % copies
        return it[0]
    for M in Ms:
        x = torch.randn((M, K), device=dev).to(torch.bfloat16)
        t_ = torch.full((M,), 0.5, device=dev)
        sd = torch.arange(M, device=dev, dtype=torch.int64) * 7919 + 13
        fns = {"lib_sampler": lambda: ops.sample(torch.nn.functional.linear(x, ws[nxt()]), t_, sd)}
        import os
        os.environ["PENNY_LM_STREAM"] = "0"     # ops.lm_head_sample -> the 256x256 tile kernel

        def tile():
            return ops.lm_head_sample(x, ws[nxt()], t_, sd)
        fns["tile_fused"] = tile
        for nf in (4, 8):
            for rm in (True, False):
                for r2 in (False, True):
                    fns[f"stream_nf{nf}_{'rm' if rm else 'tiled'}{'_r2' if r2 else ''}"] = (
                        lambda nf=nf, rm=rm, r2=r2: ops.lm_head_stream_sample(
                            x, ws[nxt()] if rm else wts[nxt()], t_, sd, nf=nf, rowmajor=rm, ring2=r2))
        t = interleaved(fns, rounds=5, iters=copies)
        os.environ.pop("PENNY_LM_STREAM", None)
        w0 = ws[0]
        ref = ops.sample(gemm.splitk_bf16(x, w0, V, 8), t_, sd)
        got = ops.lm_head_stream_sample(x, w0, t_, sd, nf=8, rowmajor=True)
        best = min((k for k in t if k.startswith("stream")), key=lambda k: t[k])
        row = {"op": "lm_head_stream", "M": M, **{k: round(v, 1) for k, v in t.items()}, "best": best,
               "best_TBps": round(V * K * 2 / t[best] / 1e6, 2), "speedup_vs_lib": round(t["lib_sampler"] / t[best], 2),
               "same_tokens_as_unfused_on_equal_logits": bool(torch.equal(ref, got))}
        print(json.dumps(row), flush=True)
        out.append(row)
    return out


def interleave16_rows(w: torch.Tensor) -> torch.Tensor:
    from ..ops.gemm import interleave16
    half = w.shape[0] // 2
    return interleave16(w[:half], w[half:])


def main(argv=None) -> int:
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="decode,prefill,elementwise,topk")
    ap.add_argument("--out", default="")
    args = ap.parse_args(argv)
    dev = torch.device("cuda")
    res = []
    for name in args.only.split(","):
        res += {"decode": bench_decode, "decode_mixed": bench_decode_mixed, "decode_lean": bench_decode_lean, "prefill": bench_prefill, "prefill_mixed": bench_prefill_mixed, "prefill_spec_split": bench_prefill_spec_split, "elementwise": bench_elementwise,
                "topk": bench_topk, "gemm": bench_gemm, "gemm_prefill": bench_gemm_prefill, "lm_head": bench_lm_head, "lm_head_fused": bench_lm_head_fused, "bge_query": bench_bge_query, "gemm_tail": bench_gemm_tail,
                "gemm_tune": bench_gemm_tune_sweep, "skinny": bench_skinny, "splitk": bench_splitk,
                "splitk_qkv": lambda d: bench_splitk(d, ("qkv",)), "gateup": bench_gateup, "moe": bench_moe,
                "moe_prefill": bench_moe_prefill, "gemm_hip": bench_gemm_hip, "gemm_hip_quick": lambda d: bench_gemm_hip(d, [512, 1024, 2048, 3072, 4096]), "gemm_hip_check": check_gemm_hip, "gemm_lds_probe": gemm_lds_probe, "prefill_policy": bench_prefill_policy, "prefill_policy_quick": lambda d: bench_prefill_policy(d, [512, 1024, 1536, 2048, 2560, 3072, 3584, 4096]), "prefill_policy_70b": lambda d: bench_prefill_policy(d, [384, 512, 768, 1024, 1536, 2048, 2560, 3072, 4096], model="70b"),
                "prefill_policy_small": lambda d: bench_prefill_policy(d, [512, 768, 1024, 1280, 1536]), "gemm_ablate": bench_gemm_ablate,
                "splitk70b": lambda d: bench_splitk(d, ("qkv", "o", "down"), SHAPES_70B),
                "gateup70b": lambda d: bench_gateup(d, 57344, 8192),
                "splitk70b_tp8": lambda d: bench_splitk(d, ("qkv", "o", "down"), SHAPES_70B_TP8),
                "gateup70b_tp8": lambda d: bench_gateup(d, 7168, 8192),
                "shard_shapes": bench_shard_shapes,
                "mid_decode": bench_mid_decode,
                "attn_overlap": bench_attn_overlap,
                "mid_8b": lambda d: bench_shard_shapes(d, names=("8b_qkv", "8b_o", "8b_down", "8b_gate_up"), Ms=(),
                                                       prefill_Ms=(320, 384, 512, 768, 1024, 1536, 2048)),
                "mid_shards": lambda d: bench_shard_shapes(d, names=("70b_tp8_qkv", "70b_tp8_o", "70b_tp8_gate_up",
                                                                     "70b_tp8_down", "70b_tp1_qkv"), Ms=()), "rm_pair": bench_rm_pair, "gemm_tiled_w": bench_gemm_tiled_w, "gemm_group": bench_gemm_group,
                "rm_pair_wide": lambda d: bench_rm_pair(d, names=("8b_qkv", "8b_o", "8b_down", "8b_gate_up", "70b_tp8_qkv",
                                                                  "70b_tp8_gate_up", "70b_tp8_down"),
                                                        Ms=(96, 112, 128, 144, 160, 192, 256)), "chunked_prefill": bench_chunked_prefill,
                "shard_shapes_tp8": lambda d: bench_shard_shapes(d, [n for n in SHARD_SHAPES if "tp8" in n]),
                "shard_shapes_tp1": lambda d: bench_shard_shapes(d, [n for n in SHARD_SHAPES if "tp1" in n]),
                "lm_head_stream": bench_lm_head_stream, "decode_8b": lambda d: bench_shard_shapes(d, names=("8b_qkv", "8b_o", "8b_down"), Ms=(32, 64, 96, 128, 160, 192, 256), prefill_Ms=()), "gateup_shapes": lambda d: bench_shard_shapes(d, names=("70b_tp8_gate_up", "70b_tp1_gate_up", "8b_gate_up"), prefill_Ms=()),
                "lm_head_stream_shard": lambda d: bench_lm_head_stream(d, V=16128, Ms=(1, 8, 32, 64, 127))}[name](dev)
    for r in res:
        print(json.dumps(r), flush=True)
    if args.out:
        with open(args.out, "w") as fh:
            for r in res:
                fh.write(json.dumps(r) + "\n")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
