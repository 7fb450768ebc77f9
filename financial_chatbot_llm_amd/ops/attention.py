"""K3-epilogue/K4/K5 (RoPE + paged KV write) and K6/K7 (paged prefill / decode attention).

Paged KV layout (see ``csrc/kernels/kv_layout.h``): blocks of ``KV_BS = 64`` tokens, one tile
of ``64*D`` elements per (block, kv head), stored in MFMA-fragment-native order::

    k_cache[layer]: [num_blocks, Hkv, 64*D]   element (key, d) at K_INDEX[D][key, d]
    v_cache[layer]: [num_blocks, Hkv, 64*D]   element (key, d) at V_INDEX[D][key, d]

The torch reference implementations here are the numerics oracle for the HIP kernels (fp32
math on the same bf16 inputs) and the CPU path used by the CI tests.
"""
from __future__ import annotations

import heapq
import math
import os
from dataclasses import dataclass
from functools import lru_cache
from typing import Dict, Optional, Tuple

import numpy as np
import torch

from . import _native as N
from .gemm import Slabs

KV_BS = 64


def k_index(key: int, d: int, D: int) -> int:
    t, r, c, g, j = key >> 4, key & 15, d >> 5, (d >> 3) & 3, d & 7
    return (((t * (D >> 5) + c) * 64 + g * 16 + r) << 3) + j


def v_index(key: int, d: int, D: int) -> int:
    dt, row, s, k = d >> 4, d & 15, key >> 5, key & 31
    g, j = (k & 15) >> 2, ((k >> 4) << 2) + (k & 3)
    return (((dt * 2 + s) * 64 + g * 16 + row) << 3) + j


@lru_cache(maxsize=None)
def kv_index_tables(D: int):
    """(K_INDEX, V_INDEX) [64, D] long tensors for head dim D."""
    ki = torch.tensor([[k_index(k, d, D) for d in range(D)] for k in range(KV_BS)], dtype=torch.long)
    vi = torch.tensor([[v_index(k, d, D) for d in range(D)] for k in range(KV_BS)], dtype=torch.long)
    return ki, vi


# --------------------------------------------------------------------------------------------
# RoPE tables
# --------------------------------------------------------------------------------------------
def rope_inv_freq(D: int, theta: float, scaling: Optional[dict] = None) -> torch.Tensor:
    inv = 1.0 / (theta ** (torch.arange(0, D, 2, dtype=torch.float64) / D))
    if scaling and scaling.get("rope_type", scaling.get("type")) == "llama3":
        factor = scaling.get("factor", 8.0)
        lo, hi = scaling.get("low_freq_factor", 1.0), scaling.get("high_freq_factor", 4.0)
        old = scaling.get("original_max_position_embeddings", 8192)
        lo_wl, hi_wl = old / lo, old / hi
        wl = 2 * math.pi / inv
        smooth = (old / wl - lo) / (hi - lo)
        scaled = torch.where(wl > lo_wl, inv / factor, inv)
        mid = (wl <= lo_wl) & (wl >= hi_wl)
        inv = torch.where(mid, (1 - smooth) * inv / factor + smooth * inv, scaled)
    return inv


def rope_cos_sin(D: int, max_pos: int, theta: float, scaling: Optional[dict] = None,
                 device=None) -> torch.Tensor:
    """[max_pos, D] f32: cos for the D/2 frequencies, then sin (host-computed, K4 table)."""
    inv = rope_inv_freq(D, theta, scaling)
    ang = torch.arange(max_pos, dtype=torch.float64)[:, None] * inv[None, :]
    return torch.cat([ang.cos(), ang.sin()], dim=-1).to(torch.float32).to(device)


def _rope_ref(x: torch.Tensor, pos: torch.Tensor, cos_sin: torch.Tensor) -> torch.Tensor:
    D = x.shape[-1]
    cs = cos_sin[pos.long()]
    cos, sin = cs[:, None, : D // 2], cs[:, None, D // 2:]
    xf = x.float()
    x1, x2 = xf[..., : D // 2], xf[..., D // 2:]
    return torch.cat([x1 * cos - x2 * sin, x2 * cos + x1 * sin], dim=-1).to(x.dtype)


# --------------------------------------------------------------------------------------------
# KV write
# --------------------------------------------------------------------------------------------
def write_kv_ref(k: torch.Tensor, v: torch.Tensor, slots: torch.Tensor, k_cache: torch.Tensor,
                 v_cache: torch.Tensor) -> None:
    """k, v [T, Hkv, D] -> paged fragment-native caches (skips slots < 0)."""
    sl = slots.long()
    keep = sl >= 0
    if not bool(keep.any()):
        return
    sl, k, v = sl[keep], k[keep], v[keep]
    D = k.shape[-1]
    ki, vi = kv_index_tables(D)
    blk, off = sl // KV_BS, sl % KV_BS
    kc, vc = k_cache.permute(0, 2, 1), v_cache.permute(0, 2, 1)   # [NB, 64*D, Hkv] views
    kc[blk[:, None], ki.to(sl.device)[off]] = k.transpose(1, 2).to(k_cache.dtype)
    vc[blk[:, None], vi.to(sl.device)[off]] = v.transpose(1, 2).to(v_cache.dtype)


def rope_kv_write(qkv: torch.Tensor, positions: torch.Tensor, cos_sin: Optional[torch.Tensor],
                  slots: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor, Hq: int, Hkv: int,
                  D: int, apply_rope: bool = True) -> torch.Tensor:
    """Rotate q/k of a fused QKV activation, write k/v into the paged cache, return q [T,Hq,D].
    ``qkv`` may be the unreduced :class:`~.gemm.Slabs` of the split-K QKV GEMM (summed here)."""
    if isinstance(qkv, Slabs):
        S, T, _ = qkv.P.shape
        if N.use_native(qkv.P):
            q = torch.empty((T, Hq, D), dtype=torch.bfloat16, device=qkv.P.device)
            N.call("penny_rope_kv_write_slabs", N.ptr(qkv.P), S, N.ptr(positions),
                   N.ptr(cos_sin) if apply_rope else None, N.ptr(slots), N.ptr(q), N.ptr(k_cache), N.ptr(v_cache),
                   T, Hq, Hkv, D, int(apply_rope), N.stream())
            return q
        qkv = qkv.materialize()
    T = qkv.shape[0]
    if N.use_native(qkv):
        q = torch.empty((T, Hq, D), dtype=qkv.dtype, device=qkv.device)
        N.call("penny_rope_kv_write", N.ptr(qkv), N.ptr(positions), N.ptr(cos_sin) if apply_rope else None,
               N.ptr(slots), N.ptr(q), N.ptr(k_cache), N.ptr(v_cache), T, Hq, Hkv, D, int(apply_rope), N.stream())
        return q
    x = qkv.view(T, Hq + 2 * Hkv, D)
    q, k, v = x[:, :Hq], x[:, Hq:Hq + Hkv], x[:, Hq + Hkv:]
    if apply_rope:
        q, k = _rope_ref(q, positions, cos_sin), _rope_ref(k, positions, cos_sin)
    write_kv_ref(k, v, slots, k_cache, v_cache)
    return q.contiguous()


# --------------------------------------------------------------------------------------------
# Attention
# --------------------------------------------------------------------------------------------
def rope_qk(qkv: torch.Tensor, positions: torch.Tensor, cos_sin: torch.Tensor, Hq: int, Hkv: int,
            D: int) -> torch.Tensor:
    """Rotated q and k heads of the fused QKV activation, no KV-cache write: [T, Hq + Hkv, D] (the
    context-parallel prefill passes K/V around the ring as tensors).  HIP (``penny_rope_qk``) on
    the GPU, the fp32 reference on CPU."""
    T = qkv.shape[0]
    if N.use_native(qkv):
        qk = torch.empty((T, Hq + Hkv, D), dtype=qkv.dtype, device=qkv.device)
        # converted inputs bound to names: a temporary passed as N.ptr(x.contiguous()) is freed before
        # the launch, and the next temporary's copy can reuse (overwrite) its block on the stream
        src, pos = qkv.contiguous(), positions.to(torch.int32).contiguous()
        N.call("penny_rope_qk", N.ptr(src), N.ptr(pos), N.ptr(cos_sin), N.ptr(qk), T, Hq, Hkv, D, N.stream())
        return qk
    return _rope_ref(qkv.view(T, -1, D)[:, :Hq + Hkv], positions, cos_sin).to(qkv.dtype)


def gather_kv_ref(k_cache: torch.Tensor, v_cache: torch.Tensor, blocks: torch.Tensor, n: int):
    """-> K, V [n, Hkv, D] for one sequence (inverse of the paged layout)."""
    Hkv = k_cache.shape[1]
    D = k_cache.shape[2] // KV_BS
    ki, vi = kv_index_tables(D)
    nb = (n + KV_BS - 1) // KV_BS
    b = blocks[:nb].long()
    kt = k_cache[b][..., ki.to(b.device).flatten()].view(nb, Hkv, KV_BS, D)
    vt = v_cache[b][..., vi.to(b.device).flatten()].view(nb, Hkv, KV_BS, D)
    k = kt.permute(0, 2, 1, 3).reshape(nb * KV_BS, Hkv, D)
    v = vt.permute(0, 2, 1, 3).reshape(nb * KV_BS, Hkv, D)
    return k[:n], v[:n]


def _attend_ref(q, k, v, scale, causal_offset: Optional[int]):
    """q [Tq,Hq,D], k/v [Tk,Hkv,D] -> [Tq,Hq,D] in fp32."""
    Hq, Hkv = q.shape[1], k.shape[1]
    G = Hq // Hkv
    kf = k.float().repeat_interleave(G, dim=1)
    vf = v.float().repeat_interleave(G, dim=1)
    s = torch.einsum("qhd,khd->hqk", q.float(), kf) * scale
    if causal_offset is not None:
        tq, tk = q.shape[0], k.shape[0]
        qi = torch.arange(tq, device=q.device)[:, None] + causal_offset
        ki = torch.arange(tk, device=q.device)[None, :]
        s = s.masked_fill((ki > qi)[None], float("-inf"))
    p = torch.softmax(s, dim=-1)
    return torch.einsum("hqk,khd->qhd", p, vf)


PREFILL_WORK_LIST = os.environ.get("PENNY_PREFILL_WORK_LIST", "1") != "0"


def prefill_work_list(cu_q: np.ndarray, ctx_lens: np.ndarray, G: int, causal: bool = True) -> Optional[np.ndarray]:
    """Host work list for the 8-wave prefill kernel: every real (sequence, 256-row tile) of a step,
    ordered by the number of KV blocks its tile walks, longest first (LPT) -- [n, 2] int32, or None
    when the step takes the 4-wave kernel (no tile above 128 rows) or the list is disabled
    (``PENNY_PREFILL_WORK_LIST=0``).  Without it the grid is (max tiles x sequences): a step with one
    1.6k-token respond chunk and eight 220-token decide chunks launches 4x the workgroups it needs,
    and every sequence's short tiles trail its long ones."""
    if not PREFILL_WORK_LIST or G <= 0 or 256 % G:
        return None
    cu = np.asarray(cu_q, np.int64)
    ql = cu[1:] - cu[:-1]
    if len(ql) == 0 or int(ql.max()) * G <= 128:
        return None
    ctx = np.asarray(ctx_lens, np.int64)
    TQ = 256 // G
    seqs, tiles, cost = [], [], []
    for s_, (n, c) in enumerate(zip(ql.tolist(), ctx.tolist())):
        for t in range((n + TQ - 1) // TQ):
            last = min((t + 1) * TQ, n) - 1
            kv_end = min(c, c - n + last + 1) if causal else c
            seqs.append(s_)
            tiles.append(t)
            cost.append((kv_end + KV_BS - 1) // KV_BS)
    order = np.argsort(-np.asarray(cost), kind="stable")
    return np.stack([np.asarray(seqs, np.int32)[order], np.asarray(tiles, np.int32)[order]], 1)


# Lean (KV-split) big-tile prefill: tiles whose KV walk is longer than the step's balanced per-CU
# share are cut into chunks run by different workgroups, each writing flash-decoding partial state
# that ``prefill_merge_kernel`` combines in chunk order (bitwise repeatable).  A step of short
# decide / speculative chunks behind 4-5k cached tokens then no longer waits on its longest walks:
# LPT over chunks instead of whole tiles.  PENNY_PREFILL_LEAN=0 keeps whole tiles.
PREFILL_LEAN = os.environ.get("PENNY_PREFILL_LEAN", "1") != "0"
LEAN_MIN_CHUNK = 8          # KV blocks: below that a chunk's partial write + merge outweigh the balance
# r6 cost gate, in KV-block units of one workgroup's walk: a split is kept only if its LPT makespan
# (+ per-workgroup prologue / epilogue, + a chunk's partial write, + the merge launch) beats the
# whole-tile plan's.  Splitting into MORE workgroups than CUs can leave the makespan where it was
# (a second round of chunks behind the longest whole tiles): on the kbench steps
# "respond-short+4decides" / "4decides+16spec" the split ran 10 % / 2.5 % slower than whole tiles
# (profiles/r6_prefill_attn_pair_barrier_rejected.jsonl pf3_prod vs pf3_q), while 1-2 decides and
# a short respond alone keep their 1.4-3x gain.  Calibrated on those five steps.
LEAN_ITEM_BLOCKS = 3        # prologue (Q load, first K/V wait) + epilogue of one workgroup
LEAN_CHUNK_BLOCKS = 1       # a chunk's partial O / (m, l) write
LEAN_MERGE_BLOCKS = 6       # prefill_merge_kernel launch + its pass
LEAN_COST_GATE = os.environ.get("PENNY_PREFILL_LEAN_GATE", "1") != "0"


def _lpt_makespan(lengths, machines: int) -> float:
    """Makespan of longest-processing-time-first list scheduling of ``lengths`` on ``machines``."""
    ls = sorted(lengths, reverse=True)
    if machines <= 0 or not ls:
        return float(sum(ls))
    if len(ls) <= machines:
        return float(ls[0])
    loads = sorted(ls[:machines])            # a sorted list is a valid min-heap
    for x in ls[machines:]:
        heapq.heapreplace(loads, loads[0] + x)
    return float(max(loads))


def prefill_lean_list(cu_q: np.ndarray, ctx_lens: np.ndarray, G: int, Hkv: int, causal: bool = True,
                      cus: int = 256, min_chunk: int = LEAN_MIN_CHUNK) -> Optional[np.ndarray]:
    """Lean work list of one step, or None when no tile needs splitting or (``LEAN_COST_GATE``)
    the makespan model prefers whole tiles: int32 [1 + n + m, 6] = header (-1, n items, m merges,
    slots, 0, 0), n items (sequence, tile, first block, end block, slot or -1, 0) longest first,
    m merges (sequence, tile, first slot, slots, 0, 0)."""
    if not PREFILL_LEAN or G <= 0 or 256 % G:
        return None
    cu = np.asarray(cu_q, np.int64)
    ql = cu[1:] - cu[:-1]
    # tiny chunks only (speculative / known-run rows: <= 128 rows per (sequence, kv head)) take the
    # 4-wave 128-row kernel, which walks each context whole on one workgroup; with the cost gate
    # they may instead split their walks on the 8-wave kernel (its whole-tile makespan stands in
    # for the 4-wave kernel's)
    if len(ql) == 0 or (int(ql.max()) * G <= 128 and not LEAN_COST_GATE):
        return None
    ctx = np.asarray(ctx_lens, np.int64)
    TQ = 256 // G
    tiles = []
    for s_, (n, c) in enumerate(zip(ql.tolist(), ctx.tolist())):
        for t in range((n + TQ - 1) // TQ):
            last = min((t + 1) * TQ, n) - 1
            kv_end = min(c, c - n + last + 1) if causal else c
            tiles.append((s_, t, (kv_end + KV_BS - 1) // KV_BS))
    total = sum(nb for _, _, nb in tiles)
    C = max(min_chunk, -(-total * Hkv // max(cus, 1)))       # balanced per-CU share of block units
    longest = max(nb for _, _, nb in tiles)
    if longest <= C:
        return None

    def plan(C):
        items, merges, slot = [], [], 0
        for s_, t, nb in tiles:
            if nb <= C:
                items.append((s_, t, 0, nb, -1, 0))
                continue
            k = -(-nb // C)
            cuts = [round(i * nb / k) for i in range(k + 1)]
            merges.append((s_, t, slot, k, 0, 0))
            items += [(s_, t, cuts[i], cuts[i + 1], slot + i, 0) for i in range(k)]
            slot += k
        items.sort(key=lambda r: -(r[3] - r[2]))              # LPT over chunks
        return items, merges, slot

    if LEAN_COST_GATE:
        # every item runs once per kv head: the heads' identical lists share the CUs evenly.  The
        # chunk size is the balanced share or a coarser cut of the longest walk into k = 2..8
        # pieces, whichever the model's makespan prefers (finer than the balanced share never won
        # on the kbench steps and costs milliseconds of host LPT); whole tiles unless a split's
        # makespan + merge beats them
        mach = max(cus // max(Hkv, 1), 1)
        whole = _lpt_makespan([nb + LEAN_ITEM_BLOCKS for _, _, nb in tiles], mach)
        best, best_c = whole, None
        for c in sorted({C} | {-(-longest // k) for k in range(2, 9)}):
            if c < C or c >= longest:
                continue
            items, _, _ = plan(c)
            ms = _lpt_makespan([e - b + LEAN_ITEM_BLOCKS + (LEAN_CHUNK_BLOCKS if sl >= 0 else 0)
                                for _, _, b, e, sl, _ in items], mach) + LEAN_MERGE_BLOCKS
            if ms < best:
                best, best_c = ms, c
        if best_c is None:
            return None
        C = best_c
    items, merges, slot = plan(C)
    out = np.zeros((1 + len(items) + len(merges), 6), np.int32)
    out[0, :4] = (-1, len(items), len(merges), slot)
    out[1:1 + len(items)] = np.asarray(items, np.int32)
    if merges:
        out[1 + len(items):] = np.asarray(merges, np.int32)
    return out


def prefill_plan(cu_q: np.ndarray, ctx_lens: np.ndarray, G: int, Hkv: int, causal: bool = True,
                 cus: int = 256) -> Optional[np.ndarray]:
    """The step's prefill-attention work list: lean ([., 6], when some walk needs splitting; every
    prefill2 variant takes it) or whole tiles in LPT order ([n, 2])."""
    if PREFILL_LEAN:
        lean = prefill_lean_list(cu_q, ctx_lens, G, Hkv, causal, cus)
        if lean is not None:
            return lean
    return prefill_work_list(cu_q, ctx_lens, G, causal)


_LEAN_WS: Dict[int, Tuple[torch.Tensor, torch.Tensor]] = {}


def _lean_workspace(dev: torch.device, slots: int, Hkv: int, D: int) -> Tuple[torch.Tensor, torch.Tensor]:
    key = torch.device(dev).index
    ws = _LEAN_WS.get(key)
    need_o, need_ml = slots * Hkv * 256 * D, slots * Hkv * 256 * 2
    if ws is None or ws[0].numel() < need_o or ws[1].numel() < need_ml:
        grow = max(slots, 64)
        ws = (torch.empty(grow * Hkv * 256 * D, dtype=torch.bfloat16, device=dev),     # O / l (bf16)
              torch.empty(grow * Hkv * 256 * 2, dtype=torch.float32, device=dev))
        _LEAN_WS[key] = ws
    return ws


def prefill_variant(v: int = -1) -> int:
    """Select the big-tile prefill kernel for this process (returns the previous choice; -1 only
    reads it): 7 = prefill3, the 32x32x16-MFMA block loop (default from r6, head dim 128), 5 =
    prefill2 with the VALU-lean softmax (the r5 default; head dim 64 under 7), 6 = 5 with prescaled Q
    (opt-in), 4 = prefill2 with pinned K/V fragment prefetch (the fallback); other values select 5
    (``PENNY_PREFILL_PP`` sets the initial value).  In-process A/B runs and tests only."""
    return int(N.load().penny_attention_prefill_variant(int(v)))


def prefill(q: torch.Tensor, cu_q: torch.Tensor, ctx_lens: torch.Tensor, block_tables: torch.Tensor,
            k_cache: torch.Tensor, v_cache: torch.Tensor, scale: float, causal: bool = True,
            max_q_len: Optional[int] = None, out: Optional[torch.Tensor] = None,
            lse: Optional[torch.Tensor] = None, work: Optional[torch.Tensor] = None,
            lean: Optional[Tuple[int, int, int]] = None, q_prescaled: bool = False) -> torch.Tensor:
    """Varlen paged attention for the new tokens of S sequences (chunked prefill / prefix hits:
    query i of sequence s sits at absolute position ctx_lens[s] - q_len[s] + i).  ``lse`` [T, Hq]
    f32 (optional) receives each row's natural-log sum-exp of the scaled scores (-inf: no key
    visible) -- what a ring-attention merge needs.  ``work``: :func:`prefill_work_list` of the same
    step on the device (optional; LPT tile order), or :func:`prefill_lean_list`'s split-KV list
    (``lean`` = its (items, merges, slots) counts, read from the header when not given).
    ``q_prescaled``: q already carries ``scale * log2(e)`` (``prefill_qkv_rope(qscale=...)``) and
    ``scale`` is ``1 / log2(e)``; the big tiles then run the prescaled-Q fold."""
    T, Hq, D = q.shape
    flags = int(causal) | (2 if q_prescaled else 0)
    Hkv = k_cache.shape[1]
    S = block_tables.shape[0]
    assert k_cache.shape[-1] == KV_BS * D
    if N.use_native(q):
        out = torch.empty_like(q) if out is None else out
        if work is not None and work.dim() == 2 and work.shape[1] == 6:
            # lean work list (prefill_lean_list): the counts ride along host-side as ``lean``
            ni, nm, nslots = lean if lean is not None else (int(work[0, 1]), int(work[0, 2]), int(work[0, 3]))
            po, pml = _lean_workspace(q.device, max(nslots, 1), Hkv, D)
            N.call("penny_attention_prefill_lean", N.ptr(q), N.ptr(cu_q), N.ptr(ctx_lens), N.ptr(block_tables),
                   N.ptr(k_cache), N.ptr(v_cache), N.ptr(out), Hq, Hkv, D, block_tables.shape[1], float(scale),
                   flags, N.ptr(lse) if lse is not None else None, N.ptr(work[1:]), int(ni),
                   N.ptr(work[1 + ni:]) if nm else None, int(nm), N.ptr(po), N.ptr(pml), N.stream())
            return out
        if max_q_len is None:
            max_q_len = int((cu_q[1:] - cu_q[:-1]).max().item())
        N.call("penny_attention_prefill", N.ptr(q), N.ptr(cu_q), N.ptr(ctx_lens), N.ptr(block_tables),
               N.ptr(k_cache), N.ptr(v_cache), N.ptr(out), S, int(max_q_len), Hq, Hkv, D, block_tables.shape[1],
               float(scale), flags, N.ptr(lse) if lse is not None else None,
               N.ptr(work) if work is not None else None, int(work.shape[0]) if work is not None else 0, N.stream())
        return out
    out = torch.empty_like(q) if out is None else out
    cu = cu_q.tolist()
    ctx = ctx_lens.tolist()
    for s in range(S):
        a, b = cu[s], cu[s + 1]
        if b <= a:
            continue
        k, v = gather_kv_ref(k_cache, v_cache, block_tables[s], ctx[s])
        out[a:b] = _attend_ref(q[a:b], k, v, scale, ctx[s] - (b - a) if causal else None).to(q.dtype)
        if lse is not None:
            lse[a:b] = _lse_ref(q[a:b], k, scale, ctx[s] - (b - a) if causal else None)
    return out


def _lse_ref(q: torch.Tensor, k: torch.Tensor, scale: float, q_offset: Optional[int]) -> torch.Tensor:
    """[Tq, Hq] natural-log sum-exp of the scaled (masked) scores, fp32."""
    G = q.shape[1] // k.shape[1]
    kk = k.float().repeat_interleave(G, dim=1)
    s = torch.einsum("qhd,khd->hqk", q.float(), kk) * scale
    if q_offset is not None:
        qi = torch.arange(q.shape[0])[:, None] + q_offset
        s = s.masked_fill((torch.arange(k.shape[0])[None, :] > qi)[None], float("-inf"))
    return torch.logsumexp(s, dim=-1).transpose(0, 1)


@dataclass
class DecodeWorkspace:
    part_m: torch.Tensor
    part_l: torch.Tensor
    part_o: torch.Tensor
    pb: int
    nparts: int
    part_stride: int = 0    # partition slots per (row, head)
    lean_meta: Optional[torch.Tensor] = None   # [64 + max_batch + 2] int32: chunk counters + lean plan

    def partitioning(self, B: int):
        """(pb, nparts) for a decode batch of B rows.  Batches of 32+ rows already fill the chip
        with (row, head) work, so they take long partitions: fewer empty workgroups in the fixed
        hipGraph grid, fewer per-workgroup prologues/merges and fewer partials to reduce."""
        if os.environ.get("PENNY_DECODE_FIXED_PB") == "1":
            return self.pb, self.nparts
        # B >= 32: 2048-key partitions (pb 32) -- the workload's batches (B 64-128, contexts
        # 1.5-6.5k) run 3-10 % faster than with 512/1024-key ones (r2_decode_partition_sweep.txt);
        # small batches keep 512-key partitions for parallelism (B=16: 18.5 vs 24.4 us).
        # PENNY_DECODE_PB_SCALE="small,large" overrides the multipliers (A/B knob).
        scale = os.environ.get("PENNY_DECODE_PB_SCALE")
        mult = tuple(int(x) for x in scale.split(",")) if scale else (1, 4)
        pb = self.pb * (mult[0] if B < 32 else mult[-1])
        nblk = self.nparts * self.pb
        return pb, (nblk + pb - 1) // pb

    @classmethod
    def create(cls, max_batch: int, Hq: int, D: int, max_ctx: int, device, pb: int = 8) -> "DecodeWorkspace":
        nblk = (max_ctx + KV_BS - 1) // KV_BS
        nparts = max(2, (nblk + pb - 1) // pb)
        stride = max(nparts, 2)
        f = dict(dtype=torch.float32, device=device)
        return cls(torch.empty((max_batch, Hq, stride), **f), torch.empty((max_batch, Hq, stride), **f),
                   torch.empty((max_batch, Hq, stride, D), **f), pb, max(nparts, 2), stride,
                   torch.zeros(LEAN_META0 + max_batch + 2, dtype=torch.int32, device=device))


_SIDE_STREAMS = {}

# Work-balanced ("lean") split-K decode for the per-row suffixes (decode_lean_kernel): every wave
# of a one-round grid streams the same number of KV blocks.  PENNY_DECODE_LEAN=0 restores the
# per-(row, head, partition) workgroup kernel; LEAN_MIN_B: smaller batches keep it (A/B knob).
DECODE_LEAN = os.environ.get("PENNY_DECODE_LEAN", "1") != "0"
LEAN_MIN_B = int(os.environ.get("PENNY_DECODE_LEAN_MIN_B", "1"))
LEAN_WG_PER_CU = 2          # 242 VGPRs per wave -> 2 waves per SIMD = 2 workgroups per CU
LEAN_MIN_PER_WAVE = 2
# lean kernel flags (attention.hip penny_attention_decode lean_flags): bit 0 = non-temporal K/V loads
# for the blocks only one row of the step reads (the host marks the shared ones: mark_shared_blocks);
# bit 1 = the merge with 4 heads per workgroup (7.5 vs 8.1 us per call, decode -0.4..-1.8 % standalone,
# profiles/r5_decode_lean_merge_hpw_ab.jsonl).
# Measured on workload batches (bench/kernels.py decode_lean, profiles/r5_decode_lean_nt_marked_ab.jsonl):
# -9..-13 % per call at B = 64-256 (-10 % with no shared prefix; every block non-temporal, shared
# ones included, gains only 3-6 % and loses 3 % on a 2k shared prefix); +4 % at B = 16, so batches
# below LEAN_NT_MIN_B keep the default policy.  Driver bench 33.29 vs 32.52 turns/s on one box.
LEAN_FLAGS = int(os.environ.get("PENNY_DECODE_LEAN_FLAGS", "3"))
LEAN_NT_MIN_B = 32
MARK_MAX_COLS = 64          # a shared prefix is looked for in the first 64 blocks (4k tokens)


@lru_cache(maxsize=1)
def _runtime():
    try:
        from .. import _penny_runtime as rt
        return rt if hasattr(rt, "mark_shared_blocks") else None
    except ImportError:
        return None


def mark_shared_blocks(bt: np.ndarray, ctx: np.ndarray) -> np.ndarray:
    """Mark, in place as ``-id - 1``, each decode row's leading KV blocks that another row of the same
    step reads at the same position (the shared prompt prefix the prefix cache deduplicated).  The
    lean decode kernel keeps the default cache policy for those -- every row sharing them hits L2 /
    MALL -- and streams each row's own blocks non-temporally.  Every decode attention path decodes
    the marks.  The native runtime's version (``_penny_runtime.mark_shared_blocks``, ~B log B per
    column) when built; this numpy form otherwise (same result)."""
    B, W = bt.shape
    if B < 2 or W == 0:
        return bt
    rt = _runtime()
    if rt is not None and bt.dtype == np.int32 and bt.flags.c_contiguous:
        rt.mark_shared_blocks(bt, np.ascontiguousarray(ctx, dtype=np.int32), MARK_MAX_COLS, KV_BS)
        return bt
    J = min(W, MARK_MAX_COLS)
    t = bt[:, :J]
    valid = np.arange(J)[None, :] < ((np.asarray(ctx) + KV_BS - 1) // KV_BS)[:, None]
    # columns past a row's context are not read: unique negative stand-ins never match
    key = np.where(valid, t.astype(np.int64), -1 - np.arange(B * J, dtype=np.int64).reshape(B, J))
    o = np.argsort(key, axis=0, kind="stable")
    srt = np.take_along_axis(key, o, 0)
    eq = srt[1:] == srt[:-1]
    d = np.zeros((B, J), bool)
    d[1:] |= eq
    d[:-1] |= eq
    dup = np.empty_like(d)
    np.put_along_axis(dup, o, d, 0)
    lead = np.cumprod(dup, axis=1).sum(1)
    mask = np.arange(J)[None, :] < lead[:, None]
    t[mask] = -t[mask] - 1
    return bt


LEAN_META0 = 64             # lean_meta[64:]: the plan published for the merge (attention.hip LEAN_META0)
_CU_COUNT = {}


def _lean_grid(device, Hkv: int) -> int:
    """One round of workgroups, a multiple of Hkv (workgroup i serves kv head i % Hkv)."""
    key = torch.device(device).index
    if key not in _CU_COUNT:
        _CU_COUNT[key] = torch.cuda.get_device_properties(device).multi_processor_count
    return max(1, LEAN_WG_PER_CU * _CU_COUNT[key] // Hkv) * Hkv


def _side_stream(device) -> "torch.cuda.Stream":
    key = torch.device(device).index
    if key not in _SIDE_STREAMS:
        _SIDE_STREAMS[key] = torch.cuda.Stream(device=device)
    return _SIDE_STREAMS[key]


_FORK_EVENTS: Dict[int, Tuple["torch.cuda.Event", "torch.cuda.Event"]] = {}


def fork_join_events(device) -> Tuple["torch.cuda.Event", "torch.cuda.Event"]:
    """Two reusable events per device for a main -> side -> main fork/join (``Stream.wait_stream``
    creates a fresh event per call: ~30 us of HIP event creation + record, 64 times a mixed step).
    Re-recording is safe: a wait enqueued earlier keeps the record it saw."""
    key = torch.device(device).index
    if key not in _FORK_EVENTS:
        _FORK_EVENTS[key] = (torch.cuda.Event(), torch.cuda.Event())   # enable_timing=False: no timestamps
    return _FORK_EVENTS[key]


def decode(q: torch.Tensor, ctx_lens: torch.Tensor, block_tables: torch.Tensor, k_cache: torch.Tensor,
           v_cache: torch.Tensor, scale: float, workspace: Optional[DecodeWorkspace] = None,
           max_ctx: Optional[int] = None, out: Optional[torch.Tensor] = None,
           stream: Optional[int] = None) -> torch.Tensor:
    """One query token per sequence against its paged context: the work-balanced split-K kernel
    (``decode_lean_kernel``) by default, the per-(row, head, partition) kernel with
    ``PENNY_DECODE_LEAN=0``.  ``stream``: raw HIP stream to launch on (default: the current one)."""
    B, Hq, D = q.shape
    Hkv = k_cache.shape[1]
    if N.use_native(q):
        out = torch.empty_like(q) if out is None else out
        if workspace is None or workspace.part_m.shape[0] < B or workspace.part_m.shape[1] < Hq:
            if max_ctx is None:
                max_ctx = int(ctx_lens.max().item())
            workspace = DecodeWorkspace.create(B, Hq, D, max(max_ctx, 1), q.device)
        ws = workspace
        lean = (DECODE_LEAN and B >= LEAN_MIN_B and ws.lean_meta is not None
                and ws.lean_meta.numel() >= LEAN_META0 + B + 2)
        pb, nparts = ws.partitioning(B) if not lean else (ws.pb, ws.nparts)
        args = [N.ptr(q), N.ptr(ctx_lens), N.ptr(block_tables), N.ptr(k_cache), N.ptr(v_cache), N.ptr(out),
                N.ptr(ws.part_m), N.ptr(ws.part_l), N.ptr(ws.part_o), B, Hq, Hkv, D, block_tables.shape[1], pb,
                nparts, ws.part_stride, float(scale)]
        lean_args = ((_lean_grid(q.device, Hkv), N.ptr(ws.lean_meta), LEAN_MIN_PER_WAVE,
                      LEAN_FLAGS if B >= LEAN_NT_MIN_B else LEAN_FLAGS & ~1) if lean else (0, None, 1, 0))
        N.call("penny_attention_decode", *args, *lean_args, N.stream() if stream is None else stream)
        return out
    out = torch.empty_like(q) if out is None else out
    ctx = ctx_lens.tolist()
    block_tables = torch.where(block_tables < 0, -block_tables - 1, block_tables)   # shared-block marks
    for b in range(B):
        k, v = gather_kv_ref(k_cache, v_cache, block_tables[b], ctx[b])
        out[b:b + 1] = _attend_ref(q[b:b + 1], k, v, scale, None).to(q.dtype)
    return out


def default_scale(D: int) -> float:
    return 1.0 / math.sqrt(D)
