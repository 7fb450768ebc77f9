"""K3-epilogue/K4/K5 (RoPE + paged KV write) and K6/K7 (paged prefill / decode attention).

Paged KV layout (see ``csrc/kernels/kv_layout.h``): blocks of ``KV_BS = 64`` tokens, one tile
of ``64*D`` elements per (block, kv head), stored in MFMA-fragment-native order::

    k_cache[layer]: [num_blocks, Hkv, 64*D]   element (key, d) at K_INDEX[D][key, d]
    v_cache[layer]: [num_blocks, Hkv, 64*D]   element (key, d) at V_INDEX[D][key, d]

The torch reference implementations here are the numerics oracle for the HIP kernels (fp32
math on the same bf16 inputs) and the CPU path used by the CI tests.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from functools import lru_cache
from typing import Optional

import torch

from . import _native as N

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
    """Rotate q/k of a fused QKV activation, write k/v into the paged cache, return q [T,Hq,D]."""
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


def prefill(q: torch.Tensor, cu_q: torch.Tensor, ctx_lens: torch.Tensor, block_tables: torch.Tensor,
            k_cache: torch.Tensor, v_cache: torch.Tensor, scale: float, causal: bool = True,
            max_q_len: Optional[int] = None, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Varlen paged attention for the new tokens of S sequences (chunked prefill / prefix hits:
    query i of sequence s sits at absolute position ctx_lens[s] - q_len[s] + i)."""
    T, Hq, D = q.shape
    Hkv = k_cache.shape[1]
    S = block_tables.shape[0]
    assert k_cache.shape[-1] == KV_BS * D
    if N.use_native(q):
        out = torch.empty_like(q) if out is None else out
        if max_q_len is None:
            max_q_len = int((cu_q[1:] - cu_q[:-1]).max().item())
        N.call("penny_attention_prefill", N.ptr(q), N.ptr(cu_q), N.ptr(ctx_lens), N.ptr(block_tables),
               N.ptr(k_cache), N.ptr(v_cache), N.ptr(out), S, int(max_q_len), Hq, Hkv, D, block_tables.shape[1],
               float(scale), int(causal), N.stream())
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
    return out


@dataclass
class DecodeWorkspace:
    part_m: torch.Tensor
    part_l: torch.Tensor
    part_o: torch.Tensor
    pb: int
    nparts: int

    @classmethod
    def create(cls, max_batch: int, Hq: int, D: int, max_ctx: int, device, pb: int = 8) -> "DecodeWorkspace":
        nblk = (max_ctx + KV_BS - 1) // KV_BS
        nparts = max(1, (nblk + pb - 1) // pb)
        f = dict(dtype=torch.float32, device=device)
        return cls(torch.empty((max_batch, Hq, nparts), **f), torch.empty((max_batch, Hq, nparts), **f),
                   torch.empty((max_batch, Hq, nparts, D), **f), pb, nparts)


def decode(q: torch.Tensor, ctx_lens: torch.Tensor, block_tables: torch.Tensor, k_cache: torch.Tensor,
           v_cache: torch.Tensor, scale: float, workspace: Optional[DecodeWorkspace] = None,
           max_ctx: Optional[int] = None, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """One query token per sequence against its paged context (split-K over partitions)."""
    B, Hq, D = q.shape
    Hkv = k_cache.shape[1]
    if N.use_native(q):
        out = torch.empty_like(q) if out is None else out
        if workspace is None or workspace.part_m.shape[0] < B or workspace.part_m.shape[1] < Hq:
            if max_ctx is None:
                max_ctx = int(ctx_lens.max().item())
            workspace = DecodeWorkspace.create(B, Hq, D, max(max_ctx, 1), q.device)
        ws = workspace
        N.call("penny_attention_decode", N.ptr(q), N.ptr(ctx_lens), N.ptr(block_tables), N.ptr(k_cache),
               N.ptr(v_cache), N.ptr(out), N.ptr(ws.part_m), N.ptr(ws.part_l), N.ptr(ws.part_o), B, Hq, Hkv, D,
               block_tables.shape[1], ws.pb, ws.nparts, float(scale), N.stream())
        return out
    out = torch.empty_like(q) if out is None else out
    ctx = ctx_lens.tolist()
    for b in range(B):
        k, v = gather_kv_ref(k_cache, v_cache, block_tables[b], ctx[b])
        out[b:b + 1] = _attend_ref(q[b:b + 1], k, v, scale, None).to(q.dtype)
    return out


def default_scale(D: int) -> float:
    return 1.0 / math.sqrt(D)
