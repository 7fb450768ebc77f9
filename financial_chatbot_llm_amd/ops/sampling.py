"""K12: temperature / Gumbel-max sampling and greedy argmax over full-vocab logits, with optional
per-row top-k / top-p filters (HIP radix-select threshold, graph-capturable; ``sampler.hip``)."""
from __future__ import annotations

from typing import Optional

import torch

from . import _native as N

SPLITS = 16  # vocab slices per row in the HIP sampler (SAMPLE_SPLITS)


def sample(logits: torch.Tensor, temperatures: torch.Tensor, seeds: torch.Tensor,
           out: Optional[torch.Tensor] = None, top_k: Optional[torch.Tensor] = None,
           top_p: Optional[torch.Tensor] = None) -> torch.Tensor:
    """logits [B, V] (bf16 or f32), temperatures [B] f32 (<= 0 -> greedy), seeds [B] int64,
    optional top_k [B] int32 (<= 0: off) and top_p [B] f32 (>= 1: off).

    Returns int32 token ids [B].  On the GPU the HIP kernel draws counter-based Gumbel noise
    from (seed, token index); the CPU reference uses torch's generator seeded per row, so the two
    paths agree exactly for greedy rows and in distribution for sampled rows.  top-k/top-p become
    a per-row logit threshold on the device (no sort, no host sync).
    """
    B, V = logits.shape
    filt = top_k is not None and top_p is not None
    if N.use_native(logits):
        out = torch.empty((B,), dtype=torch.int32, device=logits.device) if out is None else out
        assert logits.stride(1) == 1 and logits.stride(0) % 8 == 0
        ws = torch.empty((B * SPLITS * 2 + B,), dtype=torch.float32, device=logits.device)
        tk = top_k.to(torch.int32).contiguous() if filt else None
        tp = top_p.to(torch.float32).contiguous() if filt else None
        N.call("penny_sample", N.ptr(logits), int(logits.dtype == torch.float32), logits.stride(0),
               N.ptr(temperatures), N.ptr(seeds), N.ptr(tk) if filt else None, N.ptr(tp) if filt else None,
               N.ptr(out), N.ptr(ws), B, V, N.stream())
        return out
    if filt:
        logits = apply_top_k_top_p(logits, top_k.to(logits.device), top_p.to(logits.device), temperatures)
    res = torch.empty((B,), dtype=torch.int32)
    lf = logits.float()
    temps = temperatures.tolist()
    sd = seeds.tolist()
    for b in range(B):
        if temps[b] <= 0:
            res[b] = int(torch.argmax(lf[b]).item())
        else:
            g = torch.Generator().manual_seed(int(sd[b]) & 0x7FFFFFFFFFFFFFFF)
            u = torch.rand(V, generator=g, dtype=torch.float64).clamp_(1e-12, 1 - 1e-12)
            res[b] = int(torch.argmax(lf[b].double() / temps[b] - torch.log(-torch.log(u))).item())
    if out is not None:
        out.copy_(res)
        return out
    return res.to(logits.device)


# Fused LM head + sampler (K11 + K12, ``gemm_prefill.hip`` EPI_SAMPLE): the vocabulary projection
# runs on the 256x256 MFMA tile kernel and every lane Gumbel-max-scores its logits in registers,
# so the [M, V] logits never reach HBM and the separate sampler pass disappears.  Its cost is
# nearly flat in M (two rounds of 501 vocab tiles over 256 CUs for Llama-3: 243-265 us at M = 1-160,
# 306 us at 256), while hipBLASLt + the sampler grows with M (190 us at M = 1, 266 at 128, 355 at
# 256): the fused path is taken from FUSED_LM_HEAD_MIN_M rows, where it ties (M = 128) or wins
# 8-16 % (M = 160-256) (bench/kernels.py lm_head_fused, profiles/r3_lm_head_fused_vs_hipblaslt.jsonl).
# Below that the 256-row tile's MFMA work and the 1.05 GB weight stream share each CU's time
# (4.2 TB/s) and the library's streaming GEMM wins.  ``PENNY_FUSED_LM_HEAD=0`` disables it,
# ``=force`` takes it at every M.
FUSED_LM_HEAD_MIN_M = 128


def fused_lm_head_ok(h: torch.Tensor, w: torch.Tensor) -> bool:
    import os
    mode = os.environ.get("PENNY_FUSED_LM_HEAD", "1")
    if mode == "0" or not N.use_native(h):
        return False
    M, K = h.shape
    V = w.shape[0]
    if V % 256 or K % 64 or h.stride(1) != 1 or h.stride(0) % 8 or not w.is_contiguous():
        return False
    return mode == "force" or M >= FUSED_LM_HEAD_MIN_M


def lm_head_sample(h: torch.Tensor, w: torch.Tensor, temperatures: torch.Tensor, seeds: torch.Tensor,
                   out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Sample one token per row of ``h`` [M, K] from softmax((h @ w.T) / T) (T <= 0: greedy) without
    materialising the logits.  Same noise as :func:`sample` (counter-based on (seed, token id)),
    scored on the bf16-rounded logits, so for equal logits both paths pick the same token.  The
    tile GEMM and hipBLASLt accumulate in different orders, though, so a row whose two best scores
    lie within logit rounding can differ between the paths (tokens are reproducible up to logit
    rounding; the rate is measured by tests/test_kernels_gpu.py::test_fused_vs_unfused_sampling_
    token_agreement).  No top-k / top-p (those rows need the whole distribution: use ``sample``)."""
    M, K = h.shape
    V = w.shape[0]
    if not N.use_native(h):
        import torch.nn.functional as F
        return sample(F.linear(h.float(), w.float()).to(h.dtype), temperatures, seeds, out=out)
    out = torch.empty((M,), dtype=torch.int32, device=h.device) if out is None else out
    ws = torch.empty((2 * M * 2 * (V // 256),), dtype=torch.float32, device=h.device)
    temps, sd = temperatures.to(torch.float32).contiguous(), seeds.contiguous()   # alive across the launch
    N.call("penny_lm_head_sample", N.ptr(h), h.stride(0), N.ptr(w), K, M, V, N.ptr(temps), N.ptr(sd), N.ptr(ws),
           N.ptr(out), N.stream())
    return out


# ----------------------------------------------------------------------------------------------
# Vocabulary-parallel sampling (SURVEY C2 "per-rank top-k then gather"): under TP each rank scores
# its own vocab shard -- Gumbel noise keyed by the GLOBAL token id -- and keeps one (score, id)
# candidate per row; the candidates ([B, 2] int32 per rank) are all-gathered and the best taken.
# Gumbel-max is exactly shard-decomposable, so this is the TP = 1 sample without the [B, V]
# logits all-gather (33 MB per decode step at B = 128 for Llama-3 TP=8).
# ----------------------------------------------------------------------------------------------
def sample_shard(logits: torch.Tensor, temperatures: torch.Tensor, seeds: torch.Tensor, voff: int,
                 vocab_total: int) -> torch.Tensor:
    """logits [B, Vs] of global vocabulary ids voff .. voff+Vs-1 -> pairs [B, 2] int32 (f32 score
    bits, global id) of each row's Gumbel-max (T <= 0: argmax) winner within the shard."""
    B, Vs = logits.shape
    if N.use_native(logits):
        assert logits.stride(1) == 1 and logits.stride(0) % 8 == 0
        pairs = torch.empty((B, 2), dtype=torch.int32, device=logits.device)
        ws = torch.empty((2 * B * SPLITS,), dtype=torch.float32, device=logits.device)
        N.call("penny_sample_shard", N.ptr(logits), int(logits.dtype == torch.float32), logits.stride(0),
               N.ptr(temperatures), N.ptr(seeds), N.ptr(pairs), N.ptr(ws), B, Vs, int(voff), N.stream())
        return pairs
    lf = logits.float()
    temps = temperatures.tolist()
    sd = seeds.tolist()
    sc = torch.empty(B, dtype=torch.float32)
    ids = torch.empty(B, dtype=torch.int32)
    for b in range(B):
        if temps[b] <= 0:
            v = lf[b]
        else:   # the same per-row noise over the WHOLE vocabulary as ``sample``, sliced to the shard
            g = torch.Generator().manual_seed(int(sd[b]) & 0x7FFFFFFFFFFFFFFF)
            u = torch.rand(vocab_total, generator=g, dtype=torch.float64).clamp_(1e-12, 1 - 1e-12)[voff:voff + Vs]
            v = (lf[b].double() / temps[b] - torch.log(-torch.log(u))).float()
        j = int(torch.argmax(v).item())
        sc[b] = v[j]
        ids[b] = voff + j
    return torch.stack([sc.view(torch.int32), ids], 1).to(logits.device)


def lm_head_sample_shard(h: torch.Tensor, w_pad: torch.Tensor, vvalid: int, voff: int, temperatures: torch.Tensor,
                         seeds: torch.Tensor) -> torch.Tensor:
    """Fused LM head + sampler on one vocab shard: ``w_pad`` [Vpad, K] (Vpad % 256 == 0) holds global
    rows voff .. voff+vvalid-1 then padding -> pairs [M, 2] as :func:`sample_shard`."""
    M, K = h.shape
    Vpad = w_pad.shape[0]
    pairs = torch.empty((M, 2), dtype=torch.int32, device=h.device)
    ws = torch.empty((2 * M * 2 * (Vpad // 256),), dtype=torch.float32, device=h.device)
    temps, sd = temperatures.to(torch.float32).contiguous(), seeds.contiguous()   # alive across the launch
    N.call("penny_lm_head_sample_shard", N.ptr(h), h.stride(0), N.ptr(w_pad), K, M, Vpad, int(vvalid), int(voff),
           N.ptr(temps), N.ptr(sd), N.ptr(ws), N.ptr(pairs), N.stream())
    return pairs


def pick_pairs(allp: torch.Tensor) -> torch.Tensor:
    """[R, B, 2] candidates of R vocab shards -> [B] int32 tokens: the highest score, ties to the
    smallest token id (the single-kernel sampler's rule).  Device ops only (graph-capturable)."""
    sc = allp[..., 0].contiguous().view(torch.float32)
    ids = allp[..., 1]
    best = sc.max(0, keepdim=True).values
    cand = torch.where(sc == best, ids, torch.full_like(ids, 0x7FFFFFFF))
    return cand.min(0).values.to(torch.int32)


def topk_topp_threshold(logits: torch.Tensor, temperatures: torch.Tensor, top_k: torch.Tensor,
                        top_p: torch.Tensor) -> torch.Tensor:
    """The HIP filter's per-row logit threshold (-inf: keep all) -- diagnostics/tests."""
    B, V = logits.shape
    th = torch.empty((B,), dtype=torch.float32, device=logits.device)
    tk, tp = top_k.to(torch.int32).contiguous(), top_p.to(torch.float32).contiguous()   # alive across the launch
    N.call("penny_topk_topp_threshold", N.ptr(logits), int(logits.dtype == torch.float32), logits.stride(0),
           N.ptr(temperatures), N.ptr(tk), N.ptr(tp), N.ptr(th), B, V, N.stream())
    return th


def apply_top_k_top_p(logits: torch.Tensor, top_k: torch.Tensor, top_p: torch.Tensor,
                      temperatures: Optional[torch.Tensor] = None) -> torch.Tensor:
    """fp32 reference: mask logits outside top-k, then outside the nucleus top-p of the
    temperature-scaled distribution renormalised over the top-k survivors (vLLM/HF order).
    Rows with k <= 0 / p >= 1 (or greedy rows) are untouched."""
    if bool((top_k <= 0).all()) and bool((top_p >= 1).all()):
        return logits
    lf = logits.float()
    B, V = lf.shape
    t = temperatures.float().to(lf.device) if temperatures is not None else torch.ones(B, device=lf.device)
    sorted_l, idx = torch.sort(lf, dim=-1, descending=True)
    ranks = torch.arange(V, device=lf.device)[None, :]
    k = torch.where(top_k > 0, top_k, torch.full_like(top_k, V)).to(lf.device)[:, None]
    kth = sorted_l.gather(1, (k - 1).clamp(max=V - 1))
    drop = sorted_l < kth                          # ties with the k-th value survive
    scaled = (sorted_l / t.clamp(min=1e-6)[:, None]).masked_fill(drop, float("-inf"))
    probs = torch.softmax(scaled, dim=-1)
    cum = probs.cumsum(-1) - probs                 # mass strictly above each token
    drop |= cum >= top_p.float().to(lf.device)[:, None]
    drop &= (t > 0)[:, None]
    drop[:, 0] = False
    sorted_l = sorted_l.masked_fill(drop, float("-inf"))
    return torch.empty_like(lf).scatter_(-1, idx, sorted_l).to(logits.dtype)
