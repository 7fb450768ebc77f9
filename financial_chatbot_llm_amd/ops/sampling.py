"""K12: temperature / Gumbel-max sampling and greedy argmax over full-vocab logits, with optional
per-row top-k / top-p filters (HIP radix-select threshold, graph-capturable; ``sampler.hip``)."""
from __future__ import annotations

from typing import Optional, Tuple

import torch

from . import _native as N

SPLITS = 16  # vocab slices per row in the HIP sampler (SAMPLE_SPLITS)


def _aligned_rows(logits: torch.Tensor) -> torch.Tensor:
    """The HIP samplers load 16-B vectors from each row: a row stride that is not a multiple of 8
    elements (a vocab shard of odd width, e.g. V/tp) is copied into a buffer whose stride is."""
    if logits.stride(1) == 1 and logits.stride(0) % 8 == 0:
        return logits
    B, V = logits.shape
    buf = torch.empty((B, -(-V // 8) * 8), dtype=logits.dtype, device=logits.device)
    buf[:, :V].copy_(logits)
    return buf[:, :V]


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
        logits = _aligned_rows(logits)
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


# Fused LM head + sampler (K11 + K12): no [M, V] logits in HBM and no separate sampler pass -- every
# lane Gumbel-max-scores its logits in registers.  Two kernels, by rows:
#   * M >= FUSED_LM_HEAD_MIN_M: the 256x256 MFMA tile kernel (``gemm_prefill.hip`` EPI_SAMPLE), whose
#     cost is nearly flat in M (two rounds of 501 vocab tiles over 256 CUs for Llama-3: 265 us at
#     M = 128-160, 306 us at 256) while hipBLASLt + the sampler grows with M (266 at 128, 355 at 256)
#     (profiles/r3_lm_head_fused_vs_hipblaslt.jsonl);
#   * M < FUSED_LM_HEAD_MIN_M (decode steps): the weight-streaming split-K kernel
#     (``gemm_splitk.hip`` SK_SAMPLE, ``penny_lm_head_stream_sample``) -- 128 vocab rows per
#     workgroup streamed through an LDS ring, all M rows per workgroup, the sampler in its
#     epilogue; below 128 rows the 256-row tile is MFMA-bound on padding rows (4.2 TB/s) and this
#     is the weight stream (profiles/r5_lm_head_stream.jsonl).
# ``PENNY_FUSED_LM_HEAD=0`` disables both (hipBLASLt logits + the sampler), ``=force`` takes the tile
# kernel at every M; ``PENNY_LM_STREAM=0`` drops the streaming kernel only.
FUSED_LM_HEAD_MIN_M = 128
STREAM_MAX_M = 127
# (max M, nf, 72-KiB ring) of the streaming kernel, first match wins (bench/kernels.py lm_head_stream,
# profiles/r5_lm_head_stream*.jsonl): 64-row vocab tiles and two workgroups per CU up to 64 rows,
# 128-row tiles above (half the X re-reads per vocab row)
STREAM_TABLE = ((64, 4, True), (STREAM_MAX_M, 8, True))


def stream_cfg(M: int) -> Tuple[int, bool]:
    for max_m, nf, r2 in STREAM_TABLE:
        if M <= max_m:
            return nf, r2
    return STREAM_TABLE[-1][1:]


def _stream_ok(M: int) -> bool:
    import os
    return M <= STREAM_MAX_M and os.environ.get("PENNY_LM_STREAM", "1") != "0"


def fused_lm_head_ok(h: torch.Tensor, w: torch.Tensor) -> bool:
    import os
    mode = os.environ.get("PENNY_FUSED_LM_HEAD", "1")
    if mode == "0" or not N.use_native(h):
        return False
    M, K = h.shape
    V = w.shape[0]
    if V % 256 or K % 64 or h.stride(1) != 1 or h.stride(0) % 8 or not w.is_contiguous():
        return False
    return mode == "force" or M >= FUSED_LM_HEAD_MIN_M or _stream_ok(M)


def lm_head_stream_sample(h: torch.Tensor, w: torch.Tensor, temperatures: torch.Tensor, seeds: torch.Tensor,
                          vvalid: Optional[int] = None, voff: int = 0, pairs: bool = False,
                          out: Optional[torch.Tensor] = None, nf: Optional[int] = None,
                          rowmajor: Optional[bool] = None, ring2: Optional[bool] = None) -> torch.Tensor:
    """The weight-streaming fused LM head + sampler (M <= 128 rows): ``w`` [Vpad, K] row-major (or,
    ``rowmajor=False``, its ``ops.gemm.tile_weight`` copy of the [Vpad, K] weight), global rows
    voff .. voff+vvalid-1 then padding.  Returns int32 tokens [M], or (``pairs``) the [M, 2]
    (score bits, global id) shard candidates of :func:`sample_shard`."""
    M, K = h.shape
    Vpad = w.shape[0] * (16 if w.dim() == 4 else 1)
    vvalid = Vpad if vvalid is None else vvalid
    d_nf, d_r2 = stream_cfg(M)
    nf = d_nf if nf is None else nf
    rowmajor = (w.dim() == 2) if rowmajor is None else rowmajor
    ring2 = d_r2 if ring2 is None else ring2
    P = Vpad // (16 * nf) * 2
    ws = torch.empty((2 * M * P,), dtype=torch.float32, device=h.device)
    temps, sd = temperatures.to(torch.float32).contiguous(), seeds.contiguous()   # alive across the launch
    if pairs:
        res = torch.empty((M, 2), dtype=torch.int32, device=h.device)
        o, pr = None, res
    else:
        res = torch.empty((M,), dtype=torch.int32, device=h.device) if out is None else out
        o, pr = res, None
    N.call("penny_lm_head_stream_sample", N.ptr(h), h.stride(0), N.ptr(w), K, M, Vpad, int(vvalid), int(voff),
           N.ptr(temps), N.ptr(sd), N.ptr(ws), N.ptr(o), N.ptr(pr), int(nf), int(rowmajor), int(ring2), N.stream())
    return res


def lm_head_sample(h: torch.Tensor, w: torch.Tensor, temperatures: torch.Tensor, seeds: torch.Tensor,
                   out: Optional[torch.Tensor] = None, wt: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Sample one token per row of ``h`` [M, K] from softmax((h @ w.T) / T) (T <= 0: greedy) without
    materialising the logits.  Same noise as :func:`sample` (counter-based on (seed, token id)),
    scored on the bf16-rounded logits, so for equal logits both paths pick the same token.  The
    MFMA kernels and hipBLASLt accumulate in different orders, though, so a row whose two best scores
    lie within logit rounding can differ between the paths (tokens are reproducible up to logit
    rounding; the rate is measured by tests/test_kernels_gpu.py::test_fused_vs_unfused_sampling_
    token_agreement).  No top-k / top-p (those rows need the whole distribution: use ``sample``).
    ``wt``: the fragment-tiled copy of ``w`` (``ops.gemm.tile_weight``), streamed instead of ``w`` by
    the decode-size kernel when given."""
    import os
    M, K = h.shape
    V = w.shape[0]
    if not N.use_native(h):
        import torch.nn.functional as F
        return sample(F.linear(h.float(), w.float()).to(h.dtype), temperatures, seeds, out=out)
    if _stream_ok(M) and os.environ.get("PENNY_FUSED_LM_HEAD") != "force" and V % (16 * stream_cfg(M)[0]) == 0:
        return lm_head_stream_sample(h, wt if wt is not None else w, temperatures, seeds, out=out)
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
        logits = _aligned_rows(logits)           # any shard width, no assert on the TP step
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
                         seeds: torch.Tensor, wt: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Fused LM head + sampler on one vocab shard: ``w_pad`` [Vpad, K] (Vpad % 256 == 0) holds global
    rows voff .. voff+vvalid-1 then padding -> pairs [M, 2] as :func:`sample_shard`."""
    import os
    M, K = h.shape
    Vpad = w_pad.shape[0]
    if _stream_ok(M) and os.environ.get("PENNY_FUSED_LM_HEAD") != "force" and Vpad % (16 * stream_cfg(M)[0]) == 0:
        return lm_head_stream_sample(h, wt if wt is not None else w_pad, temperatures, seeds, vvalid=vvalid,
                                     voff=voff, pairs=True)
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
