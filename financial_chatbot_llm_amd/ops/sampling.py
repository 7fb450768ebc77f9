"""K12: temperature / Gumbel-max sampling and greedy argmax over full-vocab logits."""
from __future__ import annotations

from typing import Optional

import torch

from . import _native as N

SPLITS = 16  # vocab slices per row in the HIP sampler (SAMPLE_SPLITS)


def sample(logits: torch.Tensor, temperatures: torch.Tensor, seeds: torch.Tensor,
           out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """logits [B, V] (bf16 or f32), temperatures [B] f32 (<= 0 -> greedy), seeds [B] int64.

    Returns int32 token ids [B].  On the GPU the HIP kernel draws counter-based Gumbel noise
    from (seed, token index); the CPU reference uses torch's generator seeded per row, so the two
    paths agree exactly for greedy rows and in distribution for sampled rows.
    """
    B, V = logits.shape
    if N.use_native(logits):
        out = torch.empty((B,), dtype=torch.int32, device=logits.device) if out is None else out
        assert logits.stride(1) == 1 and logits.stride(0) % 8 == 0
        ws = torch.empty((B * SPLITS * 2,), dtype=torch.float32, device=logits.device)
        N.call("penny_sample", N.ptr(logits), int(logits.dtype == torch.float32), logits.stride(0),
               N.ptr(temperatures), N.ptr(seeds), N.ptr(out), N.ptr(ws), B, V, N.stream())
        return out
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


def apply_top_k_top_p(logits: torch.Tensor, top_k: torch.Tensor, top_p: torch.Tensor) -> torch.Tensor:
    """Mask logits outside top-k / nucleus top-p (rows with k<=0 / p>=1 untouched)."""
    if bool((top_k <= 0).all()) and bool((top_p >= 1).all()):
        return logits
    lf = logits.float()
    sorted_l, idx = torch.sort(lf, dim=-1, descending=True)
    V = lf.shape[-1]
    ranks = torch.arange(V, device=lf.device)[None, :]
    k = torch.where(top_k > 0, top_k, torch.full_like(top_k, V))[:, None]
    drop = ranks >= k
    probs = torch.softmax(sorted_l, dim=-1)
    cum = probs.cumsum(-1) - probs
    drop |= cum > top_p[:, None].float()
    sorted_l = sorted_l.masked_fill(drop, float("-inf"))
    return torch.empty_like(lf).scatter_(-1, idx, sorted_l).to(logits.dtype)
