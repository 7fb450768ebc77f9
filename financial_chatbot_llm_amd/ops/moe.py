"""K13 MoE helpers: router top-k softmax, token bucketing by expert, fp8-e4m3 (OCP) weights.

gfx950 uses the OCP ``e4m3fn`` encoding (not MI300's ``fnuz``), which is torch.float8_e4m3fn.
"""
from __future__ import annotations

from typing import Tuple

import torch

FP8 = torch.float8_e4m3fn
FP8_MAX = 448.0


def topk_softmax(logits: torch.Tensor, k: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """HF Mixtral routing: softmax over all experts (f32), top-k, renormalise."""
    p = torch.softmax(logits.float(), dim=-1)
    w, i = torch.topk(p, k, dim=-1)
    w = w / w.sum(-1, keepdim=True)
    return w, i.to(torch.int32)


def route(topi: torch.Tensor, topw: torch.Tensor, num_experts: int):
    """Bucket (token, expert) pairs by expert.

    Returns ``order`` (permutation of the flattened pairs), ``offsets`` [E+1] (bucket bounds),
    ``tok_idx`` (token of each sorted pair) and ``tok_w`` (its routing weight)."""
    T, k = topi.shape
    flat_e = topi.reshape(-1).long()
    order = torch.argsort(flat_e, stable=True)
    counts = torch.bincount(flat_e, minlength=num_experts)
    offsets = torch.zeros(num_experts + 1, dtype=torch.long, device=topi.device)
    offsets[1:] = counts.cumsum(0)
    tok_idx = (order // k)
    tok_w = topw.reshape(-1)[order].float()
    return order, offsets, tok_idx, tok_w


def quantize_fp8_rowwise(w: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """w [..., out, in] -> (fp8 e4m3fn, f32 scale [..., out]) with w ~= q * scale[..., None]."""
    amax = w.float().abs().amax(dim=-1).clamp_min(1e-12)
    scale = amax / FP8_MAX
    q = (w.float() / scale[..., None]).clamp(-FP8_MAX, FP8_MAX).to(FP8)
    return q, scale


def dequant_fp8(q: torch.Tensor, scale: torch.Tensor, dtype=torch.bfloat16) -> torch.Tensor:
    return (q.float() * scale[..., None]).to(dtype)
