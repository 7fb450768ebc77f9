"""K9 epilogue (SiLU(gate) * up) and BERT GELU."""
from __future__ import annotations

import torch

from . import _native as N


def deinterleave16(gu: torch.Tensor):
    """Split a 16-column-interleaved gate/up activation into (gate, up)."""
    F = gu.shape[-1] // 2
    v = gu.reshape(*gu.shape[:-1], F // 16, 2, 16)
    return v[..., 0, :].reshape(*gu.shape[:-1], F), v[..., 1, :].reshape(*gu.shape[:-1], F)


def silu_mul(gu: torch.Tensor, interleave16: bool = False) -> torch.Tensor:
    """gu [T, 2F] (gate | up, or 16-column interleaved) -> silu(gate) * up  [T, F]."""
    F = gu.shape[-1] // 2
    T = gu.numel() // gu.shape[-1]
    if N.use_native(gu):
        out = torch.empty(gu.shape[:-1] + (F,), dtype=gu.dtype, device=gu.device)
        N.call("penny_silu_mul", N.ptr(gu), N.ptr(out), T, F, int(interleave16), N.stream())
        return out
    g, u = deinterleave16(gu) if interleave16 else (gu[..., :F], gu[..., F:])
    return (torch.nn.functional.silu(g.float()).to(gu.dtype).float() * u.float()).to(gu.dtype)


def gelu_(x: torch.Tensor) -> torch.Tensor:
    if N.use_native(x):
        N.call("penny_gelu", N.ptr(x), x.numel(), N.stream())
        return x
    x.copy_(torch.nn.functional.gelu(x.float()).to(x.dtype))
    return x
