"""K2/K14 normalisation ops: fused residual-add + RMSNorm, residual-add + LayerNorm."""
from __future__ import annotations

from typing import Optional, Tuple, Union

import torch

from . import _native as N
from .gemm import ResidualSum, Slabs


def _rms_ref(x: torch.Tensor, w: torch.Tensor, eps: float) -> torch.Tensor:
    xf = x.float()
    y = (xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + eps)).to(x.dtype)
    return (y.float() * w.float()).to(x.dtype)


def rms_norm(x: Union[torch.Tensor, Slabs], w: torch.Tensor, eps: float, residual: Optional[torch.Tensor] = None,
             out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """``residual is None``: y = rms(x).  Otherwise residual <- x + residual (in place, bf16) and
    y = rms(residual) -- the Llama pre-norm pattern, one HBM pass.  ``x`` may be the unreduced
    :class:`~.gemm.Slabs` of a split-K GEMM: the slabs are summed in the same pass."""
    if isinstance(x, ResidualSum):    # the GEMM epilogue already added x into the residual stream
        assert residual is None or residual is x.t
        return rms_norm(x.t, w, eps, None, out)
    if isinstance(x, Slabs):
        S, T, H = x.P.shape
        if N.use_native(x.P):
            out = torch.empty((T, H), dtype=torch.bfloat16, device=x.P.device) if out is None else out
            N.call("penny_rmsnorm_slabs", N.ptr(x.P), S, N.ptr(residual), N.ptr(w), N.ptr(out), T, H, float(eps),
                   int(residual is not None), N.stream())
            return out
        x = x.materialize()
    H = x.shape[-1]
    T = x.numel() // H
    if N.use_native(x):
        out = torch.empty_like(x) if out is None else out
        N.call("penny_rmsnorm", N.ptr(x), N.ptr(residual), N.ptr(w), N.ptr(out), T, H, float(eps),
               int(residual is not None), N.stream())
        return out
    if residual is not None:
        residual.copy_((x + residual).to(residual.dtype))
        x = residual
    y = _rms_ref(x, w, eps)
    if out is not None:
        out.copy_(y)
        return out
    return y


def layer_norm(x: torch.Tensor, g: torch.Tensor, b: torch.Tensor, eps: float,
               residual: Optional[torch.Tensor] = None) -> torch.Tensor:
    """y = LN(x + residual) (residual optional), f32 statistics, bf16 out."""
    H = x.shape[-1]
    T = x.numel() // H
    if N.use_native(x):
        out = torch.empty_like(x)
        N.call("penny_layernorm", N.ptr(x), N.ptr(residual), N.ptr(g), N.ptr(b), N.ptr(out), T, H, float(eps),
               int(residual is not None), N.stream())
        return out
    xf = x.float() + (residual.float() if residual is not None else 0.0)
    return torch.nn.functional.layer_norm(xf, (H,), g.float(), b.float(), eps).to(x.dtype)
