"""Mixtral-8x7B sparse-MoE decoder (north-star config 5).

Attention, norms and embeddings are shared with :class:`~.llama.DecoderModel`; the MLP is a
top-2-of-8 mixture of SiLU-gated experts:

    router  p = softmax(h W_r^T)  (f32), top-2, renormalised (HF Mixtral semantics)
    expert  y_e = W2_e (silu(W1_e h) * W3_e h)
    combine out = sum_k p_k y_{e_k}

Two execution forms, chosen per step:
* grouped (prefill, large T): tokens are bucketed by expert (``ops.moe.route``) and each expert
  runs ONE GEMM pair over its bucket -- 2/8 of the dense FLOPs.
* dense-masked (decode, small T, hipGraph-capturable): every expert runs over the whole batch
  and the routing weights (zero for unselected experts) scale the combine.  At decode batch
  sizes every expert's weights are streamed anyway, so this costs no extra HBM traffic and has
  no data-dependent shapes.

TP shards every expert's intermediate dimension (column-parallel W1|W3, row-parallel W2); the
partial sums join the O-projection's all-reduce pattern (C1).  Expert weights may be stored in
OCP fp8-e4m3 with per-output-channel scales (``fp8=True``), halving the expert bytes streamed
per decode step.
"""
from __future__ import annotations

from typing import Dict

import torch
import torch.nn.functional as F

from .. import ops
from ..ops import moe as moe_ops
from ..parallel import comm
from .llama import DecoderModel


class MixtralModel(DecoderModel):
    dense_threshold = 64   # tokens per step at or below which the dense-masked form is used

    def __init__(self, *a, fp8: bool = False, **kw):
        super().__init__(*a, **kw)
        self.fp8 = fp8

    def mlp_shapes(self, p: str) -> Dict[str, tuple]:
        c = self.cfg
        E, H, F_ = c.num_experts, c.hidden_size, c.intermediate_size
        return {p + "router": (E, H), p + "w13": (E, 2 * F_, H), p + "w2": (E, H, F_)}

    def init_random(self, seed: int = 0, std: float = 0.02) -> "MixtralModel":
        super().init_random(seed, std)
        if self.fp8:
            self.quantize_experts()
        return self

    def quantize_experts(self) -> None:
        for i in range(self.cfg.num_layers):
            p = f"layers.{i}."
            for k in ("w13", "w2"):
                q, s = moe_ops.quantize_fp8_rowwise(self.w[p + k])
                self.w[p + k] = q
                self.w[p + k + "_scale"] = s

    def _expert_weights(self, p: str, e: int):
        w13, w2 = self.w[p + "w13"][e], self.w[p + "w2"][e]
        if self.fp8:
            w13 = moe_ops.dequant_fp8(w13, self.w[p + "w13_scale"][e])
            w2 = moe_ops.dequant_fp8(w2, self.w[p + "w2_scale"][e])
        return w13, w2

    def mlp(self, i: int, h: torch.Tensor) -> torch.Tensor:
        p = f"layers.{i}."
        c = self.cfg
        T = h.shape[0]
        logits = F.linear(h, self.w[p + "router"])
        topw, topi = moe_ops.topk_softmax(logits, c.top_k_experts)
        out = torch.zeros_like(h)
        if T <= self.dense_threshold:
            dense_w = torch.zeros((T, c.num_experts), dtype=torch.float32, device=h.device)
            dense_w.scatter_(1, topi.long(), topw)
            for e in range(c.num_experts):
                w13, w2 = self._expert_weights(p, e)
                y = F.linear(ops.silu_mul(F.linear(h, w13)), w2)
                out += (y.float() * dense_w[:, e:e + 1]).to(h.dtype)
        else:
            order, offsets, tok_idx, tok_w = moe_ops.route(topi, topw, c.num_experts)
            offs = offsets.tolist()
            xs = h.index_select(0, tok_idx)
            ys = torch.empty_like(xs)
            for e in range(c.num_experts):
                a, b = offs[e], offs[e + 1]
                if b > a:
                    w13, w2 = self._expert_weights(p, e)
                    ys[a:b] = F.linear(ops.silu_mul(F.linear(xs[a:b], w13)), w2)
            out.index_add_(0, tok_idx, (ys.float() * tok_w[:, None]).to(h.dtype))
        return comm.tp_all_reduce(out) if self.tp_size > 1 else out
