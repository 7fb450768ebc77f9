"""Mixtral-8x7B sparse-MoE decoder (north-star config 5).

Attention, norms and embeddings are shared with :class:`~.llama.DecoderModel`; the MLP is a
top-2-of-8 mixture of SiLU-gated experts:

    router  p = softmax(h W_r^T)  (f32), top-2, renormalised (HF Mixtral semantics)
    expert  y_e = W2_e (silu(W1_e h) * W3_e h)
    combine out = sum_k p_k y_{e_k}

Execution forms:
* fp8 experts on the GPU, decode-sized steps (T*top_k <= 4096): the HIP pipeline of
  ``csrc/kernels/moe.hip`` -- device routing + counting sort, dynamic per-token fp8
  activations, grouped fp8 x fp8 MFMA GEMMs over expert buckets with fused SiLU / routing-weight
  epilogues, atomics-free combine.  Weights are OCP e4m3 with per-output-row scales, stored in
  MFMA-fragment tiles, halving the expert bytes streamed per decode step vs bf16.
* fp8 experts, prefill-sized steps: ``ops.moe.moe_prefill_fp8_tiles`` -- device routing, grouped
  256x256 fp8 tile GEMMs over the expert buckets (``gemm_prefill.hip``, block-scaled 16x16x128
  MFMA) with the SiLU / routing-weight epilogues, no host sync: 1.48-1.79 PF/s per MoE layer at
  T = 4096-16384 vs 1.18-1.88 for the per-expert hipBLASLt loop it replaced
  (``profiles/r3_moe_prefill_tiles_vs_hipblaslt.jsonl``; ``PENNY_MOE_PREFILL_TILES=0`` restores it).
* bf16 experts, decode-sized steps: every expert densely over the step's rows, weighted by the
  routing weights (decode streams every expert's weights anyway; no host sync, so hipGraph
  decode captures it).
* otherwise (bf16 prefill, CPU): tokens are bucketed by expert (``ops.moe.route``) and each
  expert runs one GEMM pair over its bucket; this form reads the bucket sizes on the host once
  per layer.

Under TP the experts are parallelised one of two ways (``moe_parallel``):
* ``"tp"`` (default, hipGraph decode path): every expert's intermediate dimension is sharded
  (column-parallel W1|W3, row-parallel W2) and the partial sums are all-reduced (C1);
* ``"ep"``: whole experts are partitioned over the TP group and routed rows travel by
  all-to-all dispatch/combine (C3, ``parallel/ep.py``).
"""
from __future__ import annotations

from typing import Dict, Optional

import torch
import torch.nn.functional as F

from .. import ops
from ..ops import moe as moe_ops
from ..ops.gemm import linear
from ..parallel import comm
from ..parallel.dist import state as pstate
from ..parallel.ep import ep_moe, expert_range
from .llama import DecoderModel

# bf16 experts: steps of at most this many (token, expert) pairs run every expert densely (no host
# sync, hipGraph-capturable); larger ones the bucketed per-expert loop
BF16_DENSE_MAX_PAIRS = 512


class MixtralModel(DecoderModel):
    def __init__(self, *a, fp8: bool = False, moe_parallel: str = "tp", prefill_dequant_cache: bool = True,
                 prefill_fp8: bool = True, **kw):
        super().__init__(*a, **kw)
        # fp8 experts, prefill-size chunks: hipBLASLt fp8 x fp8 GEMMs (torch._scaled_mm, per-row
        # activation x per-row weight scales) on an untiled copy of the SAME quantized experts --
        # the arithmetic of the decode fp8 MFMA pipeline (dynamic per-row fp8 activations) at
        # 1.4-1.8x the bf16 GEMM rate (profiles/r1_scaled_mm_probe.jsonl); otherwise a resident bf16
        # dequantized copy (``prefill_dequant_cache``) or per-step dequantization
        self.prefill_fp8 = prefill_fp8 and self.device.type == "cuda" and hasattr(torch, "_scaled_mm")
        self.prefill_dequant_cache = prefill_dequant_cache and not self.prefill_fp8
        if moe_parallel not in ("tp", "ep"):
            raise ValueError(f"moe_parallel must be 'tp' or 'ep', got {moe_parallel!r}")
        self.fp8 = fp8
        self.ep = moe_parallel == "ep" and self.tp_size > 1
        if self.ep:
            self.expert_lo, self.expert_hi = expert_range(self.cfg.num_experts, self.tp_rank, self.tp_size)
        self._moe_ws = None

    def shard(self, name: str, full: torch.Tensor) -> torch.Tensor:
        if self.ep and name.rsplit(".", 1)[-1] in ("w13", "w2"):
            return full[self.expert_lo:self.expert_hi].contiguous()   # whole local experts
        return super().shard(name, full)

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
        """bf16 experts -> fp8 e4m3 (per-row scales), W1|W3 interleaved by 16 rows, fragment-tiled."""
        for i in range(self.cfg.num_layers):
            p = f"layers.{i}."
            w13 = self.w.pop(p + "w13")
            half = w13.shape[1] // 2
            w13 = torch.stack([ops.gemm.interleave16(w13[e, :half], w13[e, half:]) for e in range(w13.shape[0])])
            for k, w in ((p + "w13", w13), (p + "w2", self.w.pop(p + "w2"))):
                q, s = moe_ops.quantize_fp8_rowwise(w)
                self.w[k + "_t"] = moe_ops.tile_fp8_weight(q)
                self.w[k + "_scale"] = s.float().contiguous()
                if self.prefill_fp8:
                    self.w[k + "_q"] = q.contiguous()          # [E, N, K] e4m3, row-major
                elif self.prefill_dequant_cache:
                    # the SAME quantized values in bf16 for the prefill GEMMs (hipBLASLt): ~90 GB for
                    # 8x7B -- HBM3E has it, and prefill stops re-dequantizing 2.8 GB per layer per step
                    self.w[k + "_deq"] = moe_ops.dequant_fp8(q, s, self.dtype)
                del q, w
        self.fp8 = True
        if self.device.type == "cuda":
            torch.cuda.empty_cache()   # return the bf16 experts to the pool before KV planning

    def _dequant(self, p: str, key: str, e: int) -> torch.Tensor:
        """One expert's fp8 weights -> [rows, cols] in the compute dtype (prefill path)."""
        cached = self.w.get(p + key + "_deq")
        if cached is not None:
            return cached[e]
        q = moe_ops.untile_fp8_weight(self.w[p + key + "_t"][e:e + 1])[0]
        return moe_ops.dequant_fp8(q, self.w[p + key + "_scale"][e], self.dtype)

    def _moe_workspace(self, T: int):
        c = self.cfg
        if self._moe_ws is None or self._moe_ws.max_tokens < T:
            f_local = self.w["layers.0.w13_scale"].shape[-1] // 2   # per-rank expert FFN width
            self._moe_ws = moe_ops.MoEWorkspace(max(T, 256), c.top_k_experts, c.num_experts, c.hidden_size,
                                                f_local, self.device)
        return self._moe_ws

    def _expert_fp8(self, p: str, rows: torch.Tensor, e: int, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """One expert on its routed rows with fp8 x fp8 hipBLASLt GEMMs (prefill-size buckets).
        ``out``: the expert's slice of the sorted-row output, written by the down GEMM directly
        (no copy kernel per expert and layer)."""
        xq, xs = moe_ops.quant_rows_fp8(rows)
        y13 = torch._scaled_mm(xq, self.w[p + "w13_q"][e].t(), scale_a=xs[:, None],
                               scale_b=self.w[p + "w13_scale"][e][None, :], out_dtype=self.dtype)
        aq, as_ = moe_ops.silu_quant_rows_fp8(y13)
        if out is not None:
            return torch._scaled_mm(aq, self.w[p + "w2_q"][e].t(), scale_a=as_[:, None],
                                    scale_b=self.w[p + "w2_scale"][e][None, :], out_dtype=self.dtype, out=out)
        return torch._scaled_mm(aq, self.w[p + "w2_q"][e].t(), scale_a=as_[:, None],
                                scale_b=self.w[p + "w2_scale"][e][None, :], out_dtype=self.dtype)

    def _expert(self, p: str, rows: torch.Tensor, e: int, out: Optional[torch.Tensor] = None) -> torch.Tensor:
        """One (local) expert on its routed rows (eager path); the result lands in ``out`` if given."""
        if self.fp8 and self.prefill_fp8 and (p + "w13_q") in self.w:
            return self._expert_fp8(p, rows, e, out)
        y = self._expert_bf16(p, rows, e)
        if out is not None:
            out.copy_(y)
            return out
        return y

    def _expert_bf16(self, p: str, rows: torch.Tensor, e: int) -> torch.Tensor:
        if self.fp8:
            act = ops.silu_mul(F.linear(rows, self._dequant(p, "w13", e)), interleave16=True)
            return F.linear(act, self._dequant(p, "w2", e))
        return F.linear(ops.silu_mul(F.linear(rows, self.w[p + "w13"][e])), self.w[p + "w2"][e])

    def mlp(self, i: int, h: torch.Tensor, reduce: bool = True, fuse_residual=None) -> torch.Tensor:
        """``reduce=False``: return the TP partial sum (the overlapped forward all-reduces it);
        expert-parallel outputs are already complete (all-gathered) either way."""
        p = f"layers.{i}."
        c = self.cfg
        T = h.shape[0]
        logits = linear(h, self.w[p + "router"])
        if self.ep:
            grouped = None
            if self.fp8 and ops._native.use_native(h):   # one grouped fp8 call, device bucket offsets
                tiles = ((p + "w13_q") in self.w and moe_ops.PREFILL_TILES
                         and self.w[p + "w13_q"].shape[1] % 256 == 0)

                def grouped(rows, ids):
                    # prefill-size receives: the 256x256 fp8 tile kernel; decode-size: the
                    # weight-streaming grouped kernel
                    if tiles and rows.shape[0] >= moe_ops.EP_TILE_MIN_ROWS:
                        return moe_ops.moe_grouped_fp8_tiles(rows.contiguous(), ids, self.w[p + "w13_q"],
                                                             self.w[p + "w13_scale"], self.w[p + "w2_q"],
                                                             self.w[p + "w2_scale"])
                    return moe_ops.moe_grouped_fp8(rows.contiguous(), ids, self.w[p + "w13_t"], self.w[p + "w13_scale"],
                                                   self.w[p + "w2_t"], self.w[p + "w2_scale"])
            return ep_moe(h, logits, c.top_k_experts, c.num_experts, lambda rows, e: self._expert(p, rows, e),
                          group=pstate().tp_group, grouped_fn=grouped)
        # fp8 MFMA pipeline while the step is weight-bandwidth-bound; bigger prefill chunks go to
        # hipBLASLt on the cached bf16 copy of the same quantized experts (compute-bound regime)
        fp8_limit = 1024 if (self.prefill_dequant_cache or self.prefill_fp8) else 4096
        if self.fp8 and ops._native.use_native(h) and T * c.top_k_experts <= fp8_limit:
            out = moe_ops.moe_decode_fp8(h.contiguous(), logits.contiguous(), self.w[p + "w13_t"],
                                         self.w[p + "w13_scale"], self.w[p + "w2_t"], self.w[p + "w2_scale"],
                                         c.top_k_experts, self._moe_workspace(T))
            return comm.tp_all_reduce(out) if self.tp_size > 1 and reduce else out
        if (self.fp8 and ops._native.use_native(h) and (p + "w13_q") in self.w
                and moe_ops.PREFILL_TILES and self.w[p + "w13_q"].shape[1] % 256 == 0):
            # prefill-size step: grouped fp8 tile GEMMs over device-side expert buckets (no host sync)
            out = moe_ops.moe_prefill_fp8_tiles(h.contiguous(), logits.contiguous(), self.w[p + "w13_q"],
                                                self.w[p + "w13_scale"], self.w[p + "w2_q"], self.w[p + "w2_scale"],
                                                c.top_k_experts)
            return comm.tp_all_reduce(out) if self.tp_size > 1 and reduce else out
        topw, topi = moe_ops.topk_softmax(logits, c.top_k_experts)
        if not self.fp8 and (T * c.top_k_experts <= BF16_DENSE_MAX_PAIRS
                             or (h.is_cuda and torch.cuda.is_current_stream_capturing())):
            # bf16 decode sizes: every expert over every row, weighted by the (mostly zero) routing
            # weights -- decode streams all experts' weights each step anyway, and this form has no
            # host sync, so it is hipGraph-capturable (the bucketed loop below reads sizes on the host)
            wfull = torch.zeros((T, c.num_experts), dtype=torch.float32, device=h.device)
            wfull.scatter_(1, topi.long(), topw.float())
            out = torch.zeros((T, h.shape[1]), dtype=torch.float32, device=h.device)
            for e in range(c.num_experts):
                out.add_(self._expert_bf16(p, h, e).float() * wfull[:, e:e + 1])
            out = out.to(h.dtype)
            return comm.tp_all_reduce(out) if self.tp_size > 1 and reduce else out
        order, offsets, tok_idx, tok_w = moe_ops.route(topi, topw, c.num_experts)
        offs = offsets.tolist()
        xs = h.index_select(0, tok_idx)
        ys = torch.empty_like(xs)
        for e in range(c.num_experts):
            a, b = offs[e], offs[e + 1]
            if b > a:
                self._expert(p, xs[a:b], e, out=ys[a:b])
        # every sorted row is written above (the buckets tile [0, T*k)); weighted gather-combine
        out = moe_ops.combine_weighted(ys, order, tok_w, T, c.top_k_experts)
        return comm.tp_all_reduce(out) if self.tp_size > 1 and reduce else out
