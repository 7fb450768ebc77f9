"""Llama-3 decoder (8B / 70B) and the shared decoder skeleton used by Mixtral.

Replaces the remote Gemini model of the reference (``llm_agent.py:34-45``) with a local
decoder whose per-layer hot path is::

    K2 add+RMSNorm -> K3 QKV GEMM -> K4/K5 RoPE + paged KV write (fused into the prefill tile GEMM's
    epilogue, or a separate HIP pass) -> K6/K7 paged attention (HIP, MFMA) -> K8 O GEMM [-> C1
    all-reduce] -> K2 add+RMSNorm -> K9 gate|up GEMM + SiLU*mul (fused epilogue) -> K10 down GEMM
    [-> C1]; the GEMM kernel per shape and step size follows ops/gemm.py (PREFILL_POLICY).

Weights are plain bf16 tensors (``[out, in]``), sharded Megatron-style over the TP group:
QKV/gate-up column-parallel (whole heads per rank), O/down row-parallel, embedding and LM head
vocab-parallel.  The batch is flat: prefill tokens of several sequences followed by one token
per decoding sequence (continuous batching); the attention split is described by
:class:`~.common.AttentionMetadata`.
"""
from __future__ import annotations

import math
import os
from typing import Dict, List, Optional

import torch
import torch.nn.functional as F

from .. import ops
from ..parallel import comm
from ..parallel.dist import state as pstate
from ..ops.attention import _side_stream, fork_join_events

_DUAL_STREAMS: Dict[int, "torch.cuda.Stream"] = {}


def _dual_stream(device) -> "torch.cuda.Stream":
    """The second decode micro-batch chain's stream (forward_decode_dual), one per device."""
    key = torch.device(device).index
    if key not in _DUAL_STREAMS:
        _DUAL_STREAMS[key] = torch.cuda.Stream(device=device)
    return _DUAL_STREAMS[key]
from ..ops.gemm import (interleave16, linear, linear_tiled, prefill_qkv_rope, qkv_rope_fused, tile_weight,
                        tiled_only, uses_tiled_weight)
from ..parallel.layers import shard_cols, shard_rows, shard_sections, vocab_range
from .common import AttentionMetadata, KVCache, random_tensor
from .configs import ModelConfig


# mixed prefill+decode steps overlap the two attention kernels on two streams (PENNY_ATTN_OVERLAP=0:
# one stream, prefill then decode)
ATTN_OVERLAP = os.environ.get("PENNY_ATTN_OVERLAP", "1") != "0"
# fused-QKV prefill steps hand the attention q prescaled by scale * log2(e) (ops.gemm.prefill_qkv_rope
# qscale; ops.prefill q_prescaled): the prescaled-Q fold's block loop (+7.5-8.6 % per prefill
# attention call, profiles/r5_prefill_attn_fold_ab.jsonl variant 6) at the exact form's precision
# (q rounded once either way: tests/test_kernels_gpu.py test_prefill_attention_prescaled_q).  Driver
# bench A/B on one box: 32.53 vs 32.51 turns/s (the prefill attention shares its steps with the decode
# rows' attention on the side stream).  PENNY_PRESCALE_Q=0 keeps q unscaled.
PRESCALE_Q = os.environ.get("PENNY_PRESCALE_Q", "1") != "0"
LOG2E = 1.4426950408889634


class DecoderModel:
    """Llama-family decoder; subclasses override the MLP (Mixtral MoE)."""

    def __init__(self, cfg: ModelConfig, device="cuda", tp_rank: Optional[int] = None,
                 tp_size: Optional[int] = None, dtype=torch.bfloat16):
        ps = pstate()
        self.cfg = cfg
        self.device = torch.device(device)
        self.dtype = dtype
        self.tp_rank = ps.tp_rank if tp_rank is None else tp_rank
        self.tp_size = ps.tp_size if tp_size is None else tp_size
        if cfg.num_heads % self.tp_size or cfg.num_kv_heads % self.tp_size:
            raise ValueError(f"heads {cfg.num_heads}/{cfg.num_kv_heads} not divisible by tp={self.tp_size}")
        self.hq = cfg.num_heads // self.tp_size
        self.hkv = cfg.num_kv_heads // self.tp_size
        self.D = cfg.head_dim
        self.scale = 1.0 / math.sqrt(self.D)
        self.vocab_start, self.vocab_end = vocab_range(cfg.vocab_size, self.tp_rank, self.tp_size)
        self.w: Dict[str, torch.Tensor] = {}
        self.wt: Dict[str, torch.Tensor] = {}
        # sequence parallelism for long prefills under TP (dense MLP only): steps of at least
        # sp_min_tokens rows run forward_sp (reduce-scatter / all-gather instead of all-reduce)
        self.sequence_parallel = False
        self.sp_min_tokens = 1024
        self.cos_sin = ops.rope_cos_sin(self.D, cfg.max_position, cfg.rope_theta, cfg.rope_scaling,
                                        device=self.device)

    # ------------------------------------------------------------------------------------
    # weights
    # ------------------------------------------------------------------------------------
    def full_shapes(self) -> Dict[str, tuple]:
        c = self.cfg
        H, F_ = c.hidden_size, c.intermediate_size
        shapes = {"embed": (c.vocab_size, H), "final_norm": (H,)}
        if not c.tie_embeddings:
            shapes["lm_head"] = (c.vocab_size, H)
        for i in range(c.num_layers):
            p = f"layers.{i}."
            shapes[p + "in_norm"] = (H,)
            shapes[p + "post_norm"] = (H,)
            shapes[p + "qkv"] = (c.q_size + 2 * c.kv_size, H)
            shapes[p + "o"] = (H, c.q_size)
            shapes.update(self.mlp_shapes(p))
        return shapes

    def mlp_shapes(self, p: str) -> Dict[str, tuple]:
        c = self.cfg
        return {p + "gate_up": (2 * c.intermediate_size, c.hidden_size), p + "down": (c.hidden_size, c.intermediate_size)}

    def shard(self, name: str, full: torch.Tensor) -> torch.Tensor:
        """Full (unsharded) parameter -> this rank's shard."""
        r, n, c = self.tp_rank, self.tp_size, self.cfg
        leaf = name.rsplit(".", 1)[-1]
        if leaf in ("embed", "lm_head"):
            if n == 1:
                return full
            a, b = self.vocab_start, self.vocab_end
            return full[a:b].contiguous()
        if leaf == "qkv":
            return shard_sections(full, [c.q_size, c.kv_size, c.kv_size], r, n)
        if leaf == "gate_up":
            # column-parallel per half, then 16-row gate/up interleave (decode GEMM's fused SiLU)
            half = full.shape[0] // 2
            return interleave16(shard_rows(full[:half], r, n), shard_rows(full[half:], r, n)).contiguous()
        if leaf == "w13":
            half = full.shape[-2] // 2
            if n == 1:
                return full
            return torch.cat([full[:, :half].chunk(n, 1)[r], full[:, half:].chunk(n, 1)[r]], 1).contiguous()
        if n == 1:
            return full
        if leaf in ("o", "down"):
            return shard_cols(full, r, n)
        if leaf == "w2":  # [E, H, F]
            return full.chunk(n, 2)[r].contiguous()
        return full

    def init_random(self, seed: int = 0, std: float = 0.02) -> "DecoderModel":
        for name, shape in self.full_shapes().items():
            kind = "ones" if name.endswith("norm") else "normal"
            full = random_tensor(name, shape, seed, self.device, self.dtype, std=std, kind=kind)
            self.w[name] = self.shard(name, full)
            del full
        self.prepare_decode_weights()
        return self

    def load_state(self, full_weights: Dict[str, torch.Tensor]) -> "DecoderModel":
        for name, t in full_weights.items():
            self.w[name] = self.shard(name, t.to(self.device, self.dtype)).contiguous()
        missing = set(self.full_shapes()) - set(self.w)
        if missing:
            raise KeyError(f"missing weights: {sorted(missing)[:5]}...")
        self.prepare_decode_weights()
        return self

    def prepare_decode_weights(self) -> None:
        """Fragment-tiled copies of the projections the decode MFMA kernels stream (QKV, O, the
        interleaved gate|up and the dense down-projection): +13.8 GB for Llama-3-8B next to 288 GB
        of HBM3E, against ~1.2 ms (split-K QKV/O/down) + the gate|up saving per B=128 decode step.
        Only shapes some decode kernel has a measured config for are tiled (``uses_tiled_weight``)."""
        self.wt: Dict[str, torch.Tensor] = {}
        if self.device.type != "cuda":
            return
        for name, t in self.w.items():
            if t.dim() != 2 or t.shape[0] % 16 or t.shape[1] % 32:
                continue
            if name.endswith((".qkv", ".o", ".down", ".gate_up")) and uses_tiled_weight(*t.shape):
                self.wt[name] = tile_weight(t)
                if name.endswith(".gate_up") and tiled_only(*t.shape):
                    self.w[name] = None          # the tiled copy is the only one (ops.gemm.TILED_ONLY)
        self._pad_vocab_shard()
        lm = self._lm_pad
        if lm is not None and lm.shape[0] % 64 == 0 and lm.shape[1] % 64 == 0 and self._tile_lm_head():
            # the decode-size streaming LM head + sampler reads 1-KiB fragment pieces (3-7 % faster
            # than the row-major stream, profiles/r5_lm_head_stream.jsonl)
            self.wt["lm_head"] = tile_weight(lm)

    def _tile_lm_head(self) -> bool:
        """A fragment-tiled LM-head copy costs its size in HBM: made when the weights use at most 40 %
        of the device (Llama-3-8B, any TP=8 shard, Mixtral fp8), not for Llama-3-70B at TP=1, whose
        KV pool is already smaller than its working set.  ``PENNY_LM_TILED=0/1`` overrides."""
        mode = os.environ.get("PENNY_LM_TILED", "auto")
        if mode in ("0", "1"):
            return mode == "1"
        total = torch.cuda.get_device_properties(self.device).total_memory
        return self.num_bytes() <= 0.4 * total

    def lm_tiled(self) -> Optional[torch.Tensor]:
        """The fragment-tiled copy of the (padded) LM-head weight, if one was made."""
        return self.wt.get("lm_head")

    def _pad_vocab_shard(self) -> None:
        """Under TP the LM-head shard (V/tp rows: 16,032 for Llama-3 at TP=8) lives in a buffer padded
        to a multiple of 256 rows, so the fused LM-head sampler's 256-row tiles can run on it
        (``sample_vocab_parallel``); ``lm_weight()`` stays the exact-size view."""
        name = "embed" if self.cfg.tie_embeddings else "lm_head"
        t = self.w.get(name)
        self._lm_pad = t
        if t is None or self.tp_size == 1 or self.device.type != "cuda" or t.shape[0] % 256 == 0:
            return
        rows = t.shape[0]
        buf = torch.zeros((-(-rows // 256) * 256, t.shape[1]), dtype=t.dtype, device=t.device)
        buf[:rows].copy_(t)
        self.w[name] = buf[:rows]
        self._lm_pad = buf

    def num_bytes(self) -> int:
        b = sum(t.numel() * t.element_size() for t in self.w.values() if t is not None)
        return b + sum(self.wt[n].numel() * self.wt[n].element_size() for n, t in self.w.items()
                       if t is None and n in self.wt)

    # ------------------------------------------------------------------------------------
    # forward
    # ------------------------------------------------------------------------------------
    def embed(self, ids: torch.Tensor) -> torch.Tensor:
        x = ops.embedding(ids, self.w["embed"], self.vocab_start, self.vocab_end)
        return comm.tp_all_reduce(x) if self.tp_size > 1 else x

    def mlp(self, i: int, h: torch.Tensor, reduce: bool = True,
            fuse_residual: Optional[torch.Tensor] = None) -> torch.Tensor:
        p = f"layers.{i}."
        w = self.w[p + "gate_up"]
        if w is None:                             # kept only fragment-tiled (ops.gemm.TILED_ONLY)
            wt = self.wt[p + "gate_up"]
            a = linear_tiled(h, wt, wt.shape[0] * 16, epilogue="silu")
        else:
            a = linear(h, w, epilogue="silu", wt=self.wt.get(p + "gate_up"))  # fused SiLU(gate)*up
        # TP=1: decode-size batches return split-K slabs, reduced by the next add+RMSNorm; prefill
        # sizes may add the residual stream in the GEMM epilogue (fuse_residual -> ResidualSum)
        out = linear(a, self.w[p + "down"], wt=self.wt.get(p + "down"), slabs=self.tp_size == 1,
                     fuse_residual=fuse_residual)
        return comm.tp_all_reduce(out) if self.tp_size > 1 and reduce else out

    def attention(self, i: int, h: torch.Tensor, positions: torch.Tensor, meta: AttentionMetadata,
                  kv: KVCache, reduce: bool = True, fuse_residual: Optional[torch.Tensor] = None) -> torch.Tensor:
        p = f"layers.{i}."
        T = h.shape[0]
        kc, vc = kv.k(i), kv.v(i)
        scale, qpre = self.scale, False
        if qkv_rope_fused(h, self.w[p + "qkv"], self.D):
            # prefill step: QKV GEMM with RoPE + paged KV write in its epilogue (K3+K4+K5, one pass).
            # PRESCALE_Q: q leaves it times scale * log2(e) at its one bf16 rounding, so the prefill
            # attention's block loop needs no per-score multiply (the prescaled-Q fold) without the
            # extra rounding of q * c that its in-kernel form pays; every attention call of the step
            # then takes scale 1 / log2(e)
            qpre = PRESCALE_Q and h.is_cuda
            q = prefill_qkv_rope(h, self.w[p + "qkv"], positions, self.cos_sin, meta.slots, kc, vc, self.hq,
                                 self.hkv, qscale=self.scale * LOG2E if qpre else 1.0)
            if qpre:
                scale = 1.0 / LOG2E
        else:
            # QKV is column-parallel: even under TP its split-K slabs go straight to the RoPE/KV-write
            # pass (no all-reduce in between), unlike the row-parallel O / down projections
            qkv = linear(h, self.w[p + "qkv"], wt=self.wt.get(p + "qkv"), slabs=True)
            q = ops.rope_kv_write(qkv, positions, self.cos_sin, meta.slots, kc, vc, self.hq, self.hkv, self.D)
        attn = torch.empty_like(q)
        tp = meta.num_prefill_tokens
        side = None
        if tp > 0 and meta.num_decode > 0 and ATTN_OVERLAP and q.is_cuda:
            # mixed step: the decode rows' attention (HBM-bound: streams their whole contexts) runs on
            # a side stream CONCURRENTLY with the prefill rows' attention (MFMA-bound) -- the two read
            # disjoint sequences' KV and write disjoint rows of attn; joined before the O projection
            # (reused fork / join events, the raw side stream passed to the launch: no per-layer event
            # creation or current-stream switching on the host)
            side = _side_stream(q.device)
            main = torch.cuda.current_stream()
            ev_fork, ev_join = fork_join_events(q.device)
            ev_fork.record(main)
            side.wait_event(ev_fork)
            ops.decode(q[tp:], meta.ctx_lens_d, meta.block_tables_d, kc, vc, scale,
                       workspace=meta.decode_ws, out=attn[tp:], stream=side.cuda_stream)
        if tp > 0:
            ops.prefill(q[:tp], meta.cu_q, meta.ctx_lens_p, meta.block_tables_p, kc, vc, scale,
                        causal=meta.causal, max_q_len=meta.max_q_len, out=attn[:tp], work=meta.prefill_work,
                        lean=meta.prefill_lean, q_prescaled=qpre)
        if side is not None:
            ev_join.record(side)
            main.wait_event(ev_join)
        elif meta.num_decode > 0:
            ops.decode(q[tp:], meta.ctx_lens_d, meta.block_tables_d, kc, vc, scale,
                       workspace=meta.decode_ws, out=attn[tp:])
        out = linear(attn.view(T, self.hq * self.D), self.w[p + "o"], wt=self.wt.get(p + "o"),
                     slabs=self.tp_size == 1, fuse_residual=fuse_residual)
        return comm.tp_all_reduce(out) if self.tp_size > 1 and reduce else out

    def uses_sp(self, T: int) -> bool:
        return (self.sequence_parallel and self.tp_size > 1 and T >= self.sp_min_tokens
                and self.cfg.arch == "llama")

    def forward_sp(self, ids: torch.Tensor, positions: torch.Tensor, meta: AttentionMetadata,
                   kv: KVCache) -> torch.Tensor:
        """Sequence-parallel forward (Megatron SP) for long prefills under TP.

        Between the row-parallel outputs and the next column-parallel input the residual stream
        is sharded by rows: reduce-scatter after the vocab-parallel embedding / O / down, norm +
        residual add on the local T/tp rows, all-gather before QKV / gate|up.  Rows are padded to
        a multiple of tp (padding rows never reach attention: they are cut before QKV)."""
        c, n = self.cfg, self.tp_size
        T = ids.shape[0]
        Tp = -(-T // n) * n

        def pad(t: torch.Tensor) -> torch.Tensor:
            return t if Tp == T else torch.cat([t, t.new_zeros((Tp - T,) + tuple(t.shape[1:]))])

        x = comm.tp_reduce_scatter_rows(pad(ops.embedding(ids, self.w["embed"], self.vocab_start, self.vocab_end)))
        residual = x
        h = ops.rms_norm(x, self.w["layers.0.in_norm"], c.norm_eps)
        for i in range(c.num_layers):
            p = f"layers.{i}."
            if i > 0:
                h = ops.rms_norm(x, self.w[p + "in_norm"], c.norm_eps, residual=residual)
            a = self.attention(i, comm.tp_all_gather_rows(h)[:T], positions, meta, kv, reduce=False)
            a = comm.tp_reduce_scatter_rows(pad(a))
            h = ops.rms_norm(a, self.w[p + "post_norm"], c.norm_eps, residual=residual)
            x = comm.tp_reduce_scatter_rows(pad(self.mlp(i, comm.tp_all_gather_rows(h)[:T], reduce=False)))
        h = ops.rms_norm(x, self.w["final_norm"], c.norm_eps, residual=residual)
        return comm.tp_all_gather_rows(h)[:T]

    def forward_overlap(self, ids: torch.Tensor, positions: torch.Tensor, metas, split: int,
                        kv: KVCache) -> torch.Tensor:
        """TP forward with the row-parallel all-reduces overlapped with compute (C1 overlap).

        The step's rows are cut into two micro-batches at row ``split`` (``metas`` holds each
        one's attention metadata; a sequence cut in two appears in both, its second part seeing
        the first part's KV, which is written earlier on the same stream).  Per layer::

            attn(A) -> AR(A) starts | attn(B) -> AR(B) starts | wait A: norm, mlp(A) -> AR(A) ...

        so each half's all-reduce is on the wire (RCCL's stream) while the other half computes,
        instead of every all-reduce stalling the whole batch.  Same arithmetic as ``forward``."""
        c = self.cfg
        x = self.embed(ids)
        xs = [x[:split], x[split:]]
        pos = [positions[:split], positions[split:]]
        res = [xs[0], xs[1]]
        hs = [ops.rms_norm(xs[k], self.w["layers.0.in_norm"], c.norm_eps) for k in (0, 1)]
        pend = [None, None]
        for i in range(c.num_layers):
            p = f"layers.{i}."
            outs = [None, None]
            for k in (0, 1):
                if i > 0:
                    pend[k].wait()
                    hs[k] = ops.rms_norm(xs[k], self.w[p + "in_norm"], c.norm_eps, residual=res[k])
                outs[k] = self.attention(i, hs[k], pos[k], metas[k], kv, reduce=False)
                pend[k] = comm.tp_all_reduce_async(outs[k])
            for k in (0, 1):
                pend[k].wait()
                hs[k] = ops.rms_norm(outs[k], self.w[p + "post_norm"], c.norm_eps, residual=res[k])
                xs[k] = self.mlp(i, hs[k], reduce=False)
                # expert-parallel MoE outputs come back complete (all-gathered): nothing to reduce
                pend[k] = comm._Done() if getattr(self, "ep", False) else comm.tp_all_reduce_async(xs[k])
        for k in (0, 1):
            pend[k].wait()
        x = torch.cat(xs)
        return ops.rms_norm(x, self.w["final_norm"], c.norm_eps, residual=torch.cat(res))

    def forward_decode_dual(self, ids: torch.Tensor, positions: torch.Tensor, metas, split: int,
                            kv: KVCache) -> torch.Tensor:
        """TP decode with the all-reduces hidden under compute (SURVEY §5.8 "micro-batches on two
        streams"): the batch is cut at row ``split`` into two micro-batches that run as two
        INDEPENDENT chains -- embedding, every layer, final norm -- one on the current stream and
        one on a second stream, each with its own custom all-reduce instance (``comm.ar_channel``:
        own IPC buffers and flag rounds) and its own decode-attention workspace (``metas[k]``).
        While one chain's one-shot all-reduce waits for its peers (a few CUs spinning on xGMI
        flags), the other chain's GEMMs and attention use the rest of the GPU, so at 70B TP=8
        (160 all-reduces per token) the exposed all-reduce latency shrinks toward the GEMM time of
        a half batch.  Inside a hipGraph capture the two chains become parallel branches joined
        before sampling.  Same arithmetic per row as ``forward``."""
        c = self.cfg
        main = torch.cuda.current_stream(ids.device)
        side = _dual_stream(ids.device)
        side.wait_stream(main)
        streams = (main, side)
        rows = ((0, split), (split, ids.shape[0]))
        st = []
        for k in (0, 1):
            a, b = rows[k]
            with torch.cuda.stream(streams[k]), comm.ar_channel(k):
                x = self.embed(ids[a:b])
                st.append([x, x, ops.rms_norm(x, self.w["layers.0.in_norm"], c.norm_eps)])
        for i in range(c.num_layers):
            p = f"layers.{i}."
            for k in (0, 1):
                a, b = rows[k]
                with torch.cuda.stream(streams[k]), comm.ar_channel(k):
                    x, res, h = st[k]
                    if i > 0:
                        h = ops.rms_norm(x, self.w[p + "in_norm"], c.norm_eps, residual=res)
                    o = self.attention(i, h, positions[a:b], metas[k], kv)
                    h = ops.rms_norm(o, self.w[p + "post_norm"], c.norm_eps, residual=res)
                    st[k] = [self.mlp(i, h), res, h]
        outs = []
        for k in (0, 1):
            with torch.cuda.stream(streams[k]):
                outs.append(ops.rms_norm(st[k][0], self.w["final_norm"], c.norm_eps, residual=st[k][1]))
        main.wait_stream(side)
        outs[1].record_stream(main)
        return torch.cat(outs)

    def forward_cp(self, ids: torch.Tensor, total_len: int, group=None, kv_sink=None, prefix_len: int = 0,
                   prefix_kv=None) -> torch.Tensor:
        """:meth:`forward_cp_iter` run to the end (returns the local rows' final hidden states)."""
        it = self.forward_cp_iter(ids, total_len, group, kv_sink, prefix_len, prefix_kv)
        while True:
            try:
                next(it)
            except StopIteration as e:
                return e.value

    def forward_cp_iter(self, ids: torch.Tensor, total_len: int, group=None, kv_sink=None, prefix_len: int = 0,
                        prefix_kv=None):
        """Context-parallel prefill of ONE long prompt (SURVEY §5.7 stretch path, >128k tokens),
        as a generator that yields after every layer (the serving leader interleaves decode steps
        between layer slices) and returns the local rows' final hidden states.

        ``ids`` is this rank's zig-zag shard (``parallel.context.zigzag_shard``) of a
        ``total_len``-token prompt; every CP rank holds the full weights (TP=1 inside the CP
        group).  Each layer: QKV on the local rows, RoPE at the rows' GLOBAL positions, ring
        attention over the CP group (K/V shards travel one xGMI hop per step; blocks on the HIP
        prefill kernel on the GPU), then O / MLP on the local rows.  Returns the final hidden
        states of the local rows.  ``kv_sink(layer, k, v)`` receives each layer's local K/V shard
        (``zigzag_unshard`` of every rank's shards is the full cache for the decode rank).
        ``prefix_len`` tokens before the sharded ones are already cached (a prefix-cache hit):
        the shard's positions start there, and ``prefix_kv(layer) -> (k, v)`` [P, Hkv, D]
        supplies that layer's prefix keys on every rank for the ring attention."""
        from ..ops.attention import rope_qk
        from ..ops.gemm import Slabs
        from ..parallel import context as cpx
        import torch.distributed as dist
        c = self.cfg
        cp = dist.get_world_size(group) if dist.is_initialized() else 1
        rank = dist.get_rank(group) if dist.is_initialized() else 0
        pos = cpx.zigzag_positions(total_len, cp, rank, device=ids.device) + prefix_len
        block = cpx.hip_block_attention if ops._native.use_native(self.w["embed"]) else cpx.torch_block_attention
        x = ops.embedding(ids, self.w["embed"])
        residual = x
        h = ops.rms_norm(x, self.w["layers.0.in_norm"], c.norm_eps)
        T = ids.shape[0]
        for i in range(c.num_layers):
            p = f"layers.{i}."
            if i > 0:
                h = ops.rms_norm(x, self.w[p + "in_norm"], c.norm_eps, residual=residual)
            qkv = linear(h, self.w[p + "qkv"])
            if isinstance(qkv, Slabs):
                qkv = qkv.materialize()
            # RoPE of q and k heads in one HIP pass at the shard's zig-zag positions (no cache write)
            qk = rope_qk(qkv, pos, self.cos_sin, self.hq, self.hkv, self.D)
            q = qk[:, :self.hq].contiguous()
            k = qk[:, self.hq:].contiguous()
            v = qkv.view(T, self.hq + 2 * self.hkv, self.D)[:, self.hq + self.hkv:].contiguous()
            if kv_sink is not None:
                kv_sink(i, k, v)
            pre = prefix_kv(i) if (prefix_kv is not None and prefix_len > 0) else None
            a = cpx.ring_attention(q, k, v, total_len, scale=self.scale, causal=True, group=group, block_fn=block,
                                   prefix=pre)
            a = linear(a.reshape(T, self.hq * self.D), self.w[p + "o"])
            h = ops.rms_norm(a, self.w[p + "post_norm"], c.norm_eps, residual=residual)
            x = self.mlp(i, h)
            yield i
        return ops.rms_norm(x, self.w["final_norm"], c.norm_eps, residual=residual)

    def forward(self, ids: torch.Tensor, positions: torch.Tensor, meta: AttentionMetadata, kv: KVCache) -> torch.Tensor:
        if self.uses_sp(ids.shape[0]):
            return self.forward_sp(ids, positions, meta, kv)
        c = self.cfg
        x = self.embed(ids)
        residual = x
        h = ops.rms_norm(x, self.w["layers.0.in_norm"], c.norm_eps)
        for i in range(c.num_layers):
            p = f"layers.{i}."
            if i > 0:
                h = ops.rms_norm(x, self.w[p + "in_norm"], c.norm_eps, residual=residual)
            # TP=1: the O / down projections may add the residual stream in their epilogue (in place)
            fr = residual if self.tp_size == 1 else None
            a = self.attention(i, h, positions, meta, kv, fuse_residual=fr)
            h = ops.rms_norm(a, self.w[p + "post_norm"], c.norm_eps, residual=residual)
            x = self.mlp(i, h, fuse_residual=fr)
        return ops.rms_norm(x, self.w["final_norm"], c.norm_eps, residual=residual)

    def lm_weight(self) -> torch.Tensor:
        """The (local shard of the) [V, H] vocabulary projection."""
        return self.w["embed"] if self.cfg.tie_embeddings else self.w["lm_head"]

    def logits(self, h: torch.Tensor) -> torch.Tensor:
        out = linear(h, self.lm_weight())
        return comm.tp_all_gather_last(out) if self.tp_size > 1 else out

    def sample_vocab_parallel(self, h: torch.Tensor, temps: torch.Tensor, seeds: torch.Tensor) -> torch.Tensor:
        """TP sampling without the logits all-gather: each rank draws its vocab shard's
        Gumbel-max candidate -- on the fused LM-head sampler from FUSED_LM_HEAD_MIN_M rows, else
        local logits + the shard sampler -- and the [B, 2] candidates are all-gathered and the best
        taken.  Same noise (keyed by the global token id) and tie rule as TP = 1: the TP = 1 token
        whenever the shard logits equal the full ones bitwise (always on the fused path)."""
        w = self.lm_weight()
        pad = getattr(self, "_lm_pad", None)
        if pad is not None and ops.fused_lm_head_ok(h, pad):
            pairs = ops.lm_head_sample_shard(h, pad, w.shape[0], self.vocab_start, temps, seeds, wt=self.lm_tiled())
        else:
            pairs = ops.sample_shard(linear(h, w), temps, seeds, self.vocab_start, self.cfg.vocab_size)
        return ops.pick_pairs(comm.tp_all_gather_pairs(pairs))


class LlamaModel(DecoderModel):
    pass
