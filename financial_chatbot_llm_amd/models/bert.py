"""BERT / bge-base-en encoder on the GPU (replaces OpenAIEmbeddings, qdrant_tool.py:28).

Post-LN BERT: embeddings (word + position + type) -> LayerNorm -> 12 x [fused QKV GEMM (+bias)
-> bidirectional attention -> O GEMM -> add+LayerNorm -> GELU MLP -> add+LayerNorm] -> CLS
pooling -> L2 normalise.  Queries are packed varlen (no padding FLOPs).  Attention reuses the
decoder's paged-KV machinery: each layer's K/V go through the RoPE-less KV writer into a small
scratch paged cache (reused by every layer) and the MFMA prefill kernel runs with
``causal=False`` at head_dim 64.
"""
from __future__ import annotations

import math
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch
import torch.nn.functional as F

from .. import ops
from ..ops.attention import KV_BS
from ..ops.gemm import linear_bias
from .common import random_tensor
from .configs import ModelConfig


class BertEncoder:
    def __init__(self, cfg: ModelConfig, device="cuda", dtype=torch.bfloat16):
        self.cfg = cfg
        self.device = torch.device(device)
        self.dtype = dtype
        self.H, self.nh, self.D = cfg.hidden_size, cfg.num_heads, cfg.head_dim
        self.w: Dict[str, torch.Tensor] = {}
        self._scratch: Optional[torch.Tensor] = None

    def shapes(self) -> Dict[str, tuple]:
        c = self.cfg
        H, F_ = c.hidden_size, c.intermediate_size
        s = {"word_emb": (c.vocab_size, H), "pos_emb": (c.max_position, H), "type_emb": (c.type_vocab_size, H),
             "emb_ln_g": (H,), "emb_ln_b": (H,)}
        for i in range(c.num_layers):
            p = f"layers.{i}."
            s.update({p + "qkv": (3 * H, H), p + "qkv_b": (3 * H,), p + "o": (H, H), p + "o_b": (H,),
                      p + "ln1_g": (H,), p + "ln1_b": (H,), p + "fc1": (F_, H), p + "fc1_b": (F_,),
                      p + "fc2": (H, F_), p + "fc2_b": (H,), p + "ln2_g": (H,), p + "ln2_b": (H,)})
        return s

    @classmethod
    def build(cls, cfg: ModelConfig, device="cuda", weights: Optional[str] = None, seed: int = 0,
              dtype=torch.bfloat16) -> "BertEncoder":
        m = cls(cfg, device, dtype)
        if weights:
            from .weights import hf_bert_to_internal, read_safetensors
            m.load_state(hf_bert_to_internal(read_safetensors(weights), cfg.num_layers))
        else:
            for name, shape in m.shapes().items():
                kind = "ones" if name.endswith("_g") else ("zeros" if name.endswith("_b") else "normal")
                m.w[name] = random_tensor("bert." + name, shape, seed, m.device, dtype, kind=kind)
        return m

    def load_state(self, sd: Dict[str, torch.Tensor]) -> "BertEncoder":
        for k, v in sd.items():
            self.w[k] = v.to(self.device, self.dtype).contiguous()
        return self

    def _kv_scratch(self, nblocks: int):
        if self._scratch is None or self._scratch.shape[1] < nblocks:
            self._scratch = torch.zeros((2, max(nblocks, 64), self.nh, KV_BS * self.D), dtype=self.dtype,
                                        device=self.device)
        return self._scratch[0], self._scratch[1]

    @torch.no_grad()
    def forward(self, ids_list: Sequence[Sequence[int]]) -> torch.Tensor:
        """-> final hidden states [T, H] of the packed batch, plus CLS row indices."""
        c, dev = self.cfg, self.device
        # packed varlen metadata, vectorised on the host (bulk ingest packs 100k+ tokens a call)
        lens = np.fromiter((len(x) for x in ids_list), np.int64, len(ids_list))
        T = int(lens.sum())
        cu = np.zeros(len(lens) + 1, np.int64)
        np.cumsum(lens, out=cu[1:])
        flat = np.fromiter((t for x in ids_list for t in x), np.int32, T)
        pos = np.arange(T, dtype=np.int64) - np.repeat(cu[:-1], lens)
        nbs = (lens + KV_BS - 1) // KV_BS
        starts = np.zeros(len(lens) + 1, np.int64)
        np.cumsum(nbs, out=starts[1:])
        W = int(nbs.max())
        cols = np.arange(W, dtype=np.int64)
        bt = np.where(cols[None, :] < nbs[:, None], starts[:-1, None] + cols[None, :], 0).astype(np.int32)
        slots = (np.repeat(starts[:-1], lens) + pos // KV_BS) * KV_BS + pos % KV_BS
        ids_t = torch.from_numpy(flat).to(dev)
        pos_t = torch.from_numpy(pos.astype(np.int32)).to(dev)
        slots_t = torch.from_numpy(slots.astype(np.int32)).to(dev)
        cu_t = torch.from_numpy(cu.astype(np.int32)).to(dev)
        lens_t = torch.from_numpy(lens.astype(np.int32)).to(dev)
        bt = torch.from_numpy(bt).to(dev)
        starts = starts.tolist()
        lens = lens.tolist()
        cu = cu.tolist()
        kc, vc = self._kv_scratch(starts[-1])
        w = self.w
        e_word = ops.embedding(ids_t, w["word_emb"])
        e_pos = ops.embedding(pos_t, w["pos_emb"])
        e_pos = (e_pos.float() + w["type_emb"][0].float()).to(self.dtype)
        x = ops.layer_norm(e_word, w["emb_ln_g"], w["emb_ln_b"], c.norm_eps, residual=e_pos)
        scale = 1.0 / math.sqrt(self.D)
        for i in range(c.num_layers):
            p = f"layers.{i}."
            qkv = linear_bias(x, w[p + "qkv"], w[p + "qkv_b"])
            q = ops.rope_kv_write(qkv, pos_t, None, slots_t, kc, vc, self.nh, self.nh, self.D, apply_rope=False)
            a = ops.prefill(q, cu_t, lens_t, bt, kc, vc, scale, causal=False, max_q_len=max(lens))
            o = linear_bias(a.view(T, self.H), w[p + "o"], w[p + "o_b"])
            x = ops.layer_norm(o, w[p + "ln1_g"], w[p + "ln1_b"], c.norm_eps, residual=x)
            h = linear_bias(x, w[p + "fc1"], w[p + "fc1_b"], gelu=True)      # bias + GELU fused
            y = linear_bias(h, w[p + "fc2"], w[p + "fc2_b"])
            x = ops.layer_norm(y, w[p + "ln2_g"], w[p + "ln2_b"], c.norm_eps, residual=x)
        return x, cu

    @torch.no_grad()
    def encode(self, ids_list: Sequence[Sequence[int]]) -> torch.Tensor:
        """CLS pooling + L2 normalisation (bge convention) -> [n, H] f32."""
        x, cu = self.forward(ids_list)
        cls = x[torch.tensor(cu[:-1], device=x.device)]
        return F.normalize(cls.float(), dim=-1)
