"""Shared model plumbing: attention metadata, paged KV cache, deterministic weight init."""
from __future__ import annotations

import zlib
from dataclasses import dataclass, field
from typing import Dict, List, Optional

import torch

from ..ops.attention import KV_BS, DecodeWorkspace


@dataclass
class AttentionMetadata:
    """Per-step batch layout: ``num_prefill_tokens`` prefill tokens first, then one token per
    decoding sequence.  All tensors live on the model's device."""

    slots: torch.Tensor                      # [T] int32 KV slot per token (-1: no write)
    num_prefill_tokens: int = 0
    cu_q: Optional[torch.Tensor] = None      # [Sp+1] int32
    ctx_lens_p: Optional[torch.Tensor] = None  # [Sp] int32 total KV length after this step
    block_tables_p: Optional[torch.Tensor] = None  # [Sp, max_blocks] int32
    max_q_len: int = 0
    num_decode: int = 0
    ctx_lens_d: Optional[torch.Tensor] = None  # [Bd]
    block_tables_d: Optional[torch.Tensor] = None
    decode_ws: Optional[DecodeWorkspace] = None
    causal: bool = True
    prefill_work: Optional[torch.Tensor] = None  # [n, 2] int32 (ops.attention.prefill_work_list) or lean [., 6]
    prefill_lean: Optional[tuple] = None          # lean list counts (items, merges, slots), host ints


class KVCache:
    """All layers' paged K/V in ONE HBM allocation: [L, 2, num_blocks, Hkv, 64*D] bf16.

    ``k(l)`` / ``v(l)`` are [num_blocks, Hkv, 64*D] tiles in MFMA-fragment-native order
    (csrc/kernels/kv_layout.h).
    """

    def __init__(self, num_layers: int, num_blocks: int, num_kv_heads: int, head_dim: int,
                 dtype=torch.bfloat16, device="cuda"):
        self.num_layers, self.num_blocks = num_layers, num_blocks
        self.num_kv_heads, self.head_dim = num_kv_heads, head_dim
        self.buf = torch.zeros((num_layers, 2, num_blocks, num_kv_heads, KV_BS * head_dim), dtype=dtype,
                               device=device)

    def k(self, layer: int) -> torch.Tensor:
        return self.buf[layer, 0]

    def v(self, layer: int) -> torch.Tensor:
        return self.buf[layer, 1]

    @staticmethod
    def bytes_per_block(num_layers: int, num_kv_heads: int, head_dim: int, elt: int = 2) -> int:
        return num_layers * 2 * num_kv_heads * KV_BS * head_dim * elt


def param_seed(base: int, name: str) -> int:
    return (base * 1_000_003 + zlib.crc32(name.encode())) & 0x7FFFFFFF


def random_tensor(name: str, shape, seed: int, device, dtype=torch.bfloat16, std: float = 0.02,
                  kind: str = "normal") -> torch.Tensor:
    """Deterministic per-name init, identical on every rank (so TP shards agree)."""
    if kind == "ones":
        return torch.ones(shape, dtype=dtype, device=device)
    if kind == "zeros":
        return torch.zeros(shape, dtype=dtype, device=device)
    g = torch.Generator(device=device)
    g.manual_seed(param_seed(seed, name))
    t = torch.randn(shape, generator=g, device=device, dtype=torch.float32 if device == "cpu" else dtype)
    return t.mul_(std).to(dtype)
