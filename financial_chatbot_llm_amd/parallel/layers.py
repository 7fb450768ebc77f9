"""Megatron-style tensor-parallel sharding helpers (TP row).

Weights are kept as plain bf16 tensors in ``[out_features, in_features]`` layout (the layout
hipBLASLt consumes as ``x @ W^T``):

* column-parallel (QKV, gate/up): each rank owns a contiguous slice of the OUTPUT rows; with
  the fused QKV weight, the slice is taken per section (q heads | k heads | v heads) so every
  rank holds whole heads; the fused gate|up weight is sliced per half.
* row-parallel (O, down): each rank owns a slice of the INPUT columns; outputs are partial sums
  completed by ``tp_all_reduce``.
* vocab-parallel (embedding, LM head): each rank owns ``V/tp`` vocabulary rows.
"""
from __future__ import annotations

from typing import List, Sequence

import torch


def shard_rows(w: torch.Tensor, rank: int, size: int) -> torch.Tensor:
    n = w.shape[0]
    assert n % size == 0, f"{n} rows not divisible by tp={size}"
    k = n // size
    return w[rank * k:(rank + 1) * k].contiguous()


def shard_cols(w: torch.Tensor, rank: int, size: int) -> torch.Tensor:
    n = w.shape[1]
    assert n % size == 0, f"{n} cols not divisible by tp={size}"
    k = n // size
    return w[:, rank * k:(rank + 1) * k].contiguous()


def shard_sections(w: torch.Tensor, sections: Sequence[int], rank: int, size: int) -> torch.Tensor:
    """Column-parallel shard of a row-concatenation of ``sections`` (e.g. q|k|v or gate|up)."""
    parts: List[torch.Tensor] = []
    start = 0
    for n in sections:
        parts.append(shard_rows(w[start:start + n], rank, size))
        start += n
    return torch.cat(parts, dim=0).contiguous()


def vocab_range(vocab: int, rank: int, size: int):
    per = (vocab + size - 1) // size
    return rank * per, min(vocab, (rank + 1) * per)
