"""K1 token-embedding gather; vocab-parallel shards return zeros for foreign ids."""
from __future__ import annotations

import torch

from . import _native as N


def embedding(ids: torch.Tensor, table: torch.Tensor, vocab_start: int = 0, vocab_end: int = -1) -> torch.Tensor:
    vocab_end = table.shape[0] + vocab_start if vocab_end < 0 else vocab_end
    H = table.shape[1]
    if N.use_native(table):
        ids32 = ids.to(torch.int32).contiguous()
        out = torch.empty((ids.numel(), H), dtype=table.dtype, device=table.device)
        N.call("penny_embedding", N.ptr(ids32), N.ptr(table), N.ptr(out), ids.numel(), H, vocab_start, vocab_end,
               N.stream())
        return out
    idx = ids.long()
    mine = (idx >= vocab_start) & (idx < vocab_end)
    out = table[(idx - vocab_start).clamp(0, table.shape[0] - 1)]
    return out * mine.unsqueeze(-1).to(out.dtype)
