"""Tensor-parallel collectives over RCCL/xGMI.

* C1 ``tp_all_reduce``: the partial sums after the row-parallel O-projection and
  down-projection (2 per layer).  In-place ``dist.all_reduce`` on the TP group; captured into
  the decode hipGraph together with the GEMMs.
* C2 ``tp_all_gather_last``: vocab-parallel LM-head logits ([B, V/tp] -> [B, V]); embedding
  partials are summed with C1.
* C4 ``broadcast_object``: the TP leader's scheduler decisions (token ids, positions, block
  tables) for a step, so non-leader ranks replay the identical forward.

xGMI is point-to-point (7 links per GPU): for 8-way TP the bandwidth-optimal ring is per-link
bound, so large messages (prefill activations) use RCCL's ring/tree; decode messages are
latency-bound (a few hundred KB).
"""
from __future__ import annotations

from typing import Any, List, Optional

import torch
import torch.distributed as dist

from .dist import state


def tp_size() -> int:
    return state().tp_size


_CUSTOM_AR = None   # CustomAllReduce for the TP group (enable_custom_all_reduce)


def enable_custom_all_reduce(max_bytes: int = 4 << 20):
    """Route small bf16 TP all-reduces (decode) through the one-shot xGMI P2P kernel
    (``custom_ar.py``); RCCL keeps everything else.  Call on every TP rank after init."""
    global _CUSTOM_AR
    s = state()
    if s.tp_size > 1 and _CUSTOM_AR is None:
        from .custom_ar import CustomAllReduce
        _CUSTOM_AR = CustomAllReduce(s.tp_group, max_bytes=max_bytes)
    return _CUSTOM_AR


def tp_all_reduce(x: torch.Tensor) -> torch.Tensor:
    s = state()
    if s.tp_size == 1:
        return x
    if _CUSTOM_AR is not None and _CUSTOM_AR.eligible(x):
        return _CUSTOM_AR.all_reduce(x, out=x)   # reads peers' staged copies, so in-place is safe
    dist.all_reduce(x, group=s.tp_group)
    return x


def tp_all_gather_last(x: torch.Tensor) -> torch.Tensor:
    """Concatenate the TP shards along the last dim."""
    s = state()
    if s.tp_size == 1:
        return x
    parts = [torch.empty_like(x) for _ in range(s.tp_size)]
    dist.all_gather(parts, x.contiguous(), group=s.tp_group)
    return torch.cat(parts, dim=-1)


def broadcast_object(obj: Any) -> Any:
    """TP leader -> all ranks of its TP group (CPU pickled; small step metadata)."""
    s = state()
    if s.tp_size == 1:
        return obj
    box: List[Any] = [obj if s.is_tp_leader else None]
    dist.broadcast_object_list(box, src=s.tp_leader_rank, group=s.tp_group)
    return box[0]


def broadcast_tensor(x: torch.Tensor) -> torch.Tensor:
    s = state()
    if s.tp_size == 1:
        return x
    dist.broadcast(x, src=s.tp_leader_rank, group=s.tp_group)
    return x
