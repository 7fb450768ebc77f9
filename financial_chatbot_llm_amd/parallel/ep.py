"""Expert parallelism for the Mixtral MoE (all-to-all dispatch / combine over RCCL).

Layout: the E experts are partitioned over the EP group (rank r owns experts
[r*E/n, (r+1)*E/n), whole -- no FFN-dim split).  Inside a TP group every rank holds the same
post-attention activations, so the MoE runs sequence-parallel: rank r takes token shard r,
routes it, and

    1. dispatch   all_to_all_single   (token rows, sorted by owner rank) -> expert owners
    2. compute    grouped GEMMs over the rows each local expert received
    3. combine    all_to_all_single   (expert outputs back to the token's home rank)
    4. weighting  routing-weighted scatter-add into the shard (on the home rank)
    5. gather     all_gather of the token shards -> every rank has the full [T, H] again

Versus TP-sharded experts (each rank computes 1/n of EVERY active expert for ALL tokens, then
all-reduces [T, H]) this moves only routed rows (top_k * T * H per layer in each direction, split
n ways) and runs each expert's GEMM unsplit, which is what pays on xGMI's point-to-point links
once experts outnumber what one GPU should hold.  Split sizes travel in a tiny first all_to_all
(one host sync per layer: EP is an eager/prefill path; TP-sharded experts stay the hipGraph
decode path).
"""
from __future__ import annotations

from typing import Callable, Optional

import torch
import torch.distributed as dist

from ..ops.moe import topk_softmax


def expert_range(num_experts: int, rank: int, size: int):
    if num_experts % size:
        raise ValueError(f"{num_experts} experts not divisible by ep={size}")
    per = num_experts // size
    return rank * per, (rank + 1) * per


def ep_moe_shard(x: torch.Tensor, router_logits: torch.Tensor, top_k: int, num_experts: int,
                 expert_fn: Callable[[torch.Tensor, int], torch.Tensor], group=None,
                 rank: Optional[int] = None, size: Optional[int] = None) -> torch.Tensor:
    """MoE output for this rank's token shard ``x`` [t, H] (t may be 0).

    ``expert_fn(rows, e_local)`` applies local expert ``e_local`` to ``rows`` [m, H] -> [m, H]."""
    size = size if size is not None else dist.get_world_size(group)
    rank = rank if rank is not None else dist.get_rank(group)
    t, H = x.shape
    per = num_experts // size
    topw, topi = topk_softmax(router_logits, top_k)                 # [t, k] f32 / int32
    flat_e = topi.reshape(-1).long()
    owner = flat_e // per
    order = torch.argsort(owner, stable=True)
    tok = order // top_k                                           # home row of each sent pair
    send = x.index_select(0, tok)
    send_e = (flat_e[order] % per).to(torch.int32)
    send_counts = torch.bincount(owner, minlength=size)
    recv_counts = torch.empty_like(send_counts)
    dist.all_to_all_single(recv_counts, send_counts, group=group)
    s_split, r_split = send_counts.tolist(), recv_counts.tolist()
    recv = x.new_empty((sum(r_split), H))
    recv_e = torch.empty(sum(r_split), dtype=torch.int32, device=x.device)
    dist.all_to_all_single(recv, send, r_split, s_split, group=group)
    dist.all_to_all_single(recv_e, send_e, r_split, s_split, group=group)
    # grouped expert compute on the received rows
    y = torch.empty_like(recv)
    if recv.shape[0]:
        eo = torch.argsort(recv_e.long(), stable=True)
        counts = torch.bincount(recv_e.long(), minlength=per).tolist()
        a = 0
        for e, c in enumerate(counts):
            if c:
                rows = eo[a:a + c]
                y.index_copy_(0, rows, expert_fn(recv.index_select(0, rows), e).to(y.dtype))
            a += c
    back = x.new_empty((sum(s_split), H))
    dist.all_to_all_single(back, y, s_split, r_split, group=group)
    out = torch.zeros((t, H), dtype=torch.float32, device=x.device)
    w = topw.reshape(-1)[order].float()
    out.index_add_(0, tok, back.float() * w[:, None])
    return out.to(x.dtype)


def ep_moe(h: torch.Tensor, router_logits: torch.Tensor, top_k: int, num_experts: int,
           expert_fn: Callable[[torch.Tensor, int], torch.Tensor], group=None) -> torch.Tensor:
    """Replicated activations [T, H] in, replicated MoE output out: shard tokens over the group,
    dispatch/compute/combine (``ep_moe_shard``), all_gather the shards back."""
    size = dist.get_world_size(group)
    rank = dist.get_rank(group)
    T, H = h.shape
    per = (T + size - 1) // size
    a, b = min(rank * per, T), min((rank + 1) * per, T)
    mine = ep_moe_shard(h[a:b], router_logits[a:b], top_k, num_experts, expert_fn, group, rank, size)
    padded = h.new_zeros((per, H))
    padded[:b - a] = mine
    parts = [torch.empty_like(padded) for _ in range(size)]
    dist.all_gather(parts, padded, group=group)
    return torch.cat(parts, 0)[:T]
