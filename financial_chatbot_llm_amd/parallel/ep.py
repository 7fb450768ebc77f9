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
once experts outnumber what one GPU should hold.

Two dispatch forms:
* **fixed capacity** (decode-size shards, ``t * top_k <= capacity_pairs``): every destination gets
  a block of ``t * top_k`` rows (the worst case), padded with expert id -1 -- equal splits, so
  the all-to-alls need no size exchange, nothing syncs with the host, and the layer is
  hipGraph-capturable.  The padding costs n x the routed bytes, which at decode sizes is a few
  hundred KB of latency-bound traffic;
* **exact splits** (prefill): split sizes travel in a tiny first all_to_all (one host read per
  layer -- ``all_to_all_single`` takes host split lists), then only routed rows move.

Expert compute is one grouped call over the received rows when the model provides
``grouped_fn(rows, local_expert_ids)`` (the fp8 MFMA grouped GEMMs with device-side bucket
offsets; padding rows carry id -1 and are skipped) -- no per-expert Python loop, no host sync.
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


def _loop_experts(recv: torch.Tensor, recv_e: torch.Tensor, per: int,
                  expert_fn: Callable[[torch.Tensor, int], torch.Tensor]) -> torch.Tensor:
    """Reference / CPU form: one expert_fn call per local expert (rows with id -1 stay zero)."""
    y = torch.zeros_like(recv)
    if recv.shape[0]:
        e_l = recv_e.long()
        for e in range(per):
            rows = (e_l == e).nonzero().flatten()
            if rows.numel():
                y.index_copy_(0, rows, expert_fn(recv.index_select(0, rows), e).to(y.dtype))
    return y


def ep_moe_shard(x: torch.Tensor, router_logits: torch.Tensor, top_k: int, num_experts: int,
                 expert_fn: Callable[[torch.Tensor, int], torch.Tensor], group=None,
                 rank: Optional[int] = None, size: Optional[int] = None,
                 grouped_fn: Optional[Callable[[torch.Tensor, torch.Tensor], torch.Tensor]] = None,
                 capacity_pairs: int = 512, shard_tokens: Optional[int] = None) -> torch.Tensor:
    """MoE output for this rank's token shard ``x`` [t, H] (t may be 0).

    ``expert_fn(rows, e_local)`` applies local expert ``e_local`` to ``rows`` [m, H] -> [m, H];
    ``grouped_fn(rows, e_local_ids)`` (optional) applies each row's expert in one call.
    ``shard_tokens``: the largest shard of the group (same on every rank); enables the
    fixed-capacity dispatch when ``shard_tokens * top_k <= capacity_pairs``."""
    size = size if size is not None else dist.get_world_size(group)
    rank = rank if rank is not None else dist.get_rank(group)
    t, H = x.shape
    per = num_experts // size
    topw, topi = topk_softmax(router_logits, top_k)                 # [t, k] f32 / int32
    flat_e = topi.reshape(-1).long()
    owner = flat_e // per
    order = torch.argsort(owner, stable=True)
    tok = order // top_k                                           # home row of each sent pair
    compute = grouped_fn or (lambda rows, ids: _loop_experts(rows, ids, per, expert_fn))
    w = topw.reshape(-1)[order].float()
    P = t * top_k
    if shard_tokens is not None and shard_tokens * top_k <= capacity_pairs:
        # fixed-capacity dispatch: destination block d holds its pairs first, then id -1 padding
        C = shard_tokens * top_k
        counts = torch.zeros(size, dtype=torch.long, device=x.device)
        counts.scatter_add_(0, owner, torch.ones_like(owner))
        starts = torch.cumsum(counts, 0) - counts
        own_sorted = owner[order]
        slot = own_sorted * C + (torch.arange(P, device=x.device) - starts[own_sorted])
        send = x.new_zeros((size * C, H))
        send_e = torch.full((size * C,), -1, dtype=torch.int32, device=x.device)
        send.index_copy_(0, slot, x.index_select(0, tok))
        send_e.index_copy_(0, slot, (flat_e[order] % per).to(torch.int32))
        recv = torch.empty_like(send)
        recv_e = torch.empty_like(send_e)
        dist.all_to_all_single(recv, send, group=group)
        dist.all_to_all_single(recv_e, send_e, group=group)
        y = compute(recv, recv_e)
        back = torch.empty_like(y)
        dist.all_to_all_single(back, y, group=group)
        back = back.index_select(0, slot)
    else:
        send = x.index_select(0, tok)
        send_e = (flat_e[order] % per).to(torch.int32)
        send_counts = torch.zeros(size, dtype=torch.long, device=x.device)
        send_counts.scatter_add_(0, owner, torch.ones_like(owner))
        recv_counts = torch.empty_like(send_counts)
        dist.all_to_all_single(recv_counts, send_counts, group=group)
        s_split, r_split = send_counts.tolist(), recv_counts.tolist()   # the one host read per layer
        recv = x.new_empty((sum(r_split), H))
        recv_e = torch.empty(sum(r_split), dtype=torch.int32, device=x.device)
        dist.all_to_all_single(recv, send, r_split, s_split, group=group)
        dist.all_to_all_single(recv_e, send_e, r_split, s_split, group=group)
        y = compute(recv, recv_e)
        back = x.new_empty((sum(s_split), H))
        dist.all_to_all_single(back, y.contiguous(), s_split, r_split, group=group)
    out = torch.zeros((t, H), dtype=torch.float32, device=x.device)
    out.index_add_(0, tok, back.float() * w[:, None])
    return out.to(x.dtype)


def ep_moe(h: torch.Tensor, router_logits: torch.Tensor, top_k: int, num_experts: int,
           expert_fn: Callable[[torch.Tensor, int], torch.Tensor], group=None,
           grouped_fn: Optional[Callable[[torch.Tensor, torch.Tensor], torch.Tensor]] = None,
           capacity_pairs: int = 512) -> torch.Tensor:
    """Replicated activations [T, H] in, replicated MoE output out: shard tokens over the group,
    dispatch/compute/combine (``ep_moe_shard``), all_gather the shards back."""
    size = dist.get_world_size(group)
    rank = dist.get_rank(group)
    T, H = h.shape
    per = (T + size - 1) // size
    a, b = min(rank * per, T), min((rank + 1) * per, T)
    mine = ep_moe_shard(h[a:b], router_logits[a:b], top_k, num_experts, expert_fn, group, rank, size,
                        grouped_fn=grouped_fn, capacity_pairs=capacity_pairs, shard_tokens=per)
    padded = h.new_zeros((per, H))
    padded[:b - a] = mine
    out = torch.empty((size * per, H), dtype=h.dtype, device=h.device)
    dist.all_gather_into_tensor(out, padded, group=group) if dist.get_backend(group) != "gloo" else \
        out.copy_(torch.cat(_gather_list(padded, size, group), 0))
    return out[:T]


def _gather_list(x: torch.Tensor, size: int, group):
    parts = [torch.empty_like(x) for _ in range(size)]
    dist.all_gather(parts, x, group=group)
    return parts
