"""Context parallelism: ring attention for one very long prefill sequence.

The reference has no long-context machinery at all -- it relies on Gemini's window and can stuff
up to 10 000 retrieved transactions into one system message (``tools/qdrant_tool.py:145``,
``llm_agent.py:234-236``).  Chunked prefill on one TP group covers every north-star config; this
module is the stretch path for prompts beyond ~128k tokens, where one GPU's prefill time (not its
KV memory -- 288 GB holds ~1.9M Llama-3-8B tokens) is the limit.

Design, for xGMI's point-to-point links:

* **Zig-zag sharding.** The sequence is cut into ``2·cp`` equal chunks and rank ``r`` owns chunks
  ``r`` and ``2·cp-1-r``.  Under a causal mask every rank then does the same amount of work in
  every ring step (a contiguous split leaves rank 0 idle for most of the ring).
* **Ring exchange.** K/V shards travel one hop per step (``batch_isend_irecv`` to ``rank+1``,
  from ``rank-1``): each step moves one shard over ONE direct xGMI link, and the transfer of step
  ``s+1``'s shard is posted before step ``s``'s block is computed, so it hides under the math.
  Positions never travel: the owner of a shard is ``(rank - s) mod cp``, and its global
  positions follow from the zig-zag layout.
* **Merge.** Each block yields ``(o, lse)`` in fp32; blocks combine with the log-sum-exp rule,
  so the result equals one softmax over the whole key range.

``block_fn`` computes one ``(q-shard × kv-shard)`` block and returns ``(o, lse)``; the default is
an fp32 torch implementation (GQA, position mask) that runs on CPU (gloo tests) and GPU alike.
"""
from __future__ import annotations

from typing import Callable, Optional, Tuple

import torch
import torch.distributed as dist

BlockFn = Callable[[torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor, torch.Tensor, float, bool],
                   Tuple[torch.Tensor, torch.Tensor]]


def zigzag_positions(total: int, cp: int, rank: int, device=None) -> torch.Tensor:
    """Global token positions owned by ``rank`` (chunks ``rank`` and ``2·cp-1-rank``)."""
    if total % (2 * cp):
        raise ValueError(f"sequence length {total} must be a multiple of 2*cp={2 * cp}")
    c = total // (2 * cp)
    a = torch.arange(rank * c, (rank + 1) * c, device=device)
    b = torch.arange((2 * cp - 1 - rank) * c, (2 * cp - rank) * c, device=device)
    return torch.cat([a, b])


def zigzag_shard(x: torch.Tensor, cp: int, rank: int, dim: int = 0) -> torch.Tensor:
    """This rank's rows of a full-sequence tensor (``dim`` indexes tokens)."""
    return x.index_select(dim, zigzag_positions(x.shape[dim], cp, rank, device=x.device))


def zigzag_unshard(parts, dim: int = 0) -> torch.Tensor:
    """Inverse of :func:`zigzag_shard` given every rank's shard in rank order."""
    cp = len(parts)
    total = sum(p.shape[dim] for p in parts)
    shape = list(parts[0].shape)
    shape[dim] = total
    out = parts[0].new_empty(shape)
    for r, p in enumerate(parts):
        out.index_copy_(dim, zigzag_positions(total, cp, r, device=p.device), p)
    return out


def torch_block_attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, pos_q: torch.Tensor,
                          pos_k: torch.Tensor, scale: float, causal: bool) -> Tuple[torch.Tensor, torch.Tensor]:
    """One attention block in fp32: q [Tq,Hq,D], k/v [Tk,Hkv,D] -> (o [Tq,Hq,D], lse [Hq,Tq]).

    Rows with no visible key get ``lse = -inf`` and ``o = 0`` (they merge as no-ops)."""
    hq, hkv = q.shape[1], k.shape[1]
    qf = q.float().transpose(0, 1)                                          # [Hq, Tq, D]
    kf = k.float().repeat_interleave(hq // hkv, dim=1).transpose(0, 1)      # [Hq, Tk, D]
    vf = v.float().repeat_interleave(hq // hkv, dim=1).transpose(0, 1)
    s = torch.matmul(qf, kf.transpose(1, 2)) * scale                        # [Hq, Tq, Tk]
    if causal:
        s = s.masked_fill((pos_k[None, :] > pos_q[:, None])[None], float("-inf"))
    lse = torch.logsumexp(s, dim=-1)                                        # [Hq, Tq]
    p = torch.exp(s - torch.where(torch.isinf(lse), torch.zeros_like(lse), lse)[..., None])
    o = torch.matmul(p, vf).transpose(0, 1)                                 # [Tq, Hq, D]
    return o, lse


def merge_blocks(o_a: torch.Tensor, lse_a: torch.Tensor, o_b: torch.Tensor,
                 lse_b: torch.Tensor) -> Tuple[torch.Tensor, torch.Tensor]:
    """Log-sum-exp merge of two partial softmax blocks (o [T,H,D] fp32, lse [H,T])."""
    lse = torch.logaddexp(lse_a, lse_b)
    safe = torch.where(torch.isinf(lse), torch.zeros_like(lse), lse)
    wa = torch.exp(lse_a - safe).transpose(0, 1)[..., None]                 # [T, H, 1]
    wb = torch.exp(lse_b - safe).transpose(0, 1)[..., None]
    return o_a * wa + o_b * wb, lse


def _ring_peers(group) -> Tuple[int, int, int, int]:
    cp = dist.get_world_size(group)
    r = dist.get_rank(group)
    to_global = (lambda i: dist.get_global_rank(group, i)) if group is not None else (lambda i: i)
    return cp, r, to_global((r + 1) % cp), to_global((r - 1) % cp)


def ring_attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, total_len: int,
                   scale: Optional[float] = None, causal: bool = True, group=None,
                   block_fn: BlockFn = torch_block_attention) -> torch.Tensor:
    """Context-parallel attention over the zig-zag shards of one sequence.

    ``q`` [Tl,Hq,D], ``k``/``v`` [Tl,Hkv,D] are this rank's shards (``zigzag_shard``) of a
    ``total_len``-token sequence; returns this rank's output rows [Tl,Hq,D] in ``q.dtype``.
    """
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        pos = torch.arange(total_len, device=q.device)
        o, _ = block_fn(q, k, v, pos, pos, scale or q.shape[-1] ** -0.5, causal)
        return o.to(q.dtype)
    cp, r, nxt, prv = _ring_peers(group)
    scale = scale if scale is not None else q.shape[-1] ** -0.5
    pos_q = zigzag_positions(total_len, cp, r, device=q.device)
    kv = torch.stack([k, v]).contiguous()                                   # one message per hop
    o = lse = None
    for step in range(cp):
        reqs = []
        if step + 1 < cp:                                                   # post next hop first
            nxt_kv = torch.empty_like(kv)
            ops_ = [dist.P2POp(dist.isend, kv, nxt, group), dist.P2POp(dist.irecv, nxt_kv, prv, group)]
            reqs = dist.batch_isend_irecv(ops_)
        src = (r - step) % cp
        pos_k = zigzag_positions(total_len, cp, src, device=q.device)
        ob, lb = block_fn(q, kv[0], kv[1], pos_q, pos_k, scale, causal)
        o, lse = (ob, lb) if o is None else merge_blocks(o, lse, ob, lb)
        for req in reqs:
            req.wait()
        if step + 1 < cp:
            kv = nxt_kv
    return o.to(q.dtype)
