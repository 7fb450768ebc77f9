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

``block_fn`` computes one ``(q-shard × kv-shard)`` block and returns ``(o, lse)``:

* :func:`hip_block_attention` (GPU): the shard pair is cut into its contiguous position chunks;
  each (q chunk, kv chunk) pair is fully visible, causal-diagonal or fully masked under the
  zig-zag layout, so it runs on the paged MFMA prefill kernel (K6) -- non-causal or causal, the
  kv chunk staged into a scratch paged cache by the KV writer -- which also emits each row's
  log-sum-exp;
* :func:`torch_block_attention`: fp32 torch (GQA, any position mask), CPU tests and fallback.

:meth:`~..models.llama.DecoderModel.forward_cp` runs a whole decoder over one long prompt this
way (each rank: its zig-zag rows through every layer; ring attention per layer).
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


def _runs(pos: torch.Tensor):
    """Contiguous runs of a sorted position vector -> [(row0, n, pos0)]."""
    p = pos.tolist()
    out, start = [], 0
    for i in range(1, len(p) + 1):
        if i == len(p) or p[i] != p[i - 1] + 1:
            out.append((start, i - start, p[start]))
            start = i
    return out


class _Scratch:
    """Reusable scratch paged KV cache for one kv chunk (fragment-native layout)."""

    def __init__(self):
        self.kc = self.vc = None

    def get(self, nblocks: int, hkv: int, d: int, dtype, device):
        from ..ops.attention import KV_BS
        if self.kc is None or self.kc.shape[0] < nblocks or self.kc.shape[1] != hkv or self.kc.device != device:
            self.kc = torch.zeros((nblocks, hkv, KV_BS * d), dtype=dtype, device=device)
            self.vc = torch.zeros_like(self.kc)
        return self.kc, self.vc


_SCRATCH = _Scratch()


def hip_block_attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, pos_q: torch.Tensor,
                        pos_k: torch.Tensor, scale: float, causal: bool) -> Tuple[torch.Tensor, torch.Tensor]:
    """One ring block on the HIP prefill kernel: (o [Tq,Hq,D] f32, lse [Hq,Tq]).

    Each (q run, kv run) pair is fully visible (all keys before every query), the causal diagonal
    (same positions), or fully masked (skipped); anything else -- never produced by the zig-zag
    layout -- falls back to :func:`torch_block_attention` for that pair."""
    from .. import ops
    from ..ops.attention import KV_BS
    Tq, Hq, D = q.shape
    Hkv = k.shape[1]
    o = torch.zeros((Tq, Hq, D), dtype=torch.float32, device=q.device)
    lse = torch.full((Hq, Tq), float("-inf"), dtype=torch.float32, device=q.device)
    q_runs, k_runs = _runs(pos_q), _runs(pos_k)
    for kr, kn, kp in k_runs:
        nb = (kn + KV_BS - 1) // KV_BS
        kc, vc = _SCRATCH.get(nb, Hkv, D, k.dtype, k.device)
        qkv = torch.cat([k.new_zeros((kn, Hq * D)), k[kr:kr + kn].reshape(kn, Hkv * D),
                         v[kr:kr + kn].reshape(kn, Hkv * D)], dim=1)
        slots = torch.arange(kn, dtype=torch.int32, device=k.device)
        ops.rope_kv_write(qkv, slots, None, slots, kc, vc, Hq, Hkv, D, apply_rope=False)
        bt = torch.arange(nb, dtype=torch.int32, device=k.device)[None]
        for qr, qn, qp in q_runs:
            if causal and kp > qp + qn - 1:
                continue                                           # every key after every query
            full = (not causal) or kp + kn - 1 <= qp
            diag = causal and kp == qp and kn == qn
            if full or diag:
                ob = torch.empty((qn, Hq, D), dtype=q.dtype, device=q.device)
                lb = torch.empty((qn, Hq), dtype=torch.float32, device=q.device)
                ops.prefill(q[qr:qr + qn].contiguous(), torch.tensor([0, qn], dtype=torch.int32, device=q.device),
                            torch.tensor([kn], dtype=torch.int32, device=q.device), bt, kc, vc, scale,
                            causal=diag, max_q_len=qn, out=ob, lse=lb)
                ob, lb = ob.float(), lb.transpose(0, 1)
            else:
                ob, lb = torch_block_attention(q[qr:qr + qn], k[kr:kr + kn], v[kr:kr + kn], pos_q[qr:qr + qn],
                                               pos_k[kr:kr + kn], scale, causal)
            mo, ml = merge_blocks(o[qr:qr + qn], lse[:, qr:qr + qn], ob, lb)
            o[qr:qr + qn] = mo
            lse[:, qr:qr + qn] = ml
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
                   block_fn: BlockFn = torch_block_attention,
                   prefix: Optional[Tuple[torch.Tensor, torch.Tensor]] = None) -> torch.Tensor:
    """Context-parallel attention over the zig-zag shards of one sequence.

    ``q`` [Tl,Hq,D], ``k``/``v`` [Tl,Hkv,D] are this rank's shards (``zigzag_shard``) of a
    ``total_len``-token sequence; returns this rank's output rows [Tl,Hq,D] in ``q.dtype``.
    ``prefix`` (k, v) [P,Hkv,D], the same on every rank: keys BEFORE the sharded tokens (a
    prefix-cache hit), visible to every query -- one extra block merged by log-sum-exp.
    """
    scale = scale if scale is not None else q.shape[-1] ** -0.5
    o = lse = None
    if prefix is not None and prefix[0].shape[0] > 0:
        P = prefix[0].shape[0]
        pos_p = torch.arange(P, device=q.device)
        pos_qp = torch.full((q.shape[0],), P, dtype=pos_p.dtype, device=q.device)
        o, lse = block_fn(q, prefix[0], prefix[1], pos_qp, pos_p, scale, False)
    if not dist.is_initialized() or dist.get_world_size(group) == 1:
        pos = torch.arange(total_len, device=q.device)
        ob, lb = block_fn(q, k, v, pos, pos, scale, causal)
        o, lse = (ob, lb) if o is None else merge_blocks(o, lse, ob, lb)
        return o.to(q.dtype)
    cp, r, nxt, prv = _ring_peers(group)
    pos_q = zigzag_positions(total_len, cp, r, device=q.device)
    kv = torch.stack([k, v]).contiguous()                                   # one message per hop
    # gloo (CPU rehearsals of the GPU path) moves host tensors only: stage the hop through host
    # memory; RCCL sends the device buffer directly over xGMI
    host_hop = kv.is_cuda and dist.get_backend(group) == "gloo"
    for step in range(cp):
        reqs = []
        if step + 1 < cp:                                                   # post next hop first
            send = kv.cpu() if host_hop else kv
            nxt_kv = torch.empty_like(send)
            ops_ = [dist.P2POp(dist.isend, send, nxt, group), dist.P2POp(dist.irecv, nxt_kv, prv, group)]
            reqs = dist.batch_isend_irecv(ops_)
        src = (r - step) % cp
        pos_k = zigzag_positions(total_len, cp, src, device=q.device)
        ob, lb = block_fn(q, kv[0], kv[1], pos_q, pos_k, scale, causal)
        o, lse = (ob, lb) if o is None else merge_blocks(o, lse, ob, lb)
        for req in reqs:
            req.wait()
        if step + 1 < cp:
            kv = nxt_kv.to(q.device) if host_hop else nxt_kv
    return o.to(q.dtype)
