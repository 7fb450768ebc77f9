"""Context-parallel prefill of very long prompts inside a serving replica.

A CP replica is ``cp_size`` ranks that each hold the FULL weights (``parallel.dist.init_cp_groups``).
Its leader runs the ordinary engine (scheduler, paged KV pool, hipGraph decode) and serves; the
other ranks wait in :meth:`ContextParallelPrefill.follower_loop`.  When the leader admits a prompt
with at least ``cp_min_tokens`` uncomputed tokens it does not chunk it through its own steps:

1. it allocates the prompt's KV blocks (no prefix-cache match: the CP pass computes every position
   from 0) and broadcasts the command (token count + ids) over the replica's gloo group;
2. every rank prefills its zig-zag shard of the first ``T`` tokens (``T`` = the prompt minus its
   last token, rounded down to a multiple of 2·cp) with ``DecoderModel.forward_cp``: QKV on the
   local rows, q/k RoPE at the rows' global positions in one HIP pass, ring attention whose K/V
   hops ride RCCL over xGMI while each block runs on the HIP prefill kernel, O / MLP on the local
   rows -- 1/cp of the GEMM FLOPs and of the causal attention work per rank;
3. each layer's K/V shards are all-gathered over the replica, un-sharded and written into the
   leader's paged, fragment-native pool at the sequence's slots by the RoPE-less KV writer;
4. the sequence then joins the scheduler with ``num_computed = T``: its last few tokens run as an
   ordinary prefill chunk against the cached prefix, which produces the first sampled token, and
   decoding continues on the leader alone.

The leader's engine loop is blocked for the duration of the CP pass (the same wall time the
prompt's chunks would have held its steps, divided across cp GPUs).  Followers keep no KV pool of
their own beyond a token one.  ``LLMEngine.stop_followers`` ends their loop.
"""
from __future__ import annotations

import time
from typing import TYPE_CHECKING, List, Optional

import torch
import torch.distributed as dist

from ..ops.attention import KV_BS, rope_kv_write
from ..parallel import context as cpx
from ..parallel.dist import state as pstate
from ..utils.logging import get_logger

if TYPE_CHECKING:
    from .llm_engine import LLMEngine
    from .sequence import Sequence

logger = get_logger(__name__)
_STOP = -1


def cp_prefix_len(num_prompt_tokens: int, cp: int) -> int:
    """Tokens prefilled context-parallel: all but the last, rounded down to a multiple of 2·cp."""
    return ((num_prompt_tokens - 1) // (2 * cp)) * (2 * cp)


class ContextParallelPrefill:
    def __init__(self, engine: "LLMEngine"):
        self.engine = engine
        self.ps = pstate()
        self.cp = self.ps.cp_size
        self.min_tokens = max(int(engine.cfg.cp_min_tokens), 4 * self.cp)
        self.queue: List["Sequence"] = []
        self.stats = {"cp_prefills": 0, "cp_tokens": 0, "cp_s": 0.0}

    # -- leader ---------------------------------------------------------------------------------
    def wants(self, seq: "Sequence") -> bool:
        return self.cp > 1 and self.ps.cp_rank == 0 and seq.num_tokens - 1 >= self.min_tokens

    def run_pending(self) -> None:
        """Leader, between engine steps: prefill every queued long prompt context-parallel, then
        hand it to the scheduler."""
        while self.queue:
            seq = self.queue.pop(0)
            if seq.finished:
                continue
            T = cp_prefix_len(seq.num_tokens, self.cp)
            eng = self.engine
            if T < 2 * self.cp or not eng.bm.grow(seq, T):
                eng.scheduler.add(seq)          # no room in the pool now: ordinary chunked prefill
                continue
            t0 = time.perf_counter()
            ids = torch.tensor(seq.prompt_ids[:T], dtype=torch.int32)
            self._broadcast(ids)
            self._prefill(ids, seq.block_table)
            seq.num_computed = T
            seq.num_prefilled += T
            eng.bm.commit(seq)
            eng.scheduler.add(seq)
            dt = time.perf_counter() - t0
            self.stats["cp_prefills"] += 1
            self.stats["cp_tokens"] += T
            self.stats["cp_s"] += dt
            logger.info(f"context-parallel prefill of {T} tokens over {self.cp} ranks in {dt:.2f}s")

    def stop(self) -> None:
        if self.cp > 1 and self.ps.cp_rank == 0:
            self._broadcast(None)

    def _broadcast(self, ids: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
        """Leader -> replica: the prefill command (token ids) or stop; followers receive it."""
        g = self.ps.cp_cpu_group
        src = self.ps.rank - self.ps.cp_rank
        head = torch.zeros(1, dtype=torch.int64)
        if self.ps.cp_rank == 0:
            head[0] = _STOP if ids is None else ids.numel()
        dist.broadcast(head, src=src, group=g)
        n = int(head[0])
        if n == _STOP:
            return None
        buf = ids if self.ps.cp_rank == 0 else torch.empty(n, dtype=torch.int32)
        dist.broadcast(buf, src=src, group=g)
        return buf

    # -- every rank -----------------------------------------------------------------------------
    @torch.no_grad()
    def _prefill(self, ids: torch.Tensor, block_table: Optional[List[int]]) -> None:
        """This rank's shard of a context-parallel prefill of ``ids`` (all ranks call it together);
        the leader (``block_table`` given) writes the gathered K/V into its paged pool."""
        eng = self.engine
        model = eng.model
        dev = eng.device
        T = ids.numel()
        local = cpx.zigzag_shard(ids.to(dev), self.cp, self.ps.cp_rank)
        leader = block_table is not None
        if leader:
            pos = torch.arange(T, dtype=torch.int32)
            bt = torch.tensor(block_table, dtype=torch.int64)
            slots = (bt[pos.long() // KV_BS] * KV_BS + pos.long() % KV_BS).to(torch.int32).to(dev)
            pos = pos.to(dev)
        g = self.ps.cp_group

        def sink(layer: int, k: torch.Tensor, v: torch.Tensor) -> None:
            kv = torch.cat([k, v], dim=1).contiguous()            # [T/cp, 2*Hkv, D]
            parts = [torch.empty_like(kv) for _ in range(self.cp)]
            dist.all_gather(parts, kv, group=g)
            if leader:
                full = cpx.zigzag_unshard(parts).reshape(T, -1)  # [T, 2*Hkv*D] in position order
                rope_kv_write(full, pos, None, slots, eng.kv.k(layer), eng.kv.v(layer), 0, model.hkv, model.D,
                              apply_rope=False)

        model.forward_cp(local, T, group=g, kv_sink=sink)
        if dev.type == "cuda":
            torch.cuda.synchronize(dev)

    def follower_loop(self) -> None:
        """CP follower: run the leader's context-parallel prefills until it broadcasts stop."""
        while True:
            ids = self._broadcast(None)
            if ids is None:
                return
            self._prefill(ids, None)
