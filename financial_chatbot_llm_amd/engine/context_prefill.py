"""Context-parallel prefill of very long prompts inside a serving replica.

A CP replica is ``cp_size`` ranks that each hold the FULL weights (``parallel.dist.init_cp_groups``).
Its leader runs the ordinary engine (scheduler, paged KV pool, hipGraph decode) and serves; the
other ranks wait in :meth:`ContextParallelPrefill.follower_loop`.  When the leader admits a prompt
with at least ``cp_min_tokens`` tokens it does not chunk it through its own steps:

1. it matches the prompt against the prefix cache (P cached tokens, a multiple of the block size);
   if fewer than ``cp_min_tokens`` uncached tokens remain the prompt goes to the scheduler as
   usual.  Otherwise it allocates the suffix's KV blocks and broadcasts the command (P + the
   suffix ids) over the replica's gloo group;
2. every rank prefills its zig-zag shard of the S suffix tokens (S = the uncached prompt minus its
   last token, rounded down to a multiple of 2·cp) with ``DecoderModel.forward_cp_iter``: QKV on
   the local rows, q/k RoPE at the rows' global positions (P + zig-zag) in one HIP pass, ring
   attention whose K/V hops ride RCCL over xGMI while each block runs on the HIP prefill kernel,
   plus one block against the cached prefix -- whose per-layer K/V the leader reads out of its
   paged pool and broadcasts -- then O / MLP on the local rows: 1/cp of the GEMM FLOPs and of the
   causal attention work per rank;
3. each layer's K/V shards are GATHERED TO THE LEADER only (the followers keep no copy), un-sharded
   and written into the leader's paged, fragment-native pool at the sequence's slots by the
   RoPE-less KV writer;
4. the sequence then joins the scheduler with ``num_computed = P + S``: its last few tokens run as
   an ordinary prefill chunk against the cached prefix, which produces the first sampled token,
   and decoding continues on the leader alone.

The pass does not stall the leader's engine loop: it runs ``layers_per_step`` layers per engine
step (``run_pending``), and the ordinary step -- the decode rows and other prefills -- follows
each slice on the same stream, so decoding sequences advance while a long prompt is prefilled.
Followers run the whole pass at once (the ring collectives pace them to the leader's slices).
``LLMEngine.stop_followers`` ends their loop.
"""
from __future__ import annotations

import time
from typing import TYPE_CHECKING, List, Optional

import torch
import torch.distributed as dist

from ..ops.attention import KV_BS, gather_kv_ref, rope_kv_write
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
        self.layers_per_step = max(1, int(getattr(engine.cfg, "cp_layers_per_step", 4)))
        self.queue: List["Sequence"] = []
        self.active = None          # (seq, layer generator, t0, P, S) of the pass in progress
        self.stats = {"cp_prefills": 0, "cp_tokens": 0, "cp_s": 0.0, "cp_prefix_tokens": 0, "cp_slices": 0}

    # -- leader ---------------------------------------------------------------------------------
    def wants(self, seq: "Sequence") -> bool:
        return self.cp > 1 and self.ps.cp_rank == 0 and seq.num_tokens - 1 >= self.min_tokens

    def busy(self) -> bool:
        return self.active is not None or bool(self.queue)

    def run_pending(self) -> None:
        """Leader, once per engine step: advance the pass in progress by ``layers_per_step``
        layers (starting the next queued prompt when none is), finishing it -- K/V in the pool,
        the sequence handed to the scheduler -- after its last layer."""
        if self.active is None:
            self._start_next()
        if self.active is None:
            return
        seq, gen, t0, P, S = self.active
        self.stats["cp_slices"] += 1
        for _ in range(self.layers_per_step):
            try:
                with torch.no_grad():
                    next(gen)
            except StopIteration:
                self.active = None
                eng = self.engine
                if seq.finished:
                    # aborted while the pass ran (Scheduler.abort cannot see it: the sequence is in
                    # neither queue, and its blocks were still being written by the K/V sink).  The
                    # followers ran the whole collective pass with us; now the blocks go back to the
                    # pool and the sequence never reaches the scheduler.
                    eng.bm.free(seq)
                    seq.block_table = []
                    self.stats["cp_aborted"] = self.stats.get("cp_aborted", 0) + 1
                    logger.info(f"context-parallel prefill of {S} tokens finished after its request was aborted: "
                                "KV blocks freed")
                    return
                seq.num_computed = P + S
                seq.num_prefilled += S
                eng.bm.commit(seq)
                eng.scheduler.add(seq)
                dt = time.perf_counter() - t0
                self.stats["cp_prefills"] += 1
                self.stats["cp_tokens"] += S
                self.stats["cp_prefix_tokens"] += P
                self.stats["cp_s"] += dt
                logger.info(f"context-parallel prefill of {S} tokens (+{P} cached) over {self.cp} ranks in {dt:.2f}s")
                return

    def _start_next(self) -> None:
        eng = self.engine
        while self.queue and self.active is None:
            seq = self.queue.pop(0)
            if seq.finished:
                continue
            P = eng.bm.match_prefix(seq) if not seq.block_table else seq.num_computed
            S = cp_prefix_len(seq.num_tokens - P, self.cp)
            if S < max(self.min_tokens, 2 * self.cp) or not eng.bm.grow(seq, P + S):
                eng.scheduler.add(seq)          # mostly cached, or no room now: ordinary chunked prefill
                continue
            ids = torch.tensor([P] + seq.prompt_ids[P:P + S], dtype=torch.int32)
            self._broadcast(ids)
            self.active = (seq, self._prefill_iter(ids, seq.block_table), time.perf_counter(), P, S)

    def stop(self) -> None:
        if self.cp > 1 and self.ps.cp_rank == 0:
            self._broadcast(None)

    def _broadcast(self, cmd: Optional[torch.Tensor]) -> Optional[torch.Tensor]:
        """Leader -> replica: the prefill command ([P, suffix ids...]) or stop; followers receive it."""
        g = self.ps.cp_cpu_group
        src = self.ps.rank - self.ps.cp_rank
        head = torch.zeros(1, dtype=torch.int64)
        if self.ps.cp_rank == 0:
            head[0] = _STOP if cmd is None else cmd.numel()
        dist.broadcast(head, src=src, group=g)
        n = int(head[0])
        if n == _STOP:
            return None
        buf = cmd if self.ps.cp_rank == 0 else torch.empty(n, dtype=torch.int32)
        dist.broadcast(buf, src=src, group=g)
        return buf

    # -- every rank -----------------------------------------------------------------------------
    def _prefill_iter(self, cmd: torch.Tensor, block_table: Optional[List[int]]):
        """This rank's shard of a context-parallel prefill (all ranks run it together, layer by
        layer): ``cmd`` = [P, suffix ids]; the leader (``block_table`` given) supplies the cached
        prefix K/V and writes the gathered suffix K/V into its paged pool."""
        eng = self.engine
        model = eng.model
        dev = eng.device
        P = int(cmd[0])
        ids = cmd[1:]
        S = ids.numel()
        local = cpx.zigzag_shard(ids.to(dev), self.cp, self.ps.cp_rank)
        leader = block_table is not None
        g = self.ps.cp_group
        src = self.ps.rank - self.ps.cp_rank
        if leader:
            pos = torch.arange(P, P + S, dtype=torch.int64)
            bt = torch.tensor(block_table, dtype=torch.int64)
            slots = (bt[pos // KV_BS] * KV_BS + pos % KV_BS).to(torch.int32).to(dev)
            pos = pos.to(torch.int32).to(dev)
            bt_dev = bt.to(torch.int32).to(dev)

        def sink(layer: int, k: torch.Tensor, v: torch.Tensor) -> None:
            kv = torch.cat([k, v], dim=1).contiguous()            # [S/cp, 2*Hkv, D]
            parts = [torch.empty_like(kv) for _ in range(self.cp)] if leader else None
            dist.gather(kv, gather_list=parts, dst=src, group=g)   # to the leader only
            if leader:
                full = cpx.zigzag_unshard(parts).reshape(S, -1)  # [S, 2*Hkv*D] in position order
                rope_kv_write(full, pos, None, slots, eng.kv.k(layer), eng.kv.v(layer), 0, model.hkv, model.D,
                              apply_rope=False)

        def prefix_kv(layer: int):
            if leader:
                k, v = gather_kv_ref(eng.kv.k(layer), eng.kv.v(layer), bt_dev, P)
                kv = torch.stack([k, v]).contiguous()             # [2, P, Hkv, D]
            else:
                kv = torch.empty((2, P, model.hkv, model.D), dtype=model.dtype, device=dev)
            dist.broadcast(kv, src=src, group=g)
            return kv[0], kv[1]

        # (callers advance the generator under torch.no_grad(): a grad-mode context held open
        # across yields would leak into the engine code that runs between the slices)
        yield from model.forward_cp_iter(local, S, group=g, kv_sink=sink, prefix_len=P,
                                         prefix_kv=prefix_kv if P > 0 else None)
        if dev.type == "cuda" and not leader:
            torch.cuda.synchronize(dev)

    def follower_loop(self) -> None:
        """CP follower: run the leader's context-parallel prefills until it broadcasts stop."""
        while True:
            cmd = self._broadcast(None)
            if cmd is None:
                return
            with torch.no_grad():
                for _ in self._prefill_iter(cmd, None):
                    pass
