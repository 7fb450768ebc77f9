"""Process-group management: one process per GPU, torch.distributed over RCCL (backend "nccl").

Topology: ``world = dp * tp``; ranks ``[d*tp, (d+1)*tp)`` form tensor-parallel group ``d``
(consecutive ranks = directly xGMI-linked GPUs of one node), and ranks with equal TP rank form
the data-parallel groups.  On CPU (tests) the same code runs on gloo.

The reference has no distributed compute at all (its only parallelism is N
gunicorn worker processes); DP replicas here are that same idea, one engine per GPU group.
"""
from __future__ import annotations

import datetime as _dt
import os
from dataclasses import dataclass
from typing import List, Optional

import torch
import torch.distributed as dist


@dataclass
class ParallelState:
    world_size: int = 1
    rank: int = 0
    local_rank: int = 0
    tp_size: int = 1
    tp_rank: int = 0
    dp_size: int = 1
    dp_rank: int = 0
    tp_group: Optional[object] = None
    dp_group: Optional[object] = None
    tp_cpu_group: Optional[object] = None   # gloo twin of tp_group: host control messages (C4)
    backend: str = "none"
    cp_size: int = 1                        # context-parallel replica (init_cp_groups)
    cp_rank: int = 0
    cp_group: Optional[object] = None
    cp_cpu_group: Optional[object] = None

    @property
    def is_tp_leader(self) -> bool:
        return self.tp_rank == 0

    @property
    def tp_leader_rank(self) -> int:
        return self.rank - self.tp_rank


_STATE = ParallelState()


def state() -> ParallelState:
    return _STATE


def set_state(s: ParallelState) -> None:
    global _STATE
    _STATE = s


def init_distributed(tp_size: int = 1, backend: Optional[str] = None, device_type: Optional[str] = None,
                     timeout_s: float = 600.0) -> ParallelState:
    """Initialise from torchrun env vars (RANK, WORLD_SIZE, LOCAL_RANK, MASTER_ADDR/PORT)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    if device_type is None:
        device_type = "cuda" if torch.cuda.is_available() else "cpu"
    if backend is None:
        # "nccl" is RCCL on ROCm; PENNY_DIST_BACKEND=gloo rehearses multi-rank paths on one GPU
        backend = os.environ.get("PENNY_DIST_BACKEND") or ("nccl" if device_type == "cuda" else "gloo")
    if device_type == "cuda":
        torch.cuda.set_device(local % max(torch.cuda.device_count(), 1))
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        kw = {}
        if backend == "nccl":
            kw["device_id"] = torch.device("cuda", torch.cuda.current_device())
        dist.init_process_group(backend=backend, rank=rank, world_size=world,
                                timeout=_dt.timedelta(seconds=timeout_s), **kw)
    if world % tp_size:
        raise ValueError(f"world size {world} not divisible by tp {tp_size}")
    dp = world // tp_size
    s = ParallelState(world, rank, local, tp_size, rank % tp_size, dp, rank // tp_size, backend=backend)
    if world > 1:
        for d in range(dp):
            ranks = list(range(d * tp_size, (d + 1) * tp_size))
            g = dist.new_group(ranks) if tp_size > 1 else None
            # C4 step metadata is host data: a gloo group moves it CPU->CPU with no device hop
            gc = (g if backend == "gloo" else dist.new_group(ranks, backend="gloo")) if tp_size > 1 else None
            if rank in ranks:
                s.tp_group = g
                s.tp_cpu_group = gc
        for t in range(tp_size):
            ranks = list(range(t, world, tp_size))
            g = dist.new_group(ranks) if dp > 1 else None
            if rank in ranks:
                s.dp_group = g
    set_state(s)
    return s


def init_cp_groups(cp_size: int) -> ParallelState:
    """Context-parallel replicas (TP = 1): consecutive ranks [g*cp, (g+1)*cp) form replica g, whose
    rank g*cp leads.  cp_group carries the ring attention's K/V hops and the K/V gather (RCCL on
    the GPU), cp_cpu_group (gloo) the leader's prefill commands."""
    s = _STATE
    if cp_size <= 1:
        return s
    if s.tp_size != 1:
        raise ValueError("context parallelism runs with tp_size 1 (every CP rank holds the full weights)")
    if s.world_size % cp_size:
        raise ValueError(f"world size {s.world_size} not divisible by cp {cp_size}")
    for gi in range(s.world_size // cp_size):
        ranks = list(range(gi * cp_size, (gi + 1) * cp_size))
        g = dist.new_group(ranks)
        gc = g if s.backend == "gloo" else dist.new_group(ranks, backend="gloo")
        if s.rank in ranks:
            s.cp_group, s.cp_cpu_group = g, gc
    s.cp_size, s.cp_rank = cp_size, s.rank % cp_size
    s.dp_size, s.dp_rank = s.world_size // cp_size, s.rank // cp_size
    return s


def barrier() -> None:
    if dist.is_initialized():
        if _STATE.backend == "nccl":
            dist.barrier(device_ids=[torch.cuda.current_device()])
        else:
            dist.barrier()


def shutdown() -> None:
    from .comm import disable_custom_all_reduce
    disable_custom_all_reduce()          # unmap peer IPC buffers before the group goes away
    if dist.is_initialized():
        dist.destroy_process_group()
    set_state(ParallelState())
