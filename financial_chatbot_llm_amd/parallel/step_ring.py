"""C4 step broadcast over a node-local shared-memory ring (``csrc/runtime/step_ring.h``).

The TP leader's scheduler decides every step and the followers replay it (``LLMEngine``).  With
gloo that is two TCP collectives per step (length header, payload) through the loopback stack;
a TP group is always inside one node (xGMI), so the leader can instead memcpy the packed
``StepInputs`` into a shared-memory slot and publish it with one release store, and each
follower picks it up with one acquire load (``_penny_runtime.StepRing``).  Messages larger than
a slot (a long prefill step's block tables) are announced in the ring and sent over gloo, so the
followers never disagree about the order of the two channels.  SURVEY C4 ("RCCL broadcast or a
shared-memory ring").

Wire format of a ring message: one tag byte, then the payload.
"""
from __future__ import annotations

import os
import socket
import uuid
from typing import Optional

import numpy as np
import torch
import torch.distributed as dist

from ..utils.logging import get_logger

logger = get_logger(__name__)

TAG_DATA, TAG_STOP, TAG_GLOO = 0, 1, 2


class StepChannel:
    """Leader -> followers byte channel of one TP group.  Construct on every rank of the group
    together (collective over ``group``, a gloo group)."""

    def __init__(self, group, leader: int, is_leader: bool, reader_index: int, nreaders: int,
                 nslots: int = 8, slot_bytes: int = 4 << 20, timeout_s: float = 600.0):
        from .. import _penny_runtime as rt
        self.group, self.leader, self.is_leader = group, leader, is_leader
        self.timeout_s = timeout_s
        box = [f"/penny_c4_{os.getpid()}_{uuid.uuid4().hex[:12]}" if is_leader else None]
        dist.broadcast_object_list(box, src=leader, group=group)
        self.name = box[0]
        self.ring = rt.StepRing(self.name, True, nslots, slot_bytes, max(nreaders, 1)) if is_leader else None
        dist.barrier(group=group)                       # created before anyone opens it
        if not is_leader:
            self.ring = rt.StepRing(self.name, False, 0, 0, 0)
        self.reader = reader_index
        dist.barrier(group=group)
        self.sent = self.received = self.fallbacks = 0

    def send(self, payload: Optional[np.ndarray]) -> None:
        """Leader: publish one message (None = stop)."""
        if payload is None:
            self.ring.put(np.array([TAG_STOP], np.uint8), self.timeout_s)
            return
        msg = np.empty(payload.size + 1, np.uint8)
        msg[0] = TAG_DATA
        msg[1:] = payload.view(np.uint8).reshape(-1)
        self.sent += 1
        if self.ring.put(msg, self.timeout_s):
            return
        self.fallbacks += 1                               # too big for a slot: announce, then gloo
        self.ring.put(np.array([TAG_GLOO], np.uint8), self.timeout_s)
        head = torch.tensor([payload.size], dtype=torch.int64)
        dist.broadcast(head, src=self.leader, group=self.group)
        dist.broadcast(torch.from_numpy(payload.view(np.uint8).reshape(-1).copy()), src=self.leader, group=self.group)

    def recv(self) -> Optional[np.ndarray]:
        """Follower: the next message's payload, or None on stop."""
        msg = self.ring.get(self.reader, self.timeout_s)
        if msg is None:
            raise TimeoutError(f"no step from the TP leader in {self.timeout_s:.0f} s")
        tag = int(msg[0])
        if tag == TAG_STOP:
            return None
        self.received += 1
        if tag == TAG_DATA:
            return msg[1:]
        head = torch.zeros(1, dtype=torch.int64)
        dist.broadcast(head, src=self.leader, group=self.group)
        buf = torch.empty(int(head[0]), dtype=torch.uint8)
        dist.broadcast(buf, src=self.leader, group=self.group)
        return buf.numpy()

    def close(self) -> None:
        if self.ring is not None:
            self.ring.close()


def same_node(group) -> bool:
    """Are all ranks of ``group`` on this host (the ring needs one shared /dev/shm)?"""
    n = dist.get_world_size(group)
    names = [None] * n
    dist.all_gather_object(names, socket.gethostname(), group=group)
    return all(x == names[0] for x in names)


def make_step_channel(state) -> Optional[StepChannel]:
    """The TP group's C4 ring, or None (TP = 1, no gloo twin, ranks on several hosts, runtime not
    built, or ``PENNY_STEP_RING=0``).  Collective over the TP group's gloo twin."""
    group = state.tp_cpu_group if state.tp_cpu_group is not None else state.tp_group
    if state.tp_size <= 1 or group is None or dist.get_backend(group) != "gloo":
        return None
    ok = os.environ.get("PENNY_STEP_RING", "1") != "0"
    try:
        from .. import _penny_runtime  # noqa: F401
    except ImportError:
        ok = False
    flags = [None] * state.tp_size
    dist.all_gather_object(flags, ok, group=group)   # every rank must agree before anyone builds it
    if not all(flags) or not same_node(group):
        return None
    ranks = dist.get_process_group_ranks(group)
    leader = state.tp_leader_rank
    followers = [r for r in ranks if r != leader]
    me = dist.get_rank()
    ch = StepChannel(group, leader, me == leader, followers.index(me) if me != leader else 0, len(followers))
    logger.info(f"C4 step broadcast over shared-memory ring {ch.name} ({len(followers)} readers)")
    return ch
