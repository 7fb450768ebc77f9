"""Tensor-parallel collectives over RCCL/xGMI.

* C1 ``tp_all_reduce``: the partial sums after the row-parallel O-projection and
  down-projection (2 per layer).  ``tp_all_reduce_async`` starts one without blocking the host:
  the prefill micro-batch pipeline (``DecoderModel.forward_overlap``) computes one half of the
  batch while the other half's all-reduce is on the wire.  In-place ``dist.all_reduce`` on the TP group; captured into
  the decode hipGraph together with the GEMMs.
* C2 ``tp_all_gather_pairs``: vocab-parallel sampling -- each rank's per-row (score, token id)
  candidate from its vocab shard ([B, 2] int32 -> [tp, B, 2]); ``tp_all_gather_last`` gathers the
  full [B, V] logits only for rows with top-k / top-p filters.  Embedding partials are summed
  with C1.
* SP ``tp_reduce_scatter_rows`` / ``tp_all_gather_rows``: sequence-parallel prefill (Megatron
  SP) -- the residual stream is sharded by rows between the row-parallel and column-parallel
  GEMMs (reduce-scatter after O/down, all-gather before QKV/gate-up).
* C4 ``broadcast_step``: the TP leader's scheduler decisions (token ids, positions, block
  tables, sampling params) for a step, so non-leader ranks replay the identical forward: ONE flat
  byte buffer (``StepInputs.pack``) -- through the node-local shared-memory ring
  (``step_ring.py``, one release store per step) when enabled, else over a gloo twin of the TP
  group (a header broadcast carries the length).  Host memory to host memory either way.

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
# a second, independent instance (own IPC buffers, signals and counters) for the second decode
# micro-batch chain (DecoderModel.forward_decode_dual): the two chains' all-reduces run on two
# streams and must never share a flag round
_CUSTOM_AR_2 = None
_CHANNEL = 0        # which instance tp_all_reduce uses (set by ar_channel)


def enable_custom_all_reduce(max_bytes: int = 4 << 20, buffer_bytes: int = 32 << 20):
    """Route small bf16 TP all-reduces (decode) through the one-shot xGMI P2P kernel and the
    vocab-parallel logits gather (up to ``buffer_bytes`` per rank) through its all-gather twin
    (``custom_ar.py``); RCCL keeps everything else.  Call on every TP rank after init."""
    global _CUSTOM_AR
    s = state()
    if s.tp_size > 1 and _CUSTOM_AR is None:
        from .custom_ar import CustomAllReduce
        _CUSTOM_AR = CustomAllReduce(s.tp_group, max_bytes=max_bytes, buffer_bytes=buffer_bytes)
    return _CUSTOM_AR


def custom_all_reduce():
    """The enabled CustomAllReduce of the TP group, or None."""
    return _CUSTOM_AR


def enable_second_channel(max_bytes: int = 4 << 20):
    """The second custom all-reduce instance (collective over the TP group; needs the first)."""
    global _CUSTOM_AR_2
    s = state()
    if s.tp_size > 1 and _CUSTOM_AR is not None and _CUSTOM_AR_2 is None:
        from .custom_ar import CustomAllReduce
        _CUSTOM_AR_2 = CustomAllReduce(s.tp_group, max_bytes=max_bytes, buffer_bytes=max_bytes)
    return _CUSTOM_AR_2


class ar_channel:
    """Context manager: TP all-reduces issued inside go through custom-AR instance ``k`` (0 or 1)."""

    def __init__(self, k: int):
        self.k = k

    def __enter__(self):
        global _CHANNEL
        self.prev, _CHANNEL = _CHANNEL, self.k
        return self

    def __exit__(self, *exc):
        global _CHANNEL
        _CHANNEL = self.prev
        return False


def _ar_instance():
    return _CUSTOM_AR_2 if _CHANNEL == 1 else _CUSTOM_AR


# what the TP group's custom all-reduce ended up as: reported in the bench JSON per rank
AR_STATUS = {"custom": False, "self_test": "not run"}


def agree_custom_all_reduce(want_second: bool = False) -> bool:
    """Presence consensus before the init self-test: one MIN all-reduce over the TP group of (instance 0
    present, instance 1 present or not wanted).  If any rank lacks an instance the others hold, every
    rank drops the custom path, so the group never issues different collective sequences.  Called by
    every TP rank, including those whose enable raised.  Returns whether the custom path stays."""
    s = state()
    if s.tp_size == 1:
        return _CUSTOM_AR is not None
    dev = _CUSTOM_AR.device if _CUSTOM_AR is not None else (
        torch.device("cuda", torch.cuda.current_device()) if torch.cuda.is_available() else torch.device("cpu"))
    if s.backend != "nccl":
        dev = torch.device("cpu")
    bits = torch.tensor([int(_CUSTOM_AR is not None), int(_CUSTOM_AR_2 is not None or not want_second)],
                        dtype=torch.int32, device=dev)
    dist.all_reduce(bits, op=dist.ReduceOp.MIN, group=s.tp_group)
    ok = bool(int(bits[0])) and bool(int(bits[1]))
    if not ok and (_CUSTOM_AR is not None or _CUSTOM_AR_2 is not None):
        import logging
        logging.getLogger(__name__).warning("custom all-reduce missing on a peer rank; RCCL carries every TP "
                                            "collective")
        disable_custom_all_reduce()
        AR_STATUS.update(custom=False, self_test="a peer rank could not enable it")
    return ok


def verify_custom_all_reduce() -> bool:
    """Init-time first contact (every TP rank together): self-test each enabled custom instance
    against the exact sum (``custom_ar.self_test``: one-shot, two-shot, all-gather, bounded-wait
    flag).  On any rank's mismatch or expired wait EVERY rank disables the custom path and RCCL
    carries all TP collectives for the process lifetime.  Returns whether the custom path stays."""
    import logging
    log = logging.getLogger(__name__)
    if _CUSTOM_AR is None:
        AR_STATUS.update(custom=False)
        return False
    for k, ar in ((0, _CUSTOM_AR), (1, _CUSTOM_AR_2)):
        if ar is None:
            continue
        ok, why = ar.self_test()
        if not ok:
            log.warning(f"custom all-reduce instance {k} failed its self-test ({why}); RCCL carries every TP "
                        "collective from now on")
            disable_custom_all_reduce()
            AR_STATUS.update(custom=False, self_test=f"failed: {why}")
            return False
    AR_STATUS.update(custom=True, self_test="ok")
    return True


def disable_custom_all_reduce() -> None:
    global _CUSTOM_AR, _CUSTOM_AR_2
    for ar in (_CUSTOM_AR_2, _CUSTOM_AR):
        if ar is not None:
            ar.close()
    _CUSTOM_AR = _CUSTOM_AR_2 = None
    while _RETIRED:
        _RETIRED.pop().close()


_RETIRED: List[Any] = []   # instances retired at runtime: mapped until shutdown (a late peer may still read)


def fallback_to_rccl(reason: str) -> None:
    """Runtime failure of the custom all-reduce (a peer missed the bounded wait, the kernels
    returned NaN with the error flag set): from the next collective on, RCCL carries every TP
    all-reduce / all-gather of this rank.  Called by EVERY TP rank at the same step boundary (the
    leader decides and sends ``StepInputs.CTRL_RCCL_FALLBACK`` over C4 before its next step), so the
    group never mixes RCCL and custom collectives.  The IPC buffers stay mapped until shutdown: a
    stalled peer can still be inside a kernel that reads them.  The reference's failure contract
    (main.py:112-122): errors reach the client, never a silently wrong answer."""
    import logging
    global _CUSTOM_AR, _CUSTOM_AR_2
    for ar in (_CUSTOM_AR, _CUSTOM_AR_2):
        if ar is not None:
            _RETIRED.append(ar)
    _CUSTOM_AR = _CUSTOM_AR_2 = None
    AR_STATUS.update(custom=False, runtime_fallback=reason,
                     runtime_fallbacks=int(AR_STATUS.get("runtime_fallbacks", 0)) + 1)
    logging.getLogger(__name__).error(f"custom all-reduce failed at runtime ({reason}); RCCL carries every TP "
                                      "collective from now on")


def tp_all_reduce(x: torch.Tensor) -> torch.Tensor:
    s = state()
    if s.tp_size == 1:
        return x
    ar = _ar_instance()
    if ar is not None and ar.eligible(x):
        return ar.all_reduce(x, out=x)           # reads peers' staged copies, so in-place is safe
    dist.all_reduce(x, group=s.tp_group)
    return x


class _Done:
    def wait(self) -> None:
        return None


def tp_all_reduce_async(x: torch.Tensor):
    """Start the TP all-reduce of ``x`` (in place) and return a handle whose ``wait()`` orders the
    CURRENT stream after it -- the host is not blocked, so compute queued meanwhile overlaps the
    transfer (RCCL runs the collective on its own stream).  Decode-size messages that the custom
    one-shot kernel takes are latency-bound and run inline (nothing to overlap)."""
    s = state()
    if s.tp_size == 1:
        return _Done()
    if _CUSTOM_AR is not None and _CUSTOM_AR.eligible(x):
        _CUSTOM_AR.all_reduce(x, out=x)
        return _Done()
    return dist.all_reduce(x, group=s.tp_group, async_op=True)


def tp_all_gather_last(x: torch.Tensor) -> torch.Tensor:
    """Concatenate the TP shards along the last dim."""
    s = state()
    if s.tp_size == 1:
        return x
    x = x.contiguous()
    if _CUSTOM_AR is not None and _CUSTOM_AR.gather_eligible(x):
        g = _CUSTOM_AR.all_gather(x)                       # [tp, ..., V/tp], graph-capturable
        return g.movedim(0, -2).reshape(tuple(x.shape[:-1]) + (s.tp_size * x.shape[-1],))
    parts = [torch.empty_like(x) for _ in range(s.tp_size)]
    dist.all_gather(parts, x, group=s.tp_group)
    return torch.cat(parts, dim=-1)


def tp_all_gather_pairs(pairs: torch.Tensor) -> torch.Tensor:
    """Vocab-parallel sampling candidates: every rank's [B, 2] int32 (score bits, token id) ->
    [tp, B, 2] in rank order.  The custom xGMI gather moves the bytes as bf16 (graph-capturable);
    RCCL / gloo otherwise."""
    s = state()
    if s.tp_size == 1:
        return pairs[None]
    B = pairs.shape[0]
    x = pairs.contiguous()
    if B % 2:                                    # the bf16 view must be a multiple of 8 elements
        x = torch.cat([x, x[:1]], 0)
    xb = x.view(torch.bfloat16)
    if _CUSTOM_AR is not None and _CUSTOM_AR.gather_eligible(xb):
        g = _CUSTOM_AR.all_gather(xb)            # [tp, B', 4] bf16
        return g.view(torch.int32).view(s.tp_size, -1, 2)[:, :B]
    if _is_gloo(s.tp_group):
        parts = [torch.empty_like(x) for _ in range(s.tp_size)]
        dist.all_gather(parts, x, group=s.tp_group)
        return torch.stack(parts, 0)[:, :B]
    out = torch.empty((s.tp_size * x.shape[0], 2), dtype=x.dtype, device=x.device)
    dist.all_gather_into_tensor(out, x, group=s.tp_group)
    return out.view(s.tp_size, -1, 2)[:, :B]


def _is_gloo(group) -> bool:
    return dist.get_backend(group) == "gloo"


def tp_reduce_scatter_rows(x: torch.Tensor) -> torch.Tensor:
    """Sequence parallel (SP): [T, H] partial sums -> this rank's [T/tp, H] row block of the sum.
    Replaces C1's all-reduce after the row-parallel O/down projections in long prefills: the
    same bytes on the wire (RS + AG = AR for ring algorithms), but the residual stream, the
    norms and the residual adds then touch 1/tp of the rows.  T must be a multiple of tp."""
    s = state()
    if s.tp_size == 1:
        return x
    T = x.shape[0]
    if T % s.tp_size:
        raise ValueError(f"{T} rows not divisible by tp={s.tp_size}")
    if _is_gloo(s.tp_group):   # gloo has no reduce_scatter: same result through all_reduce (CI)
        dist.all_reduce(x, group=s.tp_group)
        return x.chunk(s.tp_size)[s.tp_rank].contiguous()
    out = torch.empty((T // s.tp_size,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    dist.reduce_scatter_tensor(out, x.contiguous(), group=s.tp_group)
    return out


def tp_all_gather_rows(x: torch.Tensor) -> torch.Tensor:
    """SP: every rank's [T/tp, H] row block -> the full [T, H] (rank order)."""
    s = state()
    if s.tp_size == 1:
        return x
    x = x.contiguous()
    if _is_gloo(s.tp_group):
        parts = [torch.empty_like(x) for _ in range(s.tp_size)]
        dist.all_gather(parts, x, group=s.tp_group)
        return torch.cat(parts, 0)
    out = torch.empty((x.shape[0] * s.tp_size,) + tuple(x.shape[1:]), dtype=x.dtype, device=x.device)
    dist.all_gather_into_tensor(out, x, group=s.tp_group)
    return out


_STOP = -1
_STEP_CHANNEL = None   # parallel.step_ring.StepChannel of the TP group (enable_step_channel)


def enable_step_channel():
    """C4 over the node-local shared-memory ring (``step_ring.py``) instead of two gloo
    broadcasts per step.  Collective over the TP group; returns the channel or None (fallback)."""
    global _STEP_CHANNEL
    s = state()
    if s.tp_size > 1 and _STEP_CHANNEL is None:
        from .step_ring import make_step_channel
        _STEP_CHANNEL = make_step_channel(s)
    return _STEP_CHANNEL


def step_channel():
    return _STEP_CHANNEL


def disable_step_channel() -> None:
    global _STEP_CHANNEL
    if _STEP_CHANNEL is not None:
        _STEP_CHANNEL.close()
    _STEP_CHANNEL = None


def broadcast_step(si: Any) -> Any:
    """Leader: ``si`` (a StepInputs, or None = stop) -> followers; followers pass None and get
    the leader's value back.  Over the shared-memory ring when enabled, else gloo."""
    s = state()
    if s.tp_size == 1:
        return si
    ch = _STEP_CHANNEL
    if ch is not None:
        if s.is_tp_leader:
            ch.send(None if si is None else si.pack())
            return si
        buf = ch.recv()
        if buf is None:
            return None
        from ..engine.model_runner import StepInputs
        return StepInputs.unpack(buf)
    import numpy as np
    group = s.tp_cpu_group if s.tp_cpu_group is not None else s.tp_group
    head = torch.zeros(1, dtype=torch.int64)
    if s.is_tp_leader:
        payload = None if si is None else si.pack()
        head[0] = _STOP if payload is None else payload.size
    dist.broadcast(head, src=s.tp_leader_rank, group=group)
    n = int(head[0])
    if n == _STOP:
        return None
    if s.is_tp_leader:
        dist.broadcast(torch.from_numpy(payload), src=s.tp_leader_rank, group=group)
        return si
    buf = torch.empty(n, dtype=torch.uint8)
    dist.broadcast(buf, src=s.tp_leader_rank, group=group)
    from ..engine.model_runner import StepInputs
    return StepInputs.unpack(buf.numpy())


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
