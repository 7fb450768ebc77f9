"""Custom one-shot / two-shot all-reduce over xGMI P2P (SURVEY C1 custom path, csrc/kernels/allreduce.hip).

Each rank allocates one uncached data buffer (two halves, alternated per call) and one signal
area, exports their IPC handles, and maps every peer's pair (``hipIpcOpenMemHandle``).  A call is
then a single kernel: copy-in, flag every peer, wait for every peer, read the n buffers over the
direct links and sum (plus a 1-thread counter bump) -- hipGraph-capturable, because the round
number lives on the device.  Messages of >= 512 KB on > 2 ranks take the two-shot form
(reduce-scatter + all-gather inside one kernel, 2(n-1)/n instead of (n-1) message-sizes read
per rank); both forms sum in the same rank order, so their results are bit-identical.

Used by ``comm.tp_all_reduce`` for bf16 messages up to ``max_bytes`` when enabled
(``PENNY_CUSTOM_AR=1`` or ``enable_custom_all_reduce``); larger messages and every other dtype go
to RCCL.  A missing peer trips the kernel's bounded wait and :meth:`check` raises.
"""
from __future__ import annotations

import ctypes
from typing import List, Optional

import torch
import torch.distributed as dist

from ..ops import _native as N

AR_MAX_RANKS = 8
AR_MAX_BLOCKS = 64
SIG_BYTES = 2 * AR_MAX_RANKS * AR_MAX_BLOCKS * 4     # [region: copy-in | reduced][source rank][block]
TWOSHOT_MIN_BYTES = 512 << 10                        # below: latency-bound, one flag round wins

_SIGS = {
    "penny_ar_handle_size": [],
    "penny_ar_alloc": [ctypes.c_size_t, ctypes.POINTER(ctypes.c_void_p), ctypes.c_void_p],
    "penny_ar_open": [ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p)],
    "penny_ar_close": [ctypes.c_void_p],
    "penny_ar_free": [ctypes.c_void_p],
    "penny_allreduce_oneshot": [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_long, ctypes.POINTER(ctypes.c_void_p),
                                ctypes.POINTER(ctypes.c_void_p), ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                ctypes.c_int, ctypes.c_long, ctypes.c_int, ctypes.c_void_p],
    "penny_allgather": [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_long, ctypes.POINTER(ctypes.c_void_p),
                        ctypes.POINTER(ctypes.c_void_p), ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                        ctypes.c_int, ctypes.c_long, ctypes.c_int, ctypes.c_void_p],
    "penny_allreduce_twoshot": [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_long, ctypes.POINTER(ctypes.c_void_p),
                                ctypes.POINTER(ctypes.c_void_p), ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                                ctypes.c_int, ctypes.c_long, ctypes.c_int, ctypes.c_void_p],
}


def _lib():
    lib = N.load()
    for name, args in _SIGS.items():
        fn = getattr(lib, name)
        fn.argtypes = args
        fn.restype = ctypes.c_int
    return lib


def _check(rc: int, what: str) -> None:
    if rc != 0:
        raise RuntimeError(f"{what} failed with hipError {rc}")


class CustomAllReduce:
    def __init__(self, group=None, device: Optional[torch.device] = None, max_bytes: int = 4 << 20,
                 buffer_bytes: Optional[int] = None):
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        if not 1 <= self.world <= AR_MAX_RANKS:
            raise ValueError(f"custom all-reduce supports up to {AR_MAX_RANKS} ranks")
        self.device = device or torch.device("cuda", torch.cuda.current_device())
        self.max_bytes = max_bytes                       # all-reduce eligibility
        buffer_bytes = max(buffer_bytes or max_bytes, max_bytes)
        self.buffer_bytes = buffer_bytes                 # per-round copy-in capacity (all-gather)
        self.half_elems = buffer_bytes // 2
        lib = self._lib = _lib()
        hs = lib.penny_ar_handle_size()
        own_data, own_sig = ctypes.c_void_p(), ctypes.c_void_p()
        hd, hsg = ctypes.create_string_buffer(hs), ctypes.create_string_buffer(hs)
        with torch.cuda.device(self.device):
            _check(lib.penny_ar_alloc(2 * buffer_bytes, ctypes.byref(own_data), hd), "penny_ar_alloc(data)")
            _check(lib.penny_ar_alloc(SIG_BYTES, ctypes.byref(own_sig), hsg), "penny_ar_alloc(signal)")
        self._own = [own_data.value, own_sig.value]
        handles: List = [None] * self.world
        dist.all_gather_object(handles, (hd.raw, hsg.raw), group=group)
        self._opened: List[int] = []
        data, sig = [], []
        with torch.cuda.device(self.device):
            for q, (d, s) in enumerate(handles):
                if q == self.rank:
                    data.append(own_data.value)
                    sig.append(own_sig.value)
                    continue
                pd, ps = ctypes.c_void_p(), ctypes.c_void_p()
                _check(lib.penny_ar_open(d, ctypes.byref(pd)), f"penny_ar_open(data of rank {q})")
                _check(lib.penny_ar_open(s, ctypes.byref(ps)), f"penny_ar_open(signal of rank {q})")
                self._opened += [pd.value, ps.value]
                data.append(pd.value)
                sig.append(ps.value)
        self._data = (ctypes.c_void_p * self.world)(*data)
        self._sig = (ctypes.c_void_p * self.world)(*sig)
        self.counter = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.err = torch.zeros(1, dtype=torch.int32, device=self.device)
        dist.barrier(group=group)

    def eligible(self, x: torch.Tensor) -> bool:
        return (x.dtype == torch.bfloat16 and x.is_cuda and x.is_contiguous() and x.numel() % 8 == 0
                and x.numel() * 2 <= self.max_bytes)

    def method_for(self, n: int) -> str:
        """one-shot (one flag round, (n-1) x bytes read per rank) for latency-bound messages;
        two-shot (two rounds, 2(n-1)/n x bytes) once the per-link bytes dominate, at > 2 ranks."""
        if self.world > 2 and n * 2 >= TWOSHOT_MIN_BYTES and n % (8 * self.world) == 0:
            return "twoshot"
        return "oneshot"

    def all_reduce(self, x: torch.Tensor, out: Optional[torch.Tensor] = None,
                   method: Optional[str] = None) -> torch.Tensor:
        if not self.eligible(x):
            raise ValueError("tensor not eligible for the custom all-reduce")
        out = torch.empty_like(x) if out is None else out
        n = x.numel()
        method = method or self.method_for(n)
        if method not in ("oneshot", "twoshot") or (method == "twoshot" and n % (8 * self.world)):
            raise ValueError(f"all-reduce method {method!r} not applicable to {n} elements")
        per_block = n // self.world if method == "twoshot" else n
        nblocks = max(1, min(AR_MAX_BLOCKS, (per_block + 2047) // 2048))
        fn = self._lib.penny_allreduce_twoshot if method == "twoshot" else self._lib.penny_allreduce_oneshot
        _check(fn(x.data_ptr(), out.data_ptr(), n, self._data, self._sig, self.counter.data_ptr(),
                  self.err.data_ptr(), self.rank, self.world, self.half_elems, nblocks, N.stream()),
               f"penny_allreduce_{method}")
        return out

    def gather_eligible(self, x: torch.Tensor) -> bool:
        return (x.dtype == torch.bfloat16 and x.is_cuda and x.is_contiguous() and x.numel() % 8 == 0
                and x.numel() * 2 <= self.buffer_bytes)

    def all_gather(self, x: torch.Tensor) -> torch.Tensor:
        """[*] per rank -> [world, *] (rank-major), one kernel (copy-in, flag round, peer reads)."""
        if not self.gather_eligible(x):
            raise ValueError("tensor not eligible for the custom all-gather")
        out = torch.empty((self.world,) + tuple(x.shape), dtype=x.dtype, device=x.device)
        n = x.numel()
        nblocks = max(1, min(AR_MAX_BLOCKS, (n + 2047) // 2048))
        _check(self._lib.penny_allgather(x.data_ptr(), out.data_ptr(), n, self._data, self._sig,
                                         self.counter.data_ptr(), self.err.data_ptr(), self.rank, self.world,
                                         self.half_elems, nblocks, N.stream()), "penny_allgather")
        return out

    def check(self) -> None:
        """Raise if any call timed out waiting for a peer (syncs the device)."""
        if int(self.err.item()):
            raise RuntimeError("custom all-reduce: a peer never arrived (bounded wait expired)")

    def close(self) -> None:
        torch.cuda.synchronize(self.device)
        for p in self._opened:
            self._lib.penny_ar_close(p)
        for p in self._own:
            self._lib.penny_ar_free(p)
        self._opened, self._own = [], []
