"""Executes scheduled batches on the GPU: input prep, forward, logits, sampling, hipGraph decode.

Per step the host packs one int32 staging buffer (token ids, positions, KV slots, context
lengths, block tables, sampling seeds) and ships it with ONE pinned H2D copy; the forward then
runs without further host round-trips, and the only D2H sync is the sampled ids.

Pure-decode steps (the hot loop: one token per running sequence) replay a hipGraph captured
per batch-size bucket (``torch.cuda.graph`` records hipGraph on ROCm): the ~10 kernels x L
layers of a decode step become one launch, removing ~1.5 us x 300+ launch gaps per token
(SURVEY §7.4).  Padding rows of a bucket write no KV (slot -1) and their outputs are dropped.
"""
from __future__ import annotations

import itertools
import math
import os
from dataclasses import dataclass
from typing import Dict, List, Optional, Tuple

import numpy as np
import torch

from .. import ops
from ..models.common import AttentionMetadata, KVCache
from ..ops import attention as _attn
from ..ops.attention import KV_BS, DecodeWorkspace, mark_shared_blocks, prefill_plan
from ..parallel import comm
from ..utils.logging import get_logger
from ..utils.profiling import marker
from .scheduler import ScheduledBatch
from .sequence import Sequence

logger = get_logger(__name__)


# prefill-step GEMM M histogram bucket upper bounds (engine stats / bench record)
PREFILL_M_BUCKETS = (256, 512, 1024, 2048, 3072, 4096, 1 << 30)


@dataclass
class StepInputs:
    """Host-side description of one forward (also what the TP leader broadcasts, C4)."""

    ids: np.ndarray                 # [T]
    positions: np.ndarray           # [T]
    slots: np.ndarray               # [T]
    cu_q: np.ndarray                # [Sp+1]
    ctx_p: np.ndarray               # [Sp]
    bt_p: np.ndarray                # [Sp, W]
    max_q_len: int
    ctx_d: np.ndarray               # [Bd]
    bt_d: np.ndarray                # [Bd, W]
    logits_idx: np.ndarray          # [S] rows whose next token is sampled
    temps: np.ndarray               # [S] f32
    seeds: np.ndarray               # [S] int64
    top_k: np.ndarray               # [S]
    top_p: np.ndarray               # [S]
    src: Optional[np.ndarray] = None  # [Bd] row of the previous step's sampled vector (-1: ids[] is real)
    pwork: Optional[np.ndarray] = None  # prefill attention work list (filled by the runner): [n, 2] or lean [., 6]

    @property
    def num_prefill_tokens(self) -> int:
        return int(self.cu_q[-1]) if len(self.cu_q) else 0

    # -- C4 wire format: one flat byte buffer (no pickling) ------------------------------------
    _ARRAYS = ("ids", "positions", "slots", "cu_q", "ctx_p", "bt_p", "ctx_d", "bt_d", "logits_idx", "temps",
               "seeds", "top_k", "top_p", "src", "pwork")

    def pack(self) -> np.ndarray:
        """[header int64: max_q_len, then (dtype code, rows, cols) per array] + raw array bytes."""
        arrs = [getattr(self, n) for n in self._ARRAYS]
        head = [self.max_q_len]
        body = []
        for a in arrs:
            if a is None:
                head += [-1, 0, 0]
                continue
            a = np.ascontiguousarray(a)
            head += [_DT_CODE[a.dtype.str], a.shape[0], a.shape[1] if a.ndim == 2 else -1]
            body.append(a.view(np.uint8).reshape(-1))
        h = np.asarray(head, np.int64).view(np.uint8)
        return np.concatenate([h] + body)

    @classmethod
    def unpack(cls, buf: np.ndarray) -> "StepInputs":
        n = len(cls._ARRAYS)
        head = buf[:8 * (1 + 3 * n)].view(np.int64)
        off = 8 * (1 + 3 * n)
        vals = {}
        for i, name in enumerate(cls._ARRAYS):
            code, rows, cols = (int(x) for x in head[1 + 3 * i: 4 + 3 * i])
            if code < 0:
                vals[name] = None
                continue
            dt = np.dtype(_DT_NAME[code])
            count = rows * (cols if cols >= 0 else 1)
            a = buf[off: off + count * dt.itemsize].view(dt)
            off += count * dt.itemsize
            vals[name] = a.reshape(rows, cols) if cols >= 0 else a
        return cls(max_q_len=int(head[0]), **vals)

    @property
    def num_decode(self) -> int:
        return len(self.ctx_d)

    # -- control messages on the C4 channel (max_q_len < 0, no arrays) -------------------------
    CTRL_RCCL_FALLBACK = -2          # every TP rank: retire the custom all-reduce, RCCL from here on

    @classmethod
    def control(cls, code: int) -> "StepInputs":
        e = np.zeros(0, np.int32)
        return cls(e, e, e, np.zeros(1, np.int32), e, np.zeros((0, 1), np.int32), code, e, np.zeros((0, 1), np.int32),
                   np.zeros(0, np.int64), np.zeros(0, np.float32), np.zeros(0, np.int64), e, np.zeros(0, np.float32))

    @property
    def control_code(self) -> int:
        return self.max_q_len if self.max_q_len < 0 else 0


_DT_NAME = ("<i4", "<i8", "<f4")
_DT_CODE = {n: i for i, n in enumerate(_DT_NAME)}


def _slots(seq: Sequence, start: int, n: int) -> List[int]:
    bt = seq.block_table
    return [bt[p // KV_BS] * KV_BS + p % KV_BS for p in range(start, start + n)]


def sample_rows(seq, n: int) -> int:
    """Sampled positions at the end of a sequence's final chunk of n tokens: the whole draft + 1
    for a speculative chunk (engine.speculative), else the last token only."""
    return max(1, min(seq.spec_rows, n))


def _table(rows: List[List[int]]) -> np.ndarray:
    """Ragged block tables -> zero-padded [len(rows), max len] int32, in one vectorised scatter."""
    lens = np.fromiter((len(r) for r in rows), np.int64, len(rows))
    w = max(int(lens.max()) if len(rows) else 1, 1)
    out = np.zeros((len(rows), w), np.int32)
    if len(rows):
        flat = np.fromiter(itertools.chain.from_iterable(rows), np.int32, int(lens.sum()))
        mask = np.arange(w)[None, :] < lens[:, None]
        out[mask] = flat
    return out


def build_step_inputs(batch: ScheduledBatch) -> StepInputs:
    """The host arrays of one step.  Per-token work is numpy (a prefill step carries ~2-4k tokens:
    a per-token Python list build cost ~1 ms of the host's critical path between GPU steps)."""
    ids_parts: List[np.ndarray] = []
    pos_parts: List[np.ndarray] = []
    slot_parts: List[np.ndarray] = []
    cu = [0]
    ctx_p, tables_p = [], []
    logits_idx, temps, seeds, tk, tp = [], [], [], [], []
    max_q = 0
    for seq, start, n in batch.prefill:
        np_ = len(seq.prompt_ids)
        if start + n <= np_:
            ids_parts.append(np.asarray(seq.prompt_ids[start:start + n], np.int32))
        else:
            ids_parts.append(np.asarray(seq.all_ids[start:start + n], np.int32))
        p = np.arange(start, start + n, dtype=np.int32)
        pos_parts.append(p)
        bt = np.asarray(seq.block_table, np.int32)
        slot_parts.append(bt[p // KV_BS] * KV_BS + p % KV_BS)
        cu.append(cu[-1] + n)
        ctx_p.append(start + n)
        tables_p.append(seq.block_table)
        max_q = max(max_q, n)
        if start + n == seq.num_tokens:
            # a speculative chunk samples its last spec_rows positions (verification), others one
            r = sample_rows(seq, n)
            k0 = len(seq.output_ids) - r + 1
            for i in range(r):
                logits_idx.append(cu[-1] - r + i)
                temps.append(seq.params.temperature)
                seeds.append(seq.step_seed_at(k0 + i))
                tk.append(seq.params.top_k)
                tp.append(seq.params.top_p)
    Tp = cu[-1]
    ids_d, pos_d, slots_d = [], [], []
    ctx_d, tables_d, src = [], [], []
    for j, seq in enumerate(batch.decode):
        p = seq.num_tokens - 1
        if seq.pending_src >= 0:      # token sampled by the step still in flight: device gather
            ids_d.append(0)
            src.append(seq.pending_src)
        else:
            ids_d.append(seq.output_ids[-1] if seq.output_ids else seq.prompt_ids[-1])
            src.append(-1)
        pos_d.append(p)
        slots_d.append(seq.block_table[p // KV_BS] * KV_BS + p % KV_BS)
        ctx_d.append(p + 1)
        tables_d.append(seq.block_table)
        logits_idx.append(Tp + j)
        temps.append(seq.params.temperature)
        seeds.append(seq.step_seed())
        tk.append(seq.params.top_k)
        tp.append(seq.params.top_p)

    i32 = lambda x: np.asarray(x, np.int32)  # noqa: E731
    cat = lambda parts, tail: np.concatenate(parts + [i32(tail)]) if parts else i32(tail)  # noqa: E731
    src_a = i32(src) if any(x >= 0 for x in src) else None
    bt_d = _table(tables_d)
    if _attn.LEAN_FLAGS & 1 and _attn.DECODE_LEAN and len(ctx_d) >= _attn.LEAN_NT_MIN_B:
        # the lean kernel's cache policy per block -- only where ops.decode keeps the NT bit
        mark_shared_blocks(bt_d, ctx_d)
    return StepInputs(cat(ids_parts, ids_d), cat(pos_parts, pos_d), cat(slot_parts, slots_d), i32(cu), i32(ctx_p),
                      _table(tables_p), max_q, i32(ctx_d), bt_d, np.asarray(logits_idx, np.int64),
                      np.asarray(temps, np.float32), np.asarray(seeds, np.int64), i32(tk), np.asarray(tp, np.float32),
                      src_a)


class CollectiveTimeout(RuntimeError):
    """A device-side collective (custom xGMI all-reduce) reported a missing peer."""


class PendingStep:
    """Sampled ids of a launched step (host copy in flight)."""

    def __init__(self, cpu_out: Optional[torch.Tensor], n: int, host: Optional[torch.Tensor], event,
                 start_event=None, stats: Optional[Dict] = None, key: str = "", check_err: bool = False):
        self._cpu, self.n, self._host, self._event = cpu_out, n, host, event
        self._start, self._stats, self._key = start_event, stats, key
        self._check_err = check_err

    def result(self) -> List[int]:
        if self.n == 0:
            return []
        if self._cpu is not None:
            return self._cpu.tolist()
        if self._event is not None:
            self._event.synchronize()
        if self._start is not None:   # device time of the step (PENNY_STEP_GPU_TIMING=1)
            st = self._stats
            st[self._key] += self._start.elapsed_time(self._event) / 1e3
            # device idle between consecutive steps: this step's start - the previous step's end
            prev_end = st.get("_prev_end_ev")
            if prev_end is not None:
                gap = prev_end.elapsed_time(self._start) / 1e3
                if gap > 0:
                    st["gpu_idle_s"] += gap
                    st["gpu_idle_gaps"] += 1
            st["_prev_end_ev"] = self._event
        if self._check_err and int(self._host[self.n]):
            raise CollectiveTimeout("custom all-reduce: a TP peer missed the bounded wait; this step's "
                                    "hidden states are stale")
        return self._host[:self.n].tolist()


class _DecodeGraph:
    def __init__(self, graph, B: int, out: torch.Tensor, fused: bool = False):
        # fused: the graph samples inside the LM head (no top-k / top-p support)
        self.graph, self.B, self.out, self.fused = graph, B, out, fused


class ModelRunner:
    def __init__(self, model, kv: KVCache, max_model_len: int, max_decode_batch: int = 256,
                 use_graphs: bool = True, graph_sizes: Tuple[int, ...] = (1, 2, 4, 8, 16, 32, 64, 128, 256)):
        self.model = model
        self.kv = kv
        self.device = model.device
        self.max_model_len = max_model_len
        self.max_blocks = (max_model_len + KV_BS - 1) // KV_BS
        self.on_gpu = self.device.type == "cuda"
        self.use_graphs = use_graphs and self.on_gpu
        self.G = model.hq // model.hkv
        self.graph_sizes = tuple(sorted(s for s in graph_sizes if s <= max_decode_batch))
        self.max_decode_batch = max(self.graph_sizes) if self.graph_sizes else max_decode_batch
        cfg = model.cfg
        self.decode_ws = DecodeWorkspace.create(max(max_decode_batch, 1), model.hq, model.D, max_model_len,
                                                self.device) if self.on_gpu else None
        # TP decode as two micro-batch chains on two streams (DecoderModel.forward_decode_dual): their
        # all-reduces hide under the other chain's compute; needs the second custom-AR channel
        # (decided at the first graph capture: the engine enables the AR channels after building us)
        self._dual: Optional[bool] = None
        self.dual_min_batch = int(os.environ.get("PENNY_TP_DUAL_MIN_BATCH", "2"))
        self._max_decode_ws = max(max_decode_batch, 1)
        self.decode_ws2 = None
        self.graphs: Dict[int, _DecodeGraph] = {}
        self.graphs_filt: Dict[int, _DecodeGraph] = {}   # top-k / top-p twins of fused buckets (lazy)
        self._filt_failed: set = set()                    # buckets whose filtered twin could not be captured
        self._static = None
        self.graph_pool = None
        self.stats = {"steps": 0, "graph_steps": 0, "tokens": 0, "prefill_steps": 0, "prefill_step_tokens": 0,
                      "prefill_tile_pad_rows": 0, "prefill_m_hist": [0] * len(PREFILL_M_BUCKETS), "gpu_graph_s": 0.0, "gpu_eager_s": 0.0,
                      "gpu_idle_s": 0.0, "gpu_idle_gaps": 0, "_prev_end_ev": None, "overlap_steps": 0}
        # TP prefill steps of >= overlap_min_rows rows run as two micro-batches whose all-reduces
        # overlap the other half's compute (PENNY_TP_OVERLAP=0 disables)
        self.tp_overlap = os.environ.get("PENNY_TP_OVERLAP", "1") == "1"
        self.overlap_min_rows = int(os.environ.get("PENNY_TP_OVERLAP_MIN_ROWS", "1024"))
        # device time of every step and the device idle between steps (two events per step: on by
        # default so every bench run reports where the non-busy GPU time is; =0 turns it off)
        self._gpu_timing = self.on_gpu and os.environ.get("PENNY_STEP_GPU_TIMING", "1") == "1"
        # sampled ids of the latest step stay on the device: the next step gathers its decode ids
        # from here when it was launched before this one's ids reached the host (overlap mode)
        # a speculative chunk samples draft + 1 rows (engine.speculative: drafts <= 16 tokens)
        self.max_samplers = 17 * max(self.max_decode_batch, max_decode_batch) + 1024
        self.last_sampled = torch.zeros(self.max_samplers, dtype=torch.int32, device=self.device)
        # one slot past the sampled ids carries the custom all-reduce's timeout flag back with them
        self._pinned_out = ([torch.zeros(self.max_samplers + 1, dtype=torch.int32).pin_memory() for _ in range(2)]
                            if self.on_gpu else None)
        self._out_flip = 0
        self._ev_ring: Optional[List[Tuple[torch.cuda.Event, torch.cuda.Event]]] = None
        self._ev_i = 0
        # eager-step inputs: one pinned staging ring slot -> ONE H2D copy per step (see _stage_inputs)
        self._staged: Optional[Dict[int, torch.Tensor]] = None
        self._stage_ring: List[Optional[torch.Tensor]] = [None] * 4
        self._stage_events: List[Optional[torch.cuda.Event]] = [None] * 4
        self._stage_flip = 0
        self._stage_enabled = os.environ.get("PENNY_STAGE_INPUTS", "1") == "1"

    # ------------------------------------------------------------------------------------
    # eager path
    # ------------------------------------------------------------------------------------
    _STAGE_DTYPES = {np.dtype(np.int32): torch.int32, np.dtype(np.int64): torch.int64,
                     np.dtype(np.float32): torch.float32}

    def _stage_inputs(self, si: StepInputs) -> None:
        """Upload every array of an eager step with ONE H2D copy: the arrays are packed (16-B
        aligned) into a pinned staging slot, copied as one byte buffer and handed out as typed
        device views by ``_to_dev``.  One copy per array meant ~12 blit kernels and pinned
        allocations per step on the compute stream."""
        self._staged = None
        if not self.on_gpu or not self._stage_enabled:
            return
        arrs = []
        total = 0
        for name in StepInputs._ARRAYS:
            a = getattr(si, name)
            if a is None or a.dtype not in self._STAGE_DTYPES:
                continue
            arrs.append((a, np.ascontiguousarray(a), total))
            total += (a.nbytes + 15) // 16 * 16
        if total == 0:
            return
        k = self._stage_flip
        self._stage_flip = (k + 1) % len(self._stage_ring)
        if self._stage_events[k] is not None:
            self._stage_events[k].synchronize()     # the copy that last read this slot is done
        buf = self._stage_ring[k]
        if buf is None or buf.numel() < total:
            buf = torch.empty(max(total, 1 << 20), dtype=torch.uint8).pin_memory()
            self._stage_ring[k] = buf
        host = buf.numpy()
        for _, c, off in arrs:
            host[off:off + c.nbytes] = c.reshape(-1).view(np.uint8)
        dev = torch.empty(total, dtype=torch.uint8, device=self.device)
        dev.copy_(buf[:total], non_blocking=True)
        ev = torch.cuda.Event()
        ev.record()
        self._stage_events[k] = ev
        self._staged = {id(a): dev[off:off + c.nbytes].view(self._STAGE_DTYPES[c.dtype]).view(c.shape)
                        for a, c, off in arrs}

    def _to_dev(self, a: np.ndarray, dtype=None) -> torch.Tensor:
        t = self._staged.get(id(a)) if self._staged is not None else None
        if t is None:
            t = torch.from_numpy(np.ascontiguousarray(a))
            if self.on_gpu:
                t = t.pin_memory().to(self.device, non_blocking=True)
        return t if dtype is None else t.to(dtype)

    def _meta(self, si: StepInputs, slots: torch.Tensor) -> AttentionMetadata:
        m = AttentionMetadata(slots=slots, num_prefill_tokens=si.num_prefill_tokens, num_decode=si.num_decode,
                              decode_ws=self.decode_ws)
        if si.num_prefill_tokens:
            m.cu_q = self._to_dev(si.cu_q)
            m.ctx_lens_p = self._to_dev(si.ctx_p)
            m.block_tables_p = self._to_dev(si.bt_p)
            m.max_q_len = si.max_q_len
            if self.on_gpu:   # LPT-ordered prefill attention tiles (staged with the step when precomputed)
                work = si.pwork if si.pwork is not None else prefill_plan(si.cu_q, si.ctx_p, self.G, self.model.hkv)
                m.prefill_work = self._to_dev(work) if work is not None else None
                if work is not None and work.shape[1] == 6:        # lean split-KV list: its counts
                    m.prefill_lean = (int(work[0, 1]), int(work[0, 2]), int(work[0, 3]))
        if si.num_decode:
            m.ctx_lens_d = self._to_dev(si.ctx_d)
            m.block_tables_d = self._to_dev(si.bt_d)
        return m

    def _gather_pending(self, ids: torch.Tensor, src: torch.Tensor, offset: int) -> None:
        """ids[offset + r] <- last_sampled[src[r]] where src[r] >= 0 (device-side, no host sync)."""
        rows = ids[offset:offset + src.shape[0]]
        rows.copy_(torch.where(src >= 0, self.last_sampled[src.clamp(min=0).long()], rows))

    def _overlap_split(self, si: StepInputs) -> Optional[int]:
        """Row at which a TP prefill step is cut into two micro-batches (None: no overlap)."""
        m = self.model
        if (getattr(m, "tp_size", 1) == 1 or not self.tp_overlap or si.num_prefill_tokens < self.overlap_min_rows
                or (hasattr(m, "uses_sp") and m.uses_sp(len(si.ids))) or not hasattr(m, "forward_overlap")):
            return None
        half = len(si.ids) // 2
        t = half // 128 * 128 if half >= 512 else half       # GEMM-friendly halves on real steps
        return max(1, min(t, si.num_prefill_tokens))

    def _split_inputs(self, si: StepInputs, t: int):
        """Two StepInputs for rows [0, t) (prefill only) and [t, T) (rest of the prefill + the
        decodes); the sequence containing row t appears in both, its first part with the
        context length it has after those rows."""
        cu = si.cu_q
        s = int(np.searchsorted(cu, t, side="right")) - 1          # sequence holding row t
        cut = t > cu[s]                                              # row t is inside sequence s
        na = s + (1 if cut else 0)
        cu_a = np.concatenate([cu[:s + 1], [t]]) if cut else cu[:s + 1]
        ctx_a = si.ctx_p[:na].copy()
        if cut:
            ctx_a[-1] = si.ctx_p[s] - (cu[s + 1] - t)
        cu_b = np.concatenate([[0], cu[s + 1:] - t]) if cut else cu[s:] - t
        empty_i = np.zeros(0, np.int32)
        a = StepInputs(si.ids[:t], si.positions[:t], si.slots[:t], cu_a.astype(np.int32), ctx_a,
                       si.bt_p[:na], si.max_q_len, empty_i, np.zeros((0, 1), np.int32), si.logits_idx[:0],
                       si.temps[:0], si.seeds[:0], si.top_k[:0], si.top_p[:0], None)
        b = StepInputs(si.ids[t:], si.positions[t:], si.slots[t:], cu_b.astype(np.int32), si.ctx_p[s:],
                       si.bt_p[s:], si.max_q_len, si.ctx_d, si.bt_d, si.logits_idx, si.temps, si.seeds,
                       si.top_k, si.top_p, None)
        return a, b

    def _hidden(self, si: StepInputs) -> torch.Tensor:
        """Final hidden states of every row of the step."""
        ids = self._to_dev(si.ids)
        if si.src is not None:
            self._gather_pending(ids, self._to_dev(si.src), si.num_prefill_tokens)
        pos = self._to_dev(si.positions)
        slots = self._to_dev(si.slots)
        t = self._overlap_split(si)
        if t is not None:    # TP prefill: micro-batch pipeline overlapping the all-reduces
            a, b = self._split_inputs(si, t)
            metas = (self._meta(a, slots[:t]), self._meta(b, slots[t:]))
            self.stats["overlap_steps"] += 1
            return self.model.forward_overlap(ids, pos, metas, t, self.kv)
        return self.model.forward(ids, pos, self._meta(si, slots), self.kv)

    def forward_logits(self, si: StepInputs) -> torch.Tensor:
        h = self._hidden(si)
        idx = self._to_dev(si.logits_idx)
        return self.model.logits(h.index_select(0, idx))

    def _fused_sampling(self, h: torch.Tensor) -> bool:
        """Does sampling the rows ``h`` run inside the LM head (fused K11 + K12)?  TP=1 only: under TP
        the vocabulary is sharded and the logits are all-gathered before sampling."""
        m = self.model
        return getattr(m, "tp_size", 1) == 1 and hasattr(m, "lm_weight") and ops.fused_lm_head_ok(h, m.lm_weight())

    def _lm_tiled(self):
        f = getattr(self.model, "lm_tiled", None)
        return f() if f is not None else None

    def _shard_sampling(self) -> bool:
        """TP: rows without top-k / top-p are sampled vocab-parallel (``sample_vocab_parallel``:
        [B, 2] candidates all-gathered instead of the [B, V] logits); ``PENNY_VOCAB_PARALLEL_SAMPLE=0``
        restores logits all-gather + sampler."""
        m = self.model
        return (getattr(m, "tp_size", 1) > 1 and hasattr(m, "sample_vocab_parallel")
                and os.environ.get("PENNY_VOCAB_PARALLEL_SAMPLE", "1") != "0")

    @staticmethod
    def _has_filters(si: StepInputs) -> bool:
        return bool((si.top_k > 0).any() or (si.top_p < 1).any())

    def logits_and_sample(self, si: StepInputs) -> torch.Tensor:
        """Forward the step, then sample one token per ``si.logits_idx`` row: fused into the LM head
        where it applies (no top-k / top-p rows), else logits -> sampler."""
        h = self._hidden(si)
        hs = h.index_select(0, self._to_dev(si.logits_idx))
        if not self._has_filters(si) and self._shard_sampling():
            self.stats["vocab_parallel_sample_steps"] = self.stats.get("vocab_parallel_sample_steps", 0) + 1
            return self.model.sample_vocab_parallel(hs, self._to_dev(si.temps), self._to_dev(si.seeds))
        if not self._has_filters(si) and self._fused_sampling(hs):
            self.stats["fused_lm_head_steps"] = self.stats.get("fused_lm_head_steps", 0) + 1
            return ops.lm_head_sample(hs, self.model.lm_weight(), self._to_dev(si.temps), self._to_dev(si.seeds),
                                      wt=self._lm_tiled())
        return self.sample(self.model.logits(hs), si)

    def sample(self, logits: torch.Tensor, si: StepInputs) -> torch.Tensor:
        temps = self._to_dev(si.temps)
        seeds = self._to_dev(si.seeds)
        if self._has_filters(si):   # device-side top-k/top-p threshold
            return ops.sample(logits.contiguous(), temps, seeds, top_k=self._to_dev(si.top_k),
                              top_p=self._to_dev(si.top_p))
        return ops.sample(logits.contiguous(), temps, seeds)

    def execute(self, si: StepInputs) -> List[int]:
        """Run one step; returns the sampled token per entry of ``si.logits_idx``."""
        return self.launch(si).result()

    def launch(self, si: StepInputs) -> "PendingStep":
        """Enqueue one step on the current stream and return without waiting for the GPU; the
        sampled ids reach the host through ``PendingStep.result()`` (pinned D2H + event)."""
        self.stats["steps"] += 1
        self.stats["tokens"] += len(si.ids)
        if si.num_prefill_tokens:   # GEMM M of the steps that run the prefill (library) GEMMs
            M = len(si.ids)
            self.stats["prefill_steps"] += 1
            self.stats["prefill_step_tokens"] += M
            # rows the 256-row prefill tiles pad (M > 256: the tile kernels' M quantisation) and the
            # step-size histogram, for the bench record
            self.stats["prefill_tile_pad_rows"] += (-M) % 256 if M > 256 else 0
            b = next(i for i, hi in enumerate(PREFILL_M_BUCKETS) if M <= hi)
            self.stats["prefill_m_hist"][b] += 1
        if len(si.logits_idx) == 0:
            self._stage_inputs(si)
            try:
                self._forward_only(si)
            finally:
                self._staged = None
            return PendingStep(None, 0, None, None)
        start_ev = end_ev = None
        if self.on_gpu:
            # a small ring of reused events (creating two timing events per step cost ~30 us of
            # host time between launches); 4 pairs cover the step in flight, the one being collected and
            # the previous step's end event the idle-gap measurement still reads
            if self._ev_ring is None:
                self._ev_ring = [(torch.cuda.Event(enable_timing=self._gpu_timing),
                                  torch.cuda.Event(enable_timing=self._gpu_timing)) for _ in range(4)]
            start_ev, end_ev = self._ev_ring[self._ev_i]
            self._ev_i = (self._ev_i + 1) % len(self._ev_ring)
            if self._gpu_timing:
                start_ev.record()
            else:
                start_ev = None
        graph = False
        if (self.use_graphs and si.num_prefill_tokens == 0 and 0 < si.num_decode <= self.max_decode_batch
                and not self._fused_graph_needs_eager(si)):
            with marker(f"decode.graph[{si.num_decode}]"):
                out = self._graph_decode(si)
            graph = True
        else:
            with marker(f"forward.eager[{len(si.ids)}]"):
                if si.num_prefill_tokens and si.pwork is None and self.on_gpu:
                    si.pwork = prefill_plan(si.cu_q, si.ctx_p, self.G, self.model.hkv)
                self._stage_inputs(si)
                try:
                    out = self.logits_and_sample(si)
                finally:
                    self._staged = None
        n = len(si.logits_idx)
        self.last_sampled[:n].copy_(out[:n].to(torch.int32), non_blocking=True)
        ar = comm.custom_all_reduce()
        if not self.on_gpu:
            cpu = out[:n].clone()
            if ar is not None:           # a host-side stand-in (tests): its flag is host memory
                return PendingStep(None, n, torch.cat([cpu.to(torch.int32), ar.err.to(torch.int32)[:1]]), None,
                                   check_err=True)
            return PendingStep(cpu, n, None, None)
        host = self._pinned_out[self._out_flip]
        self._out_flip ^= 1
        host[:n].copy_(out[:n], non_blocking=True)
        if ar is not None:
            # the xGMI all-reduce never raises from the device: a peer that missed its bounded wait
            # sets ar.err and the step's sums are stale, so the flag rides the per-step host sync
            host[n:n + 1].copy_(ar.err, non_blocking=True)
        ev = end_ev
        ev.record()
        return PendingStep(None, n, host, ev, start_ev, self.stats, "gpu_graph_s" if graph else "gpu_eager_s",
                           check_err=ar is not None)

    def _forward_only(self, si: StepInputs) -> None:
        self._hidden(si)

    def drop_graphs(self) -> None:
        """Forget every captured decode graph (they bake in the custom all-reduce kernels and its
        buffers): after a runtime fallback to RCCL (comm.fallback_to_rccl) decode runs eagerly."""
        if self.on_gpu:
            torch.cuda.synchronize(self.device)
        self.graphs.clear()
        self.graphs_filt.clear()
        self.use_graphs = False
        self._dual = False

    # ------------------------------------------------------------------------------------
    # hipGraph decode
    # ------------------------------------------------------------------------------------
    def _alloc_static(self) -> None:
        B, W = self.max_decode_batch, self.max_blocks
        # ids | pos | slots | ctx | block tables | gather rows | top-k live in ONE device buffer fed
        # by ONE pinned H2D copy
        self._src_off = 4 * B + B * W          # pending-token gather rows (-1: host id)
        self._topk_off = self._src_off + B     # per-row top-k (0: off)
        self._dev_i32 = torch.zeros(self._topk_off + B, dtype=torch.int32, device=self.device)
        d = self._dev_i32
        self._static = {
            "ids": d[0:B], "pos": d[B:2 * B], "slots": d[2 * B:3 * B], "ctx": d[3 * B:4 * B],
            "bt": d[4 * B:self._src_off].view(B, W),
            "src": d[self._src_off:self._topk_off],
            "top_k": d[self._topk_off:self._topk_off + B],
            "f32": torch.zeros(2 * B, dtype=torch.float32, device=self.device),     # temps | top_p
            "seeds": torch.zeros(B, dtype=torch.int64, device=self.device),
        }
        self._static["slots"].fill_(-1)
        self._static["ctx"].fill_(1)
        self._static["src"].fill_(-1)
        self._static["temps"], self._static["top_p"] = self._static["f32"][:B], self._static["f32"][B:]
        self._static["top_p"].fill_(1.0)
        # two pinned staging sets, alternated per graph step: in overlap mode the host packs step
        # N+1 while step N's H2D copy may still be queued behind step N-1 on the stream, so a
        # single buffer could be overwritten before the DMA reads it
        self._pinned_sets = [(torch.zeros(self._topk_off + B, dtype=torch.int32).pin_memory(),
                              torch.zeros(2 * B, dtype=torch.float32).pin_memory(),
                              torch.zeros(B, dtype=torch.int64).pin_memory()) for _ in range(2)]
        self._pin_flip = 0
        self._pinned_i32, self._pinned_f, self._pinned_l = self._pinned_sets[0]

    @property
    def dual_decode(self) -> bool:
        if self._dual is None:
            m = self.model
            self._dual = bool(self.on_gpu and getattr(m, "tp_size", 1) > 1 and hasattr(m, "forward_decode_dual")
                              and getattr(m.cfg, "arch", "") == "llama" and comm.custom_all_reduce() is not None
                              and getattr(comm, "_CUSTOM_AR_2", None) is not None
                              and os.environ.get("PENNY_TP_DUAL_DECODE", "1") != "0")
            if self._dual:
                # each chain's all-reduce must fit ITS custom instance: a half batch falling back to
                # RCCL would put two streams' RCCL collectives on one communicator inside one graph
                need = ((self.max_decode_batch + 1) // 2) * m.cfg.hidden_size * 2
                cap = min(comm.custom_all_reduce().max_bytes, comm._CUSTOM_AR_2.max_bytes)
                if need > cap:
                    logger.warning(f"TP dual decode disabled: a half batch all-reduces {need} B > the custom "
                                   f"all-reduce's {cap} B")
                    self._dual = False
            if self._dual:
                self.decode_ws2 = DecodeWorkspace.create(self._max_decode_ws, m.hq, m.D, self.max_model_len,
                                                         self.device)
        return self._dual

    def _run_static(self, B: int, filtered: bool = False) -> torch.Tensor:
        s = self._static
        self._gather_pending(s["ids"], s["src"][:B], 0)
        if self.dual_decode and B >= self.dual_min_batch:
            k = B // 2                       # two chains: rows [0, k) and [k, B)
            metas = [AttentionMetadata(slots=s["slots"][a:b], num_prefill_tokens=0, num_decode=b - a,
                                       ctx_lens_d=s["ctx"][a:b], block_tables_d=s["bt"][a:b], decode_ws=ws)
                     for (a, b), ws in (((0, k), self.decode_ws), ((k, B), self.decode_ws2))]
            self.stats["dual_decode_graphs"] = self.stats.get("dual_decode_graphs", 0) + 1
            h = self.model.forward_decode_dual(s["ids"][:B], s["pos"][:B], metas, k, self.kv)
        else:
            meta = AttentionMetadata(slots=s["slots"][:B], num_prefill_tokens=0, num_decode=B,
                                     ctx_lens_d=s["ctx"][:B], block_tables_d=s["bt"][:B], decode_ws=self.decode_ws)
            h = self.model.forward(s["ids"][:B], s["pos"][:B], meta, self.kv)
        if not filtered:
            if self._shard_sampling():     # TP: top-k / top-p rows of this bucket replay eagerly
                return self.model.sample_vocab_parallel(h, s["temps"][:B], s["seeds"][:B])
            if self._fused_sampling(h):
                return ops.lm_head_sample(h, self.model.lm_weight(), s["temps"][:B], s["seeds"][:B],
                                          wt=self._lm_tiled())
        logits = self.model.logits(h)
        # the top-k/top-p threshold kernel is always in the graph: unfiltered rows (k=0, p=1) exit
        # after reading their parameters
        return ops.sample(logits, s["temps"][:B], s["seeds"][:B], top_k=s["top_k"][:B], top_p=s["top_p"][:B])

    def capture_graphs(self) -> None:
        if not self.use_graphs:
            return
        if self._static is None:
            self._alloc_static()
        torch.cuda.synchronize()
        for B in sorted(self.graph_sizes, reverse=True):
            # warm up (allocator + hipBLASLt heuristics) outside the capture
            for _ in range(2):
                self._run_static(B)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, pool=self.graph_pool):
                out = self._run_static(B)
            if self.graph_pool is None:
                self.graph_pool = g.pool()
            fused = self._shard_sampling() or self._fused_sampling(
                torch.empty((B, self.model.cfg.hidden_size), dtype=torch.bfloat16, device=self.device))
            self.graphs[B] = _DecodeGraph(g, B, out, fused)
        torch.cuda.synchronize()
        logger.info(f"captured decode hipGraphs for batch sizes {sorted(self.graphs)}")

    def _fused_graph_needs_eager(self, si: StepInputs) -> bool:
        """A decode step with top-k / top-p rows whose bucket's graph samples inside the LM head: at
        TP=1 it replays the bucket's FILTERED twin (logits -> threshold -> sampler), captured on the
        first such step; under TP (vocab-parallel candidates) it runs eagerly."""
        if not self._has_filters(si):
            return False
        if not self.graphs:
            self.capture_graphs()
        B = self._bucket(si.num_decode)
        G = self.graphs.get(B)
        if G is None or not G.fused:
            return False
        if getattr(self.model, "tp_size", 1) > 1:
            return True
        if B in self._filt_failed:
            return True
        if B not in self.graphs_filt:
            try:
                self._capture_filtered(B)
            except Exception as e:  # noqa: BLE001 - e.g. out of memory after the KV pool took HBM
                # (ADVICE r5): this bucket's filtered rows stay on the eager path for good
                logger.warning(f"filtered decode graph for batch {B} not captured ({e}); running it eagerly")
                self._filt_failed.add(B)
                torch.cuda.synchronize(self.device)
                return True
        return False

    def _capture_filtered(self, B: int) -> None:
        """Capture mid-serving: the static inputs still hold the step in flight, so the warm-up and
        capture passes run with every KV slot masked (< 0: no cache write) and no pending-token
        gather -- they must not rewrite live sequences' KV -- and the inputs are restored after."""
        s = self._static
        saved = (s["slots"][:B].clone(), s["src"][:B].clone())
        s["slots"][:B].fill_(-1)
        s["src"][:B].fill_(-1)
        try:
            for _ in range(2):
                self._run_static(B, filtered=True)
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, pool=self.graph_pool):
                out = self._run_static(B, filtered=True)
            self.graphs_filt[B] = _DecodeGraph(g, B, out, False)
        finally:                                  # the step in flight keeps its inputs either way
            s["slots"][:B].copy_(saved[0])
            s["src"][:B].copy_(saved[1])
            torch.cuda.synchronize()

    def _bucket(self, n: int) -> int:
        for b in self.graph_sizes:
            if b >= n:
                return b
        return self.graph_sizes[-1]

    def _graph_decode(self, si: StepInputs) -> List[int]:
        if not self.graphs:
            self.capture_graphs()
        n = si.num_decode
        B = self._bucket(n)
        G = self.graphs[B]
        if G.fused and self._has_filters(si) and B in self.graphs_filt:
            G = self.graphs_filt[B]
        S, W = self.max_decode_batch, self.max_blocks
        self._pinned_i32, self._pinned_f, self._pinned_l = self._pinned_sets[self._pin_flip]
        self._pin_flip ^= 1
        buf = self._pinned_i32.numpy()
        # layout: ids | pos | slots | ctx | bt  (each section sized for the largest bucket)
        buf[0:n] = si.ids
        buf[S:S + n] = si.positions
        buf[2 * S:2 * S + B] = -1
        buf[2 * S:2 * S + n] = si.slots
        buf[3 * S:3 * S + B] = 1
        buf[3 * S:3 * S + n] = si.ctx_d
        bt = buf[4 * S:4 * S + S * W].reshape(S, W)
        bt[:B] = 0
        bt[:n, :si.bt_d.shape[1]] = si.bt_d
        src = buf[self._src_off:self._src_off + S]
        src[:B] = -1
        if si.src is not None:
            src[:n] = si.src
        tk = buf[self._topk_off:self._topk_off + S]
        tk[:B] = 0
        tk[:n] = si.top_k
        f = self._pinned_f.numpy()
        f[:n] = si.temps
        f[S:S + B] = 1.0
        f[S:S + n] = si.top_p
        self._pinned_l.numpy()[:n] = si.seeds
        self._dev_i32.copy_(self._pinned_i32, non_blocking=True)
        s = self._static
        s["f32"].copy_(self._pinned_f, non_blocking=True)
        s["seeds"].copy_(self._pinned_l, non_blocking=True)
        G.graph.replay()
        self.stats["graph_steps"] += 1
        return G.out[:n]
