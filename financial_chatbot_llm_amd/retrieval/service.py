"""Micro-batched retrieval service: embed (R2) + filtered top-k (R3) for concurrent turns.

The reference embeds and searches once per tool call over HTTPS (``tools/qdrant_tool.py:136-153``).
Here concurrent tool calls that arrive within ``window_s`` are coalesced into ONE encoder
forward and ONE filtered-top-k launch, executed off the event loop on a dedicated HIP stream so
they overlap the LLM engine's own stream.
"""
from __future__ import annotations

import asyncio
import threading
from typing import List, Optional, Sequence, Tuple

from ..utils.logging import get_logger
from ..utils.metrics import METRICS, now
from ..utils.profiling import marker
from .store import Hit

logger = get_logger(__name__)


class RetrievalService:
    def __init__(self, embedder, store, max_batch: int = 64, window_s: float = 0.002):
        self.embedder, self.store = embedder, store
        self.max_batch, self.window_s = max_batch, window_s
        self._pending: List[Tuple[str, str, Optional[int], int, asyncio.Future]] = []
        self._flush_task: Optional[asyncio.Task] = None
        self._lock = threading.Lock()
        self._stream = None

    # -- synchronous core --------------------------------------------------------------
    def run_batch(self, queries: Sequence[str], user_ids: Sequence[str],
                  date_gte: Sequence[Optional[int]], limits: Sequence[int]) -> List[List[Hit]]:
        with self._lock, marker("retrieval.batch"):
            t0 = now()
            ctx = self._stream_ctx()
            with ctx:
                q = self.embedder.embed(list(queries))
                hits = self.store.search_batch(q, list(user_ids), list(date_gte), list(limits))
            METRICS.inc("retrieval_queries_total", len(queries))
            METRICS.inc("retrieval_batches_total")
            METRICS.set_gauge("retrieval_last_batch_s", now() - t0)
            return hits

    def _stream_ctx(self):
        import contextlib
        dev = getattr(self.store, "device", None)
        if dev is None or getattr(dev, "type", "cpu") != "cuda":
            return contextlib.nullcontext()
        import torch
        if self._stream is None:
            self._stream = torch.cuda.Stream(device=dev)
        return torch.cuda.stream(self._stream)

    def search_sync(self, query: str, user_id: str, date_gte: Optional[int], limit: int) -> List[Hit]:
        return self.run_batch([query], [user_id], [date_gte], [limit])[0]

    # -- async micro-batching --------------------------------------------------------------
    async def search(self, query: str, user_id: str, date_gte: Optional[int], limit: int) -> List[Hit]:
        loop = asyncio.get_running_loop()
        fut: asyncio.Future = loop.create_future()
        self._pending.append((query, user_id, date_gte, limit, fut))
        if len(self._pending) >= self.max_batch:
            self._kick(loop, 0.0)
        elif self._flush_task is None:
            self._kick(loop, self.window_s)
        return await fut

    def _kick(self, loop, delay: float) -> None:
        batch, self._pending = self._pending, []
        if self._flush_task is not None and delay > 0:
            self._pending = batch
            return
        self._flush_task = loop.create_task(self._flush(batch, delay))

    async def _flush(self, batch, delay: float) -> None:
        try:
            if delay > 0:
                await asyncio.sleep(delay)
                batch = batch + self._pending
                self._pending = []
            self._flush_task = None
            if not batch:
                return
            qs, us, ds, ks, futs = zip(*batch)
            try:
                res = await asyncio.to_thread(self.run_batch, qs, us, ds, ks)
            except Exception as e:  # noqa: BLE001
                for f in futs:
                    if not f.done():
                        f.set_exception(e)
                return
            for f, r in zip(futs, res):
                if not f.done():
                    f.set_result(r)
        finally:
            if self._flush_task is not None and self._flush_task.done():
                self._flush_task = None
            if self._pending and self._flush_task is None:
                self._kick(asyncio.get_running_loop(), self.window_s)
