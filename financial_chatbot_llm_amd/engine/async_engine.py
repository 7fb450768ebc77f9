"""Asyncio front-end for the engine: one background thread owns the GPU and steps continuously.

Every concurrent chat turn (decide call, respond stream) is a request in the SAME continuous
batch.  Submissions and aborts cross into the engine thread through a lock-protected queue; per
request outputs come back to the event loop with ``call_soon_threadsafe``.  The event loop never
blocks on the GPU, so ``/health`` and Kafka polling stay responsive while the engine runs
(the reference blocks its loop on every LLM call).
"""
from __future__ import annotations

import asyncio
import itertools
import os
import sys
import threading
import time
from typing import AsyncIterator, Dict, List, Optional, Sequence as Seq, Tuple

from ..config import EngineConfig
from ..utils.logging import get_logger
from ..utils.metrics import METRICS
from .llm_engine import LLMEngine, StepOutput
from .sequence import SamplingParams

logger = get_logger(__name__)
_rid = itertools.count()


def _deliver(items) -> None:
    for q, o in items:
        q.put_nowait(o)


class AsyncEngine:
    def __init__(self, cfg: Optional[EngineConfig] = None, engine: Optional[LLMEngine] = None, start: bool = True,
                 warmup: bool = True):
        self.engine = engine or LLMEngine(cfg or EngineConfig.from_env())
        if warmup:
            self.engine.warmup()
        self.tokenizer = self.engine.tokenizer
        self._lock = threading.Lock()
        self._wake = threading.Event()
        self._pending: List[Tuple[str, Seq[int], SamplingParams]] = []
        self._aborts: List[str] = []
        self._sinks: Dict[str, Tuple[asyncio.AbstractEventLoop, asyncio.Queue]] = {}
        self._stop = False
        self.error: Optional[BaseException] = None
        self.step_times: List[float] = []
        self._step_started: Optional[float] = None   # perf_counter of the in-flight step
        self.stalled = False
        self.step_timeout_s = float(getattr(self.engine.cfg, "step_timeout_s", 0) or 0)
        # The engine thread shares the GIL with the serving event loop (hundreds of streams).
        # CPython's default 5 ms switch interval lets a busy event loop hold the GIL for up to
        # 5 ms while the engine thread waits to launch the next GPU step; a short interval keeps
        # the GPU fed (PENNY_GIL_SWITCH_MS, 0 = leave the interpreter default).
        sw = float(os.environ.get("PENNY_GIL_SWITCH_MS", "0.5"))
        if sw > 0:
            sys.setswitchinterval(sw / 1e3)
        self._thread = threading.Thread(target=self._loop, name="penny-engine", daemon=True)
        self._stop_evt = threading.Event()
        self._watchdog = threading.Thread(target=self._watch, name="penny-watchdog", daemon=True)
        if start:
            self._thread.start()
            if self.step_timeout_s > 0:
                self._watchdog.start()

    # -- engine thread ---------------------------------------------------------------------
    def _loop(self) -> None:
        eng = self.engine
        if eng.device.type == "cuda":
            import torch
            torch.cuda.set_device(eng.device)
        prof_dir = os.environ.get("PENNY_PYPROFILE")   # host-side cProfile of the engine thread
        prof = None
        if prof_dir:
            import cProfile
            prof = cProfile.Profile()
            prof.enable()
        try:
            self._run_loop(eng)
        finally:
            if prof is not None:
                prof.disable()
                os.makedirs(prof_dir, exist_ok=True)
                prof.dump_stats(os.path.join(prof_dir, f"engine_r{os.environ.get('RANK', '0')}.prof"))

    def _run_loop(self, eng: LLMEngine) -> None:
        while not self._stop:
            with self._lock:
                pending, self._pending = self._pending, []
                aborts, self._aborts = self._aborts, []
            for rid in aborts:
                eng.abort(rid)
            for rid, ids, params in pending:
                try:
                    eng.add_request(rid, ids, params)
                except Exception as e:  # noqa: BLE001
                    self._emit(rid, e)
            if not eng.has_work():
                self._wake.wait(0.05)
                self._wake.clear()
                continue
            try:
                t0 = time.perf_counter()
                self._step_started = t0
                outs = eng.step()
                self._step_started = None
                self.stalled = False
                self.step_times.append(time.perf_counter() - t0)
                if len(self.step_times) > 4096:
                    del self.step_times[:2048]
            except BaseException as e:  # noqa: BLE001 - surface GPU errors to every waiter
                self._step_started = None
                logger.exception("engine step failed")
                self.error = e
                for rid in list(self._sinks):
                    self._emit(rid, e)
                    eng.abort(rid)
                continue
            self._emit_batch(outs)
        eng.stop_followers()

    def _watch(self) -> None:
        """GPU-step watchdog: a step running past ``step_timeout_s`` (a wedged kernel,
        a dead TP peer inside a collective) fails every waiting request with TimeoutError so the
        serving layer emits its error/timeout events instead of hanging, and flags the engine
        unhealthy (``/health`` reports it).  A kernel cannot be cancelled from the host, so the
        requests are failed, not the step; the flag clears if the step ever completes."""
        period = min(1.0, self.step_timeout_s / 4)
        while not self._stop:
            if self._stop_evt.wait(period):
                return
            t0 = self._step_started
            if t0 is None or self.stalled or time.perf_counter() - t0 < self.step_timeout_s:
                continue
            self.stalled = True
            err = TimeoutError(f"engine step exceeded {self.step_timeout_s:.1f}s")
            logger.error(f"watchdog: {err}; failing {len(self._sinks)} waiting request(s)")
            METRICS.inc("engine_step_timeouts")
            for rid in list(self._sinks):
                self._emit(rid, err)

    def _emit_batch(self, outs) -> None:
        """One thread-safe wakeup per event loop per step (not per token): with hundreds of
        streams, per-item call_soon_threadsafe self-pipe writes cost ~1 ms/step and GIL churn."""
        by_loop: Dict = {}
        for o in outs:
            sink = self._sinks.get(o.request_id)
            if sink is not None:
                by_loop.setdefault(sink[0], []).append((sink[1], o))
        for loop, items in by_loop.items():
            try:
                loop.call_soon_threadsafe(_deliver, items)
            except RuntimeError:  # loop closed
                pass

    def _emit(self, rid: str, item) -> None:  # single item (errors, aborts)
        sink = self._sinks.get(rid)
        if sink is None:
            return
        loop, q = sink
        try:
            loop.call_soon_threadsafe(q.put_nowait, item)
        except RuntimeError:  # loop closed
            self._sinks.pop(rid, None)

    # -- public API --------------------------------------------------------------------------
    async def generate(self, prompt_ids: Seq[int], params: SamplingParams,
                       request_id: Optional[str] = None) -> AsyncIterator[StepOutput]:
        rid = request_id or f"req-{next(_rid)}"
        q: asyncio.Queue = asyncio.Queue()
        self._sinks[rid] = (asyncio.get_running_loop(), q)
        with self._lock:
            self._pending.append((rid, list(prompt_ids), params))
        self._wake.set()
        done = False
        try:
            while True:
                item = await q.get()
                if isinstance(item, BaseException):
                    done = True
                    raise item
                done = item.finished
                yield item
                if done:
                    return
        finally:
            self._sinks.pop(rid, None)
            if not done:  # consumer went away mid-stream (timeout / disconnect): free the KV
                with self._lock:
                    self._aborts.append(rid)
                self._wake.set()

    async def generate_all(self, prompt_ids: Seq[int], params: SamplingParams) -> StepOutput:
        last = None
        async for o in self.generate(prompt_ids, params):
            last = o
        return last

    def stats(self) -> Dict[str, float]:
        s = self.engine.stats()
        if self.step_times:
            st = sorted(self.step_times[-512:])
            s["step_p50_ms"] = 1e3 * st[len(st) // 2]
        s["stalled"] = float(self.stalled)
        return s

    def shutdown(self) -> None:
        self._stop = True
        self._stop_evt.set()
        self._wake.set()
        if self._thread.is_alive():
            self._thread.join(timeout=30)
        if self._watchdog.is_alive():
            self._watchdog.join(timeout=5)
