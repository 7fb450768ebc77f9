"""Engine-core process: the GPU step loop in its own interpreter, off the serving GIL.

``AsyncEngine`` runs ``LLMEngine.step()`` on a thread of the serving process, so the engine's
host work (schedule, input packing, token bookkeeping) shares one GIL with the event loop that
detokenises, renders and produces every streamed chunk.  Measured on MI355X (128 conversations,
``PENNY_PYPROFILE`` cProfiles + a rocprofv3 kernel trace): the two together need more host time
per decode step than the 7.6 ms the GPU needs, so the next step's inputs reach the device ~0.9 ms
after the previous step drained -- ~10 % of the serving phase with the GPU idle.

``ProcessAsyncEngine`` keeps the ``AsyncEngine`` API (``generate`` / ``generate_all`` / ``stats``
/ ``shutdown`` / ``tokenizer``) but spawns the engine core as a child process that owns the GPU
step loop (one process per GPU stays the deployment model: the child is this rank's GPU
worker).  Two one-way pipes connect them:

* parent -> child: ``("add", rid, prompt_ids, params)``, ``("abort", rid)``, ``("stats",)``,
  ``("stop",)`` -- drained by the child between steps, never waited for inside a step;
* child -> parent: one message per engine step, ``("out", [(rid, new_ids, finished, reason)...])``
  (a few KB at B=128), plus ``("ready", info)``, ``("stats", dict)``, ``("error", rid|None, text)``.

A reader thread in the parent blocks in ``recv`` (GIL released) and hands each step's outputs to
the event loop with ONE ``call_soon_threadsafe`` per loop, exactly as ``AsyncEngine`` does.
Tensor parallelism keeps the in-process ``AsyncEngine`` (its TP peers are the rank processes).
"""
from __future__ import annotations

import asyncio
import itertools
import multiprocessing as mp
import os
import threading
import time
from dataclasses import dataclass, field
from typing import AsyncIterator, Dict, List, Optional, Sequence as Seq, Tuple

from ..config import EngineConfig
from ..utils.logging import get_logger
from .llm_engine import StepOutput
from .sequence import SamplingParams

logger = get_logger(__name__)
_rid = itertools.count()


@dataclass
class RemoteSeq:
    """Parent-side stand-in for the child's ``Sequence``: the tokens streamed so far."""
    output_ids: List[int] = field(default_factory=list)
    finish_reason: Optional[str] = None


def _engine_main(cfg: EngineConfig, device_index: Optional[int], req_conn, out_conn, warmup: bool) -> None:
    """Child process: build the engine on this rank's GPU and serve the two pipes."""
    import torch

    from .llm_engine import LLMEngine

    if device_index is not None and torch.cuda.is_available():
        torch.cuda.set_device(device_index)
    try:
        eng = LLMEngine(cfg)
        if warmup:
            eng.warmup()
    except BaseException as e:  # noqa: BLE001 - report start-up failures to the parent
        out_conn.send(("error", None, f"{type(e).__name__}: {e}"))
        return
    out_conn.send(("ready", {"model": eng.model.cfg.name}))
    step_times: List[float] = []
    prof = None
    if os.environ.get("PENNY_PYPROFILE"):
        import cProfile
        prof = cProfile.Profile()
        prof.enable()
    stop = False
    try:
        while not stop:
            # drain control messages between steps; block (50 ms) only when there is nothing to step
            timeout = 0 if eng.has_work() else 0.05
            while not stop and req_conn.poll(timeout):
                timeout = 0
                msg = req_conn.recv()
                kind = msg[0]
                if kind == "add":
                    _, rid, ids, params = msg
                    try:
                        eng.add_request(rid, ids, params)
                    except Exception as e:  # noqa: BLE001
                        out_conn.send(("error", rid, f"{type(e).__name__}: {e}"))
                elif kind == "abort":
                    eng.abort(msg[1])
                elif kind == "stats":
                    s = eng.stats()
                    if step_times:
                        st = sorted(step_times[-512:])
                        s["step_p50_ms"] = 1e3 * st[len(st) // 2]
                    s["stalled"] = 0.0
                    out_conn.send(("stats", s))
                elif kind == "stop":
                    stop = True
            if stop or not eng.has_work():
                continue
            t0 = time.perf_counter()
            try:
                outs = eng.step()
            except BaseException as e:  # noqa: BLE001 - surface GPU errors to every waiter
                logger.exception("engine step failed")
                out_conn.send(("error", None, f"{type(e).__name__}: {e}"))
                for rid in list(eng.requests):
                    eng.abort(rid)
                continue
            step_times.append(time.perf_counter() - t0)
            if len(step_times) > 4096:
                del step_times[:2048]
            if outs:
                out_conn.send(("out", [(o.request_id, o.new_token_ids, o.finished, o.finish_reason) for o in outs]))
    finally:
        if prof is not None:
            prof.disable()
            os.makedirs(os.environ["PENNY_PYPROFILE"], exist_ok=True)
            prof.dump_stats(os.path.join(os.environ["PENNY_PYPROFILE"],
                                         f"engine_proc_r{os.environ.get('RANK', '0')}.prof"))
        eng.stop_followers()
        out_conn.send(("stopped", None))


def _deliver(items) -> None:
    for q, o in items:
        q.put_nowait(o)


class ProcessAsyncEngine:
    """``AsyncEngine`` API over an engine-core child process (see module docstring)."""

    def __init__(self, cfg: EngineConfig, device_index: Optional[int] = None, warmup: bool = True,
                 start_timeout_s: float = 900.0):
        if cfg.tp_size != 1:
            raise ValueError("ProcessAsyncEngine serves TP=1 replicas; use AsyncEngine under tensor parallelism")
        from ..models.configs import get_model_config
        from .tokenizer import load_tokenizer

        self.cfg = cfg
        self.tokenizer = load_tokenizer(cfg.tokenizer, get_model_config(cfg.model).vocab_size)
        ctx = mp.get_context("spawn")   # a fresh interpreter: never fork a process that holds a GPU context
        req_r, self._req_w = ctx.Pipe(duplex=False)
        self._out_r, out_w = ctx.Pipe(duplex=False)
        self._proc = ctx.Process(target=_engine_main, args=(cfg, device_index, req_r, out_w, warmup),
                                 name="penny-engine-core", daemon=True)
        self._proc.start()
        req_r.close()
        out_w.close()
        self._send_lock = threading.Lock()
        self._sinks: Dict[str, Tuple[asyncio.AbstractEventLoop, asyncio.Queue]] = {}
        self._seqs: Dict[str, RemoteSeq] = {}
        self._stats_evt = threading.Event()
        self._stats: Dict[str, float] = {}
        self.error: Optional[BaseException] = None
        self._closed = False
        t0 = time.perf_counter()
        while True:   # wait for the child's engine (weights, KV pool, graph capture)
            if self._out_r.poll(1.0):
                msg = self._out_r.recv()
                if msg[0] == "ready":
                    break
                if msg[0] == "error":
                    self._proc.join(timeout=10)
                    raise RuntimeError(f"engine process failed to start: {msg[2]}")
            elif not self._proc.is_alive():
                raise RuntimeError(f"engine process exited during start-up (code {self._proc.exitcode})")
            if time.perf_counter() - t0 > start_timeout_s:
                self._proc.kill()
                raise TimeoutError("engine process start-up timed out")
        self._reader = threading.Thread(target=self._read, name="penny-engine-reader", daemon=True)
        self._reader.start()

    @property
    def stalled(self) -> bool:
        return not self._closed and not self._proc.is_alive()

    # -- child -> parent ------------------------------------------------------------------------
    def _read(self) -> None:
        while True:
            try:
                msg = self._out_r.recv()
            except (EOFError, OSError):
                if not self._closed:
                    self._fail_all(RuntimeError(f"engine process died (code {self._proc.exitcode})"))
                return
            kind = msg[0]
            if kind == "out":
                by_loop: Dict = {}
                for rid, new_ids, finished, reason in msg[1]:
                    sink = self._sinks.get(rid)
                    if sink is None:
                        continue
                    seq = self._seqs.get(rid)
                    if seq is not None:
                        seq.output_ids.extend(new_ids)
                        if finished:
                            seq.finish_reason = reason
                    by_loop.setdefault(sink[0], []).append((sink[1], StepOutput(rid, new_ids, finished, reason, seq)))
                for loop, items in by_loop.items():
                    try:
                        loop.call_soon_threadsafe(_deliver, items)
                    except RuntimeError:
                        pass
            elif kind == "stats":
                self._stats = msg[1]
                self._stats_evt.set()
            elif kind == "error":
                err = RuntimeError(msg[2])
                if msg[1] is None:
                    self.error = err
                    self._fail_all(err)
                else:
                    self._emit(msg[1], err)
            elif kind == "stopped":
                return

    def _emit(self, rid: str, item) -> None:
        sink = self._sinks.get(rid)
        if sink is None:
            return
        try:
            sink[0].call_soon_threadsafe(sink[1].put_nowait, item)
        except RuntimeError:
            self._sinks.pop(rid, None)

    def _fail_all(self, err: BaseException) -> None:
        for rid in list(self._sinks):
            self._emit(rid, err)

    def _send(self, msg) -> None:
        with self._send_lock:
            self._req_w.send(msg)

    # -- public API (same as AsyncEngine) -------------------------------------------------------
    async def generate(self, prompt_ids: Seq[int], params: SamplingParams,
                       request_id: Optional[str] = None) -> AsyncIterator[StepOutput]:
        rid = request_id or f"preq-{next(_rid)}"
        q: asyncio.Queue = asyncio.Queue()
        self._sinks[rid] = (asyncio.get_running_loop(), q)
        self._seqs[rid] = RemoteSeq()
        self._send(("add", rid, list(prompt_ids), params))
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
            self._seqs.pop(rid, None)
            if not done and not self._closed:   # consumer went away mid-stream: free the KV
                self._send(("abort", rid))

    async def generate_all(self, prompt_ids: Seq[int], params: SamplingParams) -> StepOutput:
        last = None
        async for o in self.generate(prompt_ids, params):
            last = o
        return last

    def stats(self, timeout_s: float = 30.0) -> Dict[str, float]:
        self._stats_evt.clear()
        self._send(("stats",))
        if not self._stats_evt.wait(timeout_s):
            return {"stalled": 1.0}
        s = dict(self._stats)
        s["engine_process"] = 1.0
        return s

    def shutdown(self, timeout_s: float = 30.0) -> None:
        if self._closed:
            return
        try:
            self._send(("stop",))
        except (BrokenPipeError, OSError):
            pass
        self._reader.join(timeout=timeout_s)
        self._closed = True
        self._proc.join(timeout=timeout_s)
        if self._proc.is_alive():
            self._proc.kill()
            self._proc.join(timeout=5)
