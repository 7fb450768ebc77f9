"""Profiling hooks around the engine (the reference has none).

* ``PENNY_MARKERS=1`` -- roctx ranges (``torch.cuda.nvtx`` is roctx on ROCm builds) around every
  engine step and around the runner's graph-replay / eager-forward launches, so
  ``rocprofv3 --marker-trace --kernel-trace`` attributes each kernel to a serving phase.
* ``PENNY_TORCH_PROFILE=<dir>`` -- ``torch.profiler`` over a window of engine steps
  (``PENNY_TORCH_PROFILE_STEPS=start:stop``, default ``20:30``): CPU + GPU activity with shapes,
  exported as a Chrome trace ``<dir>/engine_rank<r>.json`` per rank.

Both are off by default and cost one env lookup at engine construction.
"""
from __future__ import annotations

import contextlib
import os
from typing import Iterator, Optional

import torch

from .logging import get_logger

logger = get_logger(__name__)


def _markers_on() -> bool:
    return os.environ.get("PENNY_MARKERS") == "1" and torch.cuda.is_available()


_MARKERS = _markers_on()


@contextlib.contextmanager
def marker(name: str) -> Iterator[None]:
    """roctx range ``name`` when PENNY_MARKERS=1, else nothing."""
    if not _MARKERS:
        yield
        return
    torch.cuda.nvtx.range_push(name)
    try:
        yield
    finally:
        torch.cuda.nvtx.range_pop()


def set_markers(on: bool) -> None:
    global _MARKERS
    _MARKERS = bool(on) and torch.cuda.is_available()


class StepProfiler:
    """torch.profiler over engine steps [start, stop) -> Chrome trace (see module doc)."""

    def __init__(self, out_dir: Optional[str] = None, window: Optional[str] = None, rank: int = 0):
        self.out_dir = out_dir if out_dir is not None else os.environ.get("PENNY_TORCH_PROFILE", "")
        window = window or os.environ.get("PENNY_TORCH_PROFILE_STEPS", "20:30")
        a, b = (int(v) for v in window.split(":"))
        if not 0 <= a < b:
            raise ValueError(f"bad profile window {window!r}")
        self.start, self.stop = a, b
        self.rank = rank
        self.step = 0
        self.trace_path: Optional[str] = None
        self._prof = None

    @property
    def enabled(self) -> bool:
        return bool(self.out_dir)

    def on_step(self) -> None:
        """Call once per engine step (before it runs)."""
        if not self.enabled:
            return
        if self.step == self.start:
            acts = [torch.profiler.ProfilerActivity.CPU]
            if torch.cuda.is_available():
                acts.append(torch.profiler.ProfilerActivity.CUDA)
            self._prof = torch.profiler.profile(activities=acts, record_shapes=True)
            self._prof.__enter__()
        elif self.step == self.stop:
            self.finish()
        self.step += 1

    def finish(self) -> Optional[str]:
        if self._prof is None:
            return self.trace_path
        if torch.cuda.is_available():
            torch.cuda.synchronize()
        self._prof.__exit__(None, None, None)
        os.makedirs(self.out_dir, exist_ok=True)
        self.trace_path = os.path.join(self.out_dir, f"engine_rank{self.rank}.json")
        self._prof.export_chrome_trace(self.trace_path)
        self._prof = None
        logger.info(f"torch.profiler trace of engine steps {self.start}:{self.stop} -> {self.trace_path}")
        return self.trace_path
