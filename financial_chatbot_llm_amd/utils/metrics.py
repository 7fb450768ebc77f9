"""Serving metrics and per-request stage tracing.

The reference has logging only.  Here every chat turn carries a :class:`TurnTrace` with
monotonic timestamps for each stage (receive, mongo, decide prefill/decode, embed, search,
respond TTFT, complete, save) and a process-wide :class:`MetricsRegistry` aggregates them
into turns/s, TTFT p50/p99, ITL and retrieval latency.  ``render_prometheus()`` backs the
``/metrics`` endpoint without requiring prometheus_client at import time.
"""
from __future__ import annotations

import threading
import time
from collections import defaultdict, deque
from dataclasses import dataclass, field
from typing import Deque, Dict, List, Optional


def now() -> float:
    return time.perf_counter()


@dataclass
class TurnTrace:
    conversation_id: str = ""
    t_receive: float = field(default_factory=now)
    stages: Dict[str, float] = field(default_factory=dict)
    t_first_chunk: Optional[float] = None
    t_complete: Optional[float] = None
    n_chunks: int = 0
    chunk_times: List[float] = field(default_factory=list)
    retrieved: int = 0
    tools_ok: int = 0            # non-retrieval tool calls that succeeded (plots rendered)
    tools_failed: int = 0
    error: bool = False

    def mark(self, stage: str) -> None:
        self.stages[stage] = now()

    def on_chunk(self) -> None:
        t = now()
        if self.t_first_chunk is None:
            self.t_first_chunk = t
        self.chunk_times.append(t)
        self.n_chunks += 1

    @property
    def ttft(self) -> Optional[float]:
        return None if self.t_first_chunk is None else self.t_first_chunk - self.t_receive

    @property
    def latency(self) -> Optional[float]:
        return None if self.t_complete is None else self.t_complete - self.t_receive

    def itls(self) -> List[float]:
        c = self.chunk_times
        return [b - a for a, b in zip(c, c[1:])]


def percentile(xs: List[float], p: float) -> Optional[float]:
    if not xs:
        return None
    s = sorted(xs)
    k = (len(s) - 1) * p / 100.0
    lo = int(k)
    hi = min(lo + 1, len(s) - 1)
    return s[lo] + (s[hi] - s[lo]) * (k - lo)


class MetricsRegistry:
    """Thread-safe rolling aggregates; the engine thread and the event loop both write."""

    def __init__(self, window: int = 4096):
        self._lock = threading.Lock()
        self._traces: Deque[TurnTrace] = deque(maxlen=window)
        self.counters: Dict[str, float] = defaultdict(float)
        self.gauges: Dict[str, float] = {}
        self._t0 = now()

    def record_turn(self, tr: TurnTrace) -> None:
        with self._lock:
            self._traces.append(tr)
            self.counters["turns_total"] += 1
            if tr.error:
                self.counters["turn_errors_total"] += 1

    def inc(self, name: str, v: float = 1.0) -> None:
        with self._lock:
            self.counters[name] += v

    def set_gauge(self, name: str, v: float) -> None:
        with self._lock:
            self.gauges[name] = v

    def snapshot(self) -> Dict[str, Optional[float]]:
        with self._lock:
            traces = list(self._traces)
            counters = dict(self.counters)
            gauges = dict(self.gauges)
        ttfts = [t.ttft for t in traces if t.ttft is not None]
        lats = [t.latency for t in traces if t.latency is not None]
        itl = [x for t in traces for x in t.itls()]
        # decide_done -> retrieval_done: embed + filtered top-k (+ tool execution), marked by the worker
        ret = [t.stages["retrieval_done"] - t.stages["decide_done"] for t in traces
               if "retrieval_done" in t.stages and "decide_done" in t.stages]
        decide = [t.stages["decide_done"] - t.t_receive for t in traces if "decide_done" in t.stages]
        done = [t.t_complete for t in traces if t.t_complete is not None]
        span = (max(done) - min(t.t_receive for t in traces)) if done else 0.0
        out: Dict[str, Optional[float]] = {
            "turns_per_s": (len(done) / span) if span > 0 else None,
            "ttft_p50_s": percentile(ttfts, 50), "ttft_p99_s": percentile(ttfts, 99),
            "latency_p50_s": percentile(lats, 50), "itl_p50_s": percentile(itl, 50),
            "retrieval_p50_s": percentile(ret, 50), "decide_p50_s": percentile(decide, 50),
        }
        out.update(counters)
        out.update(gauges)
        return out

    def render_prometheus(self) -> str:
        lines = []
        for k, v in sorted(self.snapshot().items()):
            if v is None:
                continue
            lines.append(f"penny_{k} {float(v):.6g}")
        return "\n".join(lines) + "\n"


METRICS = MetricsRegistry()
