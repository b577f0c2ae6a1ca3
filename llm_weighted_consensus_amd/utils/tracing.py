"""Tracing and timing (SURVEY.md §5 "Tracing / profiling"; the reference has none).

* ``span(name)`` — a context manager around an engine phase (schedule / prefill / decode.launch /
  decode.process / embed ...).  It always feeds a cheap in-process aggregator (count, total and max
  seconds per phase, exported on ``/metrics``), and when ``LWC_TRACE=1`` it also pushes a ROCTX range
  (``libroctx64.so`` via ctypes), so ``rocprofv3 --marker-trace`` timelines show the host phases next
  to the kernels.
* ``RequestTimer`` — per-request latency: queue time, time to first token (TTFT), time per output
  token (TPOT), recorded into the same registry as summaries.

No dependency beyond ctypes; when the ROCTX library is missing the ranges are silently skipped (the
aggregator still works), because tracing must never change what the engine computes.
"""
from __future__ import annotations

import ctypes
import os
import threading
import time
from contextlib import contextmanager
from typing import Dict, Optional


class _Roctx:
    def __init__(self):
        self.lib = None
        if os.environ.get("LWC_TRACE") != "1":
            return
        for path in ("libroctx64.so", "/opt/rocm/lib/libroctx64.so"):
            try:
                lib = ctypes.CDLL(path)
                lib.roctxRangePushA.argtypes = [ctypes.c_char_p]
                lib.roctxRangePushA.restype = ctypes.c_int
                lib.roctxRangePop.restype = ctypes.c_int
                self.lib = lib
                break
            except OSError:
                continue

    def push(self, name: str) -> None:
        if self.lib is not None:
            self.lib.roctxRangePushA(name.encode())

    def pop(self) -> None:
        if self.lib is not None:
            self.lib.roctxRangePop()


class Stats:
    """Thread-safe phase aggregator + latency summaries."""

    def __init__(self):
        self._lock = threading.Lock()
        self.phases: Dict[str, list] = {}      # name -> [count, total_s, max_s]
        self.latency: Dict[str, list] = {}     # name -> [count, total_s, max_s]

    def add(self, table: Dict[str, list], name: str, dt: float) -> None:
        with self._lock:
            v = table.get(name)
            if v is None:
                table[name] = [1, dt, dt]
            else:
                v[0] += 1
                v[1] += dt
                if dt > v[2]:
                    v[2] = dt

    def prometheus(self) -> str:
        out = []
        with self._lock:
            for kind, table in (("phase", self.phases), ("latency", self.latency)):
                for name, (n, tot, mx) in sorted(table.items()):
                    key = name.replace(".", "_")
                    out.append(f'lwc_{kind}_seconds_count{{name="{key}"}} {n}')
                    out.append(f'lwc_{kind}_seconds_sum{{name="{key}"}} {tot:.6f}')
                    out.append(f'lwc_{kind}_seconds_max{{name="{key}"}} {mx:.6f}')
        return "\n".join(out) + ("\n" if out else "")

    def snapshot(self) -> dict:
        with self._lock:
            return {"phases": {k: list(v) for k, v in self.phases.items()},
                    "latency": {k: list(v) for k, v in self.latency.items()}}


ROCTX = _Roctx()
STATS = Stats()


@contextmanager
def span(name: str):
    ROCTX.push(name)
    t0 = time.perf_counter()
    try:
        yield
    finally:
        STATS.add(STATS.phases, name, time.perf_counter() - t0)
        ROCTX.pop()


class RequestTimer:
    """Queue / TTFT / TPOT of one request (a sequence group); all times host-side perf_counter."""

    __slots__ = ("t_submit", "t_start", "t_first", "t_last", "tokens", "trace_id")

    def __init__(self):
        self.trace_id = None  # the request context's trace id (context.RequestContext), when given
        self.t_submit = time.perf_counter()
        self.t_start: Optional[float] = None
        self.t_first: Optional[float] = None
        self.t_last: Optional[float] = None
        self.tokens = 0

    def started(self) -> None:
        if self.t_start is None:
            self.t_start = time.perf_counter()
            STATS.add(STATS.latency, "queue", self.t_start - self.t_submit)

    def token(self, n: int = 1) -> None:
        now = time.perf_counter()
        if self.t_first is None:
            self.t_first = now
            STATS.add(STATS.latency, "ttft", now - self.t_submit)
        self.t_last = now
        self.tokens += n

    def finished(self) -> None:
        if self.t_first is not None and self.t_last is not None and self.tokens > 1:
            STATS.add(STATS.latency, "tpot", (self.t_last - self.t_first) / (self.tokens - 1))
        STATS.add(STATS.latency, "e2e", time.perf_counter() - self.t_submit)
