"""asyncio bridge to an LLMEngine running in its own thread (one engine per GPU per process).

The HTTP front end is a single asyncio event loop (no shared mutable state across threads except
the engine's lock-protected waiting queue); the engine thread owns the GPU and runs `step()` in a
loop.  Token events are handed back with `loop.call_soon_threadsafe`, batched per engine step.  Abort (client disconnect)
is queued and applied by the engine thread between steps.
"""
from __future__ import annotations

import asyncio
import threading
import time
import traceback
from dataclasses import dataclass
from typing import List, Optional

from .engine import LLMEngine, SequenceGroup, TokenEvent
from .sampling import SamplingParams


@dataclass
class EngineFailure:
    message: str
    kind: str = "error"  # "error" (engine exception) | "deadline" (the request's deadline passed)


class EngineService:
    def __init__(self, engine: LLMEngine, name: str = "local"):
        self.engine = engine
        self.name = name
        self._cv = threading.Condition()
        self._aborts: List[SequenceGroup] = []
        self._stop = False
        self._pending: dict = {}  # event loop -> [(queue, event)] produced by the current step
        self._thread = threading.Thread(target=self._run, name=f"engine-{name}", daemon=True)
        self._thread.start()
        self.failures = 0
        self.last_step_s = 0.0

    # ------------------------------------------------------------------ async API
    def submit(self, prompt_ids, params: SamplingParams, n: int, loop: asyncio.AbstractEventLoop,
               queue: asyncio.Queue, ctx=None) -> SequenceGroup:
        # events are buffered per event loop during an engine step and handed over with ONE thread-safe
        # call per loop per step (a per-token call_soon_threadsafe is a self-pipe write each, and hundreds
        # per step of them compete with the engine thread for the GIL)
        def cb(ev: TokenEvent):
            self._pending.setdefault(loop, []).append((queue, ev))

        kw = {"ctx": ctx} if ctx is not None else {}
        g = self.engine.add_request(prompt_ids, params, n=n, callback=cb, **kw)
        g.loop, g.queue = loop, queue
        with self._cv:
            self._cv.notify()
        return g

    def abort(self, g: SequenceGroup) -> None:
        with self._cv:
            self._aborts.append(g)
            self._cv.notify()

    def close(self) -> None:
        with self._cv:
            self._stop = True
            self._cv.notify()
        self._thread.join(timeout=10)

    @property
    def load(self) -> int:
        e = self.engine
        return len(e.running) + sum(g.n for g in list(e.waiting))

    # ------------------------------------------------------------------ engine thread
    def _run(self) -> None:
        eng = self.engine
        while True:
            with self._cv:
                while not self._stop and not eng.has_work() and not self._aborts:
                    self._cv.wait(timeout=0.5)
                if self._stop:
                    return
                aborts, self._aborts = self._aborts, []
            for g in aborts:
                eng.abort(g)
            for g in (eng.expire() if hasattr(eng, "expire") else ()):  # request deadlines (RequestContext)
                loop, q = getattr(g, "loop", None), getattr(g, "queue", None)
                if loop is not None:
                    loop.call_soon_threadsafe(q.put_nowait, EngineFailure("request deadline exceeded", "deadline"))
            self._flush()  # events an abort produced
            if not eng.has_work():
                continue
            t0 = time.perf_counter()
            try:
                eng.step()
            except Exception as e:  # fail every in-flight group loudly, keep serving
                self.failures += 1
                msg = f"{type(e).__name__}: {e}"
                traceback.print_exc()
                self._flush()  # tokens of the failed step first, then the failures
                for g in eng.fail_all(msg):
                    loop, q = getattr(g, "loop", None), getattr(g, "queue", None)
                    if loop is not None:
                        loop.call_soon_threadsafe(q.put_nowait, EngineFailure(msg))
            self._flush()
            self.last_step_s = time.perf_counter() - t0

    @staticmethod
    def _deliver(batch) -> None:
        for q, ev in batch:
            q.put_nowait(ev)

    def _flush(self) -> None:
        pending, self._pending = self._pending, {}
        for loop, batch in pending.items():
            try:
                loop.call_soon_threadsafe(self._deliver, batch)
            except RuntimeError:  # the client's loop is gone
                pass
