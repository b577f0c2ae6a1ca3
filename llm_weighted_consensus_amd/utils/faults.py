"""Fault injection for the local engine (SURVEY.md §5 "Failure detection / recovery / fault injection").

``LWC_FAULT`` is a comma-separated list of ``kind[:arg]``:

  worker_crash:N   the engine's N-th step raises (default N=1; "N+" = that step and every later one,
                   a dead worker) -> EngineService fails every in-flight
                   group; each affected voter becomes an error choice, all voters failing gives the
                   reference's AllVotesFailed status unification (src/score/completions/client.rs:385-409)
  slow_decode:MS   every step sleeps MS milliseconds (exercises the first/other-chunk timeouts,
                   src/main.rs:17-20)
  bad_logprobs     token logprobs are replaced by NaN (the vote extractor must fall back to one-hot)
  oom:N            the N-th admitted request raises torch.cuda.OutOfMemoryError at admission

The injector is consulted at fixed hooks only; with LWC_FAULT unset every hook is a no-op attribute
check, so production paths pay nothing.
"""
from __future__ import annotations

import os
import time
from typing import Dict, Optional


class InjectedFault(RuntimeError):
    pass


class FaultInjector:
    def __init__(self, spec: Optional[str] = None):
        self.spec: Dict[str, Optional[str]] = {}
        for part in (spec or "").split(","):
            part = part.strip()
            if not part:
                continue
            kind, _, arg = part.partition(":")
            if kind not in ("worker_crash", "slow_decode", "bad_logprobs", "oom"):
                raise ValueError(f"unknown LWC_FAULT kind {kind!r}")
            self.spec[kind] = arg or None
        self.active = bool(self.spec)
        self.steps = 0
        self.admitted = 0

    @classmethod
    def from_env(cls) -> "FaultInjector":
        return cls(os.environ.get("LWC_FAULT"))

    def on_step(self) -> None:
        if not self.active:
            return
        self.steps += 1
        if "slow_decode" in self.spec:
            time.sleep(float(self.spec["slow_decode"] or 100) / 1000.0)
        if "worker_crash" in self.spec:
            arg = self.spec["worker_crash"] or "1"
            n = int(arg.rstrip("+"))
            if self.steps == n or (arg.endswith("+") and self.steps >= n):
                raise InjectedFault(f"injected worker crash at step {self.steps}")

    def on_admit(self) -> None:
        if not self.active or "oom" not in self.spec:
            return
        self.admitted += 1
        if self.admitted == int(self.spec["oom"] or 1):
            import torch

            raise torch.cuda.OutOfMemoryError("injected out-of-memory at admission")

    @property
    def bad_logprobs(self) -> bool:
        return self.active and "bad_logprobs" in self.spec
