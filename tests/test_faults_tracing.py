"""Fault injection and tracing (CPU): LWC_FAULT parsing and hooks; the EngineService failure path (a
crashing engine fails every in-flight group, keeps serving the next ones); phase spans and request
latency summaries on /metrics."""
import asyncio

import pytest

from llm_weighted_consensus_amd.utils.faults import FaultInjector, InjectedFault
from llm_weighted_consensus_amd.utils.tracing import STATS, RequestTimer, span


def test_fault_injector_parse_and_hooks():
    f = FaultInjector("worker_crash:3,bad_logprobs")
    assert f.active and f.bad_logprobs
    f.on_step()
    f.on_step()
    with pytest.raises(InjectedFault):
        f.on_step()
    f.on_step()  # only the N-th step crashes
    assert not FaultInjector(None).active and not FaultInjector("").bad_logprobs
    dead = FaultInjector("worker_crash:2+")
    dead.on_step()
    for _ in range(3):
        with pytest.raises(InjectedFault):
            dead.on_step()
    with pytest.raises(ValueError):
        FaultInjector("meteor_strike")


class _Seq:
    def __init__(self, g):
        self.group, self.finished, self.tokens = g, False, []


class _Group:
    def __init__(self, n, cb):
        self.seqs = [_Seq(self) for _ in range(n)]
        self.callback, self.n = cb, n


class FakeEngine:
    """Engine-shaped stub (add_request/has_work/step/abort/fail_all) that emits one token per sequence
    per step and consults the same FaultInjector hooks as LLMEngine.step()."""

    def __init__(self, faults):
        self.faults, self.groups, self.running, self.waiting = faults, [], [], []

    def add_request(self, prompt_ids, params, n=1, callback=None):
        g = _Group(n, callback)
        self.groups.append(g)
        return g

    def has_work(self):
        return any(not s.finished for g in self.groups for s in g.seqs)

    def step(self):
        self.faults.on_step()
        from llm_weighted_consensus_amd.engine.engine import TokenEvent

        for g in self.groups:
            for s in g.seqs:
                if s.finished:
                    continue
                s.tokens.append(7)
                ev = TokenEvent(s, 7, "x", 0.0, [])
                if len(s.tokens) >= 3:
                    s.finished, ev.finished, ev.finish_reason = True, True, "length"
                g.callback(ev)

    def abort(self, g):
        for s in g.seqs:
            s.finished = True

    def fail_all(self, msg):
        out = [g for g in self.groups if any(not s.finished for s in g.seqs)]
        for g in out:
            self.abort(g)
        return out


def test_engine_service_survives_injected_crash():
    from llm_weighted_consensus_amd.engine.service import EngineFailure, EngineService

    eng = FakeEngine(FaultInjector("worker_crash:2"))
    svc = EngineService(eng, "fake")

    async def go():
        loop = asyncio.get_running_loop()
        q1 = asyncio.Queue()
        svc.submit([1, 2], None, 2, loop, q1)
        got = []
        while True:
            ev = await asyncio.wait_for(q1.get(), 10)
            got.append(ev)
            if isinstance(ev, EngineFailure):
                break
        assert "injected worker crash" in got[-1].message
        # the service keeps serving after the failure
        q2 = asyncio.Queue()
        svc.submit([3], None, 1, loop, q2)
        evs = [await asyncio.wait_for(q2.get(), 10) for _ in range(3)]
        assert evs[-1].finished and evs[-1].finish_reason == "length"

    try:
        asyncio.run(go())
    finally:
        svc.close()
    assert svc.failures == 1


def test_spans_and_request_timer_on_metrics():
    with span("unit.test_phase"):
        pass
    t = RequestTimer()
    t.started()
    t.token()
    t.token(4)
    t.finished()
    text = STATS.prometheus()
    assert 'lwc_phase_seconds_count{name="unit_test_phase"}' in text
    for k in ("queue", "ttft", "tpot", "e2e"):
        assert f'lwc_latency_seconds_count{{name="{k}"}}' in text
