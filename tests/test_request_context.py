"""RequestContext (context.py): headers -> trace id / tenant / priority / deadline; the engine admits by
priority and drops requests past their deadline (CPU: the scheduler paths that need no GPU)."""
import time

from llm_weighted_consensus_amd.context import RequestContext


def test_from_headers():
    c = RequestContext.from_headers({"traceparent": "00-abcdef0123456789abcdef0123456789-0011223344556677-01",
                                     "x-priority": "3", "x-timeout-ms": "1500", "x-tenant": "acme"})
    assert c.trace_id == "abcdef0123456789abcdef0123456789" and c.priority == 3 and c.tenant == "acme"
    assert 1.0 < c.remaining() <= 1.5 and not c.expired()
    assert c.expired(time.monotonic() + 2)
    d = RequestContext.from_headers({"x-request-id": "r-1"}, default_timeout_s=None)
    assert d.trace_id == "r-1" and d.deadline is None and d.priority == 0 and d.remaining() is None
    d["seq"] = 7  # layers attach their own fields: it is a dict
    assert d["seq"] == 7 and isinstance(d, dict)


class _Eng:
    """The scheduler state LLMEngine.add_request / expire touch, without a model or a GPU."""

    def __init__(self):
        import threading
        from collections import deque

        self.waiting, self.prefilling, self.swapped, self.running = deque(), [], deque(), []
        self.lock = threading.Lock()
        self._deadlines = 0


def test_engine_priority_order_and_deadline_expiry(monkeypatch):
    from llm_weighted_consensus_amd.engine import engine as E
    from llm_weighted_consensus_amd.engine.sampling import SamplingParams

    eng = _Eng()
    eng.cfg = type("C", (), {"vocab_size": 512})()
    eng.max_model_len = 4096
    eng.tokenizer = None
    monkeypatch.setattr(E.SequenceGroup, "__init__", lambda self, engine, p, params, n, cb: (
        setattr(self, "id", next(E.SequenceGroup._ids)), setattr(self, "engine", engine), setattr(self, "params", params),
        setattr(self, "seqs", [type("S", (), {"finished": False, "finish_reason": None})() for _ in range(n)]),
        setattr(self, "timer", type("T", (), {})()), setattr(self, "prefilled", None), setattr(self, "priority", 0),
        setattr(self, "deadline", None), setattr(self, "trace_id", None), setattr(self, "n", n)) and None)
    monkeypatch.setattr(E.SequenceGroup, "finished", property(lambda self: all(s.finished for s in self.seqs)))
    add = E.LLMEngine.add_request
    sp = SamplingParams(max_tokens=4)
    now = time.monotonic()
    a = add(eng, [1, 2], sp, ctx=RequestContext(priority=0))
    b = add(eng, [1, 2], sp, ctx=RequestContext(priority=5, deadline=now - 1))
    c = add(eng, [1, 2], sp, ctx=RequestContext(priority=5))
    d = add(eng, [1, 2], sp, ctx=RequestContext(priority=1))
    assert list(eng.waiting) == [b, c, d, a]  # higher priority first, FIFO within a priority
    gone = E.LLMEngine.expire(eng, now)
    assert gone == [b] and list(eng.waiting) == [c, d, a]
    assert all(s.finished and s.finish_reason == "deadline" for s in b.seqs)
