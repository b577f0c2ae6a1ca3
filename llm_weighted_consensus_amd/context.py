"""Per-request context that flows from the HTTP layer down to the engine scheduler.

The reference threads a generic ``CTX`` through every trait (``chat::completions::Client<CTX>``,
``CtxHandler::handle`` rewriting the API bases per request: src/chat/completions/client.rs:25-32, 56-79;
the OSS binary passes ``()``: src/main.rs:152,175,197,220).  Here the context carries what a serving
deployment needs per request (SURVEY §1 [NEW]):

* ``trace_id``  — ``traceparent`` / ``x-request-id`` header or a fresh id; tags the engine's spans and
  timers and is echoed back in the ``x-request-id`` response header;
* ``tenant``    — ``x-tenant`` header (BYOK / tenant routing hook, the reference's ``CtxHandler``);
* ``priority``  — ``x-priority`` header, higher first: the engine admits waiting requests by priority,
  FIFO within a priority;
* ``deadline``  — ``x-timeout-ms`` header (absolute ``time.monotonic()`` seconds): the engine drops a
  request still waiting, or aborts one still generating, once it has passed, and the chat client ends
  the stream with a timeout error.

It is a ``dict`` so that layers can attach their own fields (the voter-sharded score client adds its
request number and seeds) and so code written against a plain dict context keeps working.
"""
from __future__ import annotations

import contextvars
import time
import uuid
from typing import Any, Mapping, Optional

# Set while a UNARY request is served (score/orchestrator.py create_unary; asyncio tasks inherit it): a
# response that is the fold of a chunk stream does not need one chunk per token.  The voter streams then
# merge each voter's output and the local chat clients emit merged chunks (a flush at the first tokens, at
# the end, and at least every COALESCE_FLUSH_S, so the first-chunk / other-chunk timeouts keep their meaning);
# chunk push is associative, so the folded response is the same.
COALESCE: contextvars.ContextVar = contextvars.ContextVar("lwc_coalesce", default=False)
COALESCE_FLUSH_S = 1.0


class RequestContext(dict):
    def __init__(self, trace_id: Optional[str] = None, tenant: Optional[str] = None, priority: int = 0,
                 deadline: Optional[float] = None, **extra: Any):
        super().__init__(extra)
        self["trace_id"] = trace_id or uuid.uuid4().hex
        self["tenant"] = tenant
        self["priority"] = int(priority)
        self["deadline"] = deadline

    @property
    def trace_id(self) -> str:
        return self["trace_id"]

    @property
    def tenant(self) -> Optional[str]:
        return self["tenant"]

    @property
    def priority(self) -> int:
        return self["priority"]

    @property
    def deadline(self) -> Optional[float]:
        return self["deadline"]

    def remaining(self) -> Optional[float]:
        """Seconds left before the deadline (None: no deadline)."""
        return None if self.deadline is None else self.deadline - time.monotonic()

    def expired(self, now: Optional[float] = None) -> bool:
        return self.deadline is not None and (time.monotonic() if now is None else now) >= self.deadline

    @classmethod
    def from_headers(cls, headers: Mapping[str, str], default_timeout_s: Optional[float] = None) -> "RequestContext":
        """Build the context of an HTTP request (header names are case-insensitive in Starlette)."""
        trace = headers.get("x-request-id")
        tp = headers.get("traceparent")
        if not trace and tp:
            parts = tp.split("-")  # W3C traceparent: version-traceid-parentid-flags
            trace = parts[1] if len(parts) >= 2 else tp
        try:
            prio = int(headers.get("x-priority", "0"))
        except ValueError:
            prio = 0
        timeout = default_timeout_s
        if headers.get("x-timeout-ms"):
            try:
                timeout = float(headers["x-timeout-ms"]) / 1000.0
            except ValueError:
                pass
        deadline = time.monotonic() + timeout if timeout is not None and timeout > 0 else None
        return cls(trace_id=trace, tenant=headers.get("x-tenant"), priority=prio, deadline=deadline)


def priority_of(ctx: Any) -> int:
    return int(ctx.get("priority", 0) or 0) if isinstance(ctx, dict) else 0


def deadline_of(ctx: Any) -> Optional[float]:
    return ctx.get("deadline") if isinstance(ctx, dict) else None


def trace_of(ctx: Any) -> Optional[str]:
    return ctx.get("trace_id") if isinstance(ctx, dict) else None
