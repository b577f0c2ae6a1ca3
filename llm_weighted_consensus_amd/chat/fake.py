"""FakeChatClient: scripted chat backend for CPU tests and the CPU plumbing config (BASELINE config 1).

A policy maps each request to a list of scripted choices (content, optional per-token logprobs) or
an error to raise before the first chunk / after k chunks — every branch of the reference's voter
handling (src/score/completions/client.rs:711-906) can be exercised without a GPU.
"""
from __future__ import annotations

import asyncio
import re
import time
import uuid
from dataclasses import dataclass
from typing import Callable, List, Optional, Sequence, Tuple

from ..errors import StatusError
from ..context import COALESCE
from ..schema import chat as C
from .base import ChatClient

KEY_LINE = re.compile(r"^- ((?:`[A-T]`)+)$", re.M)
CHOICE_MAP = re.compile(r'^  "((?:`[A-T]`)+)": (.*?),?$', re.M)


@dataclass
class Scripted:
    content: str
    # per generated token: (token text, [(alt text, logprob)])  — None = no logprobs
    logprobs: Optional[List[Tuple[str, List[Tuple[str, float]]]]] = None
    finish_reason: str = "stop"
    tool_call: bool = False
    usage: Optional[Tuple[int, int]] = (10, 3)


@dataclass
class Failure:
    error: StatusError
    after_chunks: int = 0  # 0 = before the first chunk


def select_keys(request: C.ChatCompletionCreateParams) -> List[Tuple[str, str]]:
    """(key, choice text as JSON) from the voter prompt the orchestrator built."""
    last = request.messages[-1]
    text = C.simple_content_text(last.content) if isinstance(last, C.SystemMessage) else ""
    return CHOICE_MAP.findall(text)


_BYTES: dict = {}


def _token_bytes(t: str) -> list:
    """UTF-8 byte list of a token text, cached (read-only lists shared by the chunks, as chat/local.py's
    _token_info)."""
    b = _BYTES.get(t)
    if b is None:
        b = _BYTES[t] = list(t.encode())
    return b


class FakeChatClient(ChatClient):
    def __init__(self, policy: Callable[[C.ChatCompletionCreateParams], Sequence], chunk_chars: int = 3,
                 delay_s: float = 0.0):
        self.policy = policy
        self.chunk_chars = chunk_chars
        self.delay_s = delay_s  # pause before every chunk (slow voters for the failure-isolation tests)
        self.requests: List[C.ChatCompletionCreateParams] = []

    async def create_streaming(self, ctx, request: C.ChatCompletionCreateParams):
        self.requests.append(request)
        cand = ctx.get("candidates") if isinstance(ctx, dict) else None
        first = 0
        if cand is not None:  # a slice of a sharded request (as the local engine client serves it)
            first, cnt, base = int(cand[0]), int(cand[1]), cand[2]
            # the policy scripts the whole request's candidates [0, first + cnt); this slice streams its own
            request = request.model_copy(update={"n": first + cnt,
                                                 "seed": request.seed if request.seed is not None else base})
        plan = self.policy(request)
        if isinstance(plan, Failure) and plan.after_chunks == 0:
            raise plan.error
        if cand is not None and not isinstance(plan, Failure):
            plan = list(plan)[first:first + cnt]
        return self._gen(request, plan, first)

    async def _gen(self, request, plan, first: int = 0):
        cid = f"chatcmpl-fake-{uuid.uuid4().hex[:8]}"
        created = int(time.time())
        fail = plan if isinstance(plan, Failure) else None
        choices: List[Scripted] = [] if fail else list(plan)
        if fail:
            choices = [Scripted("partial output that never finishes")]
        # emit content in pieces, interleaving choices, then finish chunks with usage
        pieces = []
        for i, sc in enumerate(choices):
            toks = sc.logprobs or [(sc.content[k:k + self.chunk_chars], None)
                                   for k in range(0, max(len(sc.content), 1), self.chunk_chars)]
            for t, alts in toks:
                pieces.append((i, t, alts))
        emitted = 0
        if COALESCE.get() and not fail and not any(sc.tool_call for sc in choices) and pieces:
            # a unary request (context.COALESCE): each choice's pieces merged into one chunk, as the local
            # engine client merges a flush's tokens (the fold is the same)
            for i, sc in enumerate(choices):
                mine = [(t, alts) for j, t, alts in pieces if j == i]
                if self.delay_s:
                    await asyncio.sleep(self.delay_s * len(mine))
                lp = None
                if any(a is not None for _, a in mine):
                    tb = _token_bytes  # (cached per token text, as the local client caches per token id)
                    lp = C.Logprobs(content=[C.Logprob.trusted(token=t, bytes=tb(t),
                                                               logprob=float(alts[0][1]) if alts else 0.0,
                                                               top_logprobs=[C.TopLogprob.trusted(
                                                                   token=a, bytes=tb(a), logprob=float(l))
                                                                   for a, l in alts])
                                             for t, alts in mine if alts is not None])
                yield C.ChatCompletionChunk(id=cid, created=created, model=request.model, provider="fake",
                                            choices=[C.StreamChoice(delta=C.Delta(role="assistant",
                                                                                  content="".join(t for t, _ in mine)),
                                                                    index=first + i, logprobs=lp)])
            pieces = []
        for i, t, alts in pieces:
            if self.delay_s:
                await asyncio.sleep(self.delay_s)
            sc = choices[i]
            d = C.Delta(role="assistant")
            if sc.tool_call:
                d.tool_calls = [C.StreamToolCall(index=0, id="call_fake", type="function",
                                                 function=C.StreamToolCallFunction(name="response_key", arguments=t))]
            else:
                d.content = t
            lp = None
            if alts is not None:
                lp = C.Logprobs(content=[C.Logprob(token=t, bytes=list(t.encode()), logprob=alts[0][1] if alts else 0.0,
                                                   top_logprobs=[C.TopLogprob(token=a, bytes=list(a.encode()), logprob=l)
                                                                 for a, l in alts])])
            yield C.ChatCompletionChunk(id=cid, created=created, model=request.model, provider="fake",
                                        choices=[C.StreamChoice(delta=d, index=first + i, logprobs=lp)])
            emitted += 1
            if fail and emitted >= fail.after_chunks:
                raise fail.error
        for i, sc in enumerate(choices):
            u = None
            if sc.usage is not None:
                u = C.Usage(prompt_tokens=sc.usage[0], completion_tokens=sc.usage[1],
                            total_tokens=sc.usage[0] + sc.usage[1], cost=0.001)
                u.with_total_cost()
            yield C.ChatCompletionChunk(id=cid, created=created, model=request.model, provider="fake", usage=u,
                                        choices=[C.StreamChoice(delta=C.Delta(), index=first + i,
                                                                finish_reason="tool_calls" if sc.tool_call
                                                                else sc.finish_reason)])
