"""Chat client interface + the helpers every backend shares.

Contract (reference src/chat/completions/client.rs:56-79): `create_streaming` either fails before the
first chunk (the awaited call raises a StatusError) or returns an async iterator of
`ChatCompletionChunk`s whose iteration may raise a StatusError mid-stream; `create_unary` folds the
stream with the merge algebra (`EmptyStream` if nothing arrives).
"""
from __future__ import annotations

import abc
from typing import Any, AsyncIterator, Optional

from ..errors import ChatError
from ..schema.chat import ChatCompletion, ChatCompletionChunk, ChatCompletionCreateParams


class ChatClient(abc.ABC):
    @abc.abstractmethod
    async def create_streaming(self, ctx: Any, request: ChatCompletionCreateParams) -> AsyncIterator[ChatCompletionChunk]:
        ...

    async def create_unary(self, ctx: Any, request: ChatCompletionCreateParams) -> ChatCompletion:
        agg: Optional[ChatCompletionChunk] = None
        stream = await self.create_streaming(ctx, request)
        async for chunk in stream:
            if agg is None:
                agg = chunk.clone()
            else:
                agg.push(chunk)
        if agg is None:
            raise ChatError.empty_stream()
        return ChatCompletion.from_chunk(agg)


async def prepend(first, rest: AsyncIterator):
    """StreamOnce(first).chain(rest)."""
    yield first
    async for x in rest:
        yield x


async def probe_first(stream: AsyncIterator):
    """Pull the first item so errors before it surface at call time; returns (first, rest) or raises
    ChatError.empty_stream()."""
    it = stream.__aiter__()
    try:
        first = await it.__anext__()
    except StopAsyncIteration:
        raise ChatError.empty_stream()
    return prepend(first, it)
