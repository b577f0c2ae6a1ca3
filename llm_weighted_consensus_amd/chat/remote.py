"""RemoteChatClient: OpenAI-compatible upstream providers over HTTP/SSE (optional fallback tier).

Same semantics as the reference DefaultClient (src/chat/completions/client.rs:193-434):
  * archive references resolved first; a CtxHandler may rewrite the api-base list per request;
  * the request is forced to `stream: true` (adding `stream_options.include_usage` if the caller was
    unary);
  * attempts = [(base, model) for base] + [(base, m) for m in models for base] — fallback models use the
    ctx-rewritten bases (the reference used the unrewritten list: SURVEY §7.4 fix);
  * each attempt probes the FIRST chunk; on error/empty the next attempt runs; the whole list is
    retried with exponential backoff (100 ms initial, x1.5, ±50 % jitter, 1 s cap, 40 s budget) using a
    per-request clock;
  * SSE loop with first-chunk / other-chunk timeouts, `[DONE]`, comments and empty events skipped,
    chunk-or-provider-error decode, `BadStatus{code, body}` capture.
"""
from __future__ import annotations

import asyncio
import json
import random
import time
from dataclasses import dataclass
from typing import Any, List, Optional

from ..errors import ChatError, CtxError, StatusError
from ..schema import chat as C
from .base import ChatClient, prepend


@dataclass
class ApiBase:
    api_base: str
    api_key: str


@dataclass
class Backoff:
    initial_interval: float = 0.1
    randomization_factor: float = 0.5
    multiplier: float = 1.5
    max_interval: float = 1.0
    max_elapsed: float = 40.0

    def intervals(self):
        cur = self.initial_interval
        while True:
            d = cur * self.randomization_factor
            yield random.uniform(cur - d, cur + d)
            cur = min(cur * self.multiplier, self.max_interval)


class NoOpCtxHandler:
    async def handle(self, ctx, api_bases: List[ApiBase]) -> List[ApiBase]:
        return api_bases


class RemoteChatClient(ChatClient):
    def __init__(self, api_bases: List[ApiBase], backoff: Optional[Backoff] = None, user_agent: Optional[str] = None,
                 x_title: Optional[str] = None, referer: Optional[str] = None, first_chunk_timeout: float = 10.0,
                 other_chunk_timeout: float = 60.0, ctx_handler=None, archive=None, http_client=None):
        self.api_bases = api_bases
        self.backoff = backoff or Backoff()
        self.user_agent, self.x_title, self.referer = user_agent, x_title, referer
        self.first_chunk_timeout, self.other_chunk_timeout = first_chunk_timeout, other_chunk_timeout
        self.ctx_handler = ctx_handler or NoOpCtxHandler()
        self.archive = archive
        self._http = http_client

    def _client(self):
        if self._http is None:
            import httpx

            self._http = httpx.AsyncClient(timeout=None, http2=False)
        return self._http

    async def create_streaming(self, ctx, request: C.ChatCompletionCreateParams):
        try:
            bases = await self.ctx_handler.handle(ctx, list(self.api_bases))
        except StatusError as e:
            raise CtxError(e.to_response_error())
        request = request.model_copy()
        if self.archive is not None:
            from ..archive.resolve import fetch_completions_from_messages, replace_completion_messages

            try:
                comps = await fetch_completions_from_messages(self.archive, ctx, request.messages)
            except StatusError as e:
                raise ChatError(e.status(), e.message())
            request.messages = list(request.messages)
            replace_completion_messages(comps, request.messages)
        if not request.stream:
            request.stream_options = C.StreamOptions(include_usage=True)
        request.stream = True
        attempts = [(b, request.model) for b in bases]
        for m in request.models or []:
            attempts += [(b, m) for b in bases]
        request.models = None
        t0 = time.monotonic()
        last_err: Optional[StatusError] = None
        for delay in self.backoff.intervals():
            for base, model in attempts:
                req = request.model_copy()
                req.model = model
                stream = self._events(base, req)
                try:
                    first = await stream.__anext__()
                    return prepend(first, stream)
                except StopAsyncIteration:
                    last_err = ChatError.empty_stream()
                except StatusError as e:
                    last_err = e
            if time.monotonic() - t0 + delay > self.backoff.max_elapsed:
                break
            await asyncio.sleep(delay)
        raise last_err or ChatError.empty_stream()

    async def _events(self, base: ApiBase, req: C.ChatCompletionCreateParams):
        headers = {"authorization": f"Bearer {base.api_key}", "content-type": "application/json",
                   "accept": "text/event-stream"}
        if self.user_agent:
            headers["user-agent"] = self.user_agent
        if self.x_title:
            headers["x-title"] = self.x_title
        if self.referer:
            headers["referer"] = self.referer
            headers["http-referer"] = self.referer
        body = req.to_json()
        client = self._client()
        try:
            async with client.stream("POST", f"{base.api_base}/chat/completions", content=body.encode(),
                                     headers=headers) as resp:
                if resp.status_code >= 400:
                    raw = (await resp.aread()).decode("utf-8", "replace")
                    try:
                        b = json.loads(raw)
                    except Exception:
                        b = raw
                    raise ChatError.bad_status(resp.status_code, b)
                first = True
                lines = resp.aiter_lines()
                data_buf: List[str] = []
                while True:
                    try:
                        line = await asyncio.wait_for(lines.__anext__(),
                                                      self.first_chunk_timeout if first else self.other_chunk_timeout)
                    except StopAsyncIteration:
                        return
                    except asyncio.TimeoutError:
                        raise ChatError.stream_timeout()
                    if line.startswith(":"):
                        continue
                    if line.startswith("data:"):
                        data_buf.append(line[5:].lstrip(" "))
                        continue
                    if line != "" or not data_buf:
                        continue
                    data, data_buf = "\n".join(data_buf), []
                    first = False
                    if data == "[DONE]":
                        return
                    if data.startswith(":") or data == "":
                        continue
                    try:
                        obj = json.loads(data)
                    except Exception as e:
                        raise ChatError.deserialization(str(e))
                    try:
                        chunk = C.ChatCompletionChunk.model_validate(obj)
                    except Exception as e:
                        err = obj.get("error") if isinstance(obj, dict) else None
                        if isinstance(err, dict):
                            raise ChatError.provider(err.get("code"), err.get("message"), err.get("metadata"))
                        raise ChatError.deserialization(str(e))
                    chunk.with_total_cost()
                    yield chunk
        except StatusError:
            raise
        except Exception as e:  # transport errors
            raise ChatError.stream_error(f"{type(e).__name__}: {e}")


class RoutingChatClient(ChatClient):
    """Local engine first for the models it serves; everything else to the remote providers."""

    def __init__(self, local, remote: Optional[RemoteChatClient]):
        self.local, self.remote = local, remote

    async def create_streaming(self, ctx, request):
        if self.local is not None and any(self.local.serves(m) for m in [request.model] + list(request.models or [])):
            return await self.local.create_streaming(ctx, request)
        if self.remote is not None:
            return await self.remote.create_streaming(ctx, request)
        raise ChatError.model_not_found(request.model)
