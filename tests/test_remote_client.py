"""RemoteChatClient (CPU) against a mock OpenAI-compatible upstream (httpx.MockTransport): forced streaming
with include_usage, attempt order over api bases and fallback models, first-chunk probing, bad-status /
provider-error / first-chunk-timeout handling, SSE comments and [DONE], backoff budget
(reference src/chat/completions/client.rs:193-434, src/main.rs:5-20)."""
import asyncio
import json

import httpx
import pytest

from llm_weighted_consensus_amd.chat.remote import ApiBase, Backoff, RemoteChatClient
from llm_weighted_consensus_amd.errors import ChatError
from llm_weighted_consensus_amd.schema import chat as C


def _chunk(content, model="m", finish=None, usage=None):
    obj = {"id": "c1", "choices": [{"delta": {"content": content}, "finish_reason": finish, "index": 0}],
           "created": 1, "model": model, "object": "chat.completion.chunk"}
    if usage:
        obj["usage"] = usage
    return f"data: {json.dumps(obj)}\n\n"


class _Slow(httpx.AsyncByteStream):
    def __init__(self, parts, delay):
        self.parts, self.delay = parts, delay

    async def __aiter__(self):
        for p in self.parts:
            await asyncio.sleep(self.delay)
            yield p.encode()


def _client(handler, bases=("http://a", "http://b"), **kw):
    http = httpx.AsyncClient(transport=httpx.MockTransport(handler))
    return RemoteChatClient([ApiBase(b, f"key-{b[-1]}") for b in bases],
                            backoff=kw.pop("backoff", Backoff(0.001, 0.0, 1.5, 0.002, 0.05)),
                            user_agent="ua", x_title="title", referer="ref", http_client=http, **kw)


def _req(**kw):
    return C.ChatCompletionCreateParams.model_validate(
        dict({"model": "m", "messages": [{"role": "user", "content": "hi"}]}, **kw))


async def _collect(stream):
    return [c async for c in stream]


def test_forced_stream_headers_and_sse_parsing():
    seen = []

    async def handler(request: httpx.Request):
        seen.append((str(request.url), dict(request.headers), json.loads(request.content)))
        body = ": keep-alive comment\n\n" + _chunk("Hel") + _chunk("lo", finish="stop") + \
            _chunk("", usage={"prompt_tokens": 3, "completion_tokens": 2, "total_tokens": 5}) + "data: [DONE]\n\n"
        return httpx.Response(200, content=body.encode(), headers={"content-type": "text/event-stream"})

    cli = _client(handler)

    async def go():
        stream = await cli.create_streaming(None, _req())
        return await _collect(stream)

    chunks = asyncio.run(go())
    text = "".join(c.choices[0].delta.content or "" for c in chunks if c.choices)
    assert text == "Hello"
    assert chunks[-1].usage.total_tokens == 5
    url, headers, body = seen[0]
    assert url == "http://a/chat/completions" and headers["authorization"] == "Bearer key-a"
    assert headers["user-agent"] == "ua" and headers["x-title"] == "title" and headers["http-referer"] == "ref"
    assert body["stream"] is True and body["stream_options"] == {"include_usage": True}  # caller was unary


def test_attempt_order_bases_then_fallback_models():
    calls = []

    async def handler(request: httpx.Request):
        body = json.loads(request.content)
        calls.append((str(request.url.host), body["model"]))
        if body["model"] == "good" and request.url.host == "b":
            return httpx.Response(200, content=(_chunk("ok", model="good") + "data: [DONE]\n\n").encode())
        return httpx.Response(503, json={"error": "down"})

    cli = _client(handler)

    async def go():
        stream = await cli.create_streaming(None, _req(model="bad", models=["worse", "good"]))
        return await _collect(stream)

    chunks = asyncio.run(go())
    assert chunks[0].model == "good"
    assert calls == [("a", "bad"), ("b", "bad"), ("a", "worse"), ("b", "worse"), ("a", "good"), ("b", "good")]


def test_all_attempts_fail_bad_status_after_backoff_budget():
    n = {"calls": 0}

    async def handler(request):
        n["calls"] += 1
        return httpx.Response(429, json={"error": {"message": "rate limited"}})

    cli = _client(handler)
    with pytest.raises(ChatError) as ei:
        asyncio.run(cli.create_streaming(None, _req()))
    assert ei.value.status() == 429 and ei.value.detail["kind"] == "bad_status"
    assert n["calls"] >= 4  # the attempt list was retried under the backoff budget


def test_provider_error_and_first_chunk_timeout_fall_through():
    async def handler(request):
        if request.url.host == "a":  # provider error object instead of a chunk
            return httpx.Response(200, content=b'data: {"error": {"code": 502, "message": "upstream"}}\n\n')
        if request.url.host == "b":  # nothing within the first-chunk timeout
            return httpx.Response(200, stream=_Slow([_chunk("late"), "data: [DONE]\n\n"], 0.5))
        return httpx.Response(200, content=(_chunk("from c") + "data: [DONE]\n\n").encode())

    cli = _client(handler, bases=("http://a", "http://b", "http://c"), first_chunk_timeout=0.1)

    async def go():
        return await _collect(await cli.create_streaming(None, _req()))

    chunks = asyncio.run(go())
    assert chunks[0].choices[0].delta.content == "from c"

    cli2 = _client(handler, bases=("http://a",))
    with pytest.raises(ChatError) as ei:
        asyncio.run(cli2.create_streaming(None, _req()))
    assert ei.value.status() == 502 and ei.value.detail["kind"] == "provider"
