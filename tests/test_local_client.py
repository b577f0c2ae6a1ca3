"""LocalChatClient attempt semantics (reference src/chat/completions/client.rs:238-305, 347-354) against
fake engine services on the CPU: fall over to the next locally served model on an engine failure or a
first-chunk timeout, commit once a chunk arrived, `stream_timeout` on a stalled committed stream, and the
aborted attempt's engine group is released."""
import asyncio
import types

import pytest

from llm_weighted_consensus_amd.chat.local import LocalChatClient
from llm_weighted_consensus_amd.engine.service import EngineFailure
from llm_weighted_consensus_amd.engine.tokenizer import ByteTokenizer
from llm_weighted_consensus_amd.errors import ChatError
from llm_weighted_consensus_amd.models.config import decoder_config
from llm_weighted_consensus_amd.schema import chat as C


class _Ev:
    def __init__(self, index, tid, last):
        self.seq = types.SimpleNamespace(index=index)
        self.token_id, self.text = tid, chr(97 + tid % 26)
        self.logprob, self.top_logprobs = -0.1, []
        self.finished, self.finish_reason = last, ("length" if last else None)


class FakeService:
    """mode: ok | fail (EngineFailure before any token) | stall (never emits) | stall_after_first."""

    def __init__(self, mode, tokens=3):
        cfg = decoder_config("llama-tiny")
        self.engine = types.SimpleNamespace(tokenizer=ByteTokenizer(cfg.vocab_size), cfg=cfg, max_model_len=2048)
        self.mode, self.tokens = mode, tokens
        self.submitted, self.aborted = 0, 0

    def submit(self, ids, sp, n, loop, q):
        self.submitted += 1
        g = object()
        if self.mode == "fail":
            loop.call_soon(q.put_nowait, EngineFailure("engine worker crashed"))
        elif self.mode in ("ok", "stall_after_first"):
            count = 1 if self.mode == "stall_after_first" else self.tokens
            for i in range(n):
                for k in range(count):
                    last = self.mode == "ok" and k == count - 1
                    loop.call_soon(q.put_nowait, _Ev(i, 65 + k, last))
        return g

    def abort(self, g):
        self.aborted += 1


def _req(model, models=None, stream=True):
    return C.ChatCompletionCreateParams.model_validate(
        {"model": model, "models": models, "stream": stream, "max_tokens": 4,
         "messages": [{"role": "user", "content": "hi"}]})


async def _drain(stream):
    return [c async for c in stream]


def test_falls_over_to_next_model_on_engine_failure():
    svcs = {"a": FakeService("fail"), "b": FakeService("ok")}
    cl = LocalChatClient(svcs)

    async def go():
        chunks = await _drain(await cl.create_streaming(None, _req("a", ["b"])))
        return chunks

    chunks = asyncio.run(go())
    assert chunks and all(c.model == "b" for c in chunks)
    assert svcs["a"].submitted == 1 and svcs["b"].submitted == 1


def test_first_chunk_timeout_tries_next_model_and_aborts_the_stalled_one():
    svcs = {"a": FakeService("stall"), "b": FakeService("ok")}
    cl = LocalChatClient(svcs, first_chunk_timeout=0.2)

    async def go():
        return await _drain(await cl.create_streaming(None, _req("a", ["b", "zzz"])))

    chunks = asyncio.run(go())
    assert chunks[0].model == "b"
    assert svcs["a"].aborted == 1  # the stalled attempt's sequences were released


def test_every_attempt_fails_raises_last_error():
    svcs = {"a": FakeService("fail"), "b": FakeService("stall")}
    cl = LocalChatClient(svcs, first_chunk_timeout=0.2)

    async def go():
        await cl.create_streaming(None, _req("a", ["b"]))

    with pytest.raises(ChatError) as ei:
        asyncio.run(go())
    assert "timeout" in str(ei.value.message()).lower() or ei.value.status() == 500


def test_other_chunk_timeout_on_committed_stream():
    svcs = {"a": FakeService("stall_after_first"), "b": FakeService("ok")}
    cl = LocalChatClient(svcs, first_chunk_timeout=1.0, other_chunk_timeout=0.2)

    async def go():
        stream = await cl.create_streaming(None, _req("a", ["b"]))
        got = []
        with pytest.raises(ChatError) as ei:
            async for c in stream:
                got.append(c)
        return got, ei.value

    got, err = asyncio.run(go())
    assert len(got) == 1 and got[0].model == "a"       # committed to "a": no silent switch mid-stream
    assert err.to_response_error().code == 500 and "timeout" in str(err.message()).lower()
    assert svcs["b"].submitted == 0 and svcs["a"].aborted == 1


def test_unknown_models_use_fallback_client():
    class Fallback:
        async def create_streaming(self, ctx, req):
            async def one():
                yield "remote"
            return one()

    cl = LocalChatClient({"a": FakeService("ok")}, fallback=Fallback())

    async def go():
        return await _drain(await cl.create_streaming(None, _req("remote-model")))

    assert asyncio.run(go()) == ["remote"]
