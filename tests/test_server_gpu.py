"""End-to-end on the GPU (the minimum slice): the ASGI server with a local
random-init Llama voter model and a local BGE encoder.  /score/completions with N voters that all map
to the local engine (json_schema output mode: constrained decoding guarantees a parseable key; votes
from real top-k logprobs), /chat/completions streaming, /multichat, /consensus, /embeddings — and
the fault path: an injected engine crash turns every voter into an error choice and the request into
the reference's AllVotesFailed status."""
import asyncio
import json
import re

import httpx
import pytest

pytestmark = pytest.mark.gpu

MODELS = {"tiny": {"arch": "llama-tiny", "weights": "random:1", "max_model_len": 2048, "max_batch": 64}}
EMBED = {"bge-small": {"arch": "bge-small-en-v1.5", "weights": "random:2"}}


def _client(monkeypatch, fault=None):
    from llm_weighted_consensus_amd.server.app import create_app
    from llm_weighted_consensus_amd.server.config import Config
    from llm_weighted_consensus_amd.server.main import build_state

    if fault:
        monkeypatch.setenv("LWC_FAULT", fault)
    else:
        monkeypatch.delenv("LWC_FAULT", raising=False)
    state = build_state(Config(models=MODELS, embed_models=EMBED, kv_fraction=0.05))
    return state, httpx.AsyncClient(transport=httpx.ASGITransport(app=create_app(state)), base_url="http://t",
                                    timeout=120)


def _close(state):
    for svc in state.services.values():
        svc.close()


SCORE = {"messages": [{"role": "user", "content": "Which city is the capital of France?"}],
         "model": {"llms": [{"model": "tiny", "output_mode": "json_schema", "top_logprobs": 5},
                            {"model": "tiny", "output_mode": "json_schema", "top_logprobs": 5, "temperature": 0.5},
                            {"model": "tiny", "output_mode": "instruction", "top_logprobs": 5,
                             "weight": {"type": "static", "weight": 2}}]},
         "choices": ["Paris", "Madrid", "Rome"]}


def test_score_chat_multichat_consensus_embeddings_local(gpu, monkeypatch):
    state, c = _client(monkeypatch)

    async def go():
        r = await c.post("/score/completions", json=SCORE)
        assert r.status_code == 200, r.text
        body = r.json()
        provided = [ch for ch in body["choices"] if ch["index"] < 3]
        assert len(provided) == 3
        # json_schema voters always produce a valid key -> their votes exist and sum to 1
        voters = [ch for ch in body["choices"] if ch["index"] >= 3]
        assert len(voters) == 3
        ok = [v for v in voters if v.get("error") is None]
        assert len(ok) >= 2
        conf = sum(ch["confidence"] or 0 for ch in provided)
        assert conf == pytest.approx(1.0, abs=1e-6)
        # streaming chat from the local engine
        r = await c.post("/chat/completions", json={"model": "tiny", "stream": True, "max_tokens": 8,
                                                    "messages": [{"role": "user", "content": "hi"}], "n": 2})
        assert r.status_code == 200 and r.text.endswith("data: [DONE]\n\n")
        chunks = [json.loads(e[6:]) for e in r.text.split("\n\n") if e.startswith("data: {")]
        assert chunks and all(ch["object"] == "chat.completion.chunk" for ch in chunks)
        r = await c.post("/consensus/completions", json={"model": "tiny", "n": 4, "max_tokens": 12,
                                                         "messages": [{"role": "user", "content": "say hi"}],
                                                         "embedding_model": "bge-small"})
        assert r.status_code == 200, r.text
        assert sum(ch["confidence"] for ch in r.json()["choices"]) == pytest.approx(1.0, abs=1e-5)
        r = await c.post("/embeddings", json={"model": "bge-small", "input": ["alpha", "beta"]})
        assert r.status_code == 200 and len(r.json()["data"][0]["embedding"]) == 384
        r = await c.get("/metrics")
        assert "lwc_latency_seconds_count" in r.text and "lwc_engine_running" in r.text

    try:
        asyncio.run(go())
    finally:
        _close(state)


def test_injected_engine_crash_gives_all_votes_failed(gpu, monkeypatch):
    state, c = _client(monkeypatch, fault="worker_crash:1+")

    async def go():
        r = await c.post("/score/completions", json=SCORE)
        # every voter failed with the engine's 500 -> AllVotesFailed(500)
        assert r.status_code == 500, r.text
        assert r.json()["kind"] == "score"

    try:
        asyncio.run(go())
    finally:
        _close(state)
    assert all(svc.failures >= 1 for svc in state.services.values())


def test_engine_group_two_workers_serve_chat(gpu, monkeypatch):
    """LWC_GPUS with two entries: an EngineGroup of two worker processes (both on the box's one GPU here)
    serves a chat request whose n candidates are split across them."""
    from llm_weighted_consensus_amd.server.app import create_app
    from llm_weighted_consensus_amd.server.config import Config
    from llm_weighted_consensus_amd.server.main import build_state

    monkeypatch.delenv("LWC_FAULT", raising=False)
    monkeypatch.setenv("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    state = build_state(Config(models=MODELS, embed_models=EMBED, gpus=[0, 0], kv_fraction=0.04))
    c = httpx.AsyncClient(transport=httpx.ASGITransport(app=create_app(state)), base_url="http://t", timeout=300)
    svc = state.services["tiny"]

    async def go():
        r = await c.post("/chat/completions", json={"model": "tiny", "max_tokens": 6, "n": 6, "seed": 3,
                                                    "messages": [{"role": "user", "content": "hello"}]})
        assert r.status_code == 200, r.text
        ch = r.json()["choices"]
        assert sorted(x["index"] for x in ch) == list(range(6))
        r = await c.get("/metrics")
        assert 'lwc_engine_workers_alive{model="tiny"} 2' in r.text
        # /consensus: both workers embed the candidates they generated; rows come back to the front end
        assert svc.embeds_in_workers("bge-small")
        r = await c.post("/consensus/completions", json={"model": "tiny", "n": 6, "max_tokens": 8, "seed": 5,
                                                         "messages": [{"role": "user", "content": "say hi"}],
                                                         "embedding_model": "bge-small"})
        assert r.status_code == 200, r.text
        ch = r.json()["choices"]
        assert len(ch) == 6 and sum(x["confidence"] for x in ch) == pytest.approx(1.0, abs=1e-5)

    try:
        assert len(svc.live_workers()) == 2
        asyncio.run(go())
    finally:
        svc.close()


def test_decoder_embedder_served_from_embed_models(gpu):
    """An embed-model spec naming a DECODER arch serves /embeddings through the decoder-as-embedder
    (e5-mistral style: last-token pooling of the final hidden state), unit-norm rows of the model's width."""
    from llm_weighted_consensus_amd.server.app import create_app
    from llm_weighted_consensus_amd.server.config import Config
    from llm_weighted_consensus_amd.server.main import build_state

    state = build_state(Config(embed_models={"e5": {"arch": "llama-tiny", "weights": "random:5", "max_tokens": 256}}))
    c = httpx.AsyncClient(transport=httpx.ASGITransport(app=create_app(state)), base_url="http://t", timeout=120)

    async def go():
        r = await c.post("/embeddings", json={"input": ["a cat", "a dog", "a cat"], "model": "e5"})
        assert r.status_code == 200, r.text
        data = r.json()["data"]
        assert len(data) == 3 and len(data[0]["embedding"]) == 512
        n = sum(x * x for x in data[0]["embedding"]) ** 0.5
        assert abs(n - 1.0) < 1e-2
        assert data[0]["embedding"] == data[2]["embedding"]  # same text -> same row (cache or not)
    asyncio.run(go())


@pytest.mark.parametrize("kind", ["bytelevel", "sentencepiece"])
def test_constrained_voters_with_real_tokenizer(gpu, tmp_path, kind):
    """json_schema and tool_call voters on a model served with a REAL tokenizer.json (built offline):
    token-level masks from the tokenizer's bytes, so every voter emits parseable JSON with a valid key
    and a vote (round-1 masks assumed id == byte and produced garbage here)."""
    from llm_weighted_consensus_amd.server.app import create_app
    from llm_weighted_consensus_amd.server.config import Config
    from llm_weighted_consensus_amd.server.main import build_state
    from tests.test_tokenizers import _bytelevel, _sentencepiece

    path = (_bytelevel if kind == "bytelevel" else _sentencepiece)(tmp_path)
    models = {"tiny": dict(MODELS["tiny"], tokenizer=path)}
    state = build_state(Config(models=models, kv_fraction=0.05))
    c = httpx.AsyncClient(transport=httpx.ASGITransport(app=create_app(state)), base_url="http://t", timeout=120)
    req = {"messages": [{"role": "user", "content": "Which city is the capital of France?"}],
           "model": {"llms": [{"model": "tiny", "output_mode": "json_schema", "top_logprobs": 5},
                              {"model": "tiny", "output_mode": "json_schema", "top_logprobs": 5, "temperature": 1.5},
                              {"model": "tiny", "output_mode": "tool_call", "top_logprobs": 5}]},
           "choices": ["Paris", "Madrid", "Rome"]}

    async def go():
        r = await c.post("/score/completions", json=req)
        assert r.status_code == 200, r.text
        body = r.json()
        voters = [ch for ch in body["choices"] if ch["index"] >= 3]
        assert len(voters) == 3
        for v in voters:
            assert v.get("error") is None, v
            msg = v["message"]
            text = msg["content"] if msg.get("content") else msg["tool_calls"][0]["function"]["arguments"]
            obj = json.loads(text)
            assert re.fullmatch(r"`[A-T]`", obj["response_key"]), text  # keys are drawn per voter (KeyTree)
            assert msg["vote"] is not None and sum(msg["vote"]) == pytest.approx(1.0, abs=1e-6)

    try:
        asyncio.run(go())
    finally:
        _close(state)
