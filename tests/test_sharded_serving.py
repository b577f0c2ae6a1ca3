"""Whole-node serving layout on the CPU: the voter-sharded deployment (``LWC_SHARD_VOTERS``) at world 8 over
gloo, requests through the real ASGI app on rank 0.

* /score/completions: unary, and streamed (SSE) — the stream's fold equals the unary response of a
  single-process server (voters, votes, tally), the initial chunk comes first, each rank's voters arrive
  as they finish;
* /consensus/completions: the request's candidates are split over the 8 ranks (each samples its slice with
  the seeds the slice has in the whole request and embeds it on its own device), the unit rows come back
  to the leader over the shard links and the response equals the single-process one (candidates,
  weights, confidences, embeddings)."""
import asyncio
import json
import math
import os
import socket

import pytest
import torch.multiprocessing as mp

from llm_weighted_consensus_amd.chat.fake import FakeChatClient, Scripted, select_keys

WORLD = int(os.environ.get("LWC_TEST_WORLD", "8"))
EMBED = {"arch": "bert-tiny", "weights": "random:1"}
ANSWERS = ["Paris is the capital of France.", "The capital is Paris.", "It is London, I think.",
           "Paris.", "Berlin", "Definitely Paris, the French capital."]


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _policy(req):
    if req.model == "cand":  # consensus candidates: candidate i's text depends on (seed, i) only
        return [Scripted(ANSWERS[(int(req.seed) * 7 + i) % len(ANSWERS)]) for i in range(int(req.n or 1))]
    keys = select_keys(req)
    good = next(k for k, v in keys if "Paris" in v)
    bad = [k for k, v in keys if "Paris" not in v]
    if req.top_logprobs:
        lp = [("`", [("`", 0.0)]), (good[1], [(good[1], math.log(0.6)), (bad[0][1], math.log(0.3))]), ("`", [("`", 0.0)])]
        return [Scripted(good, logprobs=lp)]
    if req.model == "wrong":
        return [Scripted(f"clearly {bad[0]}")]
    return [Scripted(f"The answer is {good}.")]


LLMS = [{"model": "a", "weight": {"type": "static", "weight": 3}}, {"model": "wrong"}, {"model": "lp", "top_logprobs": 5},
        {"model": "b"}, {"model": "a", "temperature": 0.5}, {"model": "wrong", "top_p": 0.9},
        {"model": "lp", "top_logprobs": 3}, {"model": "b", "weight": {"type": "static", "weight": 2}},
        {"model": "a", "temperature": 0.2}, {"model": "wrong", "temperature": 0.3}]


def _score_body(stream):
    return {"messages": [{"role": "user", "content": "What is the capital of France?"}], "model": {"llms": LLMS},
            "choices": ["Paris", "London", "Berlin"], "stream": stream}


def _consensus_body(n):
    return {"messages": [{"role": "user", "content": "Capital of France?"}], "model": "cand", "n": n, "seed": 11,
            "embedding_model": "e", "tau": 0.1}


def _state(chat, rng_seed=7):
    from llm_weighted_consensus_amd.embeddings.service import build_embedding_service
    from llm_weighted_consensus_amd.score.multichat import ConsensusClient, MultichatClient
    from llm_weighted_consensus_amd.score.orchestrator import ScoreClient
    from llm_weighted_consensus_amd.server.app import AppState

    emb = {"e": build_embedding_service("e", EMBED, "cpu")}
    score = ScoreClient(chat, rng_seed=rng_seed)
    return AppState(chat, score, MultichatClient(score, None), ConsensusClient(chat, emb), embedders=emb)


def _summary_score(obj):
    return {"n": len(obj["choices"]),
            "provided": sorted((c["index"], round(c["weight"], 6), round(c["confidence"], 6))
                               for c in obj["choices"] if c["index"] < 3),
            "voters": sorted((c["model_index"], c["message"].get("vote") and tuple(c["message"]["vote"]),
                              round(c["weight"], 6)) for c in obj["choices"] if c["index"] >= 3),
            "prompt_tokens": obj["usage"]["prompt_tokens"]}


def _summary_consensus(obj):
    return {"choices": sorted((c["index"], c["message"]["content"], c["weight"], c["confidence"])
                              for c in obj["choices"]),
            "emb": [e["embedding"][:8] for e in obj["weight_data"]["embeddings_response"]["data"]],
            "usage": (obj["usage"]["prompt_tokens"], obj["usage"]["completion_tokens"])}


def _same_consensus(a, b):
    """Same candidates in the same order, usage equal; weights / confidences / embeddings equal up to the
    float noise of embedding the candidates in other batches (each rank embeds its own slice)."""
    assert a["usage"] == b["usage"]
    assert [c[:2] for c in a["choices"]] == [c[:2] for c in b["choices"]]
    for x, y in zip(a["choices"], b["choices"]):
        assert x[2] == pytest.approx(y[2], abs=1e-4) and x[3] == pytest.approx(y[3], abs=1e-4)
    for x, y in zip(a["emb"], b["emb"]):
        assert x == pytest.approx(y, abs=1e-4)


async def _drive(app):
    """The client side: unary score, streamed score (SSE), consensus at two sizes, concurrent mix."""
    import httpx

    client = httpx.AsyncClient(transport=httpx.ASGITransport(app=app), base_url="http://t", timeout=300)
    out = {}
    r = await client.post("/score/completions", json=_score_body(False))
    assert r.status_code == 200, r.text
    out["unary"] = _summary_score(r.json())
    chunks = []
    async with client.stream("POST", "/score/completions", json=_score_body(True)) as resp:
        assert resp.status_code == 200
        async for line in resp.aiter_lines():
            if line.startswith("data: ") and line != "data: [DONE]":
                chunks.append(json.loads(line[6:]))
    out["n_chunks"] = len(chunks)
    from llm_weighted_consensus_amd.schema import score as S

    agg = S.ScoreCompletionChunk.model_validate(chunks[0])
    for c in chunks[1:]:
        agg.push(S.ScoreCompletionChunk.model_validate(c))
    out["stream"] = _summary_score(S.ScoreCompletion.from_chunk(agg).to_obj())
    out["first_chunk_choices"] = len(chunks[0]["choices"])
    for n in (12, 5):
        r = await client.post("/consensus/completions", json=_consensus_body(n))
        assert r.status_code == 200, r.text
        out[f"consensus{n}"] = _summary_consensus(r.json())
    many = await asyncio.gather(*([client.post("/score/completions", json=_score_body(False)) for _ in range(3)]
                                  + [client.post("/consensus/completions", json=_consensus_body(9)) for _ in range(3)]))
    out["many"] = [(m.status_code, len(m.json()["choices"])) for m in many]
    await client.aclose()
    return out


def _rank(rank, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(WORLD), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    import torch

    torch.set_num_threads(1)
    from llm_weighted_consensus_amd.parallel import dist as pdist
    from llm_weighted_consensus_amd.server.app import create_app
    from llm_weighted_consensus_amd.server.main import shard_voters

    try:
        pdist.init_from_env("cpu")
        state = _state(FakeChatClient(_policy))
        lead = shard_voters(state, rng_seed=7)
        if rank == 0:
            res = asyncio.run(_drive(create_app(state)))
            lead.close()
        else:
            res = lead.serve()
        q.put((rank, res))
    except BaseException as e:  # noqa: BLE001
        import traceback

        q.put((rank, f"ERROR {type(e).__name__}: {e}\n{traceback.format_exc()}"))
    finally:
        pdist.shutdown()


@pytest.mark.timeout(600)
def test_world8_sharded_serving_matches_single_process():
    from llm_weighted_consensus_amd.server.app import create_app

    # single process, same request numbering: score request k's voters seeded from (7, k)
    single = _state(FakeChatClient(_policy))

    async def want_all():
        import httpx

        client = httpx.AsyncClient(transport=httpx.ASGITransport(app=create_app(single)), base_url="http://t")
        from llm_weighted_consensus_amd.schema import score as S

        out = {}
        for k in (0, 1):  # score requests 0 (unary) and 1 (streamed): voters seeded from (7, k)
            req = S.ScoreCompletionCreateParams.model_validate(_score_body(False))
            out[f"score{k}"] = _summary_score((await single.score.create_unary({"seed": 7 * 1000003 + k}, req)).to_obj())
        for n in (12, 5):
            r = await client.post("/consensus/completions", json=_consensus_body(n))
            out[f"consensus{n}"] = _summary_consensus(r.json())
        return out

    want = asyncio.run(want_all())
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, port, q)) for r in range(WORLD)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=500) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    for r in range(WORLD):
        assert not (isinstance(got[r], str) and got[r].startswith("ERROR")), got[r]
    lead = got[0]
    # unary and streamed score: every voter of the request (10 voters + 3 choices), streamed fold == unary shape
    assert lead["unary"] == want["score0"]
    assert lead["stream"] == want["score1"]  # the fold of the SSE stream is the single-process response
    assert lead["n_chunks"] >= 3 and lead["first_chunk_choices"] == 3  # initial chunk first, then voters
    for n in (12, 5):  # consensus: the 8-way split equals one process
        _same_consensus(lead[f"consensus{n}"], want[f"consensus{n}"])
    assert lead["many"] == [(200, 3 + len(LLMS))] * 3 + [(200, 9)] * 3
    # followers get work only for what they own: every score request (10 voters over 8 ranks), a slice of every
    # consensus request whose candidate count reaches them (12 and 9: all ranks; 5: ranks 1-4)
    assert all(got[r] == 5 + 1 + (1 if r < 5 else 0) + 3 for r in range(1, WORLD)), got
