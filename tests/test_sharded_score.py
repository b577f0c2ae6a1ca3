"""Voter-sharded scoring over a process group (C2; gloo, world 2, CPU): a score request's voters split
across ranks give the single-process tally, confidences, votes and usage; ids agree on every rank;
"every vote failed" is decided globally (every rank raises, error codes unified over all ranks); a rank
that owns no voter still takes part; requests run concurrently (combines ordered by request number)."""
import asyncio
import math
import os
import socket

import pytest
import torch.multiprocessing as mp

from llm_weighted_consensus_amd.chat.fake import Failure, FakeChatClient, Scripted, select_keys
from llm_weighted_consensus_amd.errors import ChatError, ScoreError
from llm_weighted_consensus_amd.schema import score as S


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _policy(req):
    if req.model.startswith("fail"):
        code = int(req.model.split("-")[1])
        return Failure(ChatError.bad_status(code, {"code": code}))
    keys = select_keys(req)
    good = next(k for k, v in keys if "Paris" in v)
    bad = [k for k, v in keys if "Paris" not in v]
    if req.top_logprobs:
        lp = [("`", [("`", 0.0)]),
              (good[1], [(good[1], math.log(0.6)), (bad[0][1], math.log(0.3)), ("zz", math.log(0.1))]),
              ("`", [("`", 0.0)])]
        return [Scripted(good, logprobs=lp)]
    if req.model == "wrong":
        return [Scripted(f"clearly {bad[0]}")]
    return [Scripted(f"The answer is {good}.")]


CASES = {
    "mixed": [{"model": "a", "weight": {"type": "static", "weight": 3}}, {"model": "wrong"},
              {"model": "lp", "top_logprobs": 5}, {"model": "b", "weight": {"type": "static", "weight": 2}},
              {"model": "fail-429"}],
    "one_voter": [{"model": "a"}],
    "all_fail": [{"model": "fail-429"}, {"model": "fail-500"}, {"model": "fail-429", "weight": {"type": "static",
                                                                                                "weight": 2}}],
}


def _request(case):
    if case == "one_choice":  # rejected before any voter runs: the request still takes its combine slot
        return S.ScoreCompletionCreateParams.model_validate(dict(
            messages=[{"role": "user", "content": "What is the capital of France?"}],
            model={"llms": CASES["one_voter"]}, choices=["Paris"], stream=False))
    return S.ScoreCompletionCreateParams.model_validate(dict(
        messages=[{"role": "user", "content": "What is the capital of France?"}],
        model={"llms": CASES[case]}, choices=["Paris", "London", "Berlin"], stream=False))


def _summary(out: S.ScoreCompletion):
    provided = sorted((c.index, c.weight, c.confidence) for c in out.choices if c.index < 3)
    voters = sorted((c.model_index, c.message.vote, c.weight, c.confidence, c.error.code if c.error else None)
                    for c in out.choices if c.index >= 3)
    return {"provided": provided, "voters": voters, "prompt_tokens": out.usage.prompt_tokens,
            "total_cost": out.usage.total_cost, "id": out.id, "n": len(out.choices),
            "indices": sorted(c.index for c in out.choices)}


def _run(client, case, ctx=None):
    try:
        return _summary(asyncio.run(client.create_unary(ctx, _request(case))))
    except ScoreError as e:
        return {"error": e.code}


async def _run_sharded(client, seq, case):
    try:
        return _summary(await client.run(seq, (1700000000, f"scrcpl-test-{seq}"), _request(case)))
    except ScoreError as e:
        return {"error": e.code}


def _worker(rank, world, port, out_q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    from llm_weighted_consensus_amd.parallel import dist as pdist
    from llm_weighted_consensus_amd.score.sharded import ShardedScoreClient

    pdist.init_from_env("cpu")
    client = ShardedScoreClient(FakeChatClient(_policy), rng_seed=7)
    # one at a time (same key-tree seeds as the single-process client), then all cases concurrently
    res = {case: asyncio.run(_run_sharded(client, i, case)) for i, case in enumerate(CASES)}

    async def concurrent():
        cases = (list(CASES) + ["one_choice"]) * 3
        outs = await asyncio.gather(*(_run_sharded(client, len(CASES) + i, c) for i, c in enumerate(cases)))
        return [(c, o) for c, o in zip(cases, outs)]

    res["concurrent"] = asyncio.run(concurrent())
    client.close()
    out_q.put((rank, res))
    pdist.shutdown()


def test_voter_sharded_score_matches_single_process():
    from llm_weighted_consensus_amd.score.orchestrator import ScoreClient

    single = ScoreClient(FakeChatClient(_policy), rng_seed=7)
    # the sharded client seeds request `seq`'s voters from (seed base 7, seq): the same seeds here
    want = {case: _run(single, case, {"seed": 7 * 1000003 + i}) for i, case in enumerate(CASES)}
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for case in ("mixed", "one_voter"):
        w, g0, g1 = want[case], got[0][case], got[1][case]
        assert g0["id"] == g1["id"]  # the request's id, identical on every rank
        for g in (g0, g1):  # every rank merges the same full response
            assert g["n"] == w["n"] and g["indices"] == list(range(w["n"]))
            assert g["prompt_tokens"] == w["prompt_tokens"]
            assert g["total_cost"] == pytest.approx(w["total_cost"])
            for (i, wt, cf), (j, wt2, cf2) in zip(w["provided"], g["provided"]):
                assert i == j and wt2 == pytest.approx(wt) and cf2 == pytest.approx(cf)
            for a, b in zip(w["voters"], g["voters"]):
                assert a[0] == b[0] and a[1] == b[1] and a[4] == b[4]
                assert b[2] == pytest.approx(a[2])
                assert (a[3] is None and b[3] is None) or b[3] == pytest.approx(a[3])
    assert want["all_fail"]["error"] == got[0]["all_fail"]["error"] == got[1]["all_fail"]["error"]
    for r in (0, 1):  # concurrent requests: same shapes and tallies (seeds differ, so not the votes)
        for case, o in got[r]["concurrent"]:
            if case == "one_choice":
                assert o == {"error": 400}
            elif case == "all_fail":
                assert o == {"error": want["all_fail"]["error"]}
            else:
                assert o["n"] == want[case]["n"] and o["prompt_tokens"] == want[case]["prompt_tokens"]
                assert sum(cf for _, _, cf in o["provided"]) == pytest.approx(1.0)


def _serve_worker(rank, world, port, out_q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    from llm_weighted_consensus_amd.parallel import dist as pdist
    from llm_weighted_consensus_amd.score.multichat import MultichatClient
    from llm_weighted_consensus_amd.score.orchestrator import ScoreClient
    from llm_weighted_consensus_amd.score.sharded import follow
    from llm_weighted_consensus_amd.server.app import AppState
    from llm_weighted_consensus_amd.server.main import shard_voters

    pdist.init_from_env("cpu")
    chat = FakeChatClient(_policy)
    score = ScoreClient(chat, rng_seed=7)
    state = AppState(chat, score, MultichatClient(score, None))
    lead = shard_voters(state, rng_seed=7)
    if rank == 0:
        async def serve():
            out = [_summary(await state.score.create_unary(None, _request("mixed")))]
            chunks = [c async for c in await state.score.create_streaming(None, _request("mixed"))]
            agg = chunks[0].clone()
            for c in chunks[1:]:
                agg.push(c)
            out.append((len(chunks), _summary(S.ScoreCompletion.from_chunk(agg))))
            try:
                await state.score.create_unary(None, _request("all_fail"))
            except ScoreError as e:
                out.append(e.code)
            many = await asyncio.gather(*(state.score.create_unary(None, _request("mixed")) for _ in range(6)))
            out.append([len(m.choices) for m in many])
            return out

        res = asyncio.run(serve())
        lead.close()
    else:
        res = follow(lead)
    out_q.put((rank, res))
    pdist.shutdown()


def test_leader_broadcasts_requests_to_followers():
    single = __import__("llm_weighted_consensus_amd.score.orchestrator", fromlist=["ScoreClient"]).ScoreClient(
        FakeChatClient(_policy), rng_seed=7)
    want = _run(single, "mixed", {"seed": 7 * 1000003 + 0})   # request 0: unary
    want_s = _run(single, "mixed", {"seed": 7 * 1000003 + 1})  # request 1: streamed
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_serve_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    mixed, (n_chunks, folded), code, many = got[0]
    assert mixed["n"] == want["n"] and [v[:2] for v in mixed["voters"]] == [v[:2] for v in want["voters"]]
    # streamed: initial chunk, this rank's voter chunks as they arrive, final chunk (remote voters + tally);
    # the fold of the stream is the unary response
    assert n_chunks >= 3
    assert folded["n"] == want_s["n"] and folded["indices"] == want_s["indices"]
    assert [v[:2] + v[4:] for v in folded["voters"]] == [v[:2] + v[4:] for v in want_s["voters"]]
    assert sum(cf for _, _, cf in folded["provided"]) == pytest.approx(1.0)
    assert code == 429 or code == want.get("error", code)
    assert many == [want["n"]] * 6  # concurrent requests: every voter of every request in the response
    assert got[1] == 9  # the follower ran all nine requests
