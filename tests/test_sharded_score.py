"""Voter-sharded scoring (C2; CPU ranks): the leader (rank 0) resolves each request once, sends every
follower its share of voters over the shard links, merges their chunks live and tallies alone.

* world 2: a request's voters split across ranks give the single-process tally, confidences, votes and
  usage; "every vote failed" is decided over all voters (codes unified); concurrent requests; streamed
  requests interleave the follower's voter chunks live (before the final chunk);
* world 4, failure isolation: a follower killed mid-load turns exactly its unfinished
  voters of the in-flight requests into ``voter_shard_lost`` error choices, those requests complete within
  the bound, later requests run on the survivors with every voter ok, and nothing waits for a process-group
  timeout;
* an abandoned stream (never iterated) leaves nothing behind: the next request completes."""
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


def _leader_worker(rank, world, port, out_q, scenario, join_file=None):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), LWC_SHARD_DEAD_S="3", LWC_SHARD_HB_S="0.2")
    if join_file:
        os.environ["LWC_SHARD_LINK_FILE"] = join_file
    from llm_weighted_consensus_amd.parallel import dist as pdist
    from llm_weighted_consensus_amd.score.multichat import MultichatClient
    from llm_weighted_consensus_amd.score.orchestrator import ScoreClient
    from llm_weighted_consensus_amd.server.app import AppState
    from llm_weighted_consensus_amd.server.main import shard_voters

    pdist.init_from_env("cpu")
    policy = _policy
    delay = 0.0
    if scenario in ("kill", "rejoin"):
        delay = 0.03  # slow voters: requests are in flight when the last rank dies
        if rank == world - 1:
            seen = [0]

            def policy(req, _p=_policy):  # noqa: F811 — rank 3 dies while starting its 4th voter stream
                seen[0] += 1
                if seen[0] == 4:
                    os._exit(17)
                return _p(req)
    chat = FakeChatClient(policy, delay_s=delay)
    score = ScoreClient(chat, rng_seed=7)
    state = AppState(chat, score, MultichatClient(score, None))
    lead = shard_voters(state, rng_seed=7)
    if rank != 0:
        res = lead.serve()
        out_q.put((rank, res))
        pdist.shutdown()
        return
    try:
        res = asyncio.run(SCENARIOS[scenario](state.score))
    except BaseException as e:  # noqa: BLE001
        import traceback

        res = f"ERROR {type(e).__name__}: {e}\n{traceback.format_exc()}"
    lead.close()
    out_q.put((rank, res))
    if scenario not in ("kill", "rejoin"):
        pdist.shutdown()


def _rejoin_worker(rank, join_file, out_q):
    """A restarted follower: no process group, back onto the links from the leader's join file."""
    os.environ.update(LWC_SHARD_HB_S="0.2")
    from llm_weighted_consensus_amd.score.multichat import MultichatClient
    from llm_weighted_consensus_amd.score.orchestrator import ScoreClient
    from llm_weighted_consensus_amd.server.app import AppState
    from llm_weighted_consensus_amd.server.main import rejoin_follower

    chat = FakeChatClient(_policy, delay_s=0.0)
    score = ScoreClient(chat, rng_seed=7)
    state = AppState(chat, score, MultichatClient(score, None))
    out_q.put((rank, ("rejoined", rejoin_follower(state, join_file, rank).serve())))


async def _equiv(client):
    out = {}
    for case in CASES:  # one at a time: request k's voters seeded from (7, k), as the single process
        try:
            out[case] = _summary(await client.create_unary(None, _request(case)))
        except ScoreError as e:
            out[case] = {"error": e.code}
    cases = (list(CASES) + ["one_choice"]) * 3

    async def one(c):
        try:
            return _summary(await client.create_unary(None, _request(c)))
        except ScoreError as e:
            return {"error": e.code}

    out["concurrent"] = list(zip(cases, await asyncio.gather(*(one(c) for c in cases))))
    # streamed: the follower's voters arrive live, not whole in the final chunk
    req = _request("mixed").model_copy(update={"stream": True})
    chunks = [c async for c in await client.create_streaming(None, req)]
    remote = {v.index for v in client.last_model_llms if v.index % 2 == 1} if hasattr(client, "last_model_llms") \
        else {1, 3}
    live = [k for k, c in enumerate(chunks[:-1]) for ch in c.choices
            if ch.model_index in remote and ch.delta.content]
    agg = chunks[0].clone()
    for c in chunks[1:]:
        agg.push(c)
    out["stream"] = {"n_chunks": len(chunks), "live_remote_chunks": len(live),
                     "summary": _summary(S.ScoreCompletion.from_chunk(agg))}
    # abandoned before iteration: nothing is announced, nothing waits; the next request completes
    await client.create_streaming(None, _request("mixed").model_copy(update={"stream": True}))
    out["after_abandon"] = _summary(await client.create_unary(None, _request("mixed")))["n"]
    return out


def test_voter_sharded_leader_matches_single_process():
    from llm_weighted_consensus_amd.score.orchestrator import ScoreClient

    single = ScoreClient(FakeChatClient(_policy), rng_seed=7)
    # the sharded leader seeds request `seq`'s voters from (seed base 7, seq): the same seeds here
    want = {case: _run(single, case, {"seed": 7 * 1000003 + i}) for i, case in enumerate(CASES)}
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_leader_worker, args=(r, 2, port, q, "equiv")) for r in range(2)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    g = got[0]
    assert isinstance(g, dict), g
    for case in ("mixed", "one_voter"):
        w, o = want[case], g[case]
        assert o["n"] == w["n"] and o["indices"] == list(range(w["n"]))
        assert o["prompt_tokens"] == w["prompt_tokens"]
        assert o["total_cost"] == pytest.approx(w["total_cost"])
        for (i, wt, cf), (j, wt2, cf2) in zip(w["provided"], o["provided"]):
            assert i == j and wt2 == pytest.approx(wt) and cf2 == pytest.approx(cf)
        for a, b in zip(w["voters"], o["voters"]):
            assert a[0] == b[0] and a[1] == b[1] and a[4] == b[4]
            assert b[2] == pytest.approx(a[2])
            assert (a[3] is None and b[3] is None) or b[3] == pytest.approx(a[3])
    assert want["all_fail"]["error"] == g["all_fail"]["error"]
    for case, o in g["concurrent"]:  # concurrent requests: same shapes and tallies (seeds differ, not votes)
        if case == "one_choice":
            assert o == {"error": 400}
        elif case == "all_fail":
            assert o == {"error": want["all_fail"]["error"]}
        else:
            assert o["n"] == want[case]["n"] and o["prompt_tokens"] == want[case]["prompt_tokens"]
            assert sum(cf for _, _, cf in o["provided"]) == pytest.approx(1.0)
    st = g["stream"]
    assert st["live_remote_chunks"] > 0  # the follower's voters' content arrived before the final chunk
    assert st["summary"]["n"] == want["mixed"]["n"] and sum(cf for _, _, cf in st["summary"]["provided"]) == \
        pytest.approx(1.0)
    assert g["after_abandon"] == want["mixed"]["n"]
    assert got[1] >= len(CASES)  # the follower ran its share of every request that had voters for it


KILL_LLMS = [{"model": "a"}, {"model": "b"}, {"model": "a", "temperature": 0.5}, {"model": "b", "top_p": 0.9},
             {"model": "a", "temperature": 0.2}, {"model": "b", "temperature": 0.3}, {"model": "a", "top_p": 0.8},
             {"model": "b", "temperature": 0.7}]


def _kill_request(stream=False):
    return S.ScoreCompletionCreateParams.model_validate(dict(
        messages=[{"role": "user", "content": "What is the capital of France? " + "x" * 40}],
        model={"llms": KILL_LLMS}, choices=["Paris", "London", "Berlin"], stream=stream))


async def _kill(client):
    import time

    t0 = time.monotonic()

    async def one(stream):
        if stream:
            chunks = [c async for c in await client.create_streaming(None, _kill_request(True))]
            agg = chunks[0].clone()
            for c in chunks[1:]:
                agg.push(c)
            return S.ScoreCompletion.from_chunk(agg)
        return await client.create_unary(None, _kill_request())

    def voters(out):
        def kind(e):
            if e is None:
                return None
            m = e.message
            err = m.get("error") if isinstance(m, dict) else None
            return err.get("kind") if isinstance(err, dict) else (m.get("kind") if isinstance(m, dict) else e.code)

        return sorted((c.model_index, c.finish_reason, kind(c.error)) for c in out.choices if c.index >= 3)

    inflight = await asyncio.gather(*(one(k % 2 == 1) for k in range(4)))
    t_inflight = time.monotonic() - t0
    later = [await one(False), await one(True)]
    return {"inflight": [voters(o) for o in inflight], "later": [voters(o) for o in later],
            "t_inflight": t_inflight, "t_total": time.monotonic() - t0, "live": client.link.live(),
            "conf": [sum(c.confidence for c in o.choices if c.index < 3) for o in inflight + later]}


@pytest.mark.timeout(240)
def test_killed_follower_isolated_as_error_choices():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_leader_worker, args=(r, 4, port, q, "kill")) for r in range(4)]
    for p in procs:
        p.start()
    got = {}
    for _ in range(3):  # rank 3 dies and reports nothing
        r, v = q.get(timeout=200)
        got[r] = v
    for p in procs:
        p.join(timeout=60)
    assert procs[3].exitcode == 17
    g = got[0]
    assert isinstance(g, dict), g
    assert g["live"] == [1, 2]
    # voters of rank 3 (voter i -> live[i % 4] at the time: i = 3, 7) in the in-flight requests: error choices
    # of kind voter_shard_lost; every other voter finished normally
    lost_any = False
    for vs in g["inflight"]:
        assert len(vs) == len(KILL_LLMS)
        for mi, fr, err in vs:
            if mi % 4 == 3 and err == "voter_shard_lost":
                assert fr == "error"
                lost_any = True
            else:
                assert err is None and fr in ("stop", None), (mi, fr, err)
    assert lost_any
    for vs in g["later"]:  # after the death: the survivors run every voter
        assert len(vs) == len(KILL_LLMS) and all(err is None for _, _, err in vs), vs
    assert all(c == pytest.approx(1.0) for c in g["conf"])
    assert g["t_total"] < 60  # bounded by the link's failure detection, not a 600 s process-group timeout
    assert got[1] >= 4 and got[2] >= 4


async def _rejoin(client):
    """In-flight requests while rank 2 dies; wait (bounded) for the restarted rank 2 to re-join; later
    requests use it again and every voter of them finishes."""
    import time

    first = await _kill(client)
    t0 = time.monotonic()
    while client.link.live() != [1, 2] and time.monotonic() - t0 < 90:
        await asyncio.sleep(0.1)
    t_rejoin = time.monotonic() - t0
    live = client.link.live()
    later = [await client.create_unary(None, _kill_request()) for _ in range(3)]
    return {"first_live": first["live"], "live": live, "t_rejoin": t_rejoin,
            "later_errors": [sum(c.error is not None for c in o.choices) for o in later],
            "later_n": [sum(c.index >= 3 for c in o.choices) for o in later]}


SCENARIOS = {"equiv": _equiv, "kill": _kill, "rejoin": _rejoin}


class _FakeLink:
    """LinkServer stand-in: one live follower (rank 1), sends recorded."""

    def __init__(self):
        self.sent = []
        self.on_message = self.on_dead = None

    def live(self):
        return [1]

    def send(self, rank, msg):
        self.sent.append((rank, msg))
        return True


def test_release_drops_a_share_whose_stream_never_ran():
    """ADVICE r3 (the pattern, on the new links): a follower share whose stream was cancelled before it ever
    ran never runs its own ``finally``; the request's ``_release`` (called from the stream's ``finally`` in
    ScoreClient._stream) drops the share and tells its follower to stop."""
    from llm_weighted_consensus_amd.score.sharded import ShardedScoreClient

    link = _FakeLink()
    client = ShardedScoreClient(FakeChatClient(_policy), link, world=2, rng_seed=1)

    async def main():
        client.hub.open(7, {1: [0, 2]})
        assert 7 in client.hub.shares
        client._release({"seq": 7})
        assert 7 not in client.hub.shares
        assert link.sent == [(1, ("cancel", 7))]
        client._release({"seq": 7})  # idempotent: nothing left to drop
        assert link.sent == [(1, ("cancel", 7))]

    asyncio.run(main())


@pytest.mark.timeout(300)
def test_restarted_follower_rejoins_and_serves(tmp_path):
    """Recovery: a follower dies mid-load (its voters become error choices), a restarted
    process re-joins the running leader through the join file, live() returns to full size and later
    requests run voters on it again."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    join_file = str(tmp_path / "links.json")
    procs = [ctx.Process(target=_leader_worker, args=(r, 3, port, q, "rejoin", join_file)) for r in range(3)]
    for p in procs:
        p.start()
    procs[2].join(timeout=200)
    assert procs[2].exitcode == 17  # died mid-load
    back = ctx.Process(target=_rejoin_worker, args=(2, join_file, q))
    back.start()
    got = {}
    for _ in range(3):  # leader, rank 1, the re-joined rank 2
        r, v = q.get(timeout=200)
        got[r] = v
    for p in procs[:2] + [back]:
        p.join(timeout=60)
    g = got[0]
    assert isinstance(g, dict), g
    assert g["first_live"] == [1] and g["live"] == [1, 2]
    assert g["t_rejoin"] < 60
    assert g["later_errors"] == [0, 0, 0] and all(n == len(KILL_LLMS) for n in g["later_n"])
    assert got[2][0] == "rejoined" and got[2][1] >= 3  # the replacement ran voters of every later request


def test_timed_out_follower_is_told_to_cancel(monkeypatch):
    """a live follower that never answers its share (slow, wedged) is given up after
    LWC_SHARD_WAIT_S — its voters become error choices and the request completes — and the leader sends it
    ("cancel", seq) so its voters stop using its GPU."""
    from llm_weighted_consensus_amd.score.sharded import ShardedScoreClient

    monkeypatch.setenv("LWC_SHARD_WAIT_S", "0.3")
    link = _FakeLink()  # rank 1 live, never replies
    client = ShardedScoreClient(FakeChatClient(_policy), link, world=2, rng_seed=1)

    async def main():
        return await client.create_unary(None, _request("mixed"))

    out = asyncio.run(main())
    scores = [m for m in link.sent if m[1][0] == "score"]
    assert scores and all(r == 1 for r, _ in scores)
    seq = scores[0][1][1]
    assert (1, ("cancel", seq)) in link.sent
    errs = [c for c in out.choices if c.error is not None]
    assert errs and any("timed out" in str(c.error) for c in errs)
    assert not client.hub.shares  # the share is closed
