"""K10b batched vote tally: the GPU kernel against the host C++ tally (bitwise: same fp64 summation order),
and the event-loop batcher (CPU: host path and batching logic; GPU: one launch for concurrent requests)."""
import asyncio
import math
import random

import pytest

from llm_weighted_consensus_amd import _runtime as RT
from llm_weighted_consensus_amd.score import tally_batch as TB


class _Delta:
    def __init__(self, vote):
        self.vote = vote


class _Choice:
    def __init__(self, vote, weight):
        self.delta = _Delta(vote)
        self.weight = weight


def _request(rng, C, L):
    choices = []
    for _ in range(L):
        if rng.random() < 0.2:
            choices.append(_Choice(None, rng.random()))  # errored voter: no vote
            continue
        v = [rng.random() for _ in range(C)]
        if rng.random() < 0.5:  # one-hot
            v = [0.0] * C
            v[rng.randrange(C)] = 1.0
        s = sum(v)
        choices.append(_Choice([x / s for x in v], rng.choice([None, rng.uniform(0.1, 5.0)])))
    return choices


def _same(a, b):
    for x, y in zip(a, b):
        assert (math.isnan(x) and math.isnan(y)) or x == y, (x, y)
    assert len(a) == len(b)


def test_batcher_host_path_matches_native():
    rng = random.Random(0)
    reqs = [(_request(rng, C, L), C) for C, L in [(2, 3), (5, 8), (3, 1), (7, 16)]]

    async def main():
        b = TB.TallyBatcher(device=None, min_batch=1)
        return b, await asyncio.gather(*(b.tally(ch, C) for ch, C in reqs))

    b, outs = asyncio.run(main())
    assert b.gpu_batches == 0
    for (ch, C), t in zip(reqs, outs):
        votes, wts = TB.vote_rows(ch)
        r = RT.tally(votes, wts, C)
        _same(t.choice_weight, r.choice_weight)
        _same(t.voter_confidence, r.voter_confidence)


def test_batcher_groups_one_turn(monkeypatch):
    """Tallies submitted in the same event-loop turn form one batch; the batch goes to the GPU path when it
    reaches min_batch (here a host stand-in for the kernel, to check the packing and unpacking)."""
    calls = []

    def fake_gpu(items, device, stream=None):
        calls.append(len(items))
        out = []
        for votes, wts, C in items:
            r = RT.tally(votes, wts, C)
            out.append(TB.Tally(list(r.choice_weight), list(r.confidence), list(r.voter_confidence)))
        return out

    monkeypatch.setattr(TB, "tally_many_gpu", fake_gpu)
    import torch

    monkeypatch.setattr(torch.cuda, "Stream", lambda device=None: None)  # no device here
    rng = random.Random(1)
    reqs = [(_request(rng, 4, 6), 4) for _ in range(5)]

    async def main():
        b = TB.TallyBatcher(device="fake", min_batch=3)
        res = await asyncio.gather(*(b.tally(ch, C) for ch, C in reqs))
        small = await asyncio.gather(*(b.tally(ch, C) for ch, C in reqs[:2]))  # below min_batch: host
        return b, res, small

    b, res, small = asyncio.run(main())
    assert calls == [5] and b.gpu_batches == 1 and b.gpu_tallies == 5
    assert len(res) == 5 and len(small) == 2


def test_batcher_device_error_falls_back_to_host(monkeypatch):
    """A failing GPU batch (device error) must not strand the awaiting requests: they get the host tally."""
    def broken(items, device, stream=None):
        raise RuntimeError("HIP error")

    monkeypatch.setattr(TB, "tally_many_gpu", broken)
    import torch

    monkeypatch.setattr(torch.cuda, "Stream", lambda device=None: None)
    rng = random.Random(4)
    reqs = [(_request(rng, 3, 5), 3) for _ in range(4)]

    async def main():
        b = TB.TallyBatcher(device="fake", min_batch=2)
        return b, await asyncio.wait_for(asyncio.gather(*(b.tally(ch, C) for ch, C in reqs)), 10)

    b, outs = asyncio.run(main())
    assert b.gpu_batches == 0
    for (ch, C), t in zip(reqs, outs):
        votes, wts = TB.vote_rows(ch)
        _same(t.choice_weight, RT.tally(votes, wts, C).choice_weight)


def test_batcher_survives_a_closed_loop():
    """A flush left scheduled on an event loop that closed (server restart, a test's asyncio.run) must not
    wedge the batcher: the next loop schedules its own."""
    rng = random.Random(5)
    b = TB.TallyBatcher(device=None, min_batch=1)
    loop = asyncio.new_event_loop()
    fut = loop.create_future()
    b._pending.append(([], [], 2, fut))
    b._scheduled, b._sched_loop = True, loop  # as if tally() ran there and the loop closed before flushing
    loop.close()
    ch = _request(rng, 3, 4)

    async def main():
        return await asyncio.wait_for(b.tally(ch, 3), 5)

    t = asyncio.run(main())
    votes, wts = TB.vote_rows(ch)
    _same(t.choice_weight, RT.tally(votes, wts, 3).choice_weight)


def test_make_batcher_spec():
    assert TB.make_batcher(None, "cuda:0") is None
    assert TB.make_batcher("0", "cuda:0") is None
    b = TB.make_batcher("4", "cuda:0")
    assert b.min_batch == 4 and b.device == "cuda:0"


@pytest.mark.gpu
def test_vote_tally_kernel_bitwise(gpu):
    rng = random.Random(2)
    items = []
    for C, L in [(2, 1), (3, 7), (20, 128), (5, 0), (64, 40), (300, 9), (1, 3)]:
        votes, wts = TB.vote_rows(_request(rng, C, L))
        items.append((votes, wts, C))
    got = TB.tally_many_gpu(items, gpu)
    for (votes, wts, C), t in zip(items, got):
        r = RT.tally(votes, wts, C)
        _same(t.choice_weight, r.choice_weight)
        _same(t.confidence, r.confidence)
        _same(t.voter_confidence, r.voter_confidence)


@pytest.mark.gpu
def test_vote_tally_batcher_gpu(gpu):
    rng = random.Random(3)
    reqs = [(_request(rng, C, 8), C) for C in (2, 3, 4, 5, 6, 7, 8, 9)]

    async def main():
        b = TB.TallyBatcher(device=gpu, min_batch=4)
        return b, await asyncio.gather(*(b.tally(ch, C) for ch, C in reqs))

    b, outs = asyncio.run(main())
    assert b.gpu_batches == 1 and b.gpu_tallies == len(reqs)
    for (ch, C), t in zip(reqs, outs):
        votes, wts = TB.vote_rows(ch)
        r = RT.tally(votes, wts, C)
        _same(t.choice_weight, r.choice_weight)
        _same(t.voter_confidence, r.voter_confidence)


def test_server_wiring(monkeypatch):
    """LWC_GPU_TALLY reaches the score client; with no local engine and no setting the host tally stays
    (no GPU context is opened by the front end); a CPU deployment never batches."""
    from llm_weighted_consensus_amd.server.config import Config
    from llm_weighted_consensus_amd.server.main import build_state

    monkeypatch.setenv("LWC_GPU_TALLY", "4")
    cfg = Config.from_env(dotenv=False)
    assert cfg.gpu_tally == "4"
    st = build_state(cfg)
    assert st.score.tally_batcher is not None and st.score.tally_batcher.min_batch == 4
    assert build_state(Config()).score.tally_batcher is None
    assert build_state(Config(device="cpu", gpu_tally="4")).score.tally_batcher is None


def test_batcher_fails_only_the_malformed_request(monkeypatch):
    """one malformed vote (wrong length) fails its own request; the rest of the batch is tallied
    (here on the host path: device None)."""
    rng = random.Random(5)
    good = [(_request(rng, 3, 4), 3) for _ in range(3)]
    bad_ch, _ = _request(rng, 3, 4), 3

    async def main():
        b = TB.TallyBatcher(device=None, min_batch=2)
        bad = [_Choice([1.0, 0.0], 1.0)] + list(bad_ch[1:])  # 2 entries for 3 choices
        return await asyncio.gather(*([b.tally(ch, C) for ch, C in good] + [b.tally(bad, 3)]),
                                    return_exceptions=True)

    outs = asyncio.run(main())
    assert isinstance(outs[-1], ValueError)
    for (ch, C), t in zip(good, outs[:-1]):
        votes, wts = TB.vote_rows(ch)
        assert list(t.confidence) == list(RT.tally(votes, wts, C).confidence)
