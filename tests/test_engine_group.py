"""EngineGroup (CPU, fake engines in spawned worker processes): candidate routing across workers with
global choice indices and split-independent seeds; a killed worker's not-yet-started portions are
rescheduled on a survivor, started ones fail with EngineFailure; abort and close."""
import asyncio
import os
import signal
import time

import pytest

from llm_weighted_consensus_amd.engine.group import EngineGroup
from llm_weighted_consensus_amd.engine.sampling import SamplingParams
from llm_weighted_consensus_amd.engine.service import EngineFailure

FACTORY = "tests.fake_engine:make"


def _collect(group, n, params, timeout=120):
    async def go():
        loop = asyncio.get_running_loop()
        q = asyncio.Queue()
        group.submit([1, 2, 3], params, n, loop, q)
        toks = {i: [] for i in range(n)}
        done = 0
        while done < n:
            ev = await asyncio.wait_for(q.get(), timeout)
            if isinstance(ev, EngineFailure):
                return toks, ev
            toks[ev.seq.index].append(ev.token_id)
            done += ev.finished
        return toks, None

    return asyncio.run(go())


def test_group_splits_candidates_and_keeps_seeds():
    g = EngineGroup({"delay": 0.0}, devices=[0, 0, 0], factory=FACTORY)
    try:
        sp = SamplingParams(max_tokens=4, seed=42)
        toks, err = _collect(g, 7, sp)
        assert err is None and sorted(toks) == list(range(7))
        for i, t in toks.items():  # candidate i used seed 42*1000003 + i regardless of its worker
            s = 42 * 1000003 + i
            assert t == [(s + k) % 1000 for k in range(4)]
        assert g.load == 0
    finally:
        g.close()


def test_group_worker_death_reschedules_or_fails():
    # death is detected from the process exit; a long heartbeat timeout keeps a loaded CI host from
    # declaring the SURVIVOR dead too
    g = EngineGroup({"delay": 0.05}, devices=[0, 0], factory=FACTORY, heartbeat_timeout=60, respawn=False)
    try:
        sp = SamplingParams(max_tokens=50, seed=1)
        victim = g.procs[0]

        async def go():
            loop = asyncio.get_running_loop()
            q = asyncio.Queue()
            g.submit([1], sp, 4, loop, q)
            # kill worker 0 only once ITS portion (choices 0-1 of 4) has started streaming: an unstarted
            # portion would be rescheduled instead of failing (a loaded host can start worker 1 first)
            while True:
                ev = await asyncio.wait_for(q.get(), 120)
                if not isinstance(ev, EngineFailure) and ev.seq.index < 2:
                    break
            os.kill(victim.pid, signal.SIGKILL)
            while True:
                ev = await asyncio.wait_for(q.get(), 120)
                if isinstance(ev, EngineFailure):
                    return ev

        ev = asyncio.run(go())
        assert "engine worker 0" in ev.message
        assert g.alive == [False, True]
        # new requests go to the survivor only
        toks, err = _collect(g, 3, SamplingParams(max_tokens=3, seed=5))
        assert err is None and len(toks) == 3
    finally:
        g.close()


def test_workers_embed_their_own_candidates():
    """/consensus over an EngineGroup: each worker embeds the candidates it generated (here a CPU BERT in
    each fake-engine worker); the front end receives unit rows in candidate order equal to embedding the
    streamed texts locally."""
    import torch

    from llm_weighted_consensus_amd.embeddings.service import build_embedding_service

    espec = {"arch": "bert-tiny", "weights": "random:1"}
    g = EngineGroup({"delay": 0.0, "embed_models": {"e": espec}, "embed_device": "cpu"}, devices=[0, 0],
                    factory=FACTORY)
    try:
        assert g.embeds_in_workers("e") and not g.embeds_in_workers("other")

        async def go():
            loop = asyncio.get_running_loop()
            q = asyncio.Queue()
            req = g.submit([1, 2, 3], SamplingParams(max_tokens=6, seed=9), 5, loop, q, embed="e")
            texts, done = {i: "" for i in range(5)}, 0
            while done < 5:
                ev = await asyncio.wait_for(q.get(), 120)
                texts[ev.seq.index] += ev.text
                done += ev.finished
            rows, ntok = await asyncio.wait_for(req.emb_future, 120)
            return texts, rows, ntok

        texts, rows, ntok = asyncio.run(go())
        assert rows.shape[0] == 5 and ntok > 0
        ref, _ = build_embedding_service("e", espec, "cpu").embed_texts([texts[i] for i in range(5)])
        assert torch.allclose(torch.from_numpy(rows), ref.float(), atol=1e-5)
        assert not g.emb_pending
    finally:
        g.close()


def test_tp_replicas_step_in_lockstep(tmp_path):
    """spec "tp": 2 over 4 devices = two replicas of two ranks; each follower replays its leader's ticks:
    both ranks of a replica step the same batches (the per-step logs are identical), only the leaders
    stream, and a killed follower takes its whole replica down (requests go to the other one)."""
    g = EngineGroup({"delay": 0.01, "tp": 2, "log_dir": str(tmp_path)}, devices=[0, 0, 0, 0], factory=FACTORY,
                    heartbeat_timeout=60, respawn=False)
    try:
        assert len(g.procs) == 2 and all(len(f) == 1 for f in g.followers)
        toks, err = _collect(g, 6, SamplingParams(max_tokens=5, seed=3))
        assert err is None and sorted(toks) == list(range(6))
        for i, t in toks.items():
            assert t == [(3 * 1000003 + i + k) % 1000 for k in range(5)]
        time.sleep(0.5)  # followers write their last step
        for w in range(2):
            lead = (tmp_path / f"w{w}_rank0.log").read_text()
            assert lead and lead == (tmp_path / f"w{w}_rank1.log").read_text()
        os.kill(g.followers[0][0][0].pid, signal.SIGKILL)
        deadline = time.time() + 60
        while g.alive[0] and time.time() < deadline:
            time.sleep(0.1)
        assert g.alive == [False, True]
        g.procs[0].join(timeout=10)
        assert not g.procs[0].is_alive()  # the leader of the broken replica is taken down with it
        toks, err = _collect(g, 3, SamplingParams(max_tokens=3, seed=5))
        assert err is None and len(toks) == 3
    finally:
        g.close()


def _wait_live(g, n, timeout=120):
    deadline = time.time() + timeout
    while len(g.live_workers()) < n and time.time() < deadline:
        time.sleep(0.05)
    return g.live_workers()


def test_dead_worker_is_respawned_and_serves_again():
    """Recovery: a worker killed mid-load is replaced by a fresh child process;
    live_workers() returns to full size within a bounded time and the replacement takes later requests."""
    g = EngineGroup({"delay": 0.02}, devices=[0, 0], factory=FACTORY, heartbeat_timeout=60, respawn_backoff_s=0.2)
    try:
        old_pid = g.procs[0].pid

        async def go():
            loop = asyncio.get_running_loop()
            q = asyncio.Queue()
            g.submit([1], SamplingParams(max_tokens=40, seed=1), 4, loop, q)
            while True:  # mid-load: worker 0 is streaming
                ev = await asyncio.wait_for(q.get(), 120)
                if not isinstance(ev, EngineFailure) and ev.seq.index < 2:
                    break
            os.kill(old_pid, signal.SIGKILL)
            while True:
                ev = await asyncio.wait_for(q.get(), 120)
                if isinstance(ev, EngineFailure):
                    return ev

        ev = asyncio.run(go())
        assert "engine worker 0" in ev.message
        t0 = time.time()
        assert _wait_live(g, 2) == [0, 1]
        assert time.time() - t0 < 60
        # generation: +1 when the slot is fenced at death, +1 for the replacement
        assert g.procs[0].pid != old_pid and g.gen[0] == 2 and g.respawns[0] == 1
        # the replacement serves: a request split over both workers completes with the usual seeds
        sp = SamplingParams(max_tokens=3, seed=8)
        toks, err = _collect(g, 6, sp)
        assert err is None and sorted(toks) == list(range(6))
        for i, t in toks.items():
            assert t == [(8 * 1000003 + i + k) % 1000 for k in range(3)]
        assert g.load == 0
    finally:
        g.close()


def test_tp_replica_is_rebuilt_as_new_processes(tmp_path):
    """A TP replica whose follower died is torn down as a unit and rebuilt (new leader + follower on a fresh
    rendezvous port); both replicas serve afterwards."""
    g = EngineGroup({"delay": 0.01, "tp": 2, "log_dir": str(tmp_path)}, devices=[0, 0, 0, 0], factory=FACTORY,
                    heartbeat_timeout=60, respawn_backoff_s=0.2)
    try:
        old = (g.procs[0].pid, g.followers[0][0][0].pid)
        os.kill(old[1], signal.SIGKILL)
        deadline = time.time() + 60
        while g.gen[0] == 0 and time.time() < deadline:
            time.sleep(0.05)
        assert _wait_live(g, 2) == [0, 1]
        assert g.procs[0].pid not in old and g.followers[0][0][0].pid not in old
        toks, err = _collect(g, 6, SamplingParams(max_tokens=4, seed=2))
        assert err is None and sorted(toks) == list(range(6))
    finally:
        g.close()


def test_respawn_is_bounded():
    """A worker that keeps dying is replaced at most max_respawns times (with backoff), then stays dead."""
    g = EngineGroup({"delay": 0.0}, devices=[0, 0], factory=FACTORY, heartbeat_timeout=60, respawn_backoff_s=0.05,
                    max_respawns=2)
    try:
        for _ in range(3):
            _wait_live(g, 2, timeout=60)
            gen = g.gen[0]
            os.kill(g.procs[0].pid, signal.SIGKILL)
            deadline = time.time() + 60
            while g.alive[0] and time.time() < deadline:
                g._check_health()
                time.sleep(0.05)
            if g.respawns[0] < 2:
                while g.gen[0] == gen and time.time() < deadline:
                    time.sleep(0.05)
        time.sleep(1.0)
        assert g.respawns[0] == 2 and not g.alive[0] and g.live_workers() == [1]
    finally:
        g.close()


def test_worker_declared_dead_is_fenced_and_killed():
    """A worker declared dead while its process still runs (a heartbeat timeout on a hung, not exited, process)
    is fenced at once: its slot's generation moves on, so late messages of the old process are dropped by the
    reader, and the process is killed — also with respawning off, where no replacement ever bumps the
    generation (a recovering hung worker could fail requests already moved to a survivor)."""
    g = EngineGroup({"delay": 0.0}, devices=[0, 0], factory=FACTORY, heartbeat_timeout=60, respawn=False)
    try:
        victim = g.procs[0]
        gen0 = g.gen[0]
        assert victim.is_alive()
        g._worker_died(0, "heartbeat timeout")
        assert g.gen[0] == gen0 + 1 and not g.alive[0]
        victim.join(timeout=30)
        assert not victim.is_alive()
        # the survivor still serves every candidate
        toks, err = _collect(g, 4, SamplingParams(max_tokens=2, seed=3))
        assert err is None and sorted(toks) == list(range(4))
    finally:
        g.close()
