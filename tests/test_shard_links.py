"""Shard links (parallel/shard_link.py) and the sharded clients' isolation paths, on the CPU:
authenticated hellos (a rogue or stalled connection is dropped, bring-up goes on), a restarted follower
re-joins and ``live()`` returns to full size, sends never block the caller on a follower that stopped
reading, a timed-out share / slice is cancelled on its follower, and a follower's failed consensus slice is
recomputed by the leader."""
import asyncio
import os
import socket
import struct
import threading
import time

import pytest
import torch

from llm_weighted_consensus_amd.chat.fake import FakeChatClient
from llm_weighted_consensus_amd.parallel.shard_link import LinkClient, LinkServer


def policy(req):  # never called: these tests drive the sharded paths directly
    return []


def _server(world=3, **kw):
    kw.setdefault("hb_s", 0.05)
    kw.setdefault("dead_s", 1.0)
    return LinkServer(world, "127.0.0.1", **kw)


def _join_all(srv, world):
    clients = {}

    def go(r):
        clients[r] = LinkClient(srv.address, r, srv.secret, hb_s=0.05, timeout=10)

    ts = [threading.Thread(target=go, args=(r,)) for r in range(1, world)]
    for t in ts:
        t.start()
    srv.accept_all(timeout=10)
    for t in ts:
        t.join(10)
    return clients


def _wait(pred, timeout=10.0):
    end = time.monotonic() + timeout
    while time.monotonic() < end:
        if pred():
            return True
        time.sleep(0.02)
    return pred()


def test_rogue_and_stalled_connections_do_not_stop_bring_up():
    srv = _server(world=3, handshake_s=0.5)
    try:
        # a rogue peer: a pickled payload instead of the answer to the challenge — never unpickled, dropped
        rogue = socket.create_connection(srv.address)
        rogue.recv(32)
        rogue.sendall(struct.pack("!I", 5) + b"\x80\x04K\x01.")
        # a stalled peer: connects, never answers
        stalled = socket.create_connection(srv.address)
        # a peer with a wrong secret
        with pytest.raises(ConnectionError):
            LinkClient(srv.address, 1, b"x" * 32, timeout=0.5)
        clients = _join_all(srv, 3)
        assert srv.live() == [1, 2]
        assert _wait(lambda: srv.rejected >= 3)
        assert rogue.recv(16) == b""  # closed by the leader
        stalled.close()
        rogue.close()
        # out-of-range rank and a duplicate of a live rank are refused too
        with pytest.raises(ConnectionError):
            LinkClient(srv.address, 7, srv.secret, timeout=0.5)
        with pytest.raises(ConnectionError):
            LinkClient(srv.address, 1, srv.secret, timeout=0.5)
        assert srv.live() == [1, 2]
        for c in clients.values():
            c.close()
    finally:
        srv.close()


def test_restarted_follower_rejoins(tmp_path):
    srv = _server(world=3)
    joined, died = [], []
    srv.on_join = joined.append
    srv.on_dead = died.append
    try:
        clients = _join_all(srv, 3)
        path = str(tmp_path / "link.json")
        srv.write_join_file(path)
        assert oct(os.stat(path).st_mode & 0o777) == "0o600"
        clients[1].close()  # the follower process "dies"
        assert _wait(lambda: srv.live() == [2])
        assert _wait(lambda: died == [1])
        t0 = time.monotonic()
        back = LinkClient.from_join_file(path, 1, hb_s=0.05, timeout=10)
        assert _wait(lambda: srv.live() == [1, 2])
        assert time.monotonic() - t0 < 5
        assert _wait(lambda: joined == [1]) and srv.joins == 1  # the callback runs just after registration
        # the re-joined link carries traffic both ways
        got = []
        srv.on_message = lambda r, m: got.append((r, m))
        assert srv.send(1, ("ping", 1))
        assert back.recv() == ("ping", 1)
        back.send(("pong", 1))
        assert _wait(lambda: got == [(1, ("pong", 1))])
        back.close()
        clients[2].close()
    finally:
        srv.close()


def test_send_never_blocks_on_a_follower_that_stopped_reading():
    srv = _server(world=3, dead_s=2.0)
    try:
        clients = _join_all(srv, 3)
        big = ("chunk", 0, b"x" * (4 << 20))
        worst = 0.0
        for _ in range(64):  # 256 MiB at a peer that never reads: far past every socket buffer
            t0 = time.perf_counter()
            srv.send(1, big)
            worst = max(worst, time.perf_counter() - t0)
        assert worst < 0.1
        # the other follower is served meanwhile
        t0 = time.perf_counter()
        assert srv.send(2, ("ping",))
        assert clients[2].recv() == ("ping",)
        assert time.perf_counter() - t0 < 0.1
        # the stuck sender times out after dead_s and declares its rank dead
        assert _wait(lambda: srv.live() == [2], timeout=15)
        for c in clients.values():
            c.close()
    finally:
        srv.close()


class _FakeLink:
    def __init__(self, ranks=(1,), on_send=None):
        self.sent = []
        self.ranks = list(ranks)
        self.on_message = self.on_dead = None
        self.on_send = on_send

    def live(self):
        return list(self.ranks)

    def send(self, rank, msg):
        self.sent.append((rank, msg))
        if self.on_send is not None:
            self.on_send(rank, msg)
        return True


def test_timed_out_share_is_cancelled_on_its_follower(monkeypatch):
    """a share that outlives its bound becomes error choices AND its follower is told to stop."""
    from llm_weighted_consensus_amd.score.orchestrator import ChoiceIndexer
    from llm_weighted_consensus_amd.score.sharded import ShardedScoreClient

    monkeypatch.setenv("LWC_SHARD_WAIT_S", "0.2")
    link = _FakeLink()
    client = ShardedScoreClient(FakeChatClient(policy), link, world=2, rng_seed=1)

    class _L:
        def __init__(self, i):
            self.index, self.id = i, f"llm{i}"

    class _M:
        id = "m"
        llms = [_L(0), _L(1)]

    async def main():
        share = client.hub.open(5, {1: [0, 1]})
        out = []
        async for ch in client._remote({"seq": 5}, share, {1: [0, 1]}, ChoiceIndexer(2), _M(), [1.0, 1.0], "rid", 0):
            out.append(ch)
        # late chunks of the given-up share are dropped, not merged into a finished voter
        return out

    out = asyncio.run(main())
    assert len(out) == 1 and all(c.finish_reason == "error" for c in out[0].choices)
    assert (1, ("cancel", 5)) in link.sent
    assert 5 not in client.hub.shares


def test_failed_consensus_slice_is_recomputed_locally():
    """a follower that replies "failed" to its consensus slice is isolated like a dead one."""
    from llm_weighted_consensus_amd.schema import chat as C
    from llm_weighted_consensus_amd.score.sharded import ShardedConsensusClient, ShardedScoreClient

    calls = []

    class _Base:
        archive = None

        def _check_n(self, request):
            pass

        def _embedder(self, name):
            class E:
                class encoder:
                    device = torch.device("cpu")
            return E

        async def generate_embedded(self, ctx, request, embedding_model):
            first, cnt, _ = ctx["candidates"]
            calls.append((first, cnt))
            comp = C.ChatCompletion.model_validate({
                "id": "x", "created": 0, "model": "m", "object": "chat.completion",
                "choices": [{"index": first + i, "finish_reason": "stop",
                             "message": {"role": "assistant", "content": f"c{first + i}"}} for i in range(cnt)]})
            return comp, torch.full((cnt, 4), float(first)), cnt

        def build(self, merged, rows, ntok, embedding_model, tau):
            return type("Out", (), {"rows": rows, "choices": merged.choices, "id": None, "created": None})()

    holder = {}

    def on_send(rank, msg):
        if msg[0] == "consensus":  # the follower answers at once: generation failed
            holder["sc"].hub._on_message(rank, ("cons", msg[1], (False, 0, 0, "OutOfMemoryError: boom", 0), b""))

    link = _FakeLink(on_send=on_send)
    sc = ShardedScoreClient(FakeChatClient(policy), link, world=2, rng_seed=1)
    holder["sc"] = sc
    cc = ShardedConsensusClient(_Base(), sc)
    req = C.ChatCompletionCreateParams.model_validate({"model": "m", "messages": [{"role": "user", "content": "q"}],
                                                        "n": 4})
    out = asyncio.run(cc.create_unary({}, req, "emb"))
    assert sorted(calls) == [(0, 2), (2, 2)]  # the follower's slice [2, 4) ran on the leader
    assert [c.index for c in out.choices] == [0, 1, 2, 3]
    assert out.rows[2:].eq(2.0).all()


def test_link_host_defaults(monkeypatch):
    """The leader's listen address: loopback for a one-node world, MASTER_ADDR across nodes, an explicit
    LWC_SHARD_LINK_HOST always; a multi-node world with only a loopback MASTER_ADDR fails fast."""
    import pytest

    from llm_weighted_consensus_amd.parallel.shard_link import link_host

    for k in ("LWC_SHARD_LINK_HOST", "WORLD_SIZE", "LOCAL_WORLD_SIZE", "MASTER_ADDR"):
        monkeypatch.delenv(k, raising=False)
    assert link_host() == "127.0.0.1"
    monkeypatch.setenv("WORLD_SIZE", "8")
    monkeypatch.setenv("LOCAL_WORLD_SIZE", "8")
    monkeypatch.setenv("MASTER_ADDR", "10.0.0.5")
    assert link_host() == "127.0.0.1"
    monkeypatch.setenv("WORLD_SIZE", "16")
    assert link_host() == "10.0.0.5"
    monkeypatch.setenv("MASTER_ADDR", "127.0.0.1")
    with pytest.raises(RuntimeError, match="LWC_SHARD_LINK_HOST"):
        link_host()
    monkeypatch.setenv("LWC_SHARD_LINK_HOST", "10.0.0.9")
    assert link_host() == "10.0.0.9"
