"""Shared-memory SPSC ring of the EngineGroup token stream (engine/shm_ring.py): record round trips,
wrap-around, a full ring blocking the producer, and a producer in another process."""
import multiprocessing as mp
import random

import pytest

from llm_weighted_consensus_amd.engine.shm_ring import ShmRing, decode_events, encode_events


def _events(seed, n):
    rnd = random.Random(seed)
    out = []
    for i in range(n):
        top = [(rnd.randrange(128256), -rnd.random() * 5) for _ in range(rnd.choice([0, 1, 5, 20]))]
        text = rnd.choice(["", "a", "café ✓", " w1x2", "`A`\n"]) * rnd.randrange(3)
        out.append((rnd.randrange(1 << 40), i, rnd.randrange(128256), text, -rnd.random(), top, rnd.random() < 0.1,
                    rnd.choice([None, "stop", "length", "abort", "error"])))
    return out


def _same(a, b):
    assert len(a) == len(b)
    for x, y in zip(a, b):
        assert x[:4] == y[:4] and x[6:] == y[6:]
        assert abs(x[4] - y[4]) < 1e-6
        assert [t for t, _ in x[5]] == [t for t, _ in y[5]]
        assert all(abs(p - q) < 1e-6 for (_, p), (_, q) in zip(x[5], y[5]))


def test_encode_decode_round_trip():
    for n in (0, 1, 7, 500):
        ev = _events(n, n)
        _same(decode_events(encode_events(ev)), ev)


def test_ring_wraps_and_preserves_order():
    r = ShmRing(cap=4096)
    try:
        sent = []
        for i in range(300):
            payload = bytes([i % 251]) * (1 + (i * 37) % 900)
            assert r.push(payload, timeout=0.1) or r.pop() is not None
            sent.append(payload)
            if i % 3 == 2:  # the consumer lags: the ring runs near full and wraps
                while (x := r.pop()) is not None:
                    assert x == sent.pop(0)
        while (x := r.pop()) is not None:
            assert x == sent.pop(0)
        assert not sent
    finally:
        r.close()


def test_full_ring_times_out_and_oversized_records_refused():
    r = ShmRing(cap=1024)
    try:
        assert r.push(b"x" * 400)
        assert not r.push(b"y" * 400, timeout=0.05) or not r.push(b"z" * 400, timeout=0.05)
        with pytest.raises(ValueError):
            r.push(b"q" * 600)
    finally:
        r.close()


def _producer(name, n):
    r = ShmRing(name, create=False)
    for i in range(n):
        assert r.push(encode_events(_events(i, 1 + i % 40)), timeout=30)
    r.shm.close()


def test_cross_process_producer():
    r = ShmRing(cap=64 << 10)
    try:
        n = 400
        p = mp.get_context("spawn").Process(target=_producer, args=(r.name, n))
        p.start()
        got = 0
        import time

        deadline = time.time() + 120
        while got < n and time.time() < deadline:
            rec = r.pop()
            if rec is None:
                time.sleep(0.0005)
                continue
            _same(decode_events(rec), _events(got, 1 + got % 40))
            got += 1
        p.join(timeout=30)
        assert got == n and p.exitcode == 0
    finally:
        r.close()


def test_embedding_record_roundtrip_and_kinds():
    """A worker's embedding rows travel as one raw float32 record; the reader tells the kinds apart."""
    import numpy as np

    from llm_weighted_consensus_amd.engine.shm_ring import decode_record, encode_embeddings

    rows = np.random.default_rng(0).standard_normal((5, 1024)).astype(np.float32)
    kind, (rid, off, got, ntok) = decode_record(encode_embeddings(77, 3, rows, 1234))
    assert kind == "emb" and (rid, off, ntok) == (77, 3, 1234) and np.array_equal(got, rows)
    ev = _events(1, 3)
    kind, got_ev = decode_record(encode_events(ev))
    assert kind == "tokens"
    _same(got_ev, ev)
