"""Shared-memory single-producer / single-consumer ring for the EngineGroup's token stream.

Round 1 shipped every engine step's token events from a worker process to the front end as one pickled
list through a ``multiprocessing.Queue`` (a feeder thread, a pipe write and an unpickle of thousands of
tuples per step).  Here a worker packs a step into ONE binary record — fixed-width columns as numpy
arrays plus a UTF-8 text blob — and copies it into a ring in POSIX shared memory; the front end's reader
copies it out and rebuilds the events.  No pickling, no pipe, no feeder thread on the hot path; the
queue remains for rare control messages (ready / fatal / error).

Ring layout (one per worker): [head u64][tail u64][pad to 64 B][data: cap bytes].  ``head`` (bytes
written) is stored only by the producer, ``tail`` (bytes consumed) only by the consumer; each is an
aligned 8-byte store, and a record's bytes are written before ``head`` moves past them (x86-64 keeps
store order), so the consumer never sees a torn record.  A record is [len u32][payload], padded to 8
bytes; a len of 0xFFFFFFFF marks "wrap to the start".  Payloads start with a kind word: one engine step's
token events, or the unit embedding rows of a request portion the worker embedded (a /consensus request's
candidates), raw float32.

The reference has no counterpart (its voters are remote HTTP streams): this is the transport of the
multi-GPU candidate fan-out (src/score/completions/client.rs:343-356) inside one node.
"""
from __future__ import annotations

import time
from multiprocessing import shared_memory
from typing import List, Optional, Sequence, Tuple

import numpy as np

_WRAP = 0xFFFFFFFF
_HDR = 64

REASONS = (None, "stop", "length", "abort", "error")
_REASON_CODE = {r: i for i, r in enumerate(REASONS)}

EVENT_DTYPE = np.dtype([("rid", "<i8"), ("idx", "<i4"), ("tid", "<i4"), ("lp", "<f4"), ("tlen", "<u4"),
                        ("fin", "u1"), ("reason", "u1"), ("ntop", "u1"), ("pad", "u1")])


class ShmRing:
    def __init__(self, name: Optional[str] = None, cap: int = 32 << 20, create: bool = True):
        cap = (cap + 7) // 8 * 8
        if create:
            self.shm = shared_memory.SharedMemory(name=name, create=True, size=_HDR + cap)
            self.shm.buf[:_HDR] = bytes(_HDR)
        else:
            self.shm = shared_memory.SharedMemory(name=name, create=False)
            cap = self.shm.size - _HDR
        self.cap = cap
        self.owner = create
        self._hdr = np.ndarray((2,), dtype=np.uint64, buffer=self.shm.buf, offset=0)
        self._data = np.ndarray((cap,), dtype=np.uint8, buffer=self.shm.buf, offset=_HDR)

    @property
    def name(self) -> str:
        return self.shm.name

    # ---- producer
    def push(self, payload, timeout: float = 30.0, on_wait=None) -> bool:
        """Append one record (blocks while the ring is full, up to ``timeout`` s; False on timeout).
        ``on_wait`` is called about every 50 ms while waiting (the worker refreshes its heartbeat: a slow
        reader is not a dead worker)."""
        mv = memoryview(payload).cast("B")
        n = len(mv)
        need = (4 + n + 7) // 8 * 8
        if need > self.cap // 2:
            raise ValueError(f"record of {n} bytes exceeds half the ring ({self.cap})")
        deadline = None
        while True:
            head, tail = int(self._hdr[0]), int(self._hdr[1])
            free = self.cap - (head - tail)
            pos = head % self.cap
            room = self.cap - pos
            if need > room:  # not contiguous: mark the rest of the ring as skipped and wrap
                if free >= room + need:
                    self._data[pos:pos + 4] = np.frombuffer(np.uint32(_WRAP).tobytes(), np.uint8)
                    self._hdr[0] = head + room
                    continue
            elif free >= need:
                self._data[pos:pos + 4] = np.frombuffer(np.uint32(n).tobytes(), np.uint8)
                self._data[pos + 4:pos + 4 + n] = np.frombuffer(mv, np.uint8)
                self._hdr[0] = head + need  # publish after the bytes
                return True
            now = time.monotonic()
            if deadline is None:
                deadline, beat = now + timeout, now
            elif now > deadline:
                return False
            if on_wait is not None and now - beat > 0.05:
                on_wait()
                beat = now
            time.sleep(0.0002)

    # ---- consumer
    def pop(self) -> Optional[bytes]:
        if self._hdr is None:  # closed
            return None
        while True:
            head, tail = int(self._hdr[0]), int(self._hdr[1])
            if head == tail:
                return None
            pos = tail % self.cap
            ln = int(self._data[pos:pos + 4].view(np.uint32)[0])
            if ln == _WRAP:
                self._hdr[1] = tail + (self.cap - pos)
                continue
            out = self._data[pos + 4:pos + 4 + ln].tobytes()
            self._hdr[1] = tail + (4 + ln + 7) // 8 * 8
            return out

    def close(self) -> None:
        self._hdr = self._data = None
        self.shm.close()
        if self.owner:
            try:
                self.shm.unlink()
            except FileNotFoundError:
                pass


# ---------------------------------------------------------------------------------------------
# one engine step's events <-> one record


KIND_EVENTS, KIND_EMB = 1, 2


def encode_embeddings(rid: int, offset: int, rows: np.ndarray, ntok: int) -> bytes:
    """A worker's unit embedding rows [n, d] float32 of one request portion as one record (no pickling)."""
    rows = np.ascontiguousarray(rows, dtype=np.float32)
    n, d = rows.shape
    head = np.array([KIND_EMB, n, d, 0], dtype=np.uint32)
    meta = np.array([rid, offset, ntok], dtype=np.int64)
    return b"".join((head.tobytes(), meta.tobytes(), rows.tobytes()))


def decode_record(buf: bytes):
    """("tokens", events) or ("emb", (rid, offset, rows [n, d] float32, ntok))."""
    kind = int(np.frombuffer(buf, dtype=np.uint32, count=1)[0])
    if kind == KIND_EMB:
        _, n, d, _ = np.frombuffer(buf, dtype=np.uint32, count=4).tolist()
        rid, offset, ntok = np.frombuffer(buf, dtype=np.int64, count=3, offset=16).tolist()
        rows = np.frombuffer(buf, dtype=np.float32, count=n * d, offset=40).reshape(n, d).copy()
        return "emb", (rid, offset, rows, ntok)
    return "tokens", decode_events(buf)


def encode_events(events: Sequence[tuple]) -> bytes:
    """events: (rid, idx, token_id, text, logprob, [(top_id, top_lp), ...], finished, reason)."""
    n = len(events)
    rec = np.zeros(n, dtype=EVENT_DTYPE)
    texts = [e[3].encode("utf-8") for e in events]
    tops = [e[5] for e in events]
    rec["rid"] = [e[0] for e in events]
    rec["idx"] = [e[1] for e in events]
    rec["tid"] = [e[2] for e in events]
    rec["lp"] = [e[4] for e in events]
    rec["tlen"] = [len(t) for t in texts]
    rec["fin"] = [1 if e[6] else 0 for e in events]
    rec["reason"] = [_REASON_CODE.get(e[7], 4) for e in events]
    rec["ntop"] = [len(t) for t in tops]
    flat = [x for t in tops for x in t]
    top_ids = np.array([x[0] for x in flat], dtype=np.int32)
    top_lps = np.array([x[1] for x in flat], dtype=np.float32)
    blob = b"".join(texts)
    head = np.array([KIND_EVENTS, n, len(flat), len(blob)], dtype=np.uint32)
    return b"".join((head.tobytes(), rec.tobytes(), top_ids.tobytes(), top_lps.tobytes(), blob))


def decode_events(buf: bytes) -> List[Tuple]:
    _, n, ntop, nblob = np.frombuffer(buf, dtype=np.uint32, count=4).tolist()
    off = 16
    rec = np.frombuffer(buf, dtype=EVENT_DTYPE, count=n, offset=off)
    off += n * EVENT_DTYPE.itemsize
    top_ids = np.frombuffer(buf, dtype=np.int32, count=ntop, offset=off).tolist()
    off += 4 * ntop
    top_lps = np.frombuffer(buf, dtype=np.float32, count=ntop, offset=off).tolist()
    off += 4 * ntop
    blob = buf[off:off + nblob]
    out = []
    t0 = k0 = 0
    for rid, idx, tid, lp, tlen, fin, reason, nt in zip(rec["rid"].tolist(), rec["idx"].tolist(), rec["tid"].tolist(),
                                                        rec["lp"].tolist(), rec["tlen"].tolist(), rec["fin"].tolist(),
                                                        rec["reason"].tolist(), rec["ntop"].tolist()):
        text = blob[t0:t0 + tlen].decode("utf-8")
        t0 += tlen
        top = list(zip(top_ids[k0:k0 + nt], top_lps[k0:k0 + nt]))
        k0 += nt
        out.append((rid, idx, tid, text, lp, top, bool(fin), REASONS[reason]))
    return out
