"""Leader <-> follower message links of the voter-sharded deployment (score/sharded.py, ``LWC_SHARD_VOTERS``).

Why point-to-point links and not collectives.  The reference isolates a failed voter: its error becomes
that voter's choice, never a failed request (src/score/completions/client.rs:711-783, 798-813), and a
request fails as a whole only when every voter failed (:385-409, 458-463).  A gloo / RCCL collective has no
such isolation: one dead member blocks every survivor until the process-group timeout and leaves the group
unusable afterwards.  So the serving plane of a voter-sharded node is a star of TCP links: every follower
rank keeps ONE connection to the leader (rank 0).  The leader sends work (a score request's share of
voters, a consensus request's slice of candidates); a follower streams results back as they are produced
(each voter chunk, already tagged with its voter, so the leader's SSE stream interleaves remote voters live,
as the reference's ``select_all`` does at client.rs:343-382).

Framing: 4-byte big-endian length + pickle (ranks of one deployment trust each other exactly as torch's
object collectives do, which pickle too).  Liveness: each follower sends a heartbeat every ``hb_s``; the
leader declares a follower dead when its socket closes (a process that exits or is killed: detected at
once) or when nothing arrived from it for ``dead_s`` (a hung process), closes the link, and reports the
death to whoever waits on that rank (score/sharded.py turns the rank's unfinished voters into error choices
and moves its share of later requests to the survivors).

The links need no process group after bring-up: the leader's (host, port) reaches the followers with one
broadcast at start-up (:func:`open_links`).
"""
from __future__ import annotations

import logging
import os
import pickle
import socket
import struct
import threading
import time
from typing import Any, Callable, Dict, List, Optional

_LEN = struct.Struct("!I")
_log = logging.getLogger(__name__)


def _send(sock: socket.socket, obj: Any) -> None:
    data = pickle.dumps(obj, protocol=pickle.HIGHEST_PROTOCOL)
    sock.sendall(_LEN.pack(len(data)) + data)


def _recv_exact(sock: socket.socket, n: int) -> bytes:
    buf = bytearray()
    while len(buf) < n:
        part = sock.recv(n - len(buf))
        if not part:
            raise ConnectionError("link closed by peer")
        buf += part
    return bytes(buf)


def _recv(sock: socket.socket) -> Any:
    (n,) = _LEN.unpack(_recv_exact(sock, _LEN.size))
    return pickle.loads(_recv_exact(sock, n))


class LinkServer:
    """The leader's end: one connection per follower rank, a reader thread each, a liveness monitor.

    ``on_message(rank, msg)`` and ``on_dead(rank)`` are called from link threads; they must hand off to
    their own event loop themselves (``loop.call_soon_threadsafe``)."""

    def __init__(self, world: int, host: str = "127.0.0.1", hb_s: float = 0.5, dead_s: float = 10.0):
        self.world, self.hb_s, self.dead_s = world, hb_s, dead_s
        self.listener = socket.create_server((host, 0))
        self.address = (host, self.listener.getsockname()[1])
        self.conns: Dict[int, socket.socket] = {}
        self.locks: Dict[int, threading.Lock] = {}
        self.last_seen: Dict[int, float] = {}
        self.dead: set = set()
        self.on_message: Callable[[int, Any], None] = lambda r, m: None
        self.on_dead: Callable[[int], None] = lambda r: None
        self._state = threading.Lock()
        self._closed = False

    def accept_all(self, timeout: float = 120.0) -> None:
        """Wait for every follower's hello (bring-up: each follower connects once)."""
        self.listener.settimeout(timeout)
        while len(self.conns) < self.world - 1:
            sock, _ = self.listener.accept()
            sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            sock.settimeout(timeout)
            hello = _recv(sock)
            if not (isinstance(hello, tuple) and hello[0] == "hello"):
                sock.close()
                continue
            rank = int(hello[1])
            # one timeout for both directions: a reader that hears nothing (not even a heartbeat) for
            # dead_s, or a send the peer stops draining, ends in socket.timeout -> the rank is dead
            sock.settimeout(self.dead_s)
            self.conns[rank] = sock
            self.locks[rank] = threading.Lock()
            self.last_seen[rank] = time.monotonic()
        self.listener.close()
        for rank in sorted(self.conns):
            threading.Thread(target=self._reader, args=(rank,), name=f"link-rx{rank}", daemon=True).start()
        threading.Thread(target=self._monitor, name="link-monitor", daemon=True).start()

    def live(self) -> List[int]:
        with self._state:
            return sorted(r for r in self.conns if r not in self.dead)

    def send(self, rank: int, msg: Any) -> bool:
        """Send to one follower; False (and the rank declared dead) when the link is gone.  A send to a
        peer that stopped reading gives up after ``dead_s`` instead of blocking the caller forever."""
        if rank in self.dead:
            return False
        sock = self.conns[rank]
        try:
            with self.locks[rank]:
                _send(sock, msg)
            return True
        except (OSError, ValueError):
            self._declare_dead(rank)
            return False

    def broadcast(self, msg: Any) -> List[int]:
        """Send to every live follower; returns the ranks that took it."""
        return [r for r in self.live() if self.send(r, msg)]

    def _reader(self, rank: int) -> None:
        sock = self.conns[rank]
        while True:
            try:
                msg = _recv(sock)
            except (OSError, ConnectionError, EOFError, pickle.UnpicklingError, struct.error):
                self._declare_dead(rank)
                return
            self.last_seen[rank] = time.monotonic()
            if isinstance(msg, tuple) and msg and msg[0] == "hb":
                continue
            try:
                self.on_message(rank, msg)
            except Exception:  # noqa: BLE001 — a bad message must not stop the link; it is logged
                _log.exception("shard link: message from rank %d dropped", rank)

    def _monitor(self) -> None:
        while not self._closed:
            time.sleep(self.hb_s)
            now = time.monotonic()
            for rank in self.live():
                if now - self.last_seen.get(rank, now) > self.dead_s:
                    self._declare_dead(rank)

    def _declare_dead(self, rank: int) -> None:
        with self._state:
            if rank in self.dead or self._closed:
                return
            self.dead.add(rank)
        try:
            self.conns[rank].close()
        except OSError:
            pass
        self.on_dead(rank)

    def close(self) -> None:
        """Tell every live follower to stop, then drop the links."""
        for r in self.live():
            self.send(r, ("stop",))
        with self._state:
            self._closed = True
        for s in self.conns.values():
            try:
                s.close()
            except OSError:
                pass


class LinkClient:
    """A follower's end: connect to the leader, heartbeat, receive work, send results (thread-safe)."""

    def __init__(self, address, rank: int, hb_s: float = 0.5, timeout: float = 120.0):
        deadline = time.monotonic() + timeout
        while True:
            try:
                self.sock = socket.create_connection(tuple(address), timeout=10)
                break
            except OSError:
                if time.monotonic() > deadline:
                    raise
                time.sleep(0.1)
        self.sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        self.sock.settimeout(None)
        self.rank, self.hb_s = rank, hb_s
        self.lock = threading.Lock()
        self.closed = False
        _send(self.sock, ("hello", rank))
        self._hb = threading.Thread(target=self._heartbeat, name="link-hb", daemon=True)
        self._hb.start()

    def _heartbeat(self) -> None:
        while not self.closed:
            if not self.send(("hb", self.rank)):
                return
            time.sleep(self.hb_s)

    def send(self, msg: Any) -> bool:
        try:
            with self.lock:
                _send(self.sock, msg)
            return True
        except OSError:
            self.closed = True
            return False

    def recv(self) -> Optional[Any]:
        """The leader's next message; None once the link is gone."""
        try:
            return _recv(self.sock)
        except (OSError, ConnectionError, EOFError, pickle.UnpicklingError, struct.error):
            self.closed = True
            return None

    def close(self) -> None:
        self.closed = True
        try:
            self.sock.close()
        except OSError:
            pass


def open_links(group=None, hb_s: Optional[float] = None, dead_s: Optional[float] = None):
    """Bring-up (a collective over ``group``, once): rank 0 returns a :class:`LinkServer` with every follower
    connected, the others a :class:`LinkClient`.  Environment: ``LWC_SHARD_HB_S`` (heartbeat period, default
    0.5 s), ``LWC_SHARD_DEAD_S`` (silence after which a follower counts as dead, default 10 s),
    ``LWC_SHARD_LINK_HOST`` (the leader's address as the followers reach it; default MASTER_ADDR)."""
    import torch.distributed as dist

    from .dist import broadcast_object

    hb = float(os.environ.get("LWC_SHARD_HB_S", "0.5")) if hb_s is None else hb_s
    dead = float(os.environ.get("LWC_SHARD_DEAD_S", "10")) if dead_s is None else dead_s
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    if rank == 0:
        host = os.environ.get("LWC_SHARD_LINK_HOST", os.environ.get("MASTER_ADDR", "127.0.0.1"))
        srv = LinkServer(world, host, hb, dead)
        broadcast_object(srv.address, 0, group)
        srv.accept_all()
        return srv
    addr = broadcast_object(None, 0, group)
    return LinkClient(addr, rank, hb)
