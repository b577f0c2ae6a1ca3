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

Authentication.  Bring-up draws a random per-deployment secret on rank 0 and broadcasts it with the
leader's address over the bring-up process group (:func:`open_links`); nothing else knows it.  A connecting
peer gets a random challenge and must answer with HMAC-SHA256(secret, challenge || rank) in a fixed-size,
non-pickled frame before the leader reads anything else from it; a wrong answer, a rank outside
1..world-1, a rank that already has a live link, or a peer that stalls in the handshake is dropped and the
listener keeps accepting.  Only authenticated links carry the pickled frames (4-byte big-endian length +
pickle: ranks of one deployment trust each other exactly as torch's object collectives do).  The listener
binds loopback unless ``LWC_SHARD_LINK_HOST`` names another interface.

Liveness and recovery.  Each follower sends a heartbeat every ``hb_s``; the leader declares a follower dead
when its socket closes (detected at once) or nothing arrived from it for ``dead_s`` (a hung process), closes
the link and reports the death (score/sharded.py turns the rank's unfinished voters into error choices and
moves later shares to the survivors).  The listener stays open after bring-up: a restarted follower (or one
whose link dropped) authenticates again with the same secret (``LWC_SHARD_LINK_FILE``: the leader writes its
address and secret there, mode 0600, for processes started outside the bring-up group) and is re-admitted —
``on_join(rank)`` fires and ``live()`` includes it again, so the node regains its capacity (the reference never
loses capacity permanently: it retries its whole attempt list until ``max_elapsed``,
src/chat/completions/client.rs:263-305).

Sends never block the caller: each link has a sender thread draining a queue; a peer that stops reading
makes only that thread's ``sendall`` time out (``dead_s``), which declares the rank dead.
"""
from __future__ import annotations

import hashlib
import hmac
import json
import logging
import os
import pickle
import queue
import secrets
import socket
import struct
import threading
import time
from typing import Any, Callable, Dict, List, Optional

_LEN = struct.Struct("!I")
_HELLO = struct.Struct("!4sI32s")  # magic, rank, HMAC-SHA256(secret, challenge || rank)
_MAGIC = b"LWC1"
_CHALLENGE = 32
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


def _mac(secret: bytes, challenge: bytes, rank: int) -> bytes:
    return hmac.new(secret, challenge + struct.pack("!I", rank), hashlib.sha256).digest()


class _Link:
    """One authenticated follower connection: the socket, its sender queue and thread."""

    def __init__(self, sock: socket.socket):
        self.sock = sock
        self.q: "queue.Queue" = queue.Queue()
        self.closed = False


class LinkServer:
    """The leader's end: one authenticated connection per follower rank, a reader and a sender thread each,
    a liveness monitor and an acceptor that keeps admitting (re)joining followers.

    ``on_message(rank, msg)``, ``on_dead(rank)`` and ``on_join(rank)`` are called from link threads; they must
    hand off to their own event loop themselves (``loop.call_soon_threadsafe``)."""

    def __init__(self, world: int, host: str = "127.0.0.1", hb_s: float = 0.5, dead_s: float = 10.0,
                 secret: Optional[bytes] = None, handshake_s: float = 5.0):
        self.world, self.hb_s, self.dead_s, self.handshake_s = world, hb_s, dead_s, handshake_s
        self.secret = secret if secret is not None else secrets.token_bytes(32)
        self.listener = socket.create_server((host, 0))
        self.address = (host, self.listener.getsockname()[1])
        self.links: Dict[int, _Link] = {}
        self.last_seen: Dict[int, float] = {}
        self.dead: set = set()
        self.joins = 0      # re-admissions after bring-up
        self.rejected = 0   # connections dropped at the handshake
        self.on_message: Callable[[int, Any], None] = lambda r, m: None
        self.on_dead: Callable[[int], None] = lambda r: None
        self.on_join: Callable[[int], None] = lambda r: None
        self._state = threading.Lock()
        self._joined = threading.Condition(self._state)
        self._closed = False
        self._started = False
        threading.Thread(target=self._acceptor, name="link-accept", daemon=True).start()

    # ------------------------------------------------------------------ admission
    def _acceptor(self) -> None:
        while not self._closed:
            try:
                sock, _ = self.listener.accept()
            except OSError:
                return  # listener closed
            threading.Thread(target=self._handshake, args=(sock,), name="link-hello", daemon=True).start()

    def _handshake(self, sock: socket.socket) -> None:
        """Challenge-response in fixed-size frames (nothing is unpickled before the peer proved the secret)."""
        try:
            sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            sock.settimeout(self.handshake_s)
            challenge = secrets.token_bytes(_CHALLENGE)
            sock.sendall(challenge)
            magic, rank, mac = _HELLO.unpack(_recv_exact(sock, _HELLO.size))
            ok = magic == _MAGIC and hmac.compare_digest(mac, _mac(self.secret, challenge, rank))
            ok = ok and 1 <= rank < self.world
            with self._state:
                ok = ok and not self._closed and (rank not in self.links or rank in self.dead)
            if ok:
                sock.sendall(b"OK")
        except (OSError, ConnectionError, struct.error):
            ok = False
        if not ok:
            self.rejected += 1
            try:
                sock.close()
            except OSError:
                pass
            return
        with self._state:
            if self._closed or (rank in self.links and rank not in self.dead):  # lost a race with a twin
                self.rejected += 1
                sock.close()
                return
            if rank in self.links:
                self.joins += 1
            link = _Link(sock)
            self.links[rank] = link
            self.dead.discard(rank)
            self.last_seen[rank] = time.monotonic()
            started = self._started  # a join after bring-up (decided with the registration, under the lock)
        # one timeout for both directions: a reader that hears nothing (not even a heartbeat) for dead_s, or
        # a send the peer stops draining, ends in socket.timeout -> the rank is dead
        sock.settimeout(self.dead_s)
        threading.Thread(target=self._reader, args=(rank, link), name=f"link-rx{rank}", daemon=True).start()
        threading.Thread(target=self._sender, args=(rank, link), name=f"link-tx{rank}", daemon=True).start()
        with self._state:
            self._joined.notify_all()
        if started:
            _log.warning("shard link: rank %d joined", rank)
            self.on_join(rank)

    def accept_all(self, timeout: float = 120.0) -> None:
        """Wait until every follower rank has joined (bring-up); bad or stalled connections are dropped and
        do not end the wait."""
        deadline = time.monotonic() + timeout
        with self._state:
            while len([r for r in self.links if r not in self.dead]) < self.world - 1:
                left = deadline - time.monotonic()
                if left <= 0:
                    raise TimeoutError(f"shard links: {len(self.links)} of {self.world - 1} followers joined")
                self._joined.wait(min(left, 0.5))
            self._started = True
        threading.Thread(target=self._monitor, name="link-monitor", daemon=True).start()

    def write_join_file(self, path: str) -> None:
        """The leader's address and secret for followers started outside the bring-up group (mode 0600)."""
        fd = os.open(path, os.O_WRONLY | os.O_CREAT | os.O_TRUNC, 0o600)
        with os.fdopen(fd, "w") as f:
            json.dump({"address": list(self.address), "secret": self.secret.hex()}, f)

    # ------------------------------------------------------------------ traffic
    def live(self) -> List[int]:
        with self._state:
            return sorted(r for r in self.links if r not in self.dead)

    def send(self, rank: int, msg: Any) -> bool:
        """Queue a message for one follower; never blocks.  False when the rank is dead (or was never
        connected); a send that later fails or times out (``dead_s``) declares the rank dead."""
        with self._state:
            link = self.links.get(rank)
            if link is None or rank in self.dead:
                return False
        link.q.put(msg)
        return True

    def broadcast(self, msg: Any) -> List[int]:
        """Send to every live follower; returns the ranks that took it."""
        return [r for r in self.live() if self.send(r, msg)]

    def _sender(self, rank: int, link: _Link) -> None:
        while True:
            msg = link.q.get()
            if msg is None or link.closed:
                return
            try:
                _send(link.sock, msg)
            except (OSError, ValueError, pickle.PicklingError):
                self._declare_dead(rank, link)
                return

    def _reader(self, rank: int, link: _Link) -> None:
        while True:
            try:
                msg = _recv(link.sock)
            except (OSError, ConnectionError, EOFError, pickle.UnpicklingError, struct.error):
                self._declare_dead(rank, link)
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
                    with self._state:
                        link = self.links.get(rank)
                    if link is not None:
                        self._declare_dead(rank, link)

    def _declare_dead(self, rank: int, link: _Link) -> None:
        with self._state:
            # a stale link (the rank already re-joined on a new one) dies quietly
            if self.links.get(rank) is not link or rank in self.dead or self._closed:
                link.closed = True
                self._close_sock(link)
                return
            self.dead.add(rank)
        link.closed = True
        link.q.put(None)
        self._close_sock(link)
        self.on_dead(rank)

    @staticmethod
    def _close_sock(link: _Link) -> None:
        try:
            link.sock.shutdown(socket.SHUT_RDWR)
        except OSError:
            pass
        try:
            link.sock.close()
        except OSError:
            pass

    def close(self) -> None:
        """Tell every live follower to stop, then drop the links and the listener."""
        links = []
        for r in self.live():
            with self._state:
                link = self.links.get(r)
            if link is not None:
                link.q.put(("stop",))
                link.q.put(None)
                links.append(link)
        for link in links:  # let the senders flush the stop (bounded)
            t_end = time.monotonic() + 2.0
            while not link.q.empty() and time.monotonic() < t_end:
                time.sleep(0.01)
        with self._state:
            self._closed = True
        try:
            self.listener.close()
        except OSError:
            pass
        for link in list(self.links.values()):
            link.closed = True
            self._close_sock(link)


class LinkClient:
    """A follower's end: connect to the leader, authenticate, heartbeat, receive work, send results
    (thread-safe)."""

    def __init__(self, address, rank: int, secret: bytes, hb_s: float = 0.5, timeout: float = 120.0):
        deadline = time.monotonic() + timeout
        while True:
            try:
                self.sock = socket.create_connection(tuple(address), timeout=10)
                self.sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                challenge = _recv_exact(self.sock, _CHALLENGE)
                self.sock.sendall(_HELLO.pack(_MAGIC, rank, _mac(secret, challenge, rank)))
                if _recv_exact(self.sock, 2) != b"OK":
                    raise ConnectionError("shard link: handshake refused")
                break
            except (OSError, ConnectionError):
                if time.monotonic() > deadline:
                    raise ConnectionError(f"shard link: rank {rank} could not join {tuple(address)}")
                time.sleep(0.1)
        self.sock.settimeout(None)
        self.rank, self.hb_s = rank, hb_s
        self.lock = threading.Lock()
        self.closed = False
        self._hb = threading.Thread(target=self._heartbeat, name="link-hb", daemon=True)
        self._hb.start()

    @classmethod
    def from_join_file(cls, path: str, rank: int, hb_s: float = 0.5, timeout: float = 120.0) -> "LinkClient":
        """(Re)join a running leader from its :meth:`LinkServer.write_join_file`."""
        with open(path) as f:
            info = json.load(f)
        return cls(tuple(info["address"]), rank, bytes.fromhex(info["secret"]), hb_s, timeout)

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
            self.sock.shutdown(socket.SHUT_RDWR)
        except OSError:
            pass
        try:
            self.sock.close()
        except OSError:
            pass


def link_host() -> str:
    """The address the leader listens on: ``LWC_SHARD_LINK_HOST`` if set; loopback when every rank runs on this
    node (WORLD_SIZE == LOCAL_WORLD_SIZE, or no torchrun sizes in the environment); otherwise ``MASTER_ADDR`` — the
    address the other nodes already reach this node by.  A multi-node world with no usable address fails here
    instead of leaving remote followers retrying a loopback address until the bring-up timeout."""
    host = os.environ.get("LWC_SHARD_LINK_HOST")
    if host:
        return host
    world = os.environ.get("WORLD_SIZE")
    local = os.environ.get("LOCAL_WORLD_SIZE")
    master = os.environ.get("MASTER_ADDR", "")
    one_node = world is None or local is None or world == local
    if one_node:
        return "127.0.0.1"
    if master in ("", "localhost", "::1") or master.startswith("127."):
        raise RuntimeError("voter-sharded links span several nodes (WORLD_SIZE %s > LOCAL_WORLD_SIZE %s) but "
                           "MASTER_ADDR is %r: set LWC_SHARD_LINK_HOST to this node's address reachable from "
                           "the other nodes" % (world, local, master))
    return master


def open_links(group=None, hb_s: Optional[float] = None, dead_s: Optional[float] = None):
    """Bring-up (a collective over ``group``, once): rank 0 returns a :class:`LinkServer` with every follower
    connected, the others a :class:`LinkClient`.  Environment: ``LWC_SHARD_HB_S`` (heartbeat period, default
    0.5 s), ``LWC_SHARD_DEAD_S`` (silence after which a follower counts as dead, default 10 s),
    ``LWC_SHARD_LINK_HOST`` (the interface the leader listens on and the followers reach; default: loopback
    when every rank is on this node, else ``MASTER_ADDR`` — :func:`link_host`), ``LWC_SHARD_LINK_FILE``
    (where the leader writes its address + secret for re-joining followers)."""
    import torch.distributed as dist

    from .dist import broadcast_object

    hb = float(os.environ.get("LWC_SHARD_HB_S", "0.5")) if hb_s is None else hb_s
    dead = float(os.environ.get("LWC_SHARD_DEAD_S", "10")) if dead_s is None else dead_s
    world, rank = dist.get_world_size(group), dist.get_rank(group)
    if rank == 0:
        host = link_host()
        srv = LinkServer(world, host, hb, dead)
        join_file = os.environ.get("LWC_SHARD_LINK_FILE")
        if join_file:
            srv.write_join_file(join_file)
        broadcast_object((srv.address, srv.secret), 0, group)
        srv.accept_all()
        return srv
    addr, secret = broadcast_object(None, 0, group)
    return LinkClient(addr, rank, secret, hb)
