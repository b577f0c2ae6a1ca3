"""EngineGroup: one engine WORKER PROCESS per GPU behind one front end (SURVEY.md §7.1 "EngineGroup (1
worker/GPU), candidate router"; §5 "worker heartbeat; on GPU/worker failure, drain and reschedule its
sequences to surviving GPUs").

* Each worker is a spawned process that owns one GPU and one `LLMEngine` (built from a JSON-able model
  spec by ``worker_factory``), reads requests from its own queue and sends each engine step's token
  events back as ONE binary record through its shared-memory ring (`shm_ring.py`; no pickling).  It
  stamps a shared heartbeat every loop; control messages (ready / fatal / error) use a queue.
* The front end exposes the `EngineService` API (`submit / abort / close / load`, plus an
  ``engine`` facade with tokenizer / cfg / max_model_len), so `LocalChatClient` serves a whole node
  through it unchanged.
* Candidate routing: a request's n candidates are split across the live workers, least-loaded first
  (candidate-parallel — the multichat / voter fan-out of the reference,
  src/score/completions/client.rs:343-356, spread over GPUs); each worker's local choice indices are
  offset into the request's global 0..n-1.  Candidate i gets seed base*1000003+i exactly as on one
  engine, so results do not depend on the split.
* Failure handling: a worker that exits or stops heart-beating is marked dead; each of its request
  portions that has not emitted a token yet is resubmitted to a surviving worker, the others fail
  with `EngineFailure` (the client turns that into an error choice / AllVotesFailed).
* Recovery: a dead worker (a whole TP replica: every rank) is torn down and a replacement is spawned as a
  FRESH child process of the front end (never a re-exec of a process that touched the GPU), with
  exponential backoff between attempts (``respawn_backoff_s`` doubling to 30 s, at most ``max_respawns``
  per worker).  It rebuilds its engine, says ready, and the router gives it requests again, so the node
  regains the capacity a fault took (the reference never loses capacity for good: it retries its attempt
  list until ``max_elapsed``, src/chat/completions/client.rs:263-305, src/main.rs:104-121).  Every worker
  message carries its process generation, so a late message of the dead process is never taken for its
  replacement's.
"""
from __future__ import annotations

import importlib
import itertools
import multiprocessing as mp
import queue as pyqueue
import random
import threading
import time
import traceback
from dataclasses import dataclass, field, replace
from typing import Any, Dict, List, Optional

from .sampling import SamplingParams
from .service import EngineFailure
from .shm_ring import ShmRing, decode_record, encode_embeddings, encode_events


@dataclass
class GroupTokenEvent:
    """Token event re-created in the front end (same fields the LocalChatClient reads)."""
    index: int
    token_id: int
    text: str
    logprob: float
    top_logprobs: list
    finished: bool
    finish_reason: Optional[str]

    @property
    def seq(self):
        return self


@dataclass
class _Portion:
    worker: int
    offset: int
    n: int
    params: SamplingParams
    emitted: int = 0
    finished: int = 0


@dataclass
class GroupRequest:
    rid: int
    prompt_ids: list
    loop: Any
    queue: Any
    portions: List[_Portion] = field(default_factory=list)
    failed: bool = False
    embed: Optional[str] = None           # embedding model the workers run on their finished candidates
    emb_parts: Dict[int, Any] = field(default_factory=dict)  # portion offset -> (unit rows [n, d], tokens)
    emb_future: Any = None                # resolves to (rows [n, d] float32 in candidate order, tokens)


def _set_future(fut, result, exc) -> None:
    if fut.done():
        return
    if exc is not None:
        fut.set_exception(exc)
    else:
        fut.set_result(result)


def _put_all(batch) -> None:
    for q, ev in batch:
        q.put_nowait(ev)


def _wire_ctx(ctx) -> Optional[dict]:
    """The part of a request context the worker's scheduler uses (priority, deadline, trace id), as a plain
    dict.  Deadlines are time.monotonic() values: CLOCK_MONOTONIC is shared by every process of the host."""
    if not isinstance(ctx, dict) or (not ctx.get("priority") and ctx.get("deadline") is None):
        return None  # nothing for the scheduler
    return {"priority": ctx.get("priority", 0), "deadline": ctx.get("deadline"), "trace_id": ctx.get("trace_id")}


def _resolve(path: str):
    mod, _, fn = path.partition(":")
    return getattr(importlib.import_module(mod), fn)


def _apply(engine, msg, groups: Dict[int, Any], cb_for, emb_req, on_error) -> None:
    """Apply one front-end message to the worker's engine (shared by TP leaders and their followers)."""
    kind = msg[0]
    if kind == "submit":
        _, rid, prompt, params, n, offset = msg[:6]
        embed = msg[6] if len(msg) > 6 else None
        wctx = msg[7] if len(msg) > 7 else None
        cb, texts = cb_for(rid, offset, n, embed)
        if embed and texts is not None:
            emb_req[rid] = (embed, offset, texts)
        try:
            kw = {"ctx": wctx} if wctx is not None else {}
            groups[rid] = engine.add_request(prompt, params, n=n, callback=cb, **kw)
        except ValueError as e:
            on_error(rid, str(e))
    elif kind == "abort":
        g = groups.pop(msg[1], None)
        if g is not None:
            engine.abort(g)


class _Tagged:
    """A worker's view of the front end's event queue: every message carries the worker's process generation
    (the front end drops messages of a generation it has already replaced)."""

    def __init__(self, q, gen: int):
        self.q, self.gen = q, gen

    def put(self, msg) -> None:
        self.q.put(tuple(msg) + (self.gen,))


def _push(ring, record: bytes, ev_q, fallback, hb, stop) -> None:
    """One record into the worker's ring: waits (heart-beating) while the ring is full — the front end's
    reader drains it — and never re-sends through the pickled queue unless there is no ring at all."""
    if ring is None:
        ev_q.put(fallback)
        return

    def beat():
        hb.value = time.time()

    while not ring.push(record, timeout=5.0, on_wait=beat):
        if stop.is_set():
            return


def worker_main(wid: int, spec: dict, factory: str, req_q, ev_q, hb, stop, ring_name: Optional[str] = None,
                mirror_out: Optional[list] = None, mirror_in=None, gen: int = 0) -> None:
    """Worker process: build the engine, serve requests until told to stop.

    Tensor-parallel replicas (spec ``tp`` > 1): the replica's rank 0 (the leader) is the worker the front end
    talks to; every engine iteration it forwards the messages it applied — submits, aborts, deadline expiries
    — and whether it steps to its followers (``mirror_out`` queues), which apply the same messages and step in
    lockstep (``mirror_in``), so every rank schedules the same batch and the all-reduce inside each forward
    pairs up.  Only the leader streams tokens and embeds candidates."""
    ev_q = _Tagged(ev_q, gen)
    if mirror_in is not None:
        return _follower_main(wid, spec, factory, ev_q, hb, stop, mirror_in)
    ring = ShmRing(ring_name, create=False) if ring_name else None
    embedders: Dict[str, Any] = {}
    emb_req: Dict[int, tuple] = {}  # rid -> (model name, offset, streamed texts)
    try:
        engine = _resolve(factory)(spec, wid)
    except BaseException as e:  # report and die: the front end marks the worker dead
        ev_q.put(("fatal", wid, f"{type(e).__name__}: {e}"))
        return
    ev_q.put(("ready", wid, None))
    groups: Dict[int, Any] = {}
    batch: List[tuple] = []

    def cb_for(rid, offset, n, embed):
        texts = [""] * n if embed else None

        def cb(ev, rid=rid, offset=offset, texts=texts):
            batch.append((rid, ev.seq.index + offset, ev.token_id, ev.text, ev.logprob,
                          list(ev.top_logprobs), ev.finished, ev.finish_reason))
            if texts is not None:
                texts[ev.seq.index] += ev.text

        return cb, texts

    def on_error(rid, msg):
        ev_q.put(("error", wid, (rid, msg)))

    failed = False
    while not stop.is_set():
        hb.value = time.time()
        applied: List[tuple] = []
        try:
            block = not engine.has_work()
            msg = req_q.get(timeout=0.2) if block else req_q.get_nowait()
        except pyqueue.Empty:
            msg = None
        while msg is not None:
            _apply(engine, msg, groups, cb_for, emb_req, on_error)
            applied.append(msg)
            try:
                msg = req_q.get_nowait()
            except pyqueue.Empty:
                msg = None
        for g in (engine.expire() if hasattr(engine, "expire") else ()):  # request deadlines (RequestContext)
            rid = next((r for r, gg in groups.items() if gg is g), None)
            if rid is not None:
                groups.pop(rid, None)
                applied.append(("abort", rid))
                ev_q.put(("error", wid, (rid, "request deadline exceeded", "deadline")))
        step = engine.has_work()
        if mirror_out and (applied or step or failed):
            tick = ("tick", applied, step, failed)
            for q in mirror_out:
                q.put(tick)
        failed = False
        if step:
            try:
                engine.step()
            except Exception as e:  # engine failure: fail in-flight groups, keep the worker alive
                traceback.print_exc()
                failed = True  # followers fail theirs at the next tick (their state stays the leader's)
                for g in engine.fail_all(f"{type(e).__name__}: {e}"):
                    rid = next((r for r, gg in groups.items() if gg is g), None)
                    if rid is not None:
                        ev_q.put(("error", wid, (rid, f"{type(e).__name__}: {e}")))
        if batch:
            _push(ring, encode_events(batch), ev_q, ("tokens", wid, batch), hb, stop)
            batch = []
        for rid in [r for r, g in groups.items() if g.finished]:
            groups.pop(rid)
            if rid in emb_req:  # embed this worker's candidates on its own GPU; only the unit rows travel
                name, offset, texts = emb_req.pop(rid)
                try:
                    svc = embedders.get(name)
                    if svc is None:
                        from ..embeddings.service import build_embedding_service

                        dev = spec.get("embed_device") or f"cuda:{int(spec.get('device', 0))}"
                        svc = embedders[name] = build_embedding_service(name, spec["embed_models"][name], dev)
                    E, ntok = svc.embed_texts(texts)
                    rows = E.float().cpu().numpy()
                    _push(ring, encode_embeddings(rid, offset, rows, int(ntok)), ev_q,
                          ("emb", wid, (rid, offset, rows, int(ntok))), hb, stop)
                except Exception as e:  # noqa: BLE001 - reported to the request, the worker keeps serving
                    ev_q.put(("emb_err", wid, (rid, f"{type(e).__name__}: {e}")))
    if mirror_out:
        for q in mirror_out:
            q.put(("stop",))


def _follower_main(wid: int, spec: dict, factory: str, ev_q, hb, stop, mirror_in) -> None:
    """A tensor-parallel follower rank: replay the leader's ticks (messages + step) on its own engine shard."""
    try:
        engine = _resolve(factory)(spec, wid)
    except BaseException as e:
        ev_q.put(("fatal", wid, f"follower rank {spec.get('tp_rank')}: {type(e).__name__}: {e}"))
        return
    groups: Dict[int, Any] = {}
    noop = lambda rid, offset, n, embed: (None, None)  # noqa: E731 - followers stream nothing
    while not stop.is_set():
        hb.value = time.time()
        try:
            tick = mirror_in.get(timeout=0.2)
        except pyqueue.Empty:
            continue
        if tick[0] == "stop":
            return
        _, applied, step, leader_failed = tick
        if leader_failed:  # the leader's last step raised: fail the same groups here
            engine.fail_all("tensor-parallel leader step failed")
            groups.clear()
        for msg in applied:
            _apply(engine, msg, groups, noop, {}, lambda rid, m: None)
        if step:
            try:
                engine.step()
            except Exception as e:  # the replica's ranks no longer agree: take the replica down
                traceback.print_exc()
                ev_q.put(("fatal", wid, f"follower rank {spec.get('tp_rank')} step failed: {type(e).__name__}: {e}"))
                return
        for rid in [r for r, g in groups.items() if g.finished]:
            groups.pop(rid)


class _EngineFacade:
    def __init__(self, tokenizer, cfg, max_model_len):
        self.tokenizer, self.cfg, self.max_model_len = tokenizer, cfg, max_model_len
        self.running, self.waiting = [], []


class EngineGroup:
    def __init__(self, spec: dict, devices: List[int], factory: str = "llm_weighted_consensus_amd.engine.group:build_engine",
                 tokenizer=None, cfg=None, max_model_len: int = 4096, heartbeat_timeout: float = 30.0,
                 start_timeout: float = 600.0, ring_bytes: int = 32 << 20, respawn: bool = True,
                 max_respawns: int = 8, respawn_backoff_s: float = 0.5):
        self.spec, self.factory = spec, factory
        self.heartbeat_timeout = heartbeat_timeout
        self.ring_bytes = ring_bytes
        self.respawn, self.max_respawns, self.respawn_backoff_s = respawn, max_respawns, respawn_backoff_s
        # tensor-parallel replicas: spec "tp" = T groups the listed GPUs in runs of T (LWC_GPUS=0,...,7 with
        # tp 2 = four TP=2 replicas); a worker index below names a replica, served by its rank-0 process
        tp = int(spec.get("tp", 1) or 1)
        devices = list(devices)
        if tp < 1 or len(devices) % tp:
            raise ValueError(f"tp {tp} must divide the number of GPUs ({len(devices)})")
        self.tp = tp
        self.replicas = [devices[i:i + tp] for i in range(0, len(devices), tp)]
        self.devices = [r[0] for r in self.replicas]
        self._mp = mp.get_context("spawn")
        self.ev_q = self._mp.Queue()
        self.stop = self._mp.Event()
        n = len(self.replicas)
        self.req_qs: List[Any] = [None] * n
        self.hbs: List[Any] = [None] * n
        self.procs: List[Any] = [None] * n
        self.rings: List[Any] = [None] * n
        self.retired: List[Any] = []  # rings and processes of replaced workers (closed / joined at close())
        self.followers: List[List[tuple]] = [[] for _ in range(n)]  # per replica: (process, hb) of ranks 1..T-1
        self.mirror_qs: List[list] = [[] for _ in range(n)]
        self.gen = [0] * n          # process generation of each worker slot
        self.respawns = [0] * n     # replacements started per slot
        self.respawning = [False] * n
        self._port0 = int(spec.get("tp_port", 0)) or (_free_port_base(n) if tp > 1 else 0)
        self.alive = [True] * n
        self.ready = [False] * n
        self.load_of = [0] * n
        self.requests: Dict[int, GroupRequest] = {}
        self.emb_pending: Dict[int, GroupRequest] = {}  # finished generating, embeddings still on the way
        self._rid = itertools.count(1)
        self._lock = threading.Lock()
        self._life = threading.RLock()  # deaths and replacements of worker slots
        self.failures = 0
        self.engine = _EngineFacade(tokenizer, cfg, max_model_len)
        for wid in range(n):
            self._spawn(wid, self._port0 + wid if tp > 1 else 0)
        self._reader = threading.Thread(target=self._read, name="lwc-group-reader", daemon=True)
        self._reader.start()
        deadline = time.time() + start_timeout
        while not all(r or not a for r, a in zip(self.ready, self.alive)):
            if time.time() > deadline:
                raise RuntimeError("EngineGroup: workers did not start")
            self._check_health()
            time.sleep(0.05)
        if not any(self.alive):
            raise RuntimeError("EngineGroup: every worker failed to start")

    def _spawn(self, wid: int, port: int) -> None:
        """Start worker slot ``wid``'s processes (a TP replica: its leader and followers) at generation
        ``self.gen[wid]``: new request queue, heartbeat values and ring — nothing is shared with a previous
        generation."""
        ctx, devs, gen = self._mp, self.replicas[wid], self.gen[wid]
        q = ctx.Queue()
        hb = ctx.Value("d", time.time())
        ring = ShmRing(cap=self.ring_bytes)
        wspec = dict(self.spec, device=devs[0])
        mirrors, fl = [], []
        if self.tp > 1:
            shared = len(set(devs)) < len(devs)  # ranks sharing a GPU (one-GPU rehearsal) split its memory
            wspec.update(tp=self.tp, tp_rank=0, tp_port=port, tp_shared=shared)
            for r in range(1, self.tp):
                mq = ctx.Queue()
                fhb = ctx.Value("d", time.time())
                fp = ctx.Process(target=worker_main,
                                 args=(wid, dict(wspec, device=devs[r], tp_rank=r), self.factory, None, self.ev_q, fhb,
                                       self.stop, None, None, mq, gen),
                                 daemon=True, name=f"lwc-worker-{wid}-tp{r}-g{gen}")
                fp.start()
                mirrors.append(mq)
                fl.append((fp, fhb))
        p = ctx.Process(target=worker_main, args=(wid, wspec, self.factory, q, self.ev_q, hb, self.stop, ring.name,
                                                  mirrors or None, None, gen),
                        daemon=True, name=f"lwc-worker-{wid}-g{gen}")
        p.start()
        self.req_qs[wid], self.hbs[wid], self.procs[wid] = q, hb, p
        self.rings[wid] = ring
        self.followers[wid] = fl
        self.mirror_qs[wid] = mirrors  # keep the queues alive: a started Process drops its args

    # ------------------------------------------------------------------ EngineService API
    @property
    def load(self) -> int:
        return sum(self.load_of)

    def live_workers(self) -> List[int]:
        return [i for i, a in enumerate(self.alive) if a and self.ready[i]]

    def embeds_in_workers(self, model: str) -> bool:
        return model in (self.spec.get("embed_models") or {})

    def submit(self, prompt_ids, params: SamplingParams, n: int, loop, queue, embed: Optional[str] = None,
               ctx=None) -> GroupRequest:
        """``embed``: an embedding model every worker embeds its finished candidates with; the rows arrive
        in ``req.emb_future`` (a future of ``loop``)."""
        self._check_health()
        live = self.live_workers()
        if not live:
            raise ValueError("no live engine workers")
        if embed is not None and not self.embeds_in_workers(embed):
            raise ValueError(f"embedding model {embed} is not hosted by the workers")
        rid = next(self._rid)
        req = GroupRequest(rid, list(prompt_ids), loop, queue, embed=embed)
        if embed is not None:
            req.emb_future = loop.create_future()
        # candidate i of the request keeps seed base*1000003+i however the n candidates are split
        base = params.seed if params.seed is not None else random.getrandbits(63)
        order = sorted(live, key=lambda w: self.load_of[w])
        share = [n // len(order) + (1 if k < n % len(order) else 0) for k in range(len(order))]
        offset = 0
        with self._lock:
            self.requests[rid] = req
            for w, m in zip(order, share):
                if m == 0:
                    continue
                p = _Portion(w, offset, m, replace(params, seed=base, seed_offset=params.seed_offset + offset))
                req.portions.append(p)
                self.load_of[w] += m
                self.req_qs[w].put(("submit", rid, req.prompt_ids, p.params, m, offset, embed, _wire_ctx(ctx)))
                offset += m
        return req

    def abort(self, req: GroupRequest) -> None:
        with self._lock:
            self.requests.pop(req.rid, None)
            for p in req.portions:
                if self.alive[p.worker]:
                    self.req_qs[p.worker].put(("abort", req.rid))
                self.load_of[p.worker] -= p.n - p.finished

    def close(self) -> None:
        self.stop.set()
        with self._life:
            procs = self.procs + [fp for fl in self.followers for fp, _ in fl] + \
                [x for x in self.retired if not isinstance(x, ShmRing)]
        for p in procs:
            p.join(timeout=10)
            if p.is_alive():
                p.kill()
        self._reader.join(timeout=5)
        if self._reader.is_alive():  # still inside a pop: leave the segments to process exit, never
            return                   # unmap them under a running reader
        for r in self.rings + [x for x in self.retired if isinstance(x, ShmRing)]:
            r.close()
        self.rings = []
        self.retired = []

    # ------------------------------------------------------------------ reader / health
    def _deliver(self, req: GroupRequest, item) -> None:
        req.loop.call_soon_threadsafe(req.queue.put_nowait, item)

    def _read(self) -> None:
        last_health = time.monotonic()
        while not self.stop.is_set():
            busy = False
            for wid, ring in enumerate(list(self.rings)):
                while self.rings[wid] is ring:  # a replaced worker's ring is dropped, not read on
                    rec = ring.pop()
                    if rec is None:
                        break
                    busy = True
                    kind, payload = decode_record(rec)
                    if kind == "tokens":
                        self._on_tokens(wid, payload)
                    else:  # a worker's embedding rows, in the ring after its candidates' last tokens
                        self._on_embeddings("emb", payload)
            try:
                kind, wid, payload, gen = self.ev_q.get_nowait()
            except pyqueue.Empty:
                if not busy:
                    time.sleep(0.0003)
                if time.monotonic() - last_health > 0.5:
                    last_health = time.monotonic()
                    self._check_health()
                continue
            except (EOFError, OSError):
                return
            if gen != self.gen[wid]:
                continue  # a replaced process's last words: its requests were already failed / moved
            if kind == "ready":
                self.ready[wid] = True
            elif kind == "fatal":
                if self.ready[wid] and self.alive[wid]:  # a TP follower lost step with its leader
                    self._worker_died(wid, str(payload))
                else:  # failed to start: try again later (bounded by max_respawns)
                    self.alive[wid] = False
                    self.failures += 1
                    self._schedule_respawn(wid, f"failed to start: {payload}")
            elif kind == "error":
                rid, msg = payload[:2]
                fkind = payload[2] if len(payload) > 2 else "error"
                with self._lock:
                    req = self.requests.get(rid)
                    # only a worker that still owns an unfinished portion of the request may fail it
                    if req is not None and any(p.worker == wid and p.finished < p.n for p in req.portions):
                        self.requests.pop(rid, None)
                    else:
                        req = None
                if req is not None:
                    if fkind != "deadline":
                        self.failures += 1
                    self._deliver(req, EngineFailure(msg, fkind))
            elif kind == "tokens":
                self._on_tokens(wid, payload)
            elif kind in ("emb", "emb_err"):
                self._on_embeddings(kind, payload)
            self._check_health()

    def _on_embeddings(self, kind: str, payload) -> None:
        import numpy as np

        rid = payload[0]
        with self._lock:
            req = self.emb_pending.get(rid) or self.requests.get(rid)
            if req is None or req.emb_future is None:
                return
            if kind == "emb_err":
                self.emb_pending.pop(rid, None)
                req.loop.call_soon_threadsafe(_set_future, req.emb_future, None, RuntimeError(payload[1]))
                return
            _, offset, rows, ntok = payload
            req.emb_parts[offset] = (rows, ntok)
            if len(req.emb_parts) < len(req.portions):
                return
            self.emb_pending.pop(rid, None)
        parts = [req.emb_parts[o] for o in sorted(req.emb_parts)]
        out = (np.concatenate([r for r, _ in parts]), sum(t for _, t in parts))
        req.loop.call_soon_threadsafe(_set_future, req.emb_future, out, None)

    def _on_tokens(self, wid: int, payload) -> None:
        # one thread-safe hand-off per client event loop per record (not one self-pipe wake-up per token)
        per_loop: Dict[Any, list] = {}
        with self._lock:
            for (rid, idx, tid, text, lp, top, fin, reason) in payload:
                req = self.requests.get(rid)
                if req is None:
                    continue
                p = next((p for p in req.portions if p.worker == wid and p.offset <= idx < p.offset + p.n), None)
                if p is None:
                    # no portion of this worker holds the row any more: a slot declared dead (its portions moved
                    # to a survivor) whose process still pushed records before it was killed
                    continue
                p.emitted += 1
                if fin:
                    p.finished += 1
                    self.load_of[wid] -= 1
                per_loop.setdefault(req.loop, []).append((req.queue, GroupTokenEvent(idx, tid, text, lp, top, fin,
                                                                                     reason)))
                if all(pp.finished == pp.n for pp in req.portions):
                    self.requests.pop(rid, None)
                    if req.embed is not None and len(req.emb_parts) < len(req.portions):
                        self.emb_pending[rid] = req
        for loop, batch in per_loop.items():
            try:
                loop.call_soon_threadsafe(_put_all, batch)
            except RuntimeError:  # the client's loop is gone
                pass

    def _check_health(self) -> None:
        now = time.time()
        with self._life:
            for w, p in enumerate(self.procs):
                if not self.alive[w] or p is None:
                    continue
                members = [(p, self.hbs[w])] + self.followers[w]
                for q, hb in members:
                    stale = self.ready[w] and now - hb.value > self.heartbeat_timeout
                    if not q.is_alive() or stale:
                        self._worker_died(w, "exited" if not q.is_alive() else "heartbeat timeout")
                        break

    def _schedule_respawn(self, w: int, why: str) -> None:
        with self._life:
            if not self.respawn or self.stop.is_set() or self.respawning[w] or self.respawns[w] >= self.max_respawns:
                return
            self.respawning[w] = True
            delay = min(30.0, self.respawn_backoff_s * (2 ** self.respawns[w]))
            self.respawns[w] += 1
        threading.Thread(target=self._respawn, args=(w, delay, why), name=f"lwc-respawn-{w}", daemon=True).start()

    def _respawn(self, w: int, delay: float, why: str) -> None:
        """Replace worker slot ``w`` (after ``delay``): tear down every process of the old generation, then
        spawn fresh ones; the slot serves again once its new engine says ready."""
        if self.stop.wait(delay):
            return
        with self._life:
            old = [self.procs[w]] + [fp for fp, _ in self.followers[w]]
        for p in old:  # a TP replica is one unit: no rank of the old generation may outlive it
            if p is not None and p.is_alive():
                p.kill()
            if p is not None:
                p.join(timeout=10)
        with self._life:
            if self.stop.is_set():
                self.respawning[w] = False
                return
            self.retired += [r for r in (self.rings[w],) if r is not None] + [p for p in old if p is not None]
            self.gen[w] += 1
            self.ready[w] = False
            port = _free_port_base(1) if self.tp > 1 else 0  # the old rendezvous port may linger
            try:
                self._spawn(w, port)
            except Exception as e:  # noqa: BLE001 - e.g. no shared memory left: try again later
                traceback.print_exc()
                self.respawning[w] = False
                self._schedule_respawn(w, f"respawn failed: {e}")
                return
            self.alive[w] = True
            self.respawning[w] = False
        print(f"[EngineGroup] worker {w} ({why}) replaced: generation {self.gen[w]}", flush=True)

    def _worker_died(self, w: int, why: str) -> None:
        with self._life:
            if not self.alive[w]:
                return
            self.alive[w] = False
            self.ready[w] = False
            # fence the slot at once: a process declared dead for a heartbeat timeout may still be running, and
            # its late 'error' / deadline messages must not match the slot's generation while its portions are
            # moved to survivors (the reader drops messages of an older generation); _respawn bumps it again
            # for the replacement
            self.gen[w] += 1
        self.failures += 1
        self.load_of[w] = 0
        # every process of the dead unit is killed here, not only after the respawn backoff (a TP replica is one
        # unit: its other ranks cannot go on alone; a hung tp=1 worker must not come back to life)
        for fp, _ in self.followers[w]:
            if fp.is_alive():
                fp.kill()
        if self.procs[w] is not None and self.procs[w].is_alive():
            self.procs[w].kill()
        live = self.live_workers()
        with self._lock:
            for rid, req in list(self.emb_pending.items()):  # generated, but this worker's rows never came
                if any(p.worker == w and p.offset not in req.emb_parts for p in req.portions):
                    self.emb_pending.pop(rid, None)
                    req.loop.call_soon_threadsafe(_set_future, req.emb_future, None,
                                                  RuntimeError(f"engine worker {w} {why}"))
            for rid, req in list(self.requests.items()):
                for p in [p for p in req.portions if p.worker == w and p.finished < p.n]:
                    if p.emitted == 0 and live:
                        # nothing streamed yet: reschedule the portion on the least-loaded survivor
                        t = min(live, key=lambda x: self.load_of[x])
                        p.worker = t
                        self.load_of[t] += p.n
                        self.req_qs[t].put(("submit", rid, req.prompt_ids, p.params, p.n, p.offset, req.embed))
                    else:
                        self.requests.pop(rid, None)
                        for q in req.portions:  # the survivors' portions of a failed request stop too
                            if q.worker != w and self.alive[q.worker]:
                                self.req_qs[q.worker].put(("abort", rid))
                                self.load_of[q.worker] -= q.n - q.finished
                        self._deliver(req, EngineFailure(f"engine worker {w} {why}"))
                        if req.emb_future is not None:
                            req.loop.call_soon_threadsafe(_set_future, req.emb_future, None,
                                                          RuntimeError(f"engine worker {w} {why}"))
                        break
        self._schedule_respawn(w, why)


def _free_port_base(n: int) -> int:
    """A base port with n consecutive free TCP ports on 127.0.0.1 (TP replica rendezvous)."""
    import socket

    for _ in range(64):
        with socket.socket() as s0:
            s0.bind(("127.0.0.1", 0))
            base = s0.getsockname()[1]
        if base + n >= 65535:
            continue
        ok = True
        for k in range(1, n):
            with socket.socket() as sk:
                try:
                    sk.bind(("127.0.0.1", base + k))
                except OSError:
                    ok = False
                    break
        if ok:
            return base
    raise RuntimeError("no free port range for the TP rendezvous")


def _tp_setup(spec: dict, dev, hidden: int):
    """Join this rank's TP replica: a gloo group over 127.0.0.1 (control: IPC handle exchange, KV sizing)
    and the IPC one-shot all-reduce (C3) the decoder's forward uses."""
    import datetime

    import torch.distributed as dist

    from ..parallel.allreduce import CustomAllReduce

    tp, rank = int(spec["tp"]), int(spec["tp_rank"])
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{int(spec['tp_port'])}", rank=rank, world_size=tp,
                            timeout=datetime.timedelta(seconds=600))
    rows = max(int(spec.get("max_batch", 512)), int(spec.get("chunked_prefill", 0) or 0) + 1, 1024)
    comm = CustomAllReduce(device=dev, max_bytes=min(64 << 20, rows * hidden * 2))
    return rank, tp, comm


def _tp_num_blocks(model, dev, kv_fraction: float) -> int:
    """Every rank of a TP replica must schedule identically: one KV pool size for the replica (the smallest
    rank's)."""
    import torch
    import torch.distributed as dist

    from ..models.llama import KVCache

    torch.cuda.synchronize(dev)
    free, _total = torch.cuda.mem_get_info(dev)
    nb = torch.tensor([max(64, int(free * kv_fraction) // KVCache.bytes_per_block(model.cfg, 16))])
    dist.all_reduce(nb, op=dist.ReduceOp.MIN)
    return int(nb.item())


def build_engine(spec: dict, wid: int):
    """Default worker factory: a decoder engine on ``spec['device']`` from a server model spec
    ({"arch", "weights": "random:<seed>" | path, "max_model_len", "max_batch", "kv_fraction", "fp8",
    "prefix_caching", "chunked_prefill", "constrained_logprobs", "tokenizer": path to a tokenizer.json}); MoE archs get the
    Mixtral model."""
    import torch

    from ..models.config import decoder_config
    from ..models.llama import LlamaModel
    from .engine import LLMEngine
    from .tokenizer import load_tokenizer

    dev = torch.device("cuda", int(spec.get("device", 0)))
    torch.cuda.set_device(dev)
    cfg = decoder_config(spec["arch"])
    w = spec.get("weights", "random:0")
    path, seed = (None, int(w.split(":", 1)[1])) if w.startswith("random:") else (w, 0)
    mlen = int(spec.get("max_model_len", 4096))
    tp = int(spec.get("tp", 1) or 1)
    kv_fraction = float(spec.get("kv_fraction", 0.85))
    num_blocks = None
    if cfg.num_experts:
        from ..models.mixtral import MixtralModel

        tp_kw = {}
        if tp > 1:
            rank, tp, comm = _tp_setup(spec, dev, cfg.hidden)
            tp_kw = dict(tp_rank=rank, tp_size=tp, tp_comm=comm)
            if spec.get("tp_shared"):
                kv_fraction /= tp
        model = MixtralModel(cfg, device=dev, seed=seed, weights_path=path, max_position=mlen + 64,
                             fp8=bool(spec.get("fp8", False)), **tp_kw)
        if tp > 1:
            num_blocks = _tp_num_blocks(model, dev, kv_fraction)
    elif tp > 1:
        from ..models.tp import TPLlamaModel

        rank, tp, comm = _tp_setup(spec, dev, cfg.hidden)
        if spec.get("tp_shared"):
            kv_fraction /= tp
        model = TPLlamaModel(cfg, device=dev, seed=seed, weights_path=path, max_position=mlen + 64,
                             fp8_dense=bool(spec.get("fp8", False)), tp_rank=rank, tp_size=tp, tp_comm=comm)
        num_blocks = _tp_num_blocks(model, dev, kv_fraction)
    else:
        model = LlamaModel(cfg, device=dev, seed=seed, weights_path=path, max_position=mlen + 64,
                           fp8_dense=bool(spec.get("fp8", False)))
    tok = load_tokenizer(spec, cfg.vocab_size, cfg.bos_token_id, cfg.eos_token_id)
    return LLMEngine(model, tok, max_batch=int(spec.get("max_batch", 512)), max_model_len=mlen,
                     kv_memory_fraction=kv_fraction, num_blocks=num_blocks,
                     use_graphs=getattr(model, "graph_safe", True),
                     prefix_caching=bool(spec.get("prefix_caching", True)),
                     # the paged-KV prefill kernel of mixed steps is built for head_dim 128
                     chunked_prefill=int(spec.get("chunked_prefill", 0)) if cfg.head_dim == 128 else 0,
                     constrained_logprobs=bool(spec.get("constrained_logprobs", False)),
                     kv_reserve_tokens=spec.get("kv_reserve_tokens", 256))
