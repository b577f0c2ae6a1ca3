"""Voter-sharded serving: one score request's voters spread over the ranks of a node (C2), with the
reference's per-voter failure isolation and live streaming of every voter.

The reference fans a request's voters out as concurrent upstream streams, yields every voter chunk as it
arrives (src/score/completions/client.rs:342-382, ``select_all``), turns a failed voter into an error choice
rather than a failed request (:711-783, 798-813) and fails the request only when every voter failed
(:385-409, 458-463).  Here the voters run on the GPUs of the node:

* rank 0 (the **leader**) serves HTTP.  For each score request it does everything the reference does before
  the fan-out — model validation, archive references, choice texts, weights — once, then assigns every
  voter to a live rank (voter ``i`` -> ``live[i % len(live)]``) and sends each follower its share with the
  resolved request, the weights and the key-tree seeds (parallel/shard_link.py: one TCP link per follower,
  no collective);
* a **follower** runs its voters' streams on its own engine and sends every chunk back the moment it is
  produced, tagged with its voter (index ``C + voter * 4096 + native choice index``);
* the leader merges its own voters and every follower's chunks into ONE stream in arrival order (remote
  voters are streamed live, not delivered whole at the end), re-indexed through the request's
  ``ChoiceIndexer`` exactly like local ones, and runs the tally alone.

Failure isolation: when a follower dies (its socket closes, or its heartbeat stops for ``LWC_SHARD_DEAD_S``)
or a request's share outlives its bound (the request deadline plus ``LWC_SHARD_GRACE_S``, else
``LWC_SHARD_WAIT_S``), every voter of that share that had not finished becomes an error choice
(``finish_reason: "error"``, error ``voter_shard_lost``) — a partially streamed voter keeps its index, one that
never started gets one — and the request completes with the other voters (AllVotesFailed only when all of
them failed).  A dead rank gets no share of later requests: they run on the survivors.

/consensus/completions: candidates [first, first + n) of a request are sampled by the rank owning that slice
(each with the seed it has in the whole request) and embedded on its GPU; the unit rows travel back over the
link.  The slice of a follower that dies, times out or fails is recomputed by the leader — same seeds, same
candidates — so the request still completes.
"""
from __future__ import annotations

import asyncio
import copy
import logging
import os
import threading
import time
from typing import Any, Dict, List, Optional

import numpy as np

from ..errors import ChatError, ResponseError, ScoreError, StatusError
from ..parallel.shard_link import LinkClient, LinkServer
from ..schema import chat as C
from ..schema import score as S
from .orchestrator import ChoiceIndexer, ScoreClient

_log = logging.getLogger(__name__)
_NATIVE = 1 << 12  # a follower tags choice (voter v, native index k) as C + v * _NATIVE + k


def _lost(rank: int, why: str) -> ChatError:
    return ChatError(500, {"kind": "voter_shard_lost", "error": f"rank {rank}: {why}"})


class _TagIndexer:
    """A follower's indexer: the leader decodes (voter, native choice) from the index it assigns."""

    def __init__(self, C_len: int):
        self.C = C_len

    def get(self, llm_index: int, native: int) -> int:
        if not 0 <= native < _NATIVE:
            raise ValueError(f"native choice index {native} out of range")
        return self.C + llm_index * _NATIVE + native


class _Share:
    """One request's work on the followers, as the leader tracks it: link messages arrive on ``q`` (put from
    link threads through the request's loop)."""

    def __init__(self, loop, ranks):
        self.loop = loop
        self.q: asyncio.Queue = asyncio.Queue()
        self.ranks = set(ranks)

    def post(self, item) -> None:
        try:
            self.loop.call_soon_threadsafe(self.q.put_nowait, item)
        except RuntimeError:  # the request's loop is gone (request abandoned): nothing waits
            pass


class _LinkHub:
    """Routes the followers' messages to the request waiting on them (by request number) and reports a
    dead follower to every request that still expects something from it."""

    def __init__(self, link: LinkServer):
        self.link = link
        self.shares: Dict[int, _Share] = {}
        self.lock = threading.Lock()
        link.on_message = self._on_message
        link.on_dead = self._on_dead

    def open(self, seq: int, ranks) -> _Share:
        sh = _Share(asyncio.get_running_loop(), ranks)
        with self.lock:
            self.shares[seq] = sh
        return sh

    def close(self, seq: int) -> Optional[_Share]:
        with self.lock:
            return self.shares.pop(seq, None)

    def _on_message(self, rank: int, msg) -> None:
        kind, seq = msg[0], msg[1]
        with self.lock:
            sh = self.shares.get(seq)
        if sh is not None:
            sh.post((kind, rank) + tuple(msg[2:]))

    def _on_dead(self, rank: int) -> None:
        with self.lock:
            shares = [sh for sh in self.shares.values() if rank in sh.ranks]
        for sh in shares:
            sh.post(("dead", rank))


def _bound(ctx) -> float:
    """Seconds a request waits for its followers: its deadline plus a grace, else LWC_SHARD_WAIT_S."""
    dl = ctx.get("deadline") if isinstance(ctx, dict) else None
    if dl is not None:
        return max(0.0, dl - time.monotonic()) + float(os.environ.get("LWC_SHARD_GRACE_S", "5"))
    return float(os.environ.get("LWC_SHARD_WAIT_S", "300"))


class ShardedScoreClient(ScoreClient):
    """Rank 0's score client in a voter-sharded deployment (see the module docstring)."""

    def __init__(self, chat_client, link: LinkServer, world: int, **kw):
        super().__init__(chat_client, **kw)
        self.link, self.world = link, world
        self.hub = _LinkHub(link)
        self.seed_base = int(self.rng.getrandbits(63) if kw.get("rng_seed") is None else kw["rng_seed"])
        self.rng.seed(self.seed_base)
        self._seq = 0
        self._seq_lock = threading.Lock()
        self.consensus = None  # ShardedConsensusClient (shard_voters)

    # ------------------------------------------------------------------ request numbering
    def next_seq(self) -> int:
        with self._seq_lock:
            s = self._seq
            self._seq += 1
        return s

    def request_ctx(self, seq: int, ids=None, ctx=None) -> dict:
        """The request's context: the caller's (deadline, trace id, ...) plus its number, response ids and
        the voters' key-tree seed base (voter seeds depend on (seed base, request number) only, so a voter's
        prompt does not depend on which rank runs it)."""
        out = copy.copy(ctx) if isinstance(ctx, dict) else {}
        out.update(seq=seq, ids=ids if ids is not None else ScoreClient._new_ids(self),
                   seed=(self.seed_base * 1000003 + seq) & ((1 << 63) - 1))
        return out

    def _new_ids(self, ctx=None):
        return tuple(ctx["ids"])

    async def create_streaming(self, ctx, request: S.ScoreCompletionCreateParams):
        if not (isinstance(ctx, dict) and "seq" in ctx):
            ctx = self.request_ctx(self.next_seq(), ctx=ctx)
        return await super().create_streaming(ctx, request)

    async def create_unary(self, ctx, request: S.ScoreCompletionCreateParams) -> S.ScoreCompletion:
        if not (isinstance(ctx, dict) and "seq" in ctx):
            ctx = self.request_ctx(self.next_seq(), ctx=ctx)
        return await super().create_unary(ctx, request)

    # ------------------------------------------------------------------ fan-out over the ranks
    def _voter_sources(self, ctx, rid, created, indexer, model, weights, request, seeds) -> list:
        live = [0] + self.link.live()
        owner = {l.index: live[l.index % len(live)] for l in model.llms}
        mine = [l for l in model.llms if owner[l.index] == 0]
        shares: Dict[int, List[int]] = {}
        for l in model.llms:
            if owner[l.index] != 0:
                shares.setdefault(owner[l.index], []).append(l.index)
        sources = []
        seq = ctx["seq"]
        if shares:
            share = self.hub.open(seq, shares)
            rem = (ctx["deadline"] - time.monotonic()) if ctx.get("deadline") is not None else None
            base = {"rid": rid, "created": created, "model": model, "request": request, "weights": list(weights),
                    "seeds": list(seeds), "remaining": rem, "trace_id": ctx.get("trace_id"),
                    "priority": ctx.get("priority", 0)}
            for rank, idx in list(shares.items()):
                if not self.link.send(rank, ("score", seq, dict(base, llms=idx))):
                    # the rank died before taking its share: its voters run here
                    share.ranks.discard(rank)
                    mine += [l for l in model.llms if l.index in set(idx)]
                    del shares[rank]
            if shares:
                sources.append(self._remote(ctx, share, shares, indexer, model, weights, rid, created))
            else:
                self.hub.close(seq)
        pos = {l.index: j for j, l in enumerate(model.llms)}
        sources += [self._voter_stream(ctx, rid, created, indexer, l, weights[l.index], request, seeds[pos[l.index]])
                    for l in mine]
        return sources

    async def _remote(self, ctx, share: _Share, shares: Dict[int, List[int]], indexer: ChoiceIndexer, model,
                      weights, rid, created):
        """The followers' voters of one request as one chunk stream: re-indexed, weights re-stamped from the
        leader's (training-table weights learn here only), finished voters tracked so that a lost share
        turns exactly its unfinished voters into error choices."""
        llms = {l.index: l for l in model.llms}
        seen: Dict[int, Dict[int, bool]] = {i: {} for idx in shares.values() for i in idx}  # voter -> native -> done
        pending = set(shares)
        unfinished: set = set()  # ranks whose share was given up (timed out / ended by us): told to cancel
        deadline = time.monotonic() + _bound(ctx)
        try:
            while pending:
                try:
                    msg = await asyncio.wait_for(share.q.get(), timeout=max(0.0, deadline - time.monotonic()))
                except asyncio.TimeoutError:
                    msg = ("timeout", None)
                kind, rank = msg[0], msg[1]
                if kind == "chunk":
                    if rank not in pending:  # a share already closed (lost / timed out): its voters are final
                        continue
                    chunk = S.ScoreCompletionChunk.model_validate(msg[2])
                    base_c = int(msg[3])
                    for ch in chunk.choices:
                        v, native = divmod(ch.index - base_c, _NATIVE)
                        ch.index = indexer.get(v, native)
                        ch.weight = weights[v] if ch.weight is not None else None
                        done = seen.setdefault(v, {})
                        done[native] = done.get(native, False) or ch.finish_reason is not None
                    yield chunk
                elif kind == "end":
                    if rank not in pending:
                        continue
                    pending.discard(rank)
                    err = msg[2] if len(msg) > 2 else None
                    if err:
                        for c in self._lost_chunks(rid, created, model.id, indexer, llms, weights, shares[rank], seen,
                                                   _lost(rank, err)):
                            yield c
                elif kind in ("dead", "timeout"):
                    ranks = [rank] if kind == "dead" else sorted(pending)
                    for r in ranks:
                        if r not in pending:
                            continue
                        pending.discard(r)
                        if kind == "timeout":
                            unfinished.add(r)  # still alive: its voters must stop using its GPU
                        why = "follower died" if kind == "dead" else "share timed out"
                        for c in self._lost_chunks(rid, created, model.id, indexer, llms, weights, shares[r], seen,
                                                   _lost(r, why)):
                            yield c
        finally:
            self.hub.close(ctx["seq"])
            # abandoned (pending) or given-up (timed-out) shares: tell those followers to drop their voters
            for r in sorted(pending | unfinished):
                self.link.send(r, ("cancel", ctx["seq"]))

    @staticmethod
    def _lost_chunks(rid, created, model_id, indexer, llms, weights, voters, seen, err: StatusError):
        """Error choices for the unfinished voters of a lost share: a voter that streamed part of its
        output gets the error on the choices it started (as a mid-stream error, client.rs:798-813), one
        that never started gets one error choice (as an error before the first chunk, client.rs:711-783)."""
        re = ResponseError.from_status_error(err)
        choices = []
        for v in voters:
            l = llms[v]
            natives = seen.get(v) or {}
            todo = [k for k, done in natives.items() if not done] if natives else [0]
            for k in todo:
                choices.append(S.ScoreStreamChoice(delta=S.ScoreDelta(), finish_reason="error",
                                                   index=indexer.get(v, k), weight=weights[v], error=re,
                                                   model=l.id, model_index=v))
        if choices:
            yield S.ScoreCompletionChunk(id=rid, created=created, model=model_id, choices=choices)

    def _release(self, ctx) -> None:
        """The request's stream ended: normally ``_remote``'s own ``finally`` has already dropped the share;
        if that stream was cancelled before it ever ran (a generator that never starts never runs its
        ``finally``), drop it here and tell its followers to stop — no hub entry or follower work outlives the
        request."""
        seq = ctx.get("seq") if isinstance(ctx, dict) else None
        sh = self.hub.close(seq) if seq is not None else None
        if sh is not None:
            for r in sorted(sh.ranks):
                self.link.send(r, ("cancel", seq))

    def close(self) -> None:
        self.link.close()


class ShardedConsensusClient:
    """/consensus/completions over the ranks of a voter-sharded deployment (module docstring)."""

    def __init__(self, base, score_client: ShardedScoreClient):
        self.base, self.sc = base, score_client

    @staticmethod
    def split(n: int, ranks: List[int]) -> List[tuple]:
        """Contiguous candidate slices (rank, first, count) over ``ranks``."""
        W = len(ranks)
        share = [n // W + (1 if i < n % W else 0) for i in range(W)]
        out, first = [], 0
        for r, c in zip(ranks, share):
            out.append((r, first, c))
            first += c
        return out

    async def create_unary(self, ctx, request: C.ChatCompletionCreateParams, embedding_model: str,
                           tau: float = 0.05) -> S.ScoreCompletion:
        seq = self.sc.next_seq()
        return await self.run(self.sc.request_ctx(seq, ctx=ctx), request, embedding_model, tau)

    async def _slice(self, ctx, request, embedding_model, first: int, cnt: int):
        c2 = dict(ctx, candidates=(first, cnt, ctx["seed"]))
        comp, E, ntok = await self.base.generate_embedded(c2, request.model_copy(update={"n": cnt}), embedding_model)
        return comp, E.float(), ntok

    async def run(self, ctx, request: C.ChatCompletionCreateParams, embedding_model: str,
                  tau: float = 0.05) -> S.ScoreCompletion:
        import torch

        self.base._check_n(request)
        emb = self.base._embedder(embedding_model)
        seq, ids = ctx["seq"], ctx["ids"]
        slices = self.split(int(request.n), [0] + self.sc.link.live())
        remote = {r: (f, c) for r, f, c in slices if r != 0 and c}
        share = self.sc.hub.open(seq, remote) if remote else None
        for r, (f, c) in list(remote.items()):
            if not self.sc.link.send(r, ("consensus", seq, {"request": request, "embedding_model": embedding_model,
                                                            "first": f, "cnt": c, "seed": ctx["seed"]})):
                del remote[r]
                share.ranks.discard(r)
        local = [(f, c) for r, f, c in slices if (r == 0 or (r not in remote)) and c]
        parts: Dict[int, tuple] = {}  # first -> (comp, rows, ntok)
        pending = dict(remote)
        unfinished: set = set()
        try:
            for f, c in local:
                parts[f] = await self._slice(ctx, request, embedding_model, f, c)
            deadline = time.monotonic() + _bound(ctx)
            while pending:
                try:
                    msg = await asyncio.wait_for(share.q.get(), timeout=max(0.0, deadline - time.monotonic()))
                except asyncio.TimeoutError:
                    msg = ("timeout", None)
                kind, rank = msg[0], msg[1]
                if kind == "cons" and rank in pending:
                    f, c = pending.pop(rank)
                    meta, raw = msg[2], msg[3]
                    if meta[0]:
                        rows = torch.from_numpy(np.frombuffer(raw, dtype=np.float32).reshape(meta[1], meta[2]).copy())
                        parts[f] = (C.ChatCompletion.model_validate(meta[3]), rows, int(meta[4]))
                    else:  # the follower failed (e.g. out of memory): isolate it like a lost one
                        _log.warning("consensus slice [%d, %d) failed on rank %d (%s): recomputed here", f, f + c,
                                     rank, meta[3])
                        parts[f] = await self._slice(ctx, request, embedding_model, f, c)
                elif kind in ("dead", "timeout"):
                    lost = [rank] if kind == "dead" else list(pending)
                    for r in lost:  # recompute the lost slice here: same seeds, same candidates
                        if r in pending:
                            f, c = pending.pop(r)
                            if kind == "timeout":
                                unfinished.add(r)
                            parts[f] = await self._slice(ctx, request, embedding_model, f, c)
        finally:
            if share is not None:
                self.sc.hub.close(seq)
            for r in sorted(set(pending) | unfinished):  # abandoned or given up: free the follower's GPU
                self.sc.link.send(r, ("cancel", seq))
        order = sorted(parts)
        merged = parts[order[0]][0]
        for f in order[1:]:
            c = parts[f][0]
            merged.choices = merged.choices + c.choices
            if merged.usage is not None and c.usage is not None:  # every slice's generation (each ran the prompt)
                merged.usage.push(c.usage)
            elif c.usage is not None:
                merged.usage = c.usage.clone()
        merged.choices.sort(key=lambda c: c.index)
        rows = torch.cat([parts[f][1].to(emb.encoder.device) for f in order])
        ntok = sum(parts[f][2] for f in order)
        out = self.base.build(merged, rows, ntok, embedding_model, tau)
        out.id = f"cnscpl-{ids[1].split('-', 1)[-1]}"
        out.created = ids[0]
        if self.base.archive is not None:
            self.base.archive.store_score(out)
        return out


# ---------------------------------------------------------------------------------------------
# followers


class ShardWorker:
    """A follower rank: runs the voter shares and candidate slices the leader sends, streaming results back."""

    def __init__(self, score: ScoreClient, consensus, link: LinkClient):
        self.score, self.consensus, self.link = score, consensus, link
        self.tasks: Dict[int, asyncio.Task] = {}

    async def _score_share(self, seq: int, p: dict) -> None:
        request, model = p["request"], p["model"]
        C_len = len(request.choices)
        indexer = _TagIndexer(C_len)
        ctx = {"trace_id": p.get("trace_id"), "priority": p.get("priority", 0), "seq": seq,
               "deadline": time.monotonic() + p["remaining"] if p.get("remaining") is not None else None}
        llms = {l.index: l for l in model.llms}
        pos = {l.index: j for j, l in enumerate(model.llms)}
        err = None

        async def one(v: int) -> None:
            l = llms[v]
            async for chunk in self.score._voter_stream(ctx, p["rid"], p["created"], indexer, l, p["weights"][v],
                                                        request, p["seeds"][pos[v]]):
                if not self.link.send(("chunk", seq, chunk.to_obj(), C_len)):
                    raise ConnectionError("leader link lost")

        tasks = [asyncio.ensure_future(one(v)) for v in p["llms"]]
        try:
            for t in asyncio.as_completed(tasks):
                await t  # the first failure ends the share: the leader isolates all of its voters at once
        except asyncio.CancelledError:
            err = "cancelled"
        except BaseException as e:  # noqa: BLE001 — reported to the leader, which isolates these voters
            err = f"{type(e).__name__}: {e}"
        finally:
            for t in tasks:  # no sibling keeps streaming after the share ended
                t.cancel()
            await asyncio.gather(*tasks, return_exceptions=True)
        self.link.send(("end", seq, err))

    async def _consensus_slice(self, seq: int, p: dict) -> None:
        meta, raw = None, b""
        try:
            ctx = {"seq": seq, "candidates": (p["first"], p["cnt"], p["seed"])}
            req = p["request"].model_copy(update={"n": p["cnt"]})
            comp, E, ntok = await self.consensus.generate_embedded(ctx, req, p["embedding_model"])
            rows = E.float().cpu().numpy()
            meta = (True, int(rows.shape[0]), int(rows.shape[1]), comp.to_obj(), int(ntok))
            raw = rows.tobytes()
        except BaseException as e:  # noqa: BLE001
            meta = (False, 0, 0, f"{type(e).__name__}: {e}", 0)
        self.link.send(("cons", seq, meta, raw))

    def serve(self) -> int:
        """Run until the leader says stop (or the link drops); returns the number of pieces of work run."""

        async def main() -> int:
            loop = asyncio.get_running_loop()
            done = asyncio.Event()
            count = [0]

            def start(msg) -> None:
                kind, seq = msg[0], msg[1]
                if kind == "cancel":
                    t = self.tasks.get(seq)
                    if t is not None:
                        t.cancel()
                    return
                count[0] += 1
                coro = self._score_share(seq, msg[2]) if kind == "score" else self._consensus_slice(seq, msg[2])
                t = asyncio.ensure_future(coro)
                self.tasks[seq] = t
                t.add_done_callback(lambda _t, s=seq: self.tasks.pop(s, None))

            def receive() -> None:
                while True:
                    msg = self.link.recv()
                    if msg is None or msg[0] == "stop":
                        loop.call_soon_threadsafe(done.set)
                        return
                    loop.call_soon_threadsafe(start, msg)

            threading.Thread(target=receive, name="shard-follow", daemon=True).start()
            await done.wait()
            if self.tasks:
                await asyncio.gather(*list(self.tasks.values()), return_exceptions=True)
            return count[0]

        n = asyncio.run(main())
        self.link.close()
        return n
