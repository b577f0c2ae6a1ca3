"""Voter-sharded scoring: one score request's voters spread over the ranks of a process group (C2).

The reference fans a request's voters out as concurrent upstream streams and tallies their votes in one
place (src/score/completions/client.rs:343-356 fan-out, :384-455 tally).  Here every rank runs the SAME
requests (SPMD) through the ordinary ``ScoreClient`` but only for the voters it owns
(``llm.index % world == rank``: the voters whose models its GPU serves), and requests run CONCURRENTLY
on every rank, as on a single server.

C2 is ONE collective per request: when a request's local voters are done, each rank contributes its
voter choices (votes, weights, errors, content) to an object all-gather; every rank then holds every
voter of the request (its own under the indices it already streamed, the others' after them by voter
index), runs the native tally over all of them and finishes the request — rank 0's response is the full
one.  Collectives of concurrent requests must be issued in
the same order on every rank, so they go through a per-rank combiner thread that runs them strictly in
request sequence order (the leader numbers requests as it broadcasts them); a request that fails before
its combine still takes its slot (an empty contribution), so the ranks never fall out of step.

Requests and their ids reach the followers over a second process group (control), so broadcasts and
combines never interleave on one group.  Both groups are gloo: the payloads are small Python objects.
"""
from __future__ import annotations

import asyncio
import threading
from typing import Any, List

import torch.distributed as dist

from ..errors import ScoreError
from ..parallel import votes as V
from ..schema import chat as C
from ..schema import score as S
from .orchestrator import ScoreClient

_SKIP = None  # a request's empty contribution (it failed before its combine on this rank)


class _Combiner:
    """Runs each request's all-gather in sequence order on a thread of its own."""

    def __init__(self, group):
        self.group = group
        self.cv = threading.Condition()
        self.pending = {}
        self.next = 0
        self.closed = False
        self.thread = threading.Thread(target=self._run, name="c2-combiner", daemon=True)
        self.thread.start()

    async def submit(self, seq: int, payload: Any) -> List[Any]:
        loop = asyncio.get_running_loop()
        fut = loop.create_future()
        with self.cv:
            self.pending[seq] = (payload, loop, fut)
            self.cv.notify()
        return await fut

    def _run(self) -> None:
        while True:
            with self.cv:
                while self.next not in self.pending and not self.closed:
                    self.cv.wait()
                if self.next not in self.pending:
                    return
                payload, loop, fut = self.pending.pop(self.next)
                self.next += 1
            try:
                # a callable runs its own collectives (consensus: object + tensor all-gathers), else one
                # object all-gather of the payload
                res = payload() if callable(payload) else V.gather_objects(payload, self.group)
                loop.call_soon_threadsafe(_resolve, fut, res, None)
            except BaseException as e:  # noqa: BLE001 — handed to the awaiting request
                loop.call_soon_threadsafe(_resolve, fut, None, e)

    def close(self) -> None:
        with self.cv:
            self.closed = True
            self.cv.notify()
        self.thread.join(timeout=60)


def _resolve(fut, res, err) -> None:
    if fut.done():
        return
    if err is not None:
        fut.set_exception(err)
    else:
        fut.set_result(res)


class ShardedScoreClient(ScoreClient):
    """``ctx`` of every request is ``{"seq": n, "ids": (created, id)}`` (from :class:`ScoreLeader` /
    :func:`follow`, or given by the caller, identical on every rank)."""

    def __init__(self, chat_client, group=None, **kw):
        super().__init__(chat_client, **kw)
        self.group = group if group is not None else dist.new_group(backend="gloo")
        self.world = dist.get_world_size(self.group)
        self.rank = dist.get_rank(self.group)
        self.voter_filter = lambda llm: llm.index % self.world == self.rank
        # one key-tree seed base on every rank (rank 0's); each request's voter seeds derive from (base,
        # request number) — not from draws in arrival order, which concurrent requests make rank-dependent
        self.seed_base = int(V.broadcast_object(
            self.rng.getrandbits(63) if kw.get("rng_seed") is None else kw["rng_seed"], 0, self.group))
        self.rng.seed(self.seed_base)
        self.combiner = _Combiner(self.group)
        # C1 (consensus): candidate embedding rows all-gathered as device tensors on the world's backend
        # (RCCL over xGMI on a GPU node; gloo — host tensors — for CPU worlds and one-GPU rehearsals)
        self.data_group = dist.new_group()
        self.data_backend = dist.get_backend(self.data_group)

    def request_ctx(self, seq: int, ids) -> dict:
        """The per-request context every rank builds identically: sequence number (combine order), the
        response ids, and the voters' key-tree seed base."""
        return {"seq": seq, "ids": ids, "seed": (self.seed_base * 1000003 + seq) & ((1 << 63) - 1)}

    def _new_ids(self, ctx=None):
        return tuple(ctx["ids"])

    async def _combine(self, ctx, aggregate: S.ScoreCompletionChunk, C_len: int, any_ok: bool, codes, usage,
                       voter_usage):
        ctx["combined"] = True
        mine = aggregate.choices[C_len:]
        parts = await self.combiner.submit(ctx["seq"], (any_ok, list(codes), [c.to_obj() for c in mine],
                                                        voter_usage.to_obj()))
        remote, n_ok, all_codes = [], 0, []
        for r, part in enumerate(parts):
            if part is _SKIP:
                continue
            ok, cds, objs, u = part
            n_ok += bool(ok)
            all_codes += cds
            if r != self.rank:
                remote += [S.ScoreStreamChoice.model_validate(o) for o in objs]
                usage.push(C.Usage.model_validate(u))  # the other ranks' voters (an embedding's usage: once)
        # this rank's voters keep the indices its stream already used; the others' follow, by voter index
        remote.sort(key=lambda c: (c.model_index if c.model_index is not None else -1, c.index))
        for k, c in enumerate(remote):
            c.index = C_len + len(mine) + k
        ctx["whole"] = {c.index for c in remote}  # complete choices: the final chunk carries them as they are
        aggregate.choices = aggregate.choices + remote
        return await self._tally(aggregate.choices[C_len:], C_len), n_ok == 0, all_codes

    async def run(self, seq: int, ids, request: S.ScoreCompletionCreateParams) -> S.ScoreCompletion:
        """One request on this rank (unary); always takes its combine slot."""
        ctx = self.request_ctx(seq, ids)
        try:
            return await self.create_unary(ctx, request)
        finally:
            if not ctx.get("combined"):
                await self.combiner.submit(seq, _SKIP)

    async def open_stream(self, seq: int, ids, request: S.ScoreCompletionCreateParams):
        """One request on this rank, streamed: pre-stream errors raise here (the HTTP layer turns them
        into a status), then this rank's voter chunks are yielded as they arrive, and the final chunk
        carries the other ranks' voters whole plus the tally (the unary fold of the stream equals
        :meth:`run`).  The combine slot is always taken, also when the client abandons the stream."""
        ctx = self.request_ctx(seq, ids)
        try:
            it = await self.create_streaming(ctx, request)
        except BaseException:
            await self.combiner.submit(seq, _SKIP)
            raise

        async def gen():
            try:
                async for item in it:
                    yield item
            finally:
                if not ctx.get("combined"):
                    await self.combiner.submit(seq, _SKIP)

        return gen()

    def close(self) -> None:
        self.combiner.close()


class ShardedConsensusClient:
    """/consensus/completions over the ranks of a voter-sharded deployment: rank r samples candidates
    [first_r, first_r + n_r) of the request (contiguous split, each with the seed it has in the whole
    request) on its own engine and embeds them on its own GPU; ONE all-gather of the unit rows (C1: device
    tensors over RCCL) assembles the [n, d] matrix and an object all-gather the candidates' texts, so every
    rank builds the same response — rank 0's is served.  Collectives run on the request-ordered combiner
    shared with score requests."""

    def __init__(self, base, score_client: ShardedScoreClient):
        self.base, self.sc = base, score_client
        self.world, self.rank = score_client.world, score_client.rank

    def split(self, n: int):
        share = [n // self.world + (1 if r < n % self.world else 0) for r in range(self.world)]
        return sum(share[:self.rank]), share[self.rank]

    def _collect(self, meta, E):
        """Combiner thread: gather every rank's (meta, rows); rows [n, d] in candidate order on this rank's
        device, or None when a rank failed (every rank sees the same metas, so all skip the tensor call)."""
        import torch

        metas = V.gather_objects(meta, self.sc.group)
        if any(m is None or not m[0] for m in metas):
            return metas, None
        counts, d = [m[1] for m in metas], metas[0][2]
        mx = max(counts)
        if self.sc.data_backend != "nccl":
            dev = torch.device("cpu")
        else:
            dev = E.device if E is not None else torch.device("cuda", torch.cuda.current_device())
        pad = torch.zeros(mx, d, dtype=torch.float32, device=dev)
        if E is not None and E.shape[0]:
            pad[:E.shape[0]].copy_(E)
        out = torch.empty(self.world * mx, d, dtype=torch.float32, device=dev)
        dist.all_gather_into_tensor(out, pad, group=self.sc.data_group)
        rows = torch.cat([out[r * mx:r * mx + c] for r, c in enumerate(counts)])
        return metas, rows

    async def run(self, seq: int, ids, request: C.ChatCompletionCreateParams, embedding_model: str,
                  tau: float = 0.05) -> S.ScoreCompletion:
        ctx = self.sc.request_ctx(seq, ids)
        meta, E, err = None, None, None
        try:
            self.base._check_n(request)
            first, cnt = self.split(int(request.n))
            ctx["candidates"] = (first, cnt, ctx["seed"])
            if cnt:
                comp, E, ntok = await self.base.generate_embedded(ctx, request.model_copy(update={"n": cnt}),
                                                                  embedding_model)
                meta = (True, cnt, int(E.shape[1]), comp.to_obj(), int(ntok))
            else:
                emb = self.base._embedder(embedding_model)
                meta = (True, 0, int(emb.encoder.cfg.hidden), None, 0)
        except BaseException as e:  # noqa: BLE001 - every rank still takes the request's combine slot
            err = e
            meta = (False, 0, 0, f"{type(e).__name__}: {e}", 0)
        metas, rows = await self.sc.combiner.submit(seq, lambda: self._collect(meta, E))
        if err is not None:
            raise err
        if rows is None:
            bad = next((r, m[3]) for r, m in enumerate(metas) if m is None or not m[0])
            raise ScoreError(500, {"kind": "consensus_shard_failed",
                                   "error": f"rank {bad[0]} failed to generate or embed its candidates: {bad[1]}"})
        comps = [C.ChatCompletion.model_validate(m[3]) for m in metas if m[3] is not None]
        merged = comps[0]
        for c in comps[1:]:
            merged.choices = merged.choices + c.choices
            if merged.usage is not None and c.usage is not None:  # every rank's generation (each ran the prompt)
                merged.usage.push(c.usage)
            elif c.usage is not None:
                merged.usage = c.usage.clone()
        merged.choices.sort(key=lambda c: c.index)
        ntok = sum(m[4] for m in metas)
        emb = self.base._embedder(embedding_model)
        out = self.base.build(merged, rows.to(emb.encoder.device), ntok, embedding_model, tau)
        out.id = f"cnscpl-{ids[1].split('-', 1)[-1]}"  # one id on every rank (the leader's)
        out.created = ids[0]
        if self.rank == 0 and self.base.archive is not None:
            self.base.archive.store_score(out)
        return out


# ---------------------------------------------------------------------------------------------
# serving: rank 0 takes the HTTP requests and leads, the other ranks follow (SPMD)


class ScoreLeader:
    """Rank 0's score client in a voter-sharded deployment (``LWC_SHARD_VOTERS=1``): every score
    request is numbered and broadcast to the follower ranks (control group), then run here like on the
    followers — concurrently with the other requests in flight.  Streaming requests stream this rank's
    voters live, then the other ranks' voters and the tally in the final chunk.  Everything else (model
    validation for multichat, ...) is the wrapped client's.

    The broadcast is a blocking gloo call: it runs on ONE dedicated thread (FIFO, so request numbers are
    assigned and broadcast in submission order), never on the event loop, which keeps serving while a
    slow follower holds a broadcast."""

    def __init__(self, client: ShardedScoreClient, control=None):
        from concurrent.futures import ThreadPoolExecutor

        self.client = client
        self.control = control if control is not None else dist.new_group(backend="gloo")
        self._seq = 0
        self._lock = threading.Lock()
        self._announcer = ThreadPoolExecutor(max_workers=1, thread_name_prefix="c2-announce")

    def __getattr__(self, name):
        return getattr(self.client, name)

    def _announce_sync(self, request, kind: str = "score") -> tuple:
        with self._lock:
            seq = self._seq
            self._seq += 1
            ids = ScoreClient._new_ids(self.client)
            V.broadcast_object((seq, ids, kind, request), 0, self.control)
        return seq, ids

    async def _announce(self, request, kind: str = "score") -> tuple:
        return await asyncio.get_running_loop().run_in_executor(self._announcer, self._announce_sync, request, kind)

    async def create_unary(self, ctx, request: S.ScoreCompletionCreateParams) -> S.ScoreCompletion:
        seq, ids = await self._announce(request)
        return await self.client.run(seq, ids, request)

    async def create_streaming(self, ctx, request: S.ScoreCompletionCreateParams):
        seq, ids = await self._announce(request)
        return await self.client.open_stream(seq, ids, request)

    async def create_consensus(self, ctx, request: C.ChatCompletionCreateParams, embedding_model: str,
                               tau: float = 0.05) -> S.ScoreCompletion:
        seq, ids = await self._announce((request, embedding_model, tau), "consensus")
        return await self.client.consensus.run(seq, ids, request, embedding_model, tau)

    def close(self) -> None:
        self._announcer.shutdown(wait=True)
        V.broadcast_object(None, 0, self.control)
        self.client.close()


class ConsensusLeader:
    """Rank 0's /consensus/completions client in a voter-sharded deployment (see ShardedConsensusClient)."""

    def __init__(self, leader: ScoreLeader):
        self.leader = leader

    async def create_unary(self, ctx, request: C.ChatCompletionCreateParams, embedding_model: str,
                           tau: float = 0.05) -> S.ScoreCompletion:
        return await self.leader.create_consensus(ctx, request, embedding_model, tau)


def follow(client: ShardedScoreClient, control=None) -> int:
    """Ranks > 0: run every request the leader broadcasts (their voters' share), concurrently, until it
    sends None; returns the number of requests run.  A failed request fails on every rank alike and the
    leader reports it, so errors are dropped here."""
    from ..errors import StatusError

    control = control if control is not None else dist.new_group(backend="gloo")

    async def main() -> int:
        loop = asyncio.get_running_loop()
        tasks: List[asyncio.Future] = []
        done = asyncio.Event()

        async def one(seq, ids, kind, request):
            try:
                if kind == "consensus":
                    await client.consensus.run(seq, ids, *request)
                else:
                    await client.run(seq, ids, request)
            except StatusError:
                pass

        def receive() -> None:
            while True:
                msg = V.broadcast_object(None, 0, control)
                if msg is None:
                    loop.call_soon_threadsafe(done.set)
                    return
                loop.call_soon_threadsafe(lambda m=msg: tasks.append(asyncio.ensure_future(one(*m))))

        t = threading.Thread(target=receive, name="c2-follow", daemon=True)
        t.start()
        await done.wait()
        await asyncio.gather(*tasks)
        return len(tasks)

    n = asyncio.run(main())
    client.close()
    return n
