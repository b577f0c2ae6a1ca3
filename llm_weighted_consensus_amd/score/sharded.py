"""Voter-sharded scoring: one score request's voters spread over the ranks of a process group (C2).

The reference fans a request's voters out as concurrent upstream streams and tallies their votes in one
place (src/score/completions/client.rs:343-356 fan-out, :384-455 tally).  Here every rank of ``group``
runs the SAME request (SPMD: same requests, same order, one at a time) through the ordinary
``ScoreClient`` but only for the voters it owns (``llm.index % world == rank``, i.e. the voters whose
models its GPU serves); the ranks then meet twice per request:

  1. tally (parallel/votes.py ``tally_across``): one all-reduce of the [choices + 1] fp64 partial
     choice weights — every rank ends with the global weights / confidences and its own voters'
     confidences, exactly the single-process tally up to summation order;
  2. response (``create_unary``): one object all-gather of every rank's voter choices and voter usage;
     the merged response lists the provided choices (global weights) followed by every voter's choice,
     ordered by voter index.

Ids, created timestamps and the key-tree seeds match on every rank (rank 0's id is broadcast; the seeds
are drawn for all voters in model order on every rank), so a voter's prompt is the same whichever rank
runs it.  Streaming is per rank (its own voters' chunks, then the global final chunk); the merged view
is the unary response.
"""
from __future__ import annotations

import torch.distributed as dist

from ..parallel import votes as V
from ..schema import chat as C
from ..schema import score as S
from .choices import message_to_delta
from .orchestrator import ScoreClient


class ShardedScoreClient(ScoreClient):
    def __init__(self, chat_client, group=None, **kw):
        super().__init__(chat_client, **kw)
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        # one key-tree seed stream on every rank (rank 0's): a voter's prompt does not depend on its rank
        self.rng.seed(V.broadcast_object(self.rng.getrandbits(63) if kw.get("rng_seed") is None else kw["rng_seed"],
                                         0, group))
        self.voter_filter = lambda llm: llm.index % self.world == self.rank

    def _new_ids(self):
        return V.broadcast_object(super()._new_ids(), 0, self.group)

    def _combine(self, votes, wts, C_len, any_ok, codes):
        tally, all_error = V.tally_across(votes, wts, C_len, any_ok, self.group)
        if all_error:  # a global decision: every rank takes this branch together
            codes = [c for part in V.gather_objects(list(codes), self.group) for c in part]
        return tally, all_error, codes

    async def create_unary(self, ctx, request: S.ScoreCompletionCreateParams) -> S.ScoreCompletion:
        C_len = len(request.choices)
        out = await self._unary(ctx, request)
        mine = ([c.to_obj() for c in out.choices if c.index >= C_len], self._last_voter_usage.to_obj())
        parts = V.gather_objects(mine, self.group)
        voters = [S.ScoreUnaryChoice.model_validate(o) for choices, _ in parts for o in choices]
        voters.sort(key=lambda c: (c.model_index if c.model_index is not None else -1, c.index))
        for k, c in enumerate(voters):
            c.index = C_len + k
        merged = out.model_copy(deep=True)
        merged.choices = [c for c in merged.choices if c.index < C_len] + voters
        # usage: this rank's total (voters + any training-table embedding, counted once) + the other
        # ranks' voter usage
        usage = out.usage.clone() if out.usage is not None else C.Usage()
        for r, (_, u) in enumerate(parts):
            if r != self.rank:
                usage.push(C.Usage.model_validate(u))
        usage.total_cost = None
        usage.with_total_cost()
        merged.usage = usage
        if self.archive is not None and self.rank == 0:
            self.archive.store_score(merged)
        return merged


# ---------------------------------------------------------------------------------------------
# serving: rank 0 takes the HTTP requests and leads, the other ranks follow (SPMD)


class ScoreLeader:
    """Rank 0's score client in a voter-sharded deployment (``LWC_SHARD_VOTERS=1``): every score
    request is broadcast to the follower ranks (``follow``) before rank 0 runs its share, one request
    at a time (the collectives of concurrent requests must not interleave).  Streaming requests get
    the merged response as one chunk.  Everything else (model validation for multichat, ...) is the
    wrapped client's."""

    def __init__(self, client: ShardedScoreClient):
        self.client = client
        self._lock = None

    def __getattr__(self, name):
        return getattr(self.client, name)

    async def create_unary(self, ctx, request: S.ScoreCompletionCreateParams) -> S.ScoreCompletion:
        import asyncio

        if self._lock is None:
            self._lock = asyncio.Lock()
        async with self._lock:
            V.broadcast_object(request, 0, self.client.group)
            return await self.client.create_unary(ctx, request)

    async def create_streaming(self, ctx, request: S.ScoreCompletionCreateParams):
        out = await self.create_unary(ctx, request)

        async def one():
            yield as_chunk(out)

        return one()

    def close(self) -> None:
        V.broadcast_object(None, 0, self.client.group)


def as_chunk(out: S.ScoreCompletion) -> S.ScoreCompletionChunk:
    choices = []
    for c in out.choices:
        delta = message_to_delta(c.message)
        delta.vote = c.message.vote
        choices.append(S.ScoreStreamChoice(
            delta=delta, finish_reason=c.finish_reason, index=c.index, logprobs=c.logprobs, weight=c.weight,
            confidence=c.confidence, error=c.error, model=c.model, model_index=c.model_index,
            completion_metadata=c.completion_metadata))
    return S.ScoreCompletionChunk(id=out.id, choices=choices, created=out.created, model=out.model, usage=out.usage,
                                  weight_data=out.weight_data)


def follow(client: ShardedScoreClient) -> int:
    """Ranks > 0: run every request the leader broadcasts (their voters' share) until it sends None.
    Returns the number of requests served.  A request that fails fails on every rank alike (the
    all-votes-failed decision is global), so errors are dropped here — the leader reports them."""
    import asyncio

    from ..errors import StatusError

    n = 0
    while True:
        request = V.broadcast_object(None, 0, client.group)
        if request is None:
            return n
        try:
            asyncio.run(client.create_unary(None, request))
        except StatusError:
            pass
        n += 1
