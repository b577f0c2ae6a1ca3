"""Multichat completions (N candidate answers from a set of LLMs) and embedding consensus.

The reference ships only the response types (src/multichat/completions/response.rs:1-226) and the
multichat identity of a score model (src/score/model/mod.rs:115-189); the generator and the
embedding-consensus scorer are this framework's [NEW] endpoints:

* ``MultichatClient.create_streaming`` — the voter fan-out without the selection prompt: every LLM of
  the model answers the conversation; choices are indexed first-arrival (ChoiceIndexer from 0) and
  carry model / model_index / completion_metadata / error like score voter choices.
* ``ConsensusClient.create_unary`` — self-consistency: sample n candidates from ONE local model
  (prefix-shared on the GPU), embed them with the BGE encoder, cosine-consensus (MFMA GEMM +
  row-reduce kernel) and return a score-format completion whose `weight` is each candidate's
  centrality and `confidence` its softmax weight.
"""
from __future__ import annotations

import asyncio
import time
import uuid
from typing import Any, List, Optional

import torch

from .. import ops
from ..errors import ResponseError, ScoreError, StatusError
from ..schema import chat as C
from ..schema import score as S
from .orchestrator import ChoiceIndexer, ScoreClient


class MultichatClient:
    def __init__(self, score_client: ScoreClient, archive=None):
        self.score = score_client
        self.chat = score_client.chat
        self.archive = archive

    async def create_streaming(self, ctx, request: S.ScoreCompletionCreateParams):
        created = int(time.time())
        rid = f"mltcpl-{uuid.uuid4().hex}-{created}"
        model = await self.score.fetch_or_validate_model(ctx, request.model)
        indexer = ChoiceIndexer(0)
        q: asyncio.Queue = asyncio.Queue()
        DONE = object()

        async def one(llm):
            b = llm.base
            params = C.ChatCompletionCreateParams(
                messages=list(b.prefix_messages or []) + list(request.messages) + list(b.suffix_messages or []),
                model=b.model, frequency_penalty=b.frequency_penalty, logit_bias=b.logit_bias,
                max_completion_tokens=b.max_completion_tokens, presence_penalty=b.presence_penalty, seed=request.seed,
                stop=b.stop, stream=request.stream, stream_options=request.stream_options, temperature=b.temperature,
                tools=request.tools, top_p=b.top_p, max_tokens=b.max_tokens, min_p=b.min_p, provider=b.provider,
                reasoning=b.reasoning, repetition_penalty=b.repetition_penalty, top_a=b.top_a, top_k=b.top_k,
                usage=request.usage, verbosity=b.verbosity, models=b.models)
            try:
                stream = await self.chat.create_streaming(ctx, params)
                async for ch in stream:
                    out = S.MultichatCompletionChunk(id=rid, created=created, model=model.multichat_id, choices=[
                        S.MultichatStreamChoice(
                            delta=c.delta, finish_reason=c.finish_reason, index=indexer.get(llm.multichat_index,
                                                                                            c.index),
                            logprobs=c.logprobs, model=llm.multichat_id, model_index=llm.multichat_index,
                            completion_metadata=S.CompletionMetadata(
                                id=ch.id, created=ch.created, model=ch.model, service_tier=ch.service_tier,
                                system_fingerprint=ch.system_fingerprint, usage=ch.usage, provider=ch.provider))
                        for c in ch.choices])
                    await q.put(out)
            except StatusError as e:
                await q.put(S.MultichatCompletionChunk(id=rid, created=created, model=model.multichat_id, choices=[
                    S.MultichatStreamChoice(delta=C.Delta(), finish_reason="error",
                                            index=indexer.get(llm.multichat_index, 0),
                                            error=ResponseError.from_status_error(e), model=llm.multichat_id,
                                            model_index=llm.multichat_index)]))
            finally:
                await q.put(DONE)

        tasks = [asyncio.create_task(one(l)) for l in model.llms]

        async def gen():
            pending = len(tasks)
            usage = C.Usage()
            try:
                while pending:
                    item = await q.get()
                    if item is DONE:
                        pending -= 1
                        continue
                    for c in item.choices:
                        if c.completion_metadata is not None and c.completion_metadata.usage is not None:
                            usage.push(c.completion_metadata.usage)
                    yield item
            finally:
                for t in tasks:
                    t.cancel()
            usage.with_total_cost()
            yield S.MultichatCompletionChunk(id=rid, created=created, model=model.multichat_id, choices=[],
                                             usage=usage)

        return gen()

    async def create_unary(self, ctx, request) -> S.MultichatCompletion:
        agg = None
        async for ch in await self.create_streaming(ctx, request):
            if agg is None:
                agg = ch.clone()
            else:
                agg.push(ch)
        out = S.MultichatCompletion.from_chunk(agg)
        if self.archive is not None:
            self.archive.store_multichat(out)
        return out


class ConsensusClient:
    """Embedding self-consistency over n sampled candidates of one local model."""

    def __init__(self, chat_client, embedders: dict, archive=None):
        self.chat = chat_client
        self.embedders = embedders
        self.archive = archive

    async def create_unary(self, ctx, request: C.ChatCompletionCreateParams, embedding_model: str,
                           tau: float = 0.05) -> S.ScoreCompletion:
        emb = self._embedder(embedding_model)
        self._check_n(request)
        comp, E, ntok = await self.generate_embedded(ctx, request, embedding_model)
        out = self.build(comp, E.to(emb.encoder.device), ntok, embedding_model, tau)
        if self.archive is not None:
            self.archive.store_score(out)
        return out

    def _embedder(self, embedding_model: str):
        emb = self.embedders.get(embedding_model)
        if emb is None:
            raise ScoreError(404, {"kind": "model_not_found", "error": f"embedding model not served: {embedding_model}"})
        return emb

    @staticmethod
    def _check_n(request) -> int:
        n = int(request.n or 1)
        if n < 2:
            raise ScoreError.expected_two_or_more_choices(n)
        return n

    async def generate_embedded(self, ctx, request: C.ChatCompletionCreateParams, embedding_model: str):
        """The request's candidates (all of them, or the ``ctx["candidates"]`` slice of a sharded request)
        and their unit embeddings: (ChatCompletion, rows [n, d] float32 in choice order, embedding tokens)."""
        emb = self._embedder(embedding_model)
        local = getattr(self.chat, "local", self.chat)
        if hasattr(local, "can_embed_in_workers") and local.can_embed_in_workers(request, embedding_model):
            # multi-GPU: every EngineGroup worker embeds the candidates it generated on its own GPU;
            # only the unit rows come back (no candidate text is re-encoded on the front end's GPU)
            comp, rows, ntok = await local.create_unary_embedded(ctx, request, embedding_model)
            return comp, torch.from_numpy(rows).to(emb.encoder.device), ntok
        comp = await self.chat.create_unary(ctx, request)
        texts = [c.message.content or "" for c in sorted(comp.choices, key=lambda c: c.index)]
        loop = asyncio.get_running_loop()
        E, ntok = await loop.run_in_executor(None, emb.embed_texts, texts)
        return comp, E.float(), ntok

    @staticmethod
    def build(comp, E: torch.Tensor, ntok: int, embedding_model: str, tau: float) -> S.ScoreCompletion:
        """The consensus response over the candidates of ``comp`` (choice c <-> row c.index of E)."""
        n = E.shape[0]
        Eb = E.to(torch.bfloat16).unsqueeze(0).contiguous()
        if Eb.is_cuda:
            _, cen, w, best = ops.cosine_consensus(Eb, tau)
            cen, w = cen[0].tolist(), w[0].tolist()
        else:  # CPU plumbing path (tests / no GPU): same math in torch
            Sm = E @ E.t()
            cen_t = (Sm.sum(1) - Sm.diagonal()) / max(1, n - 1)
            cen, w = cen_t.tolist(), torch.softmax(cen_t / tau, 0).tolist()
        created = int(time.time())
        usage = comp.usage.clone() if comp.usage else C.Usage()
        usage.push(C.Usage(prompt_tokens=ntok, total_tokens=ntok))
        choices = []
        for c in comp.choices:
            m = S.ScoreUnaryMessage(**{k: getattr(c.message, k) for k in C.UnaryMessage.model_fields})
            choices.append(S.ScoreUnaryChoice(message=m, finish_reason=c.finish_reason, index=c.index,
                                              logprobs=c.logprobs, weight=cen[c.index], confidence=w[c.index],
                                              model=comp.model, completion_metadata=S.CompletionMetadata(
                                                  id=comp.id, created=comp.created, model=comp.model,
                                                  provider=comp.provider)))
        return S.ScoreCompletion(id=f"cnscpl-{uuid.uuid4().hex}-{created}", choices=choices, created=created,
                                 model=comp.model, usage=usage,
                                 weight_data=S.WeightDataTrainingTable(embeddings_response=S.CreateEmbeddingResponse(
                                     data=[S.EmbeddingItem(embedding=[float(x) for x in r], index=i)
                                           for i, r in enumerate(E.double().cpu().tolist())],
                                     model=embedding_model, usage=C.Usage(prompt_tokens=ntok, total_tokens=ntok))))
