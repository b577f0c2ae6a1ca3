"""Voter weight fetchers.

* ``StaticWeights`` — each voter's static weight (reference src/score/completions/weight.rs:76-97).
* ``TrainingTableWeights`` — the reference ships only a panicking stub (:99-117) for this mode; the
  types (src/score/model/mod.rs:278-306: embeddings model + `top`; per-voter base/min/max weights in
  src/score/llm/mod.rs:663-688) imply the design implemented here [INFERRED, documented]:
    1. embed the request transcript (`template_content()`, truncated to `embeddings.max_tokens`) with
       the local BGE encoder (K9*, L2-normalised);
    2. find the `top` most similar rows of the model's training table (cosine = one MFMA GEMV);
    3. each voter's weight = clamp(base_weight * 2 * a, min_weight, max_weight), where a is the
       similarity-weighted mean of that voter's historical agreement with the consensus (its score
       `confidence`) on those neighbours (a = 0.5 -> base weight; no neighbours -> base weight).
  The table learns online: after each scored request the orchestrator records the transcript
  embedding and every voter's confidence (`record`).  The embeddings response is returned to the
  client in `weight_data` exactly as the reference's `TrainingTableData` carries it.
"""
from __future__ import annotations

import asyncio
import threading
from typing import Any, Dict, List, Optional, Tuple

import torch

from ..errors import ResponseError, ResponseErrorException
from ..schema import chat as C
from ..schema import score as S
from .model import Model


class StaticWeights:
    async def fetch(self, ctx: Any, request, model: Model) -> Tuple[List[float], Any]:
        return [l.base.weight.weight for l in model.llms], S.WeightDataStatic()


class TrainingTable:
    """Rows of (unit embedding, {training_table_index: agreement}) for one training-table id."""

    def __init__(self, dim: int, device):
        self.E = torch.empty(0, dim, dtype=torch.float32, device=device)
        self.scores: List[Dict[int, float]] = []

    def add(self, e: torch.Tensor, s: Dict[int, float]) -> None:
        self.E = torch.cat([self.E, e.view(1, -1).to(self.E)], 0)
        self.scores.append(dict(s))


class TrainingTableWeights:
    def __init__(self, embedder=None):
        """`embedder(texts, max_tokens) -> (unit f32 [n, d], usage_tokens)`; None => 501 Not Implemented."""
        self.embedder = embedder
        self.tables: Dict[str, TrainingTable] = {}
        self.lock = threading.Lock()

    def _embed(self, text: str, max_tokens: int):
        if self.embedder is None:
            raise ResponseErrorException(ResponseError(code=501, message={
                "kind": "not_implemented", "error": "training-table weights need an embeddings model"}))
        return self.embedder([text], max_tokens)

    async def fetch(self, ctx: Any, request, model: Model) -> Tuple[List[float], Any]:
        w = model.weight
        text = request.template_content()
        loop = asyncio.get_running_loop()
        E, ntok = await loop.run_in_executor(None, self._embed, text, w.embeddings.max_tokens)
        e = E[0].float()
        with self.lock:
            table = self.tables.get(model.training_table_id)
        weights = []
        if table is None or table.E.shape[0] == 0:
            agree = {}
        else:
            sims = table.E @ e.to(table.E)
            k = min(w.top, sims.numel())
            vals, idx = sims.topk(k)
            vals = vals.clamp_min(0).tolist()
            idx = idx.tolist()
            agree = {}
            for l in model.llms:
                num = den = 0.0
                for s, i in zip(vals, idx):
                    a = table.scores[i].get(l.training_table_index)
                    if a is not None:
                        num += s * a
                        den += s
                if den > 0:
                    agree[l.index] = num / den
        for l in model.llms:
            tw = l.base.weight
            a = agree.get(l.index, 0.5)
            weights.append(min(max(tw.base_weight * 2.0 * a, tw.min_weight), tw.max_weight))
        resp = S.CreateEmbeddingResponse(
            data=[S.EmbeddingItem(embedding=[float(x) for x in e.tolist()], index=0)],
            model=w.embeddings.model,
            usage=C.Usage(prompt_tokens=ntok, total_tokens=ntok))
        return weights, S.WeightDataTrainingTable(embeddings_response=resp)

    def record(self, model: Model, embedding: List[float], voter_conf: Dict[int, float]) -> None:
        """Add one scored request: voter_conf maps llm.index -> confidence (agreement) in [0, 1]."""
        if model.training_table_id is None or not embedding:
            return
        e = torch.tensor(embedding, dtype=torch.float32)
        with self.lock:
            t = self.tables.get(model.training_table_id)
            if t is None:
                t = TrainingTable(e.numel(), "cpu")
                self.tables[model.training_table_id] = t
            by_tt = {model.llms[i].training_table_index: c for i, c in voter_conf.items()}
            t.add(e, by_tt)


class WeightFetchers:
    """Dispatch on the model's weight type (reference weight.rs:40-64)."""

    def __init__(self, static=None, training_table=None):
        self.static = static or StaticWeights()
        self.training_table = training_table or TrainingTableWeights()

    async def fetch(self, ctx, request, model: Model):
        if model.weight_type == "static":
            return await self.static.fetch(ctx, request, model)
        return await self.training_table.fetch(ctx, request, model)
