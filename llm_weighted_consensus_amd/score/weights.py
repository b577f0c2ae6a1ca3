"""Voter weight fetchers.

* ``StaticWeights`` — each voter's static weight (reference src/score/completions/weight.rs:76-97).
* ``TrainingTableWeights`` — the reference ships only a panicking stub (:99-117) for this mode; the
  types (src/score/model/mod.rs:278-306: embeddings model + `top`; per-voter base/min/max weights in
  src/score/llm/mod.rs:663-688) imply the design implemented here [INFERRED, documented]:
    1. embed the request transcript (`template_content()`, truncated to `embeddings.max_tokens`) with
       the local BGE encoder (K9*, L2-normalised);
    2. find the `top` most similar rows of the model's training table (cosine = one GEMV over the
       table, resident on the embedder's GPU);
    3. each voter's weight = clamp(base_weight * 2 * a, min_weight, max_weight), where a is the
       similarity-weighted mean of that voter's historical agreement with the consensus (its score
       `confidence`) on those neighbours (a = 0.5 -> base weight; no neighbours -> base weight).
  The table learns online: after each scored request the orchestrator records the transcript
  embedding and every voter's confidence (`record`), appended to ``LWC_TRAINING_TABLE_PATH`` (JSONL)
  and replayed on start.  The embeddings response is returned to the
  client in `weight_data` exactly as the reference's `TrainingTableData` carries it.
"""
from __future__ import annotations

import asyncio
import json
import os
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
    """Rows of (unit embedding, per-voter agreement) for one training-table id, resident on the
    embedder's device.  Storage is preallocated and doubled on demand (amortised O(1) per row — no
    per-row concatenation); agreements are a dense [rows, voters] matrix with NaN where a voter (by its
    ``training_table_index``) took no part or failed."""

    def __init__(self, dim: int, device, capacity: int = 64):
        self.dim = dim
        self.device = torch.device(device)
        self.n = 0
        self._E = torch.zeros(capacity, dim, dtype=torch.float32, device=self.device)
        self._A = torch.full((capacity, 1), float("nan"), dtype=torch.float32, device=self.device)

    @property
    def E(self) -> torch.Tensor:
        return self._E[:self.n]

    @property
    def A(self) -> torch.Tensor:
        return self._A[:self.n]

    def add(self, e: torch.Tensor, s: Dict[int, float]) -> None:
        cols = max(s, default=-1) + 1
        if self.n == self._E.shape[0] or cols > self._A.shape[1]:
            cap = self._E.shape[0] * (2 if self.n == self._E.shape[0] else 1)
            E2 = torch.zeros(cap, self.dim, dtype=torch.float32, device=self.device)
            E2[:self.n] = self._E[:self.n]
            A2 = torch.full((cap, max(cols, self._A.shape[1])), float("nan"), dtype=torch.float32, device=self.device)
            A2[:self.n, :self._A.shape[1]] = self._A[:self.n]
            self._E, self._A = E2, A2
        self._E[self.n] = e.reshape(-1).to(self._E)
        if s:
            row = torch.full((self._A.shape[1],), float("nan"), dtype=torch.float32)
            for k, v in s.items():
                row[int(k)] = float(v)
            self._A[self.n] = row.to(self.device)
        self.n += 1

    def agreement(self, e: torch.Tensor, top: int, tt_indices: List[int]) -> List[Optional[float]]:
        """Similarity-weighted mean agreement of each voter (by training-table index) over the ``top``
        nearest rows (cosine = one GEMV over the resident table; negative similarities weigh 0).  None
        where the voter has no neighbour rows."""
        if self.n == 0:
            return [None] * len(tt_indices)
        sims = self.E @ e.reshape(-1).to(self._E)
        k = min(int(top), self.n)
        vals, idx = sims.topk(k)
        vals = vals.clamp_min(0)
        cols = torch.tensor([i if i < self._A.shape[1] else 0 for i in tt_indices], dtype=torch.int64,
                            device=self.device)
        Ak = self._A[idx][:, cols]                                 # [k, voters]
        if any(i >= self._A.shape[1] for i in tt_indices):
            Ak[:, [j for j, i in enumerate(tt_indices) if i >= self._A.shape[1]]] = float("nan")
        have = ~torch.isnan(Ak)
        w = vals[:, None] * have
        den = w.sum(0)
        num = (w * torch.nan_to_num(Ak)).sum(0)
        out = torch.where(den > 0, num / den.clamp_min(1e-30), torch.full_like(den, float("nan"))).tolist()
        return [None if v != v else v for v in out]


class TrainingTableWeights:
    def __init__(self, embedder=None, path: Optional[str] = None, device=None):
        """`embedder(texts, max_tokens) -> (unit f32 [n, d], usage_tokens)`; None => 501 Not Implemented.
        ``path``: append-only JSONL of recorded rows, replayed on start (checkpoint / resume of what the
        tables have learned).  ``device``: where the tables live (default: the embedder's output device)."""
        self.embedder = embedder
        self.tables: Dict[str, TrainingTable] = {}
        self.lock = threading.Lock()
        self.device = device
        self.path = path
        if path and os.path.exists(path):
            self._replay(path)

    def _replay(self, path: str) -> None:
        with open(path, "r", encoding="utf-8") as f:
            for line in f:
                line = line.strip()
                if not line:
                    continue
                try:
                    o = json.loads(line)
                    self._add(o["table"], torch.tensor(o["embedding"], dtype=torch.float32),
                              {int(k): float(v) for k, v in o["scores"].items()})
                except (ValueError, KeyError, TypeError):
                    continue  # a torn last line after a crash

    def _add(self, table_id: str, e: torch.Tensor, by_tt: Dict[int, float]) -> None:
        t = self.tables.get(table_id)
        if t is None:
            t = TrainingTable(e.numel(), self.device or e.device)
            self.tables[table_id] = t
        t.add(e, by_tt)

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
        if self.device is None:
            self.device = e.device
        with self.lock:
            table = self.tables.get(model.training_table_id)
            agree = table.agreement(e, w.top, [l.training_table_index for l in model.llms]) if table else None
        weights = []
        for j, l in enumerate(model.llms):
            tw = l.base.weight
            a = agree[j] if agree is not None and agree[j] is not None else 0.5
            weights.append(min(max(tw.base_weight * 2.0 * a, tw.min_weight), tw.max_weight))
        resp = S.CreateEmbeddingResponse(
            data=[S.EmbeddingItem(embedding=[float(x) for x in e.tolist()], index=0)],
            model=w.embeddings.model,
            usage=C.Usage(prompt_tokens=ntok, total_tokens=ntok))
        return weights, S.WeightDataTrainingTable(embeddings_response=resp)

    def record(self, model: Model, embedding: List[float], voter_conf: Dict[int, float]) -> None:
        """Add one scored request: voter_conf maps llm.index -> confidence (agreement with the consensus)
        in [0, 1].  Called by the score orchestrator after every tally of a training-table model."""
        if model.training_table_id is None or not embedding or not voter_conf:
            return
        e = torch.tensor(embedding, dtype=torch.float32)
        by_tt = {model.llms[i].training_table_index: float(c) for i, c in voter_conf.items()}
        with self.lock:
            self._add(model.training_table_id, e, by_tt)
            if self.path:
                with open(self.path, "a", encoding="utf-8") as f:
                    f.write(json.dumps({"table": model.training_table_id, "embedding": [float(x) for x in embedding],
                                        "scores": {str(k): v for k, v in by_tt.items()}}) + "\n")


class WeightFetchers:
    """Dispatch on the model's weight type (reference weight.rs:40-64)."""

    def __init__(self, static=None, training_table=None):
        self.static = static or StaticWeights()
        self.training_table = training_table or TrainingTableWeights()

    async def fetch(self, ctx, request, model: Model):
        if model.weight_type == "static":
            return await self.static.fetch(ctx, request, model)
        return await self.training_table.fetch(ctx, request, model)
