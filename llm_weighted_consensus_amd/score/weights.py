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
    embedder's device.  Storage is preallocated and doubled on demand up to ``max_rows`` (amortised O(1) per
    row — no per-row concatenation), then a ring: the oldest row is overwritten (bounded memory, recent
    history wins).  Agreements are a dense [rows, voters] matrix with NaN where a voter (by its
    ``training_table_index``) took no part or failed."""

    def __init__(self, dim: int, device, capacity: int = 64, max_rows: int = 1 << 20):
        self.dim = dim
        self.device = torch.device(device)
        self.max_rows = max(1, int(max_rows))
        self.n = 0      # rows held (<= max_rows)
        self.head = 0   # next row to overwrite once the ring is full (= the oldest row)
        capacity = min(capacity, self.max_rows)
        self._seq = [0] * capacity  # the journal sequence number of each row (compaction cut-off)
        self._E = torch.zeros(capacity, dim, dtype=torch.float32, device=self.device)
        self._A = torch.full((capacity, 1), float("nan"), dtype=torch.float32, device=self.device)

    @property
    def E(self) -> torch.Tensor:
        return self._E[:self.n]

    @property
    def A(self) -> torch.Tensor:
        return self._A[:self.n]

    def _grow(self, rows: int, cols: int) -> None:
        E2 = torch.zeros(rows, self.dim, dtype=torch.float32, device=self.device)
        E2[:self.n] = self._E[:self.n]
        A2 = torch.full((rows, cols), float("nan"), dtype=torch.float32, device=self.device)
        A2[:self.n, :self._A.shape[1]] = self._A[:self.n]
        self._E, self._A = E2, A2
        self._seq = self._seq + [0] * (rows - len(self._seq))

    def add(self, e: torch.Tensor, s: Dict[int, float], seq: int = 0) -> None:
        cols = max(max(s, default=-1) + 1, self._A.shape[1])
        cap = self._E.shape[0]
        grow_rows = self.n == cap and cap < self.max_rows
        if grow_rows or cols > self._A.shape[1]:
            self._grow(min(self.max_rows, cap * 2) if grow_rows else cap, cols)
        if self.n < self._E.shape[0]:
            i = self.n
            self.n += 1
        else:  # full ring: overwrite the oldest row
            i = self.head
            self.head = (self.head + 1) % self.n
        self._E[i] = e.reshape(-1).to(self._E)
        self._seq[i] = seq
        row = torch.full((self._A.shape[1],), float("nan"), dtype=torch.float32)
        for k, v in s.items():
            row[int(k)] = float(v)
        self._A[i] = row.to(self.device)

    def rows_in_order(self, upto: Optional[int] = None):
        """(E, A) on the host, oldest row first (compaction rewrites the journal in this order); ``upto``: only
        the rows recorded with journal sequence numbers <= upto."""
        order = list(range(self.head, self.n)) + list(range(0, self.head))
        if upto is not None:
            order = [i for i in order if self._seq[i] <= upto]
        idx = torch.tensor(order, dtype=torch.int64, device=self.device)
        return self._E.index_select(0, idx).cpu(), self._A.index_select(0, idx).cpu()

    def nearest(self, e: torch.Tensor, k: int):
        """(similarities [k], rows [k]) of the k nearest rows: the K10c kernel on the GPU, torch elsewhere."""
        q = e.reshape(-1).to(self._E)
        if self._E.is_cuda and k <= 64 and self.dim % 4 == 0:
            from .. import ops

            return ops.knn_topk(self.E, q, k)
        return (self.E @ q).topk(k)

    def agreement(self, e: torch.Tensor, top: int, tt_indices: List[int]) -> List[Optional[float]]:
        """Similarity-weighted mean agreement of each voter (by training-table index) over the ``top``
        nearest rows (negative similarities weigh 0).  None where the voter has no neighbour rows."""
        if self.n == 0:
            return [None] * len(tt_indices)
        k = min(int(top), self.n)
        vals, idx = self.nearest(e, k)
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


class _Journal:
    """Append-only JSONL of training-table rows, written by a thread of its own (the event loop only
    enqueues), compacted once it holds ``compact_factor`` x the retained rows: rewritten from the in-memory
    tables (oldest row first) into a temporary file that atomically replaces it."""

    def __init__(self, path: str, snapshot, lines: int = 0, compact_factor: float = 2.0, min_lines: int = 4096):
        import queue

        self.path, self.snapshot = path, snapshot
        self.lines, self.compact_factor, self.min_lines = lines, compact_factor, min_lines
        self.q: "queue.Queue" = queue.Queue()
        self.compactions = 0
        self.thread = threading.Thread(target=self._run, name="training-table-journal", daemon=True)
        self.thread.start()

    def append(self, table_id: str, embedding, scores: Dict[int, float], retained: int, seq: int) -> None:
        self.q.put((table_id, embedding, scores, retained, seq))

    def flush(self) -> None:
        self.q.join()

    def _run(self) -> None:
        while True:
            item = self.q.get()
            try:
                if item is None:
                    return
                table_id, emb, scores, retained, seq = item
                line = json.dumps({"table": table_id, "embedding": [float(x) for x in emb],
                                   "scores": {str(k): v for k, v in scores.items()}})
                with open(self.path, "a", encoding="utf-8") as f:
                    f.write(line + "\n")
                self.lines += 1
                if self.lines > max(self.min_lines, self.compact_factor * retained):
                    self._compact(seq)
            except Exception:  # noqa: BLE001 - the journal never takes the server down
                import traceback

                traceback.print_exc()
            finally:
                self.q.task_done()

    def _compact(self, upto: int) -> None:
        # the rows recorded up to this line (the ones recorded since are still queued: appended after)
        rows = self.snapshot(upto)  # [(table id, embedding, {tt index: score})], each table oldest row first
        tmp = self.path + ".compact"
        with open(tmp, "w", encoding="utf-8") as f:
            for table_id, emb, scores in rows:
                f.write(json.dumps({"table": table_id, "embedding": emb,
                                    "scores": {str(k): v for k, v in scores.items()}}) + "\n")
        os.replace(tmp, self.path)
        self.lines = len(rows)
        self.compactions += 1

    def close(self) -> None:
        self.q.put(None)
        self.thread.join(timeout=30)


class TrainingTableWeights:
    def __init__(self, embedder=None, path: Optional[str] = None, device=None, max_rows: Optional[int] = None,
                 compact_min_lines: int = 4096):
        """`embedder(texts, max_tokens) -> (unit f32 [n, d], usage_tokens)`; None => 501 Not Implemented.
        ``path``: append-only JSONL of recorded rows, replayed on start (checkpoint / resume of what the
        tables have learned), appended by a background thread and compacted as it grows.  ``device``: where the
        tables live (default: the embedder's output device).  ``max_rows``: rows kept per table
        (``LWC_TRAINING_TABLE_MAX_ROWS``, default 1 M): beyond it the oldest row is dropped."""
        self.embedder = embedder
        self.tables: Dict[str, TrainingTable] = {}
        self.lock = threading.Lock()
        self.device = device
        self.path = path
        self.max_rows = int(max_rows or os.environ.get("LWC_TRAINING_TABLE_MAX_ROWS", 1 << 20))
        self._seq_no = 0
        lines = self._replay(path) if path and os.path.exists(path) else 0
        self.journal = _Journal(path, self._snapshot, lines, min_lines=compact_min_lines) if path else None

    def _replay(self, path: str) -> int:
        lines = 0
        with open(path, "r", encoding="utf-8") as f:
            for line in f:
                line = line.strip()
                if not line:
                    continue
                lines += 1
                try:
                    o = json.loads(line)
                    self._add(o["table"], torch.tensor(o["embedding"], dtype=torch.float32),
                              {int(k): float(v) for k, v in o["scores"].items()})
                except (ValueError, KeyError, TypeError):
                    continue  # a torn last line after a crash
        return lines

    def _snapshot(self, upto: Optional[int] = None):
        with self.lock:
            views = [(tid, t.rows_in_order(upto)) for tid, t in self.tables.items()]
        out = []
        for tid, (E, A) in views:
            for e, a in zip(E.tolist(), A.tolist()):
                out.append((tid, e, {j: v for j, v in enumerate(a) if v == v}))
        return out

    def retained(self) -> int:
        return sum(t.n for t in self.tables.values())

    def _add(self, table_id: str, e: torch.Tensor, by_tt: Dict[int, float]) -> int:
        t = self.tables.get(table_id)
        if t is None:
            t = TrainingTable(e.numel(), self.device or e.device, max_rows=self.max_rows)
            self.tables[table_id] = t
        self._seq_no += 1
        t.add(e, by_tt, self._seq_no)
        return self._seq_no

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
            seq = self._add(model.training_table_id, e, by_tt)
            retained = self.retained()
        if self.journal is not None:  # the row is resident now; its journal line is the journal thread's
            self.journal.append(model.training_table_id, embedding, by_tt, retained, seq)

    def flush(self) -> None:
        """Wait until every recorded row is in the journal file."""
        if self.journal is not None:
            self.journal.flush()


class WeightFetchers:
    """Dispatch on the model's weight type (reference weight.rs:40-64)."""

    def __init__(self, static=None, training_table=None):
        self.static = static or StaticWeights()
        self.training_table = training_table or TrainingTableWeights()

    async def fetch(self, ctx, request, model: Model):
        if model.weight_type == "static":
            return await self.static.fetch(ctx, request, model)
        return await self.training_table.fetch(ctx, request, model)
