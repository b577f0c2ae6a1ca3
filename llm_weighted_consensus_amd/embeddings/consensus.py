"""Embedding-consensus scorer: N candidate answers -> encoder embeddings -> cosine consensus.

The MI355X form of "weighted consensus" over sampled candidates (self-consistency, BASELINE.json
configs 1-4): every candidate is embedded by the BGE encoder (K9*), the pairwise cosine matrix of
the unit embeddings is ONE MFMA GEMM (K10a) and a row-reduce gives each candidate's centrality
c_i = mean_{j != i} cos(e_i, e_j); confidence = softmax(c / tau).  The answer is argmax c.

Candidate-parallel across GPUs: each rank embeds its shard of every request's candidates and one
RCCL all-gather (C1) assembles [requests, N, d] on every rank before the (tiny) consensus kernel.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional, Sequence

import torch

from .. import ops
from ..parallel import dist as pdist


@dataclass
class ConsensusResult:
    best: List[int]                 # per request: index of the consensus candidate
    weights: torch.Tensor           # [R, N] softmax(centrality / tau)
    centrality: torch.Tensor        # [R, N]
    similarity: torch.Tensor        # [R, N, N]


class EmbeddingConsensus:
    def __init__(self, encoder, tau: float = 0.05, max_tokens: Optional[int] = None):
        self.encoder = encoder
        self.tau = tau
        self.max_tokens = max_tokens

    def embed(self, candidates: Sequence[Sequence[int]]):
        return self.encoder.embed(candidates, self.max_tokens)

    def score_local(self, E: torch.Tensor) -> ConsensusResult:
        """E: [R, N, d] bf16 unit rows."""
        S, cen, w, best = ops.cosine_consensus(E, self.tau)
        return ConsensusResult(best.tolist(), w, cen, S)

    def score(self, requests: Sequence[Sequence[Sequence[int]]], gather: bool = False) -> ConsensusResult:
        """requests[r][i] = token ids of candidate i of request r (this rank's shard when gather=True;
        every rank must hold the same R and the same shard size)."""
        R = len(requests)
        n_local = len(requests[0])
        flat = [c for req in requests for c in req]
        _, eb = self.embed(flat)
        E = eb.view(R, n_local, -1)
        if gather and pdist.info().enabled:
            G = pdist.all_gather(E)                         # [W, R, n_local, d]
            E = G.permute(1, 0, 2, 3).reshape(R, -1, E.shape[-1])
        return self.score_local(E.contiguous())
