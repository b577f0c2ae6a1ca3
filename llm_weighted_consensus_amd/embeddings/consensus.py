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
from typing import List, Optional, Sequence, Union

import torch

from .. import ops
from ..parallel import dist as pdist


@dataclass
class ConsensusResult:
    best: Union[List[int], torch.Tensor]  # per request: index of the consensus candidate (device tensor until
                                          # resolve() when the result was deferred)
    weights: torch.Tensor           # [R, N] softmax(centrality / tau)
    centrality: torch.Tensor        # [R, N]
    similarity: torch.Tensor        # [R, N, N]
    # True when a failed candidate all-gather left this rank with only its own shard: best / weights then
    # cover candidates [candidate_offset, candidate_offset + n_local) of each request; ``best`` is already
    # mapped to the request's global candidate numbering
    partial: bool = False
    candidate_offset: int = 0

    def resolve(self) -> "ConsensusResult":
        """A deferred result (``score(..., defer=True)``) holds ``best`` as a device tensor so the host can
        queue more work before waiting for the encoder; this reads it back (one sync) as a list."""
        if isinstance(self.best, torch.Tensor):
            off = self.candidate_offset if self.partial else 0
            self.best = [b + off for b in self.best.tolist()]
        return self


def consensus_reference(E: torch.Tensor, tau: float) -> ConsensusResult:
    """fp32 torch form of K10a (CPU plumbing path and the numerics oracle)."""
    Ef = E.float()
    S = Ef @ Ef.transpose(1, 2)
    n = E.shape[1]
    cen = (S.sum(-1) - S.diagonal(dim1=1, dim2=2)) / max(1, n - 1)
    w = torch.softmax(cen / tau, -1)
    return ConsensusResult(cen.argmax(-1).tolist(), w, cen, S)


def gather_candidates(E_local: torch.Tensor, group=None) -> torch.Tensor:
    """Candidate-parallel all-gather (C1): [R, n_local, d] per rank -> [R, cp*n_local, d] with group rank
    r's shard at candidates [r*n_local, (r+1)*n_local) (``group`` = the candidate-parallel ranks)."""
    if not pdist.info().enabled:
        return E_local
    R, n_local, d = E_local.shape
    G = pdist.all_gather(E_local, group)  # [cp, R, n_local, d]
    return G.permute(1, 0, 2, 3).reshape(R, -1, d).contiguous()


LAST_VERIFY: dict = {}  # this process's last verify_sharded numbers (the benches put them in their JSON)


def verify_sharded(scorer: "EmbeddingConsensus", local: Sequence[Sequence[int]], res: ConsensusResult,
                   group=None, request: int = 0, atol: float = 0.03) -> bool:
    """Self-check of a candidate-parallel consensus (a collective over every rank of the job).

    ``local`` = this rank's candidates (token ids) of request ``request`` of ``res``; the candidate group
    (``group``) exchanges them (an object all-gather over the host, independent of the C1 tensor all-gather
    under test), embeds all N on ONE device here and recomputes the consensus with the fp32 reference.  It
    must match what the sharded path produced: the similarity matrix within ``atol`` (a shard in the wrong
    place, a zeroed or stale shard moves whole rows by O(1)) and the same best candidate unless the top two
    centralities are within ``atol``.  Returns the verdict of the WHOLE job (a MIN over all ranks), so every
    rank can fail the run when one group mismatched."""
    import torch.distributed as tdist

    on = pdist.info().enabled
    if on and group is not None:
        parts: List = [None] * tdist.get_world_size(group)
        tdist.all_gather_object(parts, [list(c) for c in local], group=group)
        full = [c for p in parts for c in p]
    else:
        full = [list(c) for c in local]
    _, eb = scorer.embed(full)
    ref = consensus_reference(eb.float().cpu().view(1, len(full), -1), scorer.tau)  # fp32 on the host
    S = res.similarity[request].float().cpu()
    cen = res.centrality[request].float().cpu()
    best = res.best[request] if not isinstance(res.best, torch.Tensor) else int(res.best[request])
    ok = not res.partial and S.shape == ref.similarity[0].shape
    LAST_VERIFY.clear()
    if ok:
        d_s = float((S - ref.similarity[0]).abs().max())
        top = torch.topk(ref.centrality[0], min(2, len(full))).values
        d_c = float((cen - ref.centrality[0]).abs().max())
        same_best = best == int(ref.best[0])
        LAST_VERIFY.update(similarity_max_abs=round(d_s, 5), centrality_max_abs=round(d_c, 5), same_best=same_best,
                           top2_gap=round(float(top[0] - top[-1]), 5), atol=atol)
        ok = d_s <= atol and (same_best or bool(top[0] - top[-1] <= atol)) and d_c <= atol
    if not on:
        return ok
    flag = torch.tensor([1.0 if ok else 0.0], device=eb.device if eb.is_cuda else "cpu")
    pdist.all_reduce_(flag, op="min")
    return bool(flag.item() == 1.0)


class EmbeddingConsensus:
    def __init__(self, encoder, tau: float = 0.05, max_tokens: Optional[int] = None):
        self.encoder = encoder
        self.tau = tau
        self.max_tokens = max_tokens

    def embed(self, candidates: Sequence[Sequence[int]]):
        return self.encoder.embed(candidates, self.max_tokens)

    def score_local(self, E: torch.Tensor, defer: bool = False) -> ConsensusResult:
        """E: [R, N, d] unit rows (bf16 on the GPU: the MFMA kernel; any dtype on CPU: torch math).
        ``defer``: leave ``best`` on the device (no host sync; call ``resolve()`` later)."""
        if E.is_cuda:
            S, cen, w, best = ops.cosine_consensus(E, self.tau)
            return ConsensusResult(best if defer else best.tolist(), w, cen, S)
        return consensus_reference(E, self.tau)

    def score(self, requests: Sequence[Sequence[Sequence[int]]], gather: bool = False,
              group=None, defer: bool = False) -> ConsensusResult:
        """requests[r][i] = token ids of candidate i of request r (this rank's shard when gather=True;
        every rank must hold the same R and the same shard size).  ``defer``: see :meth:`score_local`."""
        R = len(requests)
        n_local = len(requests[0])
        flat = [c for req in requests for c in req]
        _, eb = self.embed(flat)
        E = eb.view(R, n_local, -1)
        partial = False
        offset = 0
        if gather and pdist.info().enabled:
            # a dead / hung peer must not take this rank's answers down: on a failed all-gather the group
            # is aborted and the consensus runs over the local shard of candidates (flagged as partial)
            crank = pdist.dist.get_rank(group) if group is not None else pdist.info().rank
            lost = []
            E = pdist.guarded(gather_candidates, E, group, fallback=lambda: lost.append(1) or E)
            if lost:
                partial, offset = True, crank * n_local
        res = self.score_local(E.contiguous(), defer=defer)
        if partial:
            res.partial, res.candidate_offset = True, offset
            if not isinstance(res.best, torch.Tensor):
                res.best = [b + offset for b in res.best]
        return res
