"""Candidate-parallel prompt sharing (C4): every rank prefills only its own requests, then the prompt KV
blocks and last-token logits are all-gathered so every rank can sample its share of the candidates of
EVERY request without recomputing any prompt.

Why: in the candidate-parallel layout (BASELINE north star: candidates sharded across the GPUs, RCCL
all-gather of the results) each rank decodes N/W candidates of all G = R*W requests.  Replicating the
prefill would cost every rank (W-1)*R extra prompts per step — at W=8, R=16, 256-token prompts that is
~29k tokens of Llama-3-8B compute (~0.4 s) — whereas moving the finished KV costs
(W-1) * R * 33.5 MB over xGMI (~12 ms at RCCL all-gather rates).  One all-gather per tensor, on flat
padded buffers (xGMI is point-to-point: few large collectives beat many small ones).

The reference has no local inference; its closest analogue is the per-voter fan-out of one request
to many upstream chat completions (src/score/completions/client.rs:343-356).
"""
from __future__ import annotations

from typing import List, Tuple

import torch

from . import dist as pdist


def _gather_flat(t: torch.Tensor, world: int, group=None) -> torch.Tensor:
    return pdist.all_gather_flat(t, group)


def all_gather_prefills(kv: torch.Tensor, logits: torch.Tensor, nblocks: List[int],
                        group=None) -> List[Tuple[torch.Tensor, torch.Tensor]]:
    """kv [L, 2, sum(nblocks), E] + logits [n, V] of this rank's prompts -> per prompt of ALL ranks
    (rank-major order) a (kv [L, 2, nb, E] view, logits [V] view) pair.

    Ranks may hold different numbers of prompts and blocks: the per-rank counts travel first (one tiny
    all-gather), then the KV and logits are padded to the largest rank and gathered once each."""
    info = pdist.info()
    if not info.enabled or group is None and info.world == 1:
        out, off = [], 0
        for i, nb in enumerate(nblocks):
            out.append((kv[:, :, off:off + nb], logits[i]))
            off += nb
        return out
    W = pdist.group_size(group)
    dev = kv.device
    n = len(nblocks)
    counts = torch.tensor([n, int(sum(nblocks))], dtype=torch.int64, device=dev)
    counts = _gather_flat(counts, W, group).cpu().tolist()
    max_n = max(c[0] for c in counts)
    max_nb = max(c[1] for c in counts)
    nbl = torch.zeros(max(max_n, 1), dtype=torch.int64, device=dev)
    if n:
        nbl[:n] = torch.tensor(nblocks, dtype=torch.int64, device=dev)
    nbl_all = _gather_flat(nbl, W, group).cpu().tolist()
    L, two, nb_here, E = kv.shape
    kv_pad = kv
    if nb_here < max_nb:
        kv_pad = torch.zeros(L, two, max_nb, E, dtype=kv.dtype, device=dev)
        kv_pad[:, :, :nb_here] = kv
    V = logits.shape[-1]
    lg_pad = logits
    if n < max(max_n, 1):
        lg_pad = torch.zeros(max(max_n, 1), V, dtype=logits.dtype, device=dev)
        lg_pad[:n] = logits
    kv_all = _gather_flat(kv_pad, W, group)       # [W, L, 2, max_nb, E]
    lg_all = _gather_flat(lg_pad, W, group)       # [W, max_n, V]
    out = []
    for r in range(W):
        off = 0
        for i in range(counts[r][0]):
            nb = nbl_all[r][i]
            out.append((kv_all[r][:, :, off:off + nb], lg_all[r][i]))
            off += nb
    return out
