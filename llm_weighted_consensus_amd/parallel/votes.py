"""C2: combine the votes of voters that ran on different ranks.

A score request's voters (reference src/score/completions/client.rs:343-356 fans them out; the tally is
client.rs:384-455) can be spread over the ranks of a process group, each rank running the voters it
owns.  The tally only needs one number per choice from every rank — the sum over its voters of
vote[i] * weight — so the combine is ONE all-reduce of a [C + 1] fp64 vector (the extra slot counts
the ranks that had a successful vote, so "every vote failed" is a global decision).  Confidences and
each local voter's confidence (sum_i confidence[i] * vote[i]) then follow on every rank with no further
traffic.  The per-voter detail for the response (votes, errors, usage) is gathered once, as objects,
at the end of the request.

fp64 on the wire: the reduced sums equal the single-process tally up to summation order (1e-16
relative), and every rank holds the bitwise-same reduced vector.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Any, List, Optional, Sequence, Tuple

import torch
import torch.distributed as dist


@dataclass
class Tally:
    """Same fields as the native tally (csrc/runtime/consensus_core.h TallyResult)."""
    choice_weight: List[float]
    confidence: List[float]
    voter_confidence: List[float]


def _device(group) -> torch.device:
    if dist.get_backend(group) == "nccl":
        return torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def partial_weights(votes: Sequence[Sequence[float]], weights: Sequence[float], C: int) -> List[float]:
    """sum over this rank's voters of vote[i] * weight (voters without a vote contribute nothing)."""
    acc = [0.0] * C
    for v, w in zip(votes, weights):
        if not v:
            continue
        if len(v) != C:
            raise ValueError("tally: vote length != choices")
        for i in range(C):
            acc[i] += v[i] * w
    return acc


def tally_across(votes: Sequence[Sequence[float]], weights: Sequence[float], C: int, any_ok: bool,
                 group=None) -> Tuple[Tally, bool]:
    """Collective over ``group``: returns (tally with THIS rank's voters' confidences, every vote failed
    on every rank)."""
    part = partial_weights(votes, weights, C) + [1.0 if any_ok else 0.0]
    t = torch.tensor(part, dtype=torch.float64, device=_device(group))
    dist.all_reduce(t, group=group)
    red = t.cpu().tolist()
    cw, n_ok = red[:C], red[C]
    total = sum(cw)
    conf = [w / total if total > 0.0 else 0.0 for w in cw]
    vc = [sum(c * x for c, x in zip(conf, v)) if v else math.nan for v in votes]
    return Tally(cw, conf, vc), n_ok == 0.0


def gather_objects(obj: Any, group=None) -> List[Any]:
    """All-gather one picklable object per rank (group rank order)."""
    out: List[Optional[Any]] = [None] * dist.get_world_size(group)
    dist.all_gather_object(out, obj, group=group)
    return out


def broadcast_object(obj: Any, src_group_rank: int = 0, group=None) -> Any:
    box = [obj]
    src = dist.get_global_rank(group, src_group_rank) if group is not None else src_group_rank
    dist.broadcast_object_list(box, src=src, group=group)
    return box[0]
