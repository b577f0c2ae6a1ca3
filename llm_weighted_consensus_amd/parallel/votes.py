"""C2 helpers: the object collectives of voter-sharded scoring (score/sharded.py).

A score request's voters (reference src/score/completions/client.rs:343-356 fans them out; the tally is
client.rs:384-455) can be spread over the ranks of a process group.  Each request needs ONE exchange: an
all-gather of every rank's finished voter choices (votes, weights, errors, content) and voter usage,
after which every rank runs the native tally over all voters.  The payloads are small Python objects
(a few KiB per voter), so the groups used for them are gloo groups; the control traffic (the leader
broadcasting each request to the followers) uses :func:`broadcast_object` on a group of its own.
"""
from __future__ import annotations

from typing import Any, List, Optional

import torch.distributed as dist


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
