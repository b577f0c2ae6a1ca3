"""models/packing.py: the numpy varlen packer gives the same ids / positions / offsets as the straightforward
per-token Python packing, for int32 arrays (the engine's Sequence.tokens) and plain lists, head (BERT) and
tail (decoder embedder: the pooled last token) truncation, empty and ragged inputs."""
import random
from array import array

import numpy as np
import pytest

from llm_weighted_consensus_amd.models.packing import pack_ids


def _naive(token_lists, cap, V, tail):
    ids, pos, cu = [], [], [0]
    for tl in token_lists:
        tl = list(tl)
        tl = (tl[-cap:] if tail else tl[:cap]) or [0]
        tl = [t % V for t in tl]
        ids += tl
        pos += list(range(len(tl)))
        cu.append(cu[-1] + len(tl))
    return ids, pos, cu, max(cu[i + 1] - cu[i] for i in range(len(cu) - 1))


@pytest.mark.parametrize("kind", ["array", "list"])
@pytest.mark.parametrize("shape", ["equal", "ragged", "with_empty", "over_cap"])
@pytest.mark.parametrize("tail", [False, True])
def test_pack_matches_naive(kind, shape, tail):
    rng = random.Random(hash((kind, shape, tail)) & 0xffff)
    V, cap = 30522, 40
    if shape == "equal":
        lens = [25] * 17
    elif shape == "ragged":
        lens = [rng.randint(1, 39) for _ in range(17)]
    elif shape == "with_empty":
        lens = [0, 5, 0, 12]
    else:
        lens = [cap + 9] * 6 + [cap + 3]
    rows = [[rng.randrange(0, 128256) for _ in range(n)] for n in lens]
    token_lists = [array("i", r) for r in rows] if kind == "array" else rows
    ids, pos, cu, mx = pack_ids(token_lists, cap, V, tail=tail)
    n_ids, n_pos, n_cu, n_mx = _naive(rows, cap, V, tail)
    assert ids.dtype == np.int32 and pos.dtype == np.int32 and cu.dtype == np.int32
    assert ids.tolist() == n_ids and pos.tolist() == n_pos and cu.tolist() == n_cu and mx == n_mx


def test_pack_empty_batch():
    ids, pos, cu, mx = pack_ids([], 8, 100)
    assert len(ids) == 0 and cu.tolist() == [0] and mx == 0
