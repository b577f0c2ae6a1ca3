"""Encoder varlen packing (models/bert.py BertEncoder.pack): the flat-iterator fast path for equal-length
candidates, truncation at max_tokens, empty candidates and vocab folding, against a plain per-token loop."""
from types import SimpleNamespace

import numpy as np
import torch

from llm_weighted_consensus_amd.models.bert import BertEncoder


def _fake(vocab=100, max_position=16):
    return SimpleNamespace(cfg=SimpleNamespace(vocab_size=vocab, max_position=max_position), device=torch.device("cpu"))


def _loop_pack(token_lists, cap, V):
    ids, pos, cu = [], [], [0]
    for tl in token_lists:
        t = list(tl)[:cap] or [0]
        ids += [x % V for x in t]
        pos += list(range(len(t)))
        cu.append(cu[-1] + len(t))
    return ids, pos, cu


def test_pack_matches_per_token_loop():
    rng = np.random.default_rng(0)
    cases = [
        [list(rng.integers(0, 1000, 8)) for _ in range(5)],             # equal lengths (fast path, no slicing)
        [list(rng.integers(0, 1000, 20)) for _ in range(4)],            # equal after truncation at 12
        [list(rng.integers(0, 1000, n)) for n in (3, 0, 12, 7)],        # ragged, one empty
        [list(rng.integers(0, 1000, n)) for n in (12, 12, 30)],         # equal capped lengths, one longer
    ]
    for tls in cases:
        ids, pos, cu, mx = BertEncoder.pack(_fake(), tls, max_tokens=12)
        rid, rpos, rcu = _loop_pack(tls, 12, 100)
        assert ids.tolist() == rid and pos.tolist() == rpos and cu.tolist() == rcu
        assert mx == max(b - a for a, b in zip(rcu, rcu[1:]))


def test_deferred_consensus_result_resolves_with_the_shard_offset():
    from llm_weighted_consensus_amd.embeddings.consensus import ConsensusResult
    z = torch.zeros(2, 4)
    r = ConsensusResult(torch.tensor([1, 3]), z, z, z)
    assert r.resolve().best == [1, 3] and r.resolve().best == [1, 3]  # idempotent
    p = ConsensusResult(torch.tensor([1, 3]), z, z, z, partial=True, candidate_offset=4)
    assert p.resolve().best == [5, 7]
