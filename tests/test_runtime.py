"""Host C++ runtime (CPU): paged-KV block manager and the consensus core key tree / votes / tally."""
import math
import random
import re

import pytest

from llm_weighted_consensus_amd import _runtime as R


def test_block_manager_fork_cow_and_free():
    bm = R.BlockManager(8, 4)
    bm.add_sequence(1, 6)  # 2 blocks, last partial
    assert bm.num_free == 6 and bm.length(1) == 6
    bm.fork(1, 2)
    bm.fork(1, 3)
    t1 = bm.block_table(1)
    assert bm.block_table(2) == t1 and bm.refcount(t1[1]) == 3
    s = bm.append_token(2)  # shared partial block -> copy-on-write
    copies = bm.take_copies()
    assert len(copies) == 1 and copies[0][0] == t1[1]
    assert bm.block_table(2)[0] == t1[0] and bm.block_table(2)[1] == copies[0][1]
    assert s == copies[0][1] * 4 + 2
    assert bm.take_copies() == []
    bm.append_token(2)
    assert bm.append_cost(2) == 1  # block full -> needs a new block
    bm.append_token(2)
    assert len(bm.block_table(2)) == 3
    for q in (1, 2, 3):
        bm.free_sequence(q)
    assert bm.num_free == 8


def test_block_manager_exhaustion():
    bm = R.BlockManager(2, 4)
    bm.add_sequence(1, 8)
    with pytest.raises(RuntimeError):
        bm.add_sequence(2, 1)
    with pytest.raises(RuntimeError):
        bm.append_token(1)


def test_prepare_decode_padding():
    bm = R.BlockManager(16, 4)
    bm.add_sequence(5, 3)
    bt, ctx, slots, pos = R.prepare_decode(bm, [5], 4, 2)
    assert bt.shape == (2, 4) and list(ctx) == [4, 1] and list(pos) == [3, 0] and slots[1] == -1
    assert slots[0] == bm.slot(5, 3)


def test_prepare_decode_into_matches_prepare_decode():
    """The staging-buffer variant writes the same tables as prepare_decode (used columns)."""
    import numpy as np

    a, b = R.BlockManager(64, 4), R.BlockManager(64, 4)
    for bm in (a, b):
        bm.add_sequence(1, 9)
        bm.add_sequence(2, 3)
        bm.fork(1, 3)
    bt, ctx, slots, pos = R.prepare_decode(a, [1, 3, 2], 6, 4)
    buf = np.full(4 * 6 + 12, 77, dtype=np.int32)
    bt2 = buf[:24].reshape(4, 6)
    R.prepare_decode_into(b, [1, 3, 2], 6, 4, bt2, buf[24:28], buf[28:32], buf[32:36])
    assert list(buf[24:28]) == list(ctx) and list(buf[28:32]) == list(slots) and list(buf[32:36]) == list(pos)
    for i in range(3):
        n = len(b.block_table([1, 3, 2][i]))
        assert list(bt2[i, :n]) == list(bt[i, :n])
    assert b.take_copies() == a.take_copies()
    with pytest.raises(RuntimeError):
        R.prepare_decode_into(b, [1], 6, 4, bt2, buf[24:28], buf[28:32], buf[32:36].astype(np.int64))


def _ref_tree_keys(n, m):
    """Python oracle of the reference SelectPfxTree shape (client.rs:1469-1517): multiset of key depths."""
    def rec(length, force):
        if not force and length <= m:
            return [1] * length
        k = (length + m - 1) // m
        k = min(k, m)
        base, extra = divmod(length, k)
        fs = base + (1 if extra else 0) > m
        out = []
        for i in range(k):
            out += [d + 1 for d in rec(base + (1 if i < extra else 0), fs)]
        return out
    return sorted(rec(n, False))


@pytest.mark.parametrize("n,m", [(2, 20), (5, 20), (20, 20), (21, 20), (45, 5), (400, 20), (9, 2), (130, 3)])
def test_key_tree_shape_matches_reference(n, m):
    t = R.KeyTree(n, m, 7)
    keys = t.keys
    assert sorted(i for _, i in keys) == list(range(n))
    assert len({k for k, _ in keys}) == n
    for k, _ in keys:
        assert re.fullmatch(r"(`[A-T]`)+", k)
    assert sorted(k.count("`") // 2 for k, _ in keys) == _ref_tree_keys(n, m)


def test_key_tree_vote_one_hot_and_last_match():
    t = R.KeyTree(4, 20, 3)
    (k0, i0), (k1, i1) = t.keys[0], t.keys[1]
    v = t.vote(f"first {k0} then finally {k1}")
    assert v[i1] == 1.0 and sum(v) == 1.0
    bare = k0.strip("`")
    v2 = t.vote(f"I choose {bare}.")
    assert v2[i0] == 1.0
    assert t.vote("no key here at all 123") is None


def test_key_tree_vote_logprobs():
    t = R.KeyTree(3, 3, 11)
    (k0, i0), (k1, i1), (k2, i2) = t.keys
    l0, l1, l2 = k0[1], k1[1], k2[1]
    content = f"{k0}"
    # tokens: "`", letter, "`" with top alternatives at the letter position
    lp = [("`", [("`", 0.0)]),
          (l0, [(l0, math.log(0.6)), (l1, math.log(0.3)), ("x", math.log(0.05)), (l2, float("nan"))]),
          ("`", [("`", 0.0)])]
    v = t.vote(content, lp)
    assert abs(v[i0] - 0.6 / 0.9) < 1e-12 and abs(v[i1] - 0.3 / 0.9) < 1e-12 and v[i2] == 0.0
    # multi-char token carrying the letter at byte offset 1
    lp2 = [(f"`{l0}", [(f"`{l0}", math.log(0.5)), (f"`{l2}", math.log(0.5))]), ("`", [("`", 0.0)])]
    v2 = t.vote(content, lp2)
    assert abs(v2[i0] - 0.5) < 1e-12 and abs(v2[i2] - 0.5) < 1e-12
    # no sibling letter among the alternatives -> one-hot fallback (reference: unreachable!())
    lp3 = [("`", []), (l0, [("zz", 0.0)]), ("`", [])]
    v3 = t.vote(content, lp3)
    assert v3[i0] == 1.0


def test_tally_and_error_codes():
    r = R.tally([[0.5, 0.5, 0.0], [], [0.0, 1.0, 0.0]], [2.0, 5.0, 1.0], 3)
    assert r.choice_weight == [1.0, 2.0, 0.0]
    assert r.confidence == pytest.approx([1 / 3, 2 / 3, 0.0])
    assert math.isnan(r.voter_confidence[1])
    assert r.voter_confidence[2] == pytest.approx(2 / 3)
    z = R.tally([[], []], [1.0, 1.0], 2)
    assert z.confidence == [0.0, 0.0]
    assert R.unify_error_codes([]) is None
    assert R.unify_error_codes([429, 429]) == 429
    assert R.unify_error_codes([429, 404]) == 400
    assert R.unify_error_codes([404, 500]) == 500


def test_prefix_cache_reuse_and_cap():
    bm = R.BlockManager(16, 4)
    bm.set_prefix_caching(True)
    p = list(range(100, 111))  # 11 tokens: 2 full blocks + a partial one
    assert bm.add_sequence_cached(1, p) == 0
    bm.cache_prefix(1, p)
    assert bm.num_cached_blocks == 2  # only blocks the prompt fills completely
    t1 = list(bm.block_table(1))
    # same prompt + a longer tail: the two full blocks are shared, the rest is fresh
    q = p[:8] + [7, 7, 7, 7, 7]
    assert bm.match_prefix(q) == 8
    assert bm.add_sequence_cached(2, q) == 8
    t2 = bm.block_table(2)
    assert t2[:2] == t1[:2] and t2[2] not in t1 and bm.refcount(t1[0]) == 2
    # a prompt that IS exactly the cached blocks still computes its last token: only 1 block reused
    assert bm.match_prefix(p[:8]) == 4
    # different first block -> nothing reused, even though the second block's tokens match
    assert bm.match_prefix([0, 0, 0, 0] + p[4:8] + [1]) == 0
    bm.set_prefix_caching(False)
    assert bm.match_prefix(q) == 0
    bm.set_prefix_caching(True)


def test_prefix_cache_lru_eviction_keeps_capacity():
    bm = R.BlockManager(6, 4)
    bm.set_prefix_caching(True)
    a = list(range(9))        # 2 full blocks + 1
    bm.add_sequence_cached(1, a)
    bm.cache_prefix(1, a)
    bm.free_sequence(1)
    # cached-but-unreferenced blocks still count as free capacity
    assert bm.num_free == 6 and bm.num_evictable == 2 and bm.num_cached_blocks == 2
    assert bm.add_sequence_cached(2, a) == 8 and bm.num_evictable == 0  # resurrected from the LRU
    bm.free_sequence(2)
    # a request that needs every block evicts the cached ones (oldest first) instead of failing
    bm.add_sequence(3, 24)
    assert bm.num_free == 0 and bm.num_cached_blocks == 0
    bm.free_sequence(3)
    assert bm.match_prefix(a) == 0 and bm.num_free == 6
    with pytest.raises(RuntimeError):
        bm.add_sequence_cached(4, list(range(30)))


def test_prefix_cache_chain_is_content_addressed():
    bm = R.BlockManager(32, 4)
    bm.set_prefix_caching(True)
    rng = random.Random(0)
    prompts = [[rng.randrange(50) for _ in range(rng.randrange(1, 30))] for _ in range(40)]
    prompts += [p[: len(p) // 2] + [1, 2, 3] for p in prompts[:10]]
    live = {}
    for i, p in enumerate(prompts):
        try:
            c = bm.add_sequence_cached(i, p)
        except RuntimeError:
            for j in list(live):
                bm.free_sequence(j)
            live.clear()
            c = bm.add_sequence_cached(i, p)
        # every reused block must have been registered for exactly these tokens: re-derive from the
        # prompts that registered them (content equality of the covered prefix)
        tab = bm.block_table(i)
        for b in range(c // 4):
            owners = [q for j, q in live.items() if j != i and b < len(bm.block_table(j))
                      and bm.block_table(j)[b] == tab[b]]
            for q in owners:
                assert q[: (b + 1) * 4] == p[: (b + 1) * 4]
        bm.cache_prefix(i, p)
        live[i] = p


def test_run_prefill_frees_parents_when_a_later_prompt_does_not_fit():
    """A wave whose later prompt runs out of KV blocks must release the transient parents (and the cached
    blocks they acquired) created before the failure (engine._run_prefill)."""
    import types

    from llm_weighted_consensus_amd import _runtime as R
    from llm_weighted_consensus_amd.engine.engine import LLMEngine

    for use_cache in (False, True):
        bm = R.BlockManager(6, 4)
        bm.set_prefix_caching(use_cache)
        fake = types.SimpleNamespace(bm=bm, device="cpu")
        fake._run_prefill_inner = lambda *a: LLMEngine._run_prefill_inner(fake, *a)
        prompts = [list(range(8)), list(range(100, 120))]  # 2 blocks, then 5 blocks: the second does not fit
        with pytest.raises(RuntimeError, match="out of KV blocks"):
            LLMEngine._run_prefill(fake, prompts, [-1, -2], use_cache=use_cache)
        assert bm.num_sequences == 0 and bm.num_free == 6 and not bm.has_sequence(-1)


def test_block_manager_swap_out_in_keeps_sharing():
    """Preemption by swapping: a forked group leaves as its distinct blocks + per-sequence index tables
    and comes back on fresh blocks with the same sharing (shared prompt blocks refcounted again)."""
    from llm_weighted_consensus_amd._runtime import BlockManager

    bm = BlockManager(64, 16)
    bm.add_sequence(1, 40)
    for c in (2, 3):
        bm.fork(1, c)
    bm.free_sequence(1)
    for c in (2, 3):
        for _ in range(30):
            bm.append_token(c)
    assert bm.append_cost_total([2, 3]) == 0
    before = {c: list(bm.block_table(c)) for c in (2, 3)}
    blocks, tables, lens = bm.swap_out([2, 3])
    assert bm.num_free == 64 and not bm.has_sequence(2)
    assert len(blocks) == len(set(blocks)) == len(set(before[2]) | set(before[3]))
    assert [[blocks[i] for i in t] for t in tables] == [before[2], before[3]]
    phys = bm.swap_in([5, 6], len(blocks), tables, lens)
    assert [bm.length(s) for s in (5, 6)] == lens == [70, 70]
    shared = [phys[i] for i in set(tables[0]) & set(tables[1])]
    assert shared and all(bm.refcount(b) == 2 for b in shared)
    for s in (5, 6):
        bm.free_sequence(s)
    assert bm.num_free == 64
