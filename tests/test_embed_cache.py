"""HBM-resident embedding archive (archive/hbm.py), exercised on CPU: LRU slab bookkeeping, content keys,
and the embedding service returning identical rows with and without the cache while encoding only the
texts it has not seen."""
import torch

from llm_weighted_consensus_amd.archive.hbm import ResidentEmbeddings, content_key


def test_content_key_truncation_and_identity():
    assert content_key([1, 2, 3], 512) == content_key([1, 2, 3], 512)
    assert content_key([1, 2, 3], 512) != content_key([1, 2, 4], 512)
    # the truncation length is part of the key, and only the kept prefix matters
    assert content_key([1, 2, 3], 2) == content_key([1, 2, 9], 2)
    assert content_key([1, 2, 3], 2) != content_key([1, 2, 3], 3)


def test_lru_eviction_and_refresh():
    c = ResidentEmbeddings(dim=4, device="cpu", budget_bytes=3 * 4 * 4)  # 3 fp32 rows
    assert c.capacity == 3
    rows = torch.arange(16, dtype=torch.float32).view(4, 4)
    c.put([b"a", b"b", b"c"], rows[:3])
    assert c.lookup([b"a"]) != [None]          # refresh a: b is now the oldest
    c.put([b"d"], rows[3:])
    assert c.lookup([b"b"]) == [None] and c.evictions == 1
    s = c.lookup([b"a", b"c", b"d"])
    assert torch.equal(c.gather(s), torch.stack([rows[0], rows[2], rows[3]]))
    assert len(c) == 3 and c.bytes_used == 48


def test_zero_budget_stores_nothing():
    c = ResidentEmbeddings(dim=8, device="cpu", budget_bytes=0)
    c.put([b"x"], torch.ones(1, 8))
    assert len(c) == 0 and c.lookup([b"x"]) == [None]


def test_embed_through_encodes_misses_once():
    c = ResidentEmbeddings(dim=3, device="cpu", budget_bytes=1 << 20)
    calls = []

    def enc(lists):
        calls.append([list(t) for t in lists])
        return torch.tensor([[float(sum(t)), float(len(t)), 1.0] for t in lists])

    a, b = [5, 6], [7]
    out, n = c.embed_through([a, b, a], 512, enc)
    assert n == 2 and calls == [[a, b]]        # the repeated text is encoded once
    assert torch.equal(out[0], out[2]) and out[1, 0] == 7
    out2, n2 = c.embed_through([b, [1, 1], a], 512, enc)
    assert n2 == 1 and calls[-1] == [[1, 1]]   # only the new text
    assert torch.equal(out2[0], out[1]) and torch.equal(out2[2], out[0])


def test_service_cache_matches_uncached_encoder():
    from llm_weighted_consensus_amd.embeddings.service import EmbeddingService
    from llm_weighted_consensus_amd.models.bert import BertEncoder
    from llm_weighted_consensus_amd.models.config import encoder_config

    enc = BertEncoder(encoder_config("bert-tiny"), device=torch.device("cpu"), seed=3)
    plain = EmbeddingService(enc, "tiny", cache_mb=0)
    cached = EmbeddingService(enc, "tiny", cache_mb=1)
    texts = ["alpha", "beta gamma", "alpha", "delta"]
    ref, ntok = plain.embed_texts(texts)
    got, ntok2 = cached.embed_texts(texts)
    assert ntok == ntok2  # usage still counts every input
    assert torch.allclose(got, ref, atol=1e-6)
    again, _ = cached.embed_texts(["delta", "alpha"])
    assert torch.allclose(again, ref[[3, 0]], atol=1e-6)
    st = cached.cache.stats()
    assert st["entries"] == 3 and st["hits"] == 2 and st["misses"] == 4  # an in-call repeat counts as a miss


def test_put_more_misses_than_capacity_keeps_rows_consistent():
    """More new keys in one put() than the slab holds: no slot is written twice, every stored key maps to
    its own row."""
    import torch

    from llm_weighted_consensus_amd.archive.hbm import ResidentEmbeddings

    r = ResidentEmbeddings(4, "cpu", budget_bytes=3 * 4 * 4)
    assert r.capacity == 3
    r.put([b"old"], torch.full((1, 4), -1.0))
    keys = [bytes([i]) * 16 for i in range(5)]
    emb = torch.arange(5, dtype=torch.float32)[:, None].repeat(1, 4)
    r.put(keys, emb)
    slots = r.lookup(keys)
    stored = [(i, s) for i, s in enumerate(slots) if s is not None]
    assert len(stored) == 3 and len({s for _, s in stored}) == 3
    for i, s in stored:
        assert torch.equal(r.gather([s])[0], emb[i])
