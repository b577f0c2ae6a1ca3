"""Training-table voter weights that LEARN (reference types src/score/model/mod.rs:278-306,
stub src/score/completions/weight.rs:99-117): every scored request of a training-table model records
the transcript embedding and each voter's agreement with the consensus; later requests with similar
transcripts weight voters by that history; the table persists as JSONL and is replayed on start."""
import asyncio

import pytest
import torch

from llm_weighted_consensus_amd.chat.fake import FakeChatClient, Scripted, select_keys
from llm_weighted_consensus_amd.schema import score as S
from llm_weighted_consensus_amd.score.orchestrator import ScoreClient
from llm_weighted_consensus_amd.score.weights import TrainingTable, TrainingTableWeights, WeightFetchers

W = {"type": "training_table", "base_weight": 1.0, "min_weight": 0.25, "max_weight": 4.0}
MODEL = {"llms": [{"model": "good-1", "weight": W}, {"model": "good-2", "weight": W}, {"model": "contrarian", "weight": W}],
         "weight": {"type": "training_table", "top": 4, "embeddings": {"model": "bge", "max_tokens": 512}}}


def _embedder(texts, max_tokens):
    """Deterministic unit embeddings: transcripts about France are close to each other, others far."""
    rows = []
    for t in texts:
        v = torch.zeros(8)
        v[0 if "France" in t else 1] = 1.0
        v[2 + len(t) % 5] = 0.2
        rows.append(v / v.norm())
    return torch.stack(rows), 7


def _policy(req):
    keys = select_keys(req)
    want = "Madrid" if req.model == "contrarian" else "Paris"
    return [Scripted(next(k for k, v in keys if want in v))]


def _request(q="Capital of France?"):
    return S.ScoreCompletionCreateParams.model_validate(
        {"messages": [{"role": "user", "content": q}], "model": MODEL, "choices": ["Paris", "Madrid"]})


def _voter_weights(resp):
    """{"good-1"/"good-2": weight, "contrarian": weight} — voters told apart by what they voted for."""
    out, good = {}, 0
    for c in sorted((c for c in resp.choices if c.index >= 2), key=lambda c: c.model_index):
        if c.message.vote[1] > 0.5:
            out["contrarian"] = c.weight
        else:
            good += 1
            out[f"good-{good}"] = c.weight
    return out


def test_table_growth_and_vectorised_agreement():
    t = TrainingTable(4, "cpu", capacity=2)
    g = torch.Generator().manual_seed(0)
    rows = [torch.nn.functional.normalize(torch.randn(4, generator=g), dim=0) for _ in range(9)]
    scores = [{0: 0.9, 2: 0.1} if i % 2 else {1: 0.5} for i in range(9)]
    for e, s in zip(rows, scores):
        t.add(e, s)
    assert t.n == 9 and t.E.shape == (9, 4) and t.A.shape[1] == 3
    q = rows[3]
    got = t.agreement(q, 5, [0, 1, 2, 7])
    sims = torch.stack(rows) @ q
    vals, idx = sims.topk(5)
    for j, col in enumerate([0, 1, 2]):
        num = den = 0.0
        for s, i in zip(vals.clamp_min(0).tolist(), idx.tolist()):
            a = scores[i].get(col)
            if a is not None:
                num, den = num + s * a, den + s
        assert (got[j] is None) == (den == 0) and (den == 0 or got[j] == pytest.approx(num / den, rel=1e-5))
    assert got[3] is None  # a voter index the table has never seen


def test_weights_learn_from_scored_requests_and_replay(tmp_path):
    path = str(tmp_path / "tt.jsonl")
    tt = TrainingTableWeights(_embedder, path=path)
    client = ScoreClient(FakeChatClient(_policy), weight_fetchers=WeightFetchers(training_table=tt))

    async def go(q):
        return await client.create_unary(None, _request(q))

    first = asyncio.run(go("Capital of France?"))
    assert set(_voter_weights(first).values()) == {1.0}  # empty table: base weight for everyone
    assert isinstance(first.weight_data, S.WeightDataTrainingTable)
    for _ in range(3):
        asyncio.run(go("Capital of France?"))
    later = _voter_weights(asyncio.run(go("What is the capital of France?")))
    # voters that agreed with the consensus gain weight, the contrarian loses it
    assert later["good-1"] > 1.0 and later["good-2"] > 1.0 and later["contrarian"] < 1.0, later
    table = next(iter(tt.tables.values()))
    assert table.n == 5
    # an unrelated transcript has no similar neighbours (cosine <= 0 weighs nothing): base weights
    other = _voter_weights(asyncio.run(go("Tell me a joke")))
    assert other == {"good-1": 1.0, "good-2": 1.0, "contrarian": 1.0}
    # resume: a fresh fetcher replays the JSONL and weights the next request identically
    tt.flush()  # the journal thread has written every recorded row
    tt2 = TrainingTableWeights(_embedder, path=path)
    c2 = ScoreClient(FakeChatClient(_policy), weight_fetchers=WeightFetchers(training_table=tt2))
    again = _voter_weights(asyncio.run(c2.create_unary(None, _request("What is the capital of France?"))))
    assert next(iter(tt2.tables.values())).n >= 6
    assert again["good-1"] == pytest.approx(later["good-1"], rel=0.2) and again["contrarian"] < 1.0


def test_table_is_a_bounded_ring_and_the_journal_compacts(tmp_path):
    """max_rows bounds a table (the oldest rows are overwritten); the journal is rewritten from the
    resident rows once it holds twice as many lines, and replaying it gives the same table."""
    from llm_weighted_consensus_amd.score.weights import TrainingTable

    t = TrainingTable(4, "cpu", capacity=2, max_rows=5)
    for i in range(12):
        t.add(torch.full((4,), float(i)), {0: i / 12})
    assert t.n == 5 and sorted(t.E[:, 0].tolist()) == [7.0, 8.0, 9.0, 10.0, 11.0]
    E, A = t.rows_in_order()
    assert E[:, 0].tolist() == [7.0, 8.0, 9.0, 10.0, 11.0] and A[:, 0].tolist() == pytest.approx([i / 12 for i in range(7, 12)])

    path = str(tmp_path / "tt.jsonl")
    tt = TrainingTableWeights(_embedder, path=path, max_rows=8, compact_min_lines=10)

    class M:  # the two fields record() reads
        training_table_id = "tbl"
        llms = [type("L", (), {"training_table_index": 0})(), type("L", (), {"training_table_index": 1})()]

    g = torch.Generator().manual_seed(0)
    embs = [torch.nn.functional.normalize(torch.randn(8, generator=g), dim=0).tolist() for _ in range(40)]
    for i, e in enumerate(embs):
        tt.record(M, e, {0: 0.25, 1: i / 40})
    tt.flush()
    assert tt.journal.compactions >= 1
    with open(path) as f:
        lines = [l for l in f if l.strip()]
    assert len(lines) <= max(10, 2 * 8)
    tt2 = TrainingTableWeights(_embedder, path=path, max_rows=8)
    a, b = tt.tables["tbl"], tt2.tables["tbl"]
    assert a.n == b.n == 8
    Ea, Aa = a.rows_in_order()
    Eb, Ab = b.rows_in_order()
    assert torch.allclose(Ea, Eb) and torch.allclose(Aa, Ab, equal_nan=True)
    assert torch.allclose(Ea, torch.tensor(embs[-8:]))  # the newest 8 survive, oldest first
