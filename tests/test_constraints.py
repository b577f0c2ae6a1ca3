"""Token-level constrained decoding (K8d host side) over REAL tokenizers: byte-level BPE (Llama-3 family)
and SentencePiece with byte fallback (Llama-2 / Mistral family), both built offline by `tokenizers`, plus
the byte tokenizer.  The score voters' json_schema / tool_call schemas (reference
src/score/completions/client.rs:1299-1339) must only ever produce parseable JSON with a valid
response key, whatever the tokenizer's id layout is.

Soundness and completeness are checked by brute force against the byte FSM: a token is allowed in a
state iff the FSM accepts all its bytes from that state."""
import json
import random

import numpy as np
import pytest

from llm_weighted_consensus_amd.engine.constraints import TokenVocab, compile_json_schema, constraint_for_schema
from llm_weighted_consensus_amd.engine.tokenizer import ByteTokenizer, HFTokenizer
from llm_weighted_consensus_amd.score.orchestrator import response_key_format

pytest.importorskip("tokenizers")
from tests.test_tokenizers import _bytelevel, _sentencepiece  # noqa: E402

KEYS = ["`A`", "`B`", "`C`", "`T`"]


def _schema(think: bool, max_len=None):
    s = response_key_format(KEYS, think).json_schema.schema_
    if think and max_len:
        s = json.loads(json.dumps(s))
        s["properties"]["_think"]["maxLength"] = max_len
    return s


def _tokenizers(tmp_path):
    bl = HFTokenizer(_bytelevel(tmp_path), bos_token_id=0, eos_token_id=1)
    sp = HFTokenizer(_sentencepiece(tmp_path), bos_token_id=1, eos_token_id=2)
    return {"bytelevel": (bl, 416), "sentencepiece": (sp, 608), "byte": (ByteTokenizer(512), 512)}


def _walk(c, rng, max_steps=400, close_bias=0.25):
    """Random walk over the allowed tokens; returns the emitted token ids (EOS excluded)."""
    st = c.start()
    out = []
    for _ in range(max_steps):
        ok, eos = c.allowed_tokens(st)
        if c.is_done(st):
            assert eos
            return out
        ids = np.nonzero(ok)[0].tolist()
        assert ids, "dead end before the schema completed"
        closing = [t for t in ids if b'"' in c.vocab.tb[t]]
        t = rng.choice(closing if closing and rng.random() < close_bias else ids)
        st = c.advance(st, t)
        out.append(t)
    raise AssertionError("schema did not complete")


@pytest.mark.parametrize("kind", ["bytelevel", "sentencepiece", "byte"])
@pytest.mark.parametrize("think", [False, True])
def test_constrained_walk_is_valid_json(tmp_path, kind, think):
    tok, V = _tokenizers(tmp_path)[kind]
    c = constraint_for_schema(_schema(think, max_len=24), tok, V)
    rng = random.Random(1)
    for _ in range(30):
        ids = _walk(c, rng)
        text = b"".join(c.vocab.tb[t] for t in ids).decode("utf-8")
        obj = json.loads(text)
        assert obj["response_key"] in KEYS
        assert list(obj) == (["_think", "response_key"] if think else ["response_key"])
        # the tokenizer's own detokenisation agrees (ids are real ids of this vocabulary)
        if kind != "byte":
            assert tok.decode(ids) == text


@pytest.mark.parametrize("kind", ["bytelevel", "sentencepiece"])
def test_token_masks_sound_and_complete(tmp_path, kind):
    """Every state reached on a walk: allowed == {t : FSM accepts bytes(t)} by brute force."""
    tok, V = _tokenizers(tmp_path)[kind]
    c = constraint_for_schema(_schema(True, max_len=12), tok, V)
    rng = random.Random(3)
    st = c.start()
    seen = 0
    while not c.is_done(st):
        ok, _ = c.allowed_tokens(st)
        brute = np.array([bool(c.vocab.tb[t]) and c.advance_bytes(st, c.vocab.tb[t]) is not None
                          for t in range(V)])
        assert np.array_equal(ok, brute), np.nonzero(ok != brute)[0][:10]
        ids = np.nonzero(ok)[0].tolist()
        st = c.advance(st, rng.choice(ids))
        seen += 1
    assert seen > 3


def test_ids_0_255_are_not_bytes_for_real_tokenizers(tmp_path):
    """The round-1 bug: masks over ids 0..255 as raw bytes.  With byte-level BPE, id 123 is not '{'."""
    tok, V = _tokenizers(tmp_path)["bytelevel"]
    c = constraint_for_schema(_schema(False), tok, V)
    ok, _ = c.allowed_tokens(c.start())
    allowed = [c.vocab.tb[t] for t in np.nonzero(ok)[0]]
    assert allowed and all(b.startswith(b"{") for b in allowed)
    brace_ids = tok.ids_for_text("{")
    assert ok[brace_ids[0]] and brace_ids[0] != ord("{") or ok[ord("{")]
    # the mask entry packs the same set, plus nothing else
    words = c.mask_entry(c.start()).words()
    bits = np.unpackbits(words.view(np.uint8), bitorder="little").astype(bool)
    assert np.array_equal(bits[:V], ok)


def test_multi_segment_tokens_allowed(tmp_path):
    """Merged tokens that span segment boundaries (e.g. '{"' or '"response_key') are allowed, not just single bytes."""
    tok, V = _tokenizers(tmp_path)["bytelevel"]
    c = constraint_for_schema(_schema(False), tok, V)
    ok, _ = c.allowed_tokens(c.start())
    lens = [len(c.vocab.tb[t]) for t in np.nonzero(ok)[0]]
    assert max(lens) > 1, [c.vocab.tb[t] for t in np.nonzero(ok)[0]]


def test_string_room_and_mask_cache(tmp_path):
    tok, V = _tokenizers(tmp_path)["byte"]
    c = constraint_for_schema(_schema(True, max_len=6), tok, V)
    st = c.advance_bytes(c.start(), b'{"_think":"abcdef')
    ok, _ = c.allowed_tokens(st)
    assert {c.vocab.tb[t] for t in np.nonzero(ok)[0]} == {b'"'}  # no room left: only the closing quote
    st2 = c.advance_bytes(c.start(), b'{"_think":"a')
    st3 = c.advance_bytes(c.start(), b'{"_think":"b')
    assert c.mask_entry(st2).key == c.mask_entry(st3).key
    assert c._key(st2) == c._key(st3)
    assert c.advance(st, tok.eos_token_id)[0] == len(c.fsm.segments)


def test_token_vocab_cached_per_tokenizer(tmp_path):
    tok, V = _tokenizers(tmp_path)["sentencepiece"]
    assert TokenVocab.of(tok, V) is TokenVocab.of(tok, V)
    assert compile_json_schema({"type": "array"}) is None
    with pytest.raises(ValueError):
        constraint_for_schema(_schema(False), tok, 607)


def test_masks_shared_across_voters_with_equal_remaining_grammar(tmp_path):
    """Voters of different requests (different key orders / sets) reuse each other's masks wherever their
    REMAINING grammar is equal: the cache key is content, not the constraint instance."""
    tok, V = _tokenizers(tmp_path)["bytelevel"]
    a = constraint_for_schema(response_key_format(["`A`", "`B`"], False).json_schema.schema_, tok, V)
    b = constraint_for_schema(response_key_format(["`B`", "`A`"], False).json_schema.schema_, tok, V)
    c = constraint_for_schema(response_key_format(["`C`", "`D`"], False).json_schema.schema_, tok, V)
    sa, sb, sc = a.start(), b.start(), c.start()
    assert a._key(sa) == b._key(sb)            # same enum SET: the same grammar from the start
    assert a._key(sa) != c._key(sc)            # a different enum: a different suffix
    ea = a.mask_entry(sa)
    assert b.mask_entry(sb) is ea              # served from the vocab-level cache
    # after the key, every voter is in the same closing literal
    ta = a.advance_bytes(sa, b'{"response_key":"`A`"')
    tc = c.advance_bytes(sc, b'{"response_key":"`C`"')
    assert a._key(ta) == c._key(tc) and np.array_equal(a.allowed_tokens(ta)[0], c.allowed_tokens(tc)[0])


def test_constraint_pickles_without_the_vocabulary(tmp_path):
    """EngineGroup ships SamplingParams to worker processes: the constraint travels as its grammar only
    and re-binds the worker's vocabulary index (and its warm mask cache)."""
    import pickle

    tok, V = _tokenizers(tmp_path)["bytelevel"]
    c = constraint_for_schema(_schema(False), tok, V)
    blob = pickle.dumps(c)
    assert len(blob) < 4096
    c2 = pickle.loads(blob)
    assert c2.vocab is None
    c2.bind(tok, V)
    assert c2.vocab is TokenVocab.of(tok, V)
    st = c.start()
    assert c2.mask_entry(st) is c.mask_entry(st)


def test_suffix_ids_never_reused_after_table_clear(tmp_path, monkeypatch):
    """bounding the suffix-id table must not hand an old id to a new grammar, or the
    vocab-level mask cache serves the old grammar's mask to it."""
    from llm_weighted_consensus_amd.engine import constraints as C

    tok, V = _tokenizers(tmp_path)["bytelevel"]
    a = constraint_for_schema(response_key_format(["`A`", "`B`"], False).json_schema.schema_, tok, V)
    a_ids = set(a.fsm.suffix_ids) - {0}
    ea = a.mask_entry(a.start())  # cached under a's start key
    monkeypatch.setattr(C, "_SUFFIX_LIMIT", 1)  # every new suffix now clears the table first
    c = constraint_for_schema(response_key_format(["`C`", "`D`"], False).json_schema.schema_, tok, V)
    # ids shared with `a` are equal grammar content (the closing literal); the new suffixes get fresh ids
    assert c.fsm.suffix_ids[0] > max(a_ids)
    assert c._key(c.start()) != a._key(a.start())
    ec = c.mask_entry(c.start())
    assert ec is not ea
    ok, _ = c.allowed_tokens(c.start())
    assert np.array_equal(ec.words(), c.mask_entry(c.start()).words())
    # a pickled copy re-derives its ids in the receiving process instead of carrying foreign ones
    import pickle

    c2 = pickle.loads(pickle.dumps(c))
    c2.bind(tok, V)
    assert np.array_equal(c2.allowed_tokens(c2.start())[0], ok)
