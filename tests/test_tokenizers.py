"""Real tokenizer.json support (HFTokenizer), exercised with tokenizers BUILT HERE by the `tokenizers`
library (no downloads): byte-level BPE (Llama-3 family), SentencePiece-style BPE with byte fallback
(Llama-2 / Mistral family) and WordPiece (BERT / BGE).  Per-token bytes must concatenate to exactly the
text — the property incremental detokenisation and vote-letter alignment rely on."""
import pytest

tokenizers = pytest.importorskip("tokenizers")

from llm_weighted_consensus_amd.engine.tokenizer import HFTokenizer, IncrementalDecoder, load_tokenizer  # noqa: E402

CORPUS = ["Select the response: `A` or `B`", "Paris is the capital of France.", "naïve café — ✓ ok",
          '{"response_key": "`C`"}', "The quick brown fox jumps over the lazy dog."] * 20
TEXTS = ["Output exactly one response key: `Q`", "café ✓ naïve", "  spaces  and\nnewlines\t!", "`A``T`"]


def _bytelevel(tmp_path):
    from tokenizers import Tokenizer, decoders, models, pre_tokenizers, trainers

    t = Tokenizer(models.BPE())
    t.pre_tokenizer = pre_tokenizers.ByteLevel(add_prefix_space=False)
    t.decoder = decoders.ByteLevel()
    t.train_from_iterator(CORPUS, trainers.BpeTrainer(vocab_size=400, special_tokens=["<|begin_of_text|>", "<|eot_id|>"],
                                                      initial_alphabet=pre_tokenizers.ByteLevel.alphabet()))
    p = tmp_path / "bl.json"
    t.save(str(p))
    return str(p)


def _sentencepiece(tmp_path):
    from tokenizers import Tokenizer, decoders, models, normalizers, pre_tokenizers, trainers

    t = Tokenizer(models.BPE(byte_fallback=True, unk_token="<unk>"))
    t.normalizer = normalizers.Replace(" ", "▁")
    t.pre_tokenizer = pre_tokenizers.Split("▁", behavior="merged_with_next")
    t.decoder = decoders.Sequence([decoders.Replace("▁", " "), decoders.ByteFallback(), decoders.Fuse()])
    byte_tokens = [f"<0x{b:02X}>" for b in range(256)]
    t.train_from_iterator(CORPUS, trainers.BpeTrainer(vocab_size=600, special_tokens=["<unk>", "<s>", "</s>"] + byte_tokens))
    p = tmp_path / "sp.json"
    t.save(str(p))
    return str(p)


def _wordpiece(tmp_path):
    from tokenizers import Tokenizer, decoders, models, normalizers, pre_tokenizers, processors, trainers

    t = Tokenizer(models.WordPiece(unk_token="[UNK]"))
    t.normalizer = normalizers.BertNormalizer(lowercase=True)
    t.pre_tokenizer = pre_tokenizers.BertPreTokenizer()
    t.decoder = decoders.WordPiece()
    t.train_from_iterator(CORPUS, trainers.WordPieceTrainer(vocab_size=300, special_tokens=["[PAD]", "[UNK]", "[CLS]", "[SEP]"]))
    t.post_processor = processors.TemplateProcessing(single="[CLS] $A [SEP]",
                                                     special_tokens=[("[CLS]", t.token_to_id("[CLS]")),
                                                                     ("[SEP]", t.token_to_id("[SEP]"))])
    p = tmp_path / "wp.json"
    t.save(str(p))
    return str(p)


@pytest.mark.parametrize("build", [_bytelevel, _sentencepiece])
def test_decoder_tokenizer_bytes_are_exact(tmp_path, build):
    tok = HFTokenizer(build(tmp_path), bos_token_id=1, eos_token_id=2)
    for text in TEXTS:
        ids = tok.encode(text)
        assert b"".join(tok.token_bytes(i) for i in ids) == text.encode("utf-8"), (tok.kind, text)
        assert tok.decode(ids) == text
        # streaming detokenisation over partial UTF-8 yields the text exactly once
        dec = IncrementalDecoder(tok)
        assert "".join(dec.push(i) for i in ids) + dec.flush() == text
    assert tok.encode("x", add_bos=True)[0] == 1


def test_wordpiece_encoder_tokenizer(tmp_path):
    tok = HFTokenizer(_wordpiece(tmp_path))
    assert tok.kind == "wordpiece"
    ids = tok.encode_with_specials("Paris is the capital")
    assert tok.token_bytes(ids[0]) == b"" and tok.token_bytes(ids[-1]) == b""  # [CLS] / [SEP]
    assert b"".join(tok.token_bytes(i) for i in ids).strip() == b"paris is the capital"


def test_load_tokenizer_from_spec(tmp_path):
    p = _bytelevel(tmp_path)
    assert isinstance(load_tokenizer({"tokenizer": p}, 500), HFTokenizer)
    assert type(load_tokenizer({}, 500)).__name__ == "ByteTokenizer"


def test_embedding_service_uses_model_tokenizer(tmp_path):
    import torch

    from llm_weighted_consensus_amd.embeddings.service import EmbeddingService
    from llm_weighted_consensus_amd.models.bert import BertEncoder
    from llm_weighted_consensus_amd.models.config import encoder_config

    tok = HFTokenizer(_wordpiece(tmp_path))
    enc = BertEncoder(encoder_config("bert-tiny"), device=torch.device("cpu"), seed=1)
    svc = EmbeddingService(enc, "tiny", cache_mb=0, tokenizer=tok)
    assert svc.tokenize("the fox") == tok.encode_with_specials("the fox")
    e, ntok = svc.embed_texts(["the fox", "a dog"])
    assert e.shape[0] == 2 and ntok == sum(len(tok.encode_with_specials(t)) for t in ["the fox", "a dog"])
