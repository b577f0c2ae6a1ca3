"""Tokenizers for the local engine.

There is no network here (no Llama / BERT tokenizer downloads), so the default is a lossless
byte-level tokenizer over the model's vocabulary:

* ids 0..255 are raw bytes (every string round-trips exactly: prompts, backtick keys, JSON);
* ids 256..V-1 decode to deterministic synthetic ASCII word pieces (" w<base36 id>") so that text
  produced by random-init weights is printable and stream-decodable;
* ``bos``/``eos`` follow the model config.

A real ``tokenizer.json`` (HF ``tokenizers``) can be supplied instead with
``HFTokenizer(path)``; both expose the same interface.
"""
from __future__ import annotations

from functools import lru_cache
from typing import List, Optional, Sequence

_B36 = "0123456789abcdefghijklmnopqrstuvwxyz"


def _b36(n: int) -> str:
    s = ""
    while True:
        n, r = divmod(n, 36)
        s = _B36[r] + s
        if n == 0:
            return s


class ByteTokenizer:
    def __init__(self, vocab_size: int, bos_token_id: Optional[int] = None, eos_token_id: Optional[int] = None):
        if vocab_size < 258:
            raise ValueError("vocab too small for the byte tokenizer")
        self.vocab_size = vocab_size
        self.bos_token_id = bos_token_id if bos_token_id is not None and bos_token_id >= 256 else vocab_size - 2
        self.eos_token_id = eos_token_id if eos_token_id is not None and eos_token_id >= 256 else vocab_size - 1
        self.special = {self.bos_token_id: "", self.eos_token_id: ""}

    def encode(self, text: str, add_bos: bool = False) -> List[int]:
        ids = list(text.encode("utf-8"))
        return ([self.bos_token_id] if add_bos else []) + ids

    @lru_cache(maxsize=1 << 16)
    def token_bytes(self, tid: int) -> bytes:
        if 0 <= tid < 256:
            return bytes([tid])
        if tid in self.special:
            return b""
        return (" w" + _b36(tid)).encode()

    def decode(self, ids: Sequence[int]) -> str:
        return b"".join(self.token_bytes(int(t)) for t in ids).decode("utf-8", errors="replace")

    def token_str(self, tid: int) -> str:
        return self.token_bytes(int(tid)).decode("utf-8", errors="replace")

    def ids_for_text(self, text: str) -> List[int]:
        """Token ids whose decoding is exactly ``text`` piecewise (used by constrained decoding)."""
        return list(text.encode("utf-8"))


class IncrementalDecoder:
    """Streams UTF-8 text out of token bytes, holding back incomplete multi-byte sequences."""

    def __init__(self, tok):
        self.tok = tok
        self.pending = b""

    def push(self, tid: int) -> str:
        self.pending += self.tok.token_bytes(int(tid))
        for cut in range(len(self.pending), max(len(self.pending) - 4, -1), -1):
            try:
                s = self.pending[:cut].decode("utf-8")
            except UnicodeDecodeError:
                continue
            self.pending = self.pending[cut:]
            return s
        return ""

    def flush(self) -> str:
        s = self.pending.decode("utf-8", errors="replace")
        self.pending = b""
        return s


def _bytes_to_unicode() -> dict:
    """The byte-level BPE alphabet (GPT-2 / Llama-3 ``ByteLevel``): printable stand-ins for all 256 bytes."""
    bs = list(range(ord("!"), ord("~") + 1)) + list(range(ord("\xa1"), ord("\xac") + 1)) + \
        list(range(ord("\xae"), ord("\xff") + 1))
    cs = bs[:]
    n = 0
    for b in range(256):
        if b not in bs:
            bs.append(b)
            cs.append(256 + n)
            n += 1
    return dict(zip(bs, (chr(c) for c in cs)))


_BYTE_OF_CHAR = {c: b for b, c in _bytes_to_unicode().items()}


class HFTokenizer:
    """A real ``tokenizer.json`` (HF ``tokenizers``, loaded from disk; nothing is downloaded).

    ``token_bytes`` is exact per token — what incremental detokenisation and the vote extractor's
    byte-offset alignment of key letters need (reference: src/score/completions/client.rs:1727-1784) —
    for the three vocabulary families in use: byte-level BPE (Llama-3, Mistral-Nemo: the GPT-2 byte
    alphabet), SentencePiece-style pieces (Llama-2 / Mistral / Mixtral: ``▁`` = space, ``<0xNN>`` byte
    fallback) and WordPiece (BERT / BGE: ``##`` continuations, a space before every other word)."""

    def __init__(self, path: str, bos_token_id: Optional[int] = None, eos_token_id: Optional[int] = None):
        import json

        from tokenizers import Tokenizer

        self._t = Tokenizer.from_file(path)
        self.vocab_size = self._t.get_vocab_size(with_added_tokens=True)
        self.bos_token_id = bos_token_id
        self.eos_token_id = eos_token_id
        with open(path, "r", encoding="utf-8") as f:
            spec = json.load(f)
        dec = json.dumps(spec.get("decoder") or {}) + json.dumps(spec.get("pre_tokenizer") or {})
        model = (spec.get("model") or {}).get("type", "")
        if "ByteLevel" in dec:
            self.kind = "bytelevel"
        elif model == "WordPiece" or "WordPiece" in dec:
            self.kind = "wordpiece"
        else:
            self.kind = "sentencepiece"
        self.special = {t["id"] for t in spec.get("added_tokens", []) if t.get("special")}
        # SentencePiece exports that prepend "▁" to the input strip it again when decoding
        self.strip_prefix_space = "Prepend" in json.dumps(spec.get("normalizer") or {})
        self._cache: dict = {}

    def encode(self, text: str, add_bos: bool = False) -> List[int]:
        ids = self._t.encode(text, add_special_tokens=False).ids
        return ([self.bos_token_id] if add_bos and self.bos_token_id is not None else []) + ids

    def encode_with_specials(self, text: str) -> List[int]:
        """The tokenizer's own post-processing (e.g. [CLS] ... [SEP] for an encoder)."""
        return self._t.encode(text, add_special_tokens=True).ids

    def token_bytes(self, tid: int) -> bytes:
        tid = int(tid)
        b = self._cache.get(tid)
        if b is not None:
            return b
        tok = self._t.id_to_token(tid)
        if tok is not None and self.kind == "sentencepiece" and len(tok) == 6 and tok.startswith("<0x") \
                and tok.endswith(">"):
            b = bytes([int(tok[3:5], 16)])  # byte-fallback piece (some exports list these as special)
        elif tok is None or tid in self.special:
            b = b""
        elif self.kind == "bytelevel":
            b = bytes(_BYTE_OF_CHAR.get(c, 0x3F) for c in tok)
        elif self.kind == "wordpiece":
            b = (tok[2:] if tok.startswith("##") else " " + tok).encode()
        else:
            b = tok.replace("\u2581", " ").encode()
        self._cache[tid] = b
        return b

    def decode(self, ids: Sequence[int]) -> str:
        if self.kind == "wordpiece":
            return self._t.decode([int(t) for t in ids])
        # exactly the concatenation the streaming path produces (special tokens decode to nothing)
        text = b"".join(self.token_bytes(t) for t in ids).decode("utf-8", errors="replace")
        return text[1:] if self.strip_prefix_space and text.startswith(" ") else text

    def token_str(self, tid: int) -> str:
        return self.token_bytes(tid).decode("utf-8", errors="replace")

    def ids_for_text(self, text: str) -> List[int]:
        return self._t.encode(text, add_special_tokens=False).ids


def load_tokenizer(spec: dict, vocab_size: int, bos_token_id: Optional[int] = None,
                   eos_token_id: Optional[int] = None):
    """Server model spec -> tokenizer: ``"tokenizer": "/path/tokenizer.json"`` loads it, otherwise the
    byte tokenizer over the model's vocabulary."""
    path = spec.get("tokenizer")
    if path:
        return HFTokenizer(path, bos_token_id, eos_token_id)
    return ByteTokenizer(vocab_size, bos_token_id, eos_token_id)
