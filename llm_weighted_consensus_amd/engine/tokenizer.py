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


class HFTokenizer:  # pragma: no cover - needs a tokenizer.json on disk
    def __init__(self, path: str, bos_token_id: Optional[int] = None, eos_token_id: Optional[int] = None):
        from tokenizers import Tokenizer

        self._t = Tokenizer.from_file(path)
        self.vocab_size = self._t.get_vocab_size()
        self.bos_token_id = bos_token_id
        self.eos_token_id = eos_token_id

    def encode(self, text: str, add_bos: bool = False) -> List[int]:
        ids = self._t.encode(text, add_special_tokens=False).ids
        return ([self.bos_token_id] if add_bos and self.bos_token_id is not None else []) + ids

    def token_bytes(self, tid: int) -> bytes:
        return self._t.decode([int(tid)], skip_special_tokens=False).encode()

    def decode(self, ids: Sequence[int]) -> str:
        return self._t.decode([int(t) for t in ids])

    def token_str(self, tid: int) -> str:
        return self._t.decode([int(tid)])

    def ids_for_text(self, text: str) -> List[int]:
        return self._t.encode(text, add_special_tokens=False).ids
