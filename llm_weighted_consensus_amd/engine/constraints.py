"""Constrained decoding (K8d host side): per-step allowed-token bitmasks from a byte-level FSM.

Used for the voters' `json_schema` and `tool_call` output modes (reference src/score/llm/mod.rs:690-696;
schema built in src/score/completions/client.rs:1299-1339, always `strict: true`): the schema is an
object with an enum `response_key` and, with synthetic reasoning, a free-text `_think` first.  It is
compiled to a sequence of segments — literal bytes, a JSON string body, or a choice among literal
alternatives (a byte trie) — and the engine applies the mask produced for each step inside the fused
sampler kernel (the `mask` operand).

The FSM runs over BYTES; the sampler masks TOKENS.  :class:`TokenConstraint` bridges the two for any
tokenizer exposing exact per-token bytes (``token_bytes``: the byte tokenizer, byte-level BPE,
SentencePiece with byte fallback): a token is allowed in a state iff the FSM accepts ALL of its bytes
from that state, and the state advances by the token's bytes.  Allowed sets are computed against a
sorted byte-string index of the vocabulary (a trie walked by bisection, guided by the FSM's allowed
bytes) and, for free-string states, vectorised over the whole vocabulary (a token stays inside a JSON
string iff every byte is string-safe; only tokens whose first unsafe byte can close the string are
walked one by one).  Masks are cached per FSM state equivalence class.
"""
from __future__ import annotations

import bisect
import hashlib
import itertools
import json
from dataclasses import dataclass
from typing import Any, Dict, List, Optional, Sequence, Tuple, Union

import numpy as np


@dataclass
class Lit:
    data: bytes


@dataclass
class Str:
    """A JSON string body (no quotes): any byte except '"', '\\' and C0 controls; bounded length."""
    max_len: int = 2048


@dataclass
class Alt:
    options: List[bytes]


Segment = Union[Lit, Str, Alt]


def _trie(options: Sequence[bytes]) -> Dict:
    """Byte trie of the options: child per byte, -1 = an option ends here, -2 = the node's prefix bytes
    (its identity across constraint instances with the same options)."""
    root: Dict = {-2: b""}
    for o in options:
        n = root
        for b in o:
            if b not in n:
                n[b] = {-2: n[-2] + bytes([b])}
            n = n[b]
        n[-1] = True  # terminal marker
    return root


# Content ids of segment-list suffixes: equal ids <=> the same remaining grammar, whichever constraint
# instance (voter, request) it belongs to — the key of the cross-request token-mask cache.
_SUFFIX_IDS: Dict[tuple, int] = {}
_SUFFIX_LIMIT = 1 << 16
# Ids come from an ever-increasing counter and are never reused: when the table is bounded by a clear,
# a grammar seen afterwards gets a FRESH id, so no mask cached under an old id (TokenVocab.masks, keyed by
# (suffix id, local state)) and no live constraint holding an old id can ever alias a different grammar.
_SUFFIX_NEXT = itertools.count(1)


def _suffix_id(desc: tuple) -> int:
    v = _SUFFIX_IDS.get(desc)
    if v is None:
        if len(_SUFFIX_IDS) >= _SUFFIX_LIMIT:
            _SUFFIX_IDS.clear()
        v = _SUFFIX_IDS[desc] = next(_SUFFIX_NEXT)
    return v


# printable ASCII minus the quote and backslash: keeps constrained text valid UTF-8 and valid JSON
_STR_ALLOWED = np.array([1 if (0x20 <= b < 0x7F and b not in (0x22, 0x5C)) else 0 for b in range(256)], dtype=bool)


class SegmentConstraint:
    """State = (segment index, segment-local state); `done` once the last segment completes, after
    which only EOS is allowed."""

    def __init__(self, segments: List[Segment], eos_id: int):
        self.segments = segments
        self.eos_id = eos_id
        self.tries = {i: _trie(s.options) for i, s in enumerate(segments) if isinstance(s, Alt)}
        # suffix_ids[i] identifies segments[i:] by content
        self.suffix_ids = [0] * (len(segments) + 1)
        nxt = 0
        for i in range(len(segments) - 1, -1, -1):
            seg = segments[i]
            d = ("L", seg.data) if isinstance(seg, Lit) else ("S", seg.max_len) if isinstance(seg, Str) \
                else ("A", tuple(sorted(seg.options)))
            nxt = self.suffix_ids[i] = _suffix_id((d, nxt, eos_id))

    def __reduce__(self):
        # suffix ids are process-local (this process's counter): a copy shipped to an EngineGroup worker
        # re-derives them there from the grammar, so they never alias ids the worker assigned itself
        return (SegmentConstraint, (self.segments, self.eos_id))

    # ---- FSM
    def start(self):
        return self._normalize((0, 0))

    def _normalize(self, st):
        """Skip completed segments (empty literal / fully matched literal)."""
        i, local = st
        while i < len(self.segments):
            seg = self.segments[i]
            if isinstance(seg, Lit) and local >= len(seg.data):
                i, local = i + 1, 0
                continue
            break
        if i < len(self.segments) and isinstance(self.segments[i], Alt) and local == 0:
            local = self.tries[i]
        return (i, local)

    def is_done(self, st) -> bool:
        return st[0] >= len(self.segments)

    def allowed_bytes(self, st) -> Tuple[np.ndarray, bool]:
        """(allowed next bytes [256] bool, eos allowed)."""
        i, local = st
        allowed = np.zeros(256, dtype=bool)
        if i >= len(self.segments):
            return allowed, True
        seg = self.segments[i]
        if isinstance(seg, Lit):
            allowed[seg.data[local]] = True
        elif isinstance(seg, Str):
            if local < seg.max_len:
                allowed |= _STR_ALLOWED
            # the string may end: the next segment's first byte (a closing quote literal) is allowed
            nxt_st = self._normalize((i + 1, 0))
            nb, _ = self.allowed_bytes(nxt_st)
            allowed |= nb
        else:  # Alt: trie node
            for b in local:
                if b >= 0:
                    allowed[b] = True
            if -1 in local:  # an option may end here
                nb, eos = self.allowed_bytes(self._normalize((i + 1, 0)))
                allowed |= nb
                return allowed, eos
        return allowed, False

    def accepts(self, st, b: int) -> bool:
        """Whether byte ``b`` is allowed in state ``st`` (allowed_bytes(st)[b] without the arrays)."""
        i, local = st
        if i >= len(self.segments):
            return False
        seg = self.segments[i]
        if isinstance(seg, Lit):
            return seg.data[local] == b
        if isinstance(seg, Str):
            if _STR_ALLOWED[b] and local < seg.max_len:
                return True
            return self.accepts(self._normalize((i + 1, 0)), b)
        if b in local:
            return True
        return -1 in local and self.accepts(self._normalize((i + 1, 0)), b)

    def advance(self, st, token: int):
        if token < 0 or token > 255:
            return (len(self.segments), 0)  # EOS or invalid: finish
        i, local = st
        if i >= len(self.segments):
            return st
        seg = self.segments[i]
        if isinstance(seg, Lit):
            return self._normalize((i, local + 1))
        if isinstance(seg, Str):
            if _STR_ALLOWED[token] and local < seg.max_len:
                return (i, local + 1)
            return self.advance(self._normalize((i + 1, 0)), token)
        # Alt
        if token in local:
            return (i, local[token])
        if -1 in local:
            return self.advance(self._normalize((i + 1, 0)), token)
        return (len(self.segments), 0)


def _lit(s: str) -> Lit:
    return Lit(s.encode("utf-8"))


def compile_json_schema(schema: Any) -> Optional[List[Segment]]:
    """Compile the subset of JSON schemas the score voters use (and similar flat objects) to segments.

    Supported: {"type":"object","properties":{...},"required":[...],"additionalProperties":false}
    whose properties are `string` (free), string `enum`, `boolean`, or `integer`-free-less (not yet).
    Properties are emitted in schema order (all of them), compact JSON as serde_json would print it.
    Returns None for schemas outside the subset (the caller then decodes unconstrained)."""
    if not isinstance(schema, dict) or schema.get("type") != "object":
        return None
    props = schema.get("properties")
    if not isinstance(props, dict) or not props:
        return None
    segs: List[Segment] = [_lit("{")]
    for k, (name, p) in enumerate(props.items()):
        if not isinstance(p, dict):
            return None
        segs.append(_lit(("," if k else "") + json.dumps(name) + ":"))
        if "enum" in p and all(isinstance(e, str) for e in p["enum"]):
            segs.append(Alt([json.dumps(e, ensure_ascii=False).encode("utf-8") for e in p["enum"]]))
        elif p.get("type") == "string":
            segs += [_lit('"'), Str(int(p.get("maxLength", 2048))), _lit('"')]
        elif p.get("type") == "boolean":
            segs.append(Alt([b"true", b"false"]))
        else:
            return None
    segs.append(_lit("}"))
    return segs


class TokenVocab:
    """Per-tokenizer index for token-level masks (built once per tokenizer and model vocab, cached on the
    tokenizer object): exact token bytes, a lexicographically sorted byte-string index (the vocabulary
    trie: a node is a contiguous range), per token the position and value of its first JSON-string-unsafe
    byte.  Ids with no bytes (specials, padding ids beyond the tokenizer) are never allowed."""

    def __init__(self, tok, vocab_size: int):
        self.vocab_size = vocab_size
        n_tok = min(vocab_size, getattr(tok, "vocab_size", vocab_size))
        self.tb: List[bytes] = [tok.token_bytes(i) for i in range(n_tok)] + [b""] * (vocab_size - n_tok)
        ids = [i for i, b in enumerate(self.tb) if b]
        ids.sort(key=lambda i: self.tb[i])
        self.keys = [self.tb[i] for i in ids]
        self.ids = ids
        self.max_len = max((len(b) for b in self.keys), default=1)
        self.lens = np.array([len(b) for b in self.tb], dtype=np.int64)
        fu = np.zeros(vocab_size, dtype=np.int64)   # index of the first string-unsafe byte (= len if none)
        fub = np.zeros(vocab_size, dtype=np.int64)  # that byte (0 if none)
        for i, b in enumerate(self.tb):
            if not b:
                continue
            arr = np.frombuffer(b, dtype=np.uint8)
            bad = np.nonzero(~_STR_ALLOWED[arr])[0]
            fu[i] = bad[0] if len(bad) else len(b)
            fub[i] = arr[bad[0]] if len(bad) else 0
        self.first_unsafe, self.first_unsafe_byte = fu, fub
        self.nonempty = self.lens > 0
        # cross-request mask cache: (grammar-suffix id, state within the segment) -> (digest, words)
        self.masks: Dict[Any, Tuple[bytes, np.ndarray]] = {}

    @staticmethod
    def of(tok, vocab_size: int) -> "TokenVocab":
        cache = tok.__dict__.setdefault("_lwc_token_vocab", {})
        tv = cache.get(vocab_size)
        if tv is None:
            tv = cache[vocab_size] = TokenVocab(tok, vocab_size)
        return tv

    def child_range(self, lo: int, hi: int, depth: int, b: int) -> Tuple[int, int]:
        """Sub-range of [lo, hi) (all sharing a prefix of length ``depth``) whose byte ``depth`` is ``b``."""
        keys = self.keys
        pre = keys[lo][:depth] if lo < hi else b""
        a = bisect.bisect_left(keys, pre + bytes([b]), lo, hi)
        z = bisect.bisect_left(keys, pre + bytes([b + 1]), a, hi) if b < 255 else hi
        return a, z


class TokenConstraint:
    """Token-level view of a byte FSM (:class:`SegmentConstraint`) for one tokenizer.  The engine calls
    ``start`` / ``advance(state, token_id)`` / ``is_done`` and ``mask_entry(state) -> (digest, uint32
    [V/32] bitmask)``; masks are cached per state equivalence class."""

    def __init__(self, fsm: SegmentConstraint, vocab: TokenVocab):
        self.fsm = fsm
        self.vocab = vocab
        self.eos_id = fsm.eos_id

    def __getstate__(self):
        # shipped to an EngineGroup worker with the request: the grammar only — the worker re-binds the
        # vocabulary index of ITS tokenizer (bind), which also keeps its cross-request mask cache warm
        return {"fsm": self.fsm, "eos_id": self.eos_id, "vocab_size": self.vocab.vocab_size if self.vocab else None}

    def __setstate__(self, st):
        self.fsm, self.eos_id, self.vocab = st["fsm"], st["eos_id"], None
        self._vocab_size = st["vocab_size"]

    def bind(self, tok, vocab_size: int) -> "TokenConstraint":
        """Attach the vocabulary index of ``tok`` (after unpickling in another process)."""
        if self.vocab is None:
            self.vocab = TokenVocab.of(tok, vocab_size)
        return self

    def start(self):
        return self.fsm.start()

    def is_done(self, st) -> bool:
        return self.fsm.is_done(st)

    def advance_bytes(self, st, data: bytes):
        """State after consuming ``data``, or None if the FSM rejects a byte."""
        fsm = self.fsm
        for b in data:
            if not fsm.accepts(st, b):
                return None
            st = fsm.advance(st, b)
        return st

    def advance(self, st, token: int):
        if token == self.eos_id or not (0 <= token < self.vocab.vocab_size):
            return (len(self.fsm.segments), 0)
        nxt = self.advance_bytes(st, self.vocab.tb[token])
        return (len(self.fsm.segments), 0) if nxt is None else nxt

    # ---- masks
    def _key(self, st):
        """Content key of the state's token mask: the remaining grammar (suffix id) and the position in
        the current segment — equal across voters / requests whose remaining grammar is equal."""
        i, local = st
        segs = self.fsm.segments
        if i >= len(segs):
            return (0, self.eos_id)
        seg = segs[i]
        sid = self.fsm.suffix_ids[i]
        if isinstance(seg, Str):  # only the remaining length matters, and only up to the longest token
            return (sid, min(seg.max_len - local, self.vocab.max_len + 1))
        if isinstance(seg, Alt):
            if -1 in local and all(k < 0 for k in local):  # a completed option: the rest of the grammar
                return self._key(self.fsm._normalize((i + 1, 0)))
            return (sid, local[-2])
        return (sid, local)

    def allowed_tokens(self, st) -> Tuple[np.ndarray, bool]:
        """(bool [V] allowed tokens, eos allowed) in FSM state ``st``."""
        sparse, dense, eos = self._allowed(st)
        if dense is None:
            dense = np.zeros(self.vocab.vocab_size, dtype=bool)
            dense[sparse] = True
        return dense, eos

    def _allowed(self, st):
        """(sorted allowed ids or None, dense bool [V] or None, eos allowed).  Literal / enum states allow a
        handful of tokens and stay sparse (no [V] arrays on the per-step path); free-string states are
        vectorised over the whole vocabulary."""
        fsm, tv = self.fsm, self.vocab
        if fsm.is_done(st):
            return [], None, True
        i, local = st
        seg = fsm.segments[i]
        if isinstance(seg, Str):
            room = seg.max_len - local
            # tokens that stay inside the string: every byte string-safe and the length fits
            ok = tv.nonempty & (tv.first_unsafe == tv.lens) & (tv.lens <= room)
            # tokens that close the string: a safe prefix, then a byte the FSM accepts to end it
            allowed, _ = fsm.allowed_bytes(st)
            cand = np.nonzero(tv.nonempty & (tv.first_unsafe < tv.lens) & (tv.first_unsafe <= room)
                              & allowed[tv.first_unsafe_byte])[0]
            for t in cand.tolist():
                k = int(tv.first_unsafe[t])
                if self.advance_bytes((i, local + k), tv.tb[t][k:]) is not None:
                    ok[t] = True
            return None, ok, False
        # literal / alternative states: walk the vocabulary trie guided by the FSM's allowed bytes
        found: List[int] = []
        stack = [(st, 0, len(tv.keys), 0)]
        ids, keys = tv.ids, tv.keys
        while stack:
            cur, lo, hi, depth = stack.pop()
            while lo < hi and len(keys[lo]) == depth:  # tokens ending exactly here were fully accepted
                if depth:
                    found.append(ids[lo])
                lo += 1
            if lo >= hi or fsm.is_done(cur):
                continue
            ci, clocal = cur
            if isinstance(fsm.segments[ci], Str):
                # entered a free string mid-token: finish the (few) tokens of this subtree one by one
                for k in range(lo, hi):
                    if self.advance_bytes(cur, keys[k][depth:]) is not None:
                        found.append(ids[k])
                continue
            for b in self._next_bytes(cur):
                a, z = tv.child_range(lo, hi, depth, b)
                if a < z:
                    stack.append((fsm.advance(cur, b), a, z, depth + 1))
        found.sort()
        return found, None, False

    def _next_bytes(self, st) -> List[int]:
        """The bytes the FSM accepts in a literal / enum state (a few; no [256] arrays)."""
        fsm = self.fsm
        i, local = st
        seg = fsm.segments[i]
        if isinstance(seg, Lit):
            return [seg.data[local]]
        if isinstance(seg, Alt):
            out = [b for b in local if b >= 0]
            if -1 in local and i + 1 < len(fsm.segments):
                out += [b for b in self._next_bytes_any(fsm._normalize((i + 1, 0))) if b not in out]
            return out
        return self._next_bytes_any(st)

    def _next_bytes_any(self, st) -> List[int]:
        if self.fsm.is_done(st):
            return []
        i, _ = st
        if isinstance(self.fsm.segments[i], Str):
            allowed, _ = self.fsm.allowed_bytes(st)
            return np.nonzero(allowed)[0].tolist()
        return self._next_bytes(st)

    def mask_entry(self, st) -> "MaskEntry":
        """The state's mask for the sampler's table: ``.key`` (content) and ``.words()`` (uint32 [V/32]),
        cached per remaining-grammar state across every voter and request of this vocabulary."""
        key = self._key(st)
        hit = self.vocab.masks.get(key)
        if hit is not None:
            return hit
        sparse, dense, eos = self._allowed(st)
        V = self.vocab.vocab_size
        if sparse is not None:
            if (eos or not sparse) and 0 <= self.eos_id < V and self.eos_id not in sparse:
                sparse = sorted(sparse + [self.eos_id])  # done, or a dead end: EOS lets the sequence stop
            hit = MaskEntry(("s", tuple(sparse)), V, ids=sparse)
        else:
            if (eos or not dense.any()) and 0 <= self.eos_id < V:
                dense[self.eos_id] = True
            words = np.packbits(dense, bitorder="little").view(np.uint32)
            hit = MaskEntry(("d", hashlib.blake2b(words.tobytes(), digest_size=16).digest()), V, words=words)
        if len(self.vocab.masks) > 8192:
            self.vocab.masks.clear()
        self.vocab.masks[key] = hit
        return hit


class MaskEntry:
    """One token mask: a hashable content key (the allowed ids themselves for sparse masks, a digest of
    the bits for dense ones) and the packed words, built only when the engine uploads a new table row."""

    __slots__ = ("key", "V", "_ids", "_words")

    def __init__(self, key, V: int, ids: Optional[List[int]] = None, words: Optional[np.ndarray] = None):
        self.key, self.V, self._ids, self._words = key, V, ids, words

    def words(self) -> np.ndarray:
        if self._words is None:
            w = np.zeros(self.V // 32, dtype=np.uint32)
            ids = np.asarray(self._ids, dtype=np.int64)
            np.bitwise_or.at(w, ids >> 5, (np.uint32(1) << (ids & 31).astype(np.uint32)))
            self._words = w
        return self._words


def constraint_for_schema(schema: Any, tok, vocab_size: Optional[int] = None) -> Optional[TokenConstraint]:
    """Schema -> token-level constraint for ``tok`` (``vocab_size`` = the model's logits width, which may
    exceed the tokenizer's vocabulary; defaults to the tokenizer's)."""
    segs = compile_json_schema(schema)
    if segs is None:
        return None
    V = vocab_size or tok.vocab_size
    if V % 32:
        raise ValueError(f"vocab size {V} is not a multiple of 32 (mask words)")
    return TokenConstraint(SegmentConstraint(segs, tok.eos_token_id), TokenVocab.of(tok, V))
