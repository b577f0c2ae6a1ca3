"""Constrained decoding (K8d host side): per-step allowed-token bitmasks from a byte-level FSM.

Used for the voters' `json_schema` and `tool_call` output modes (reference src/score/llm/mod.rs:690-696;
schema built in src/score/completions/client.rs:1299-1339, always `strict: true`): the schema is an
object with an enum `response_key` and, with synthetic reasoning, a free-text `_think` first.  It is
compiled to a sequence of segments — literal bytes, a JSON string body, or a choice among literal
alternatives (a byte trie) — and the engine applies the mask produced for each step inside the fused
sampler kernel (the `mask` operand).  Works on the byte-level tokenizer (token id == byte for
0..255); multi-byte synthetic tokens are never allowed inside a constrained span.
"""
from __future__ import annotations

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
    root: Dict = {}
    for o in options:
        n = root
        for b in o:
            n = n.setdefault(b, {})
        n[-1] = True  # terminal marker
    return root


# printable ASCII minus the quote and backslash: keeps constrained text valid UTF-8 and valid JSON
_STR_ALLOWED = np.array([1 if (0x20 <= b < 0x7F and b not in (0x22, 0x5C)) else 0 for b in range(256)], dtype=bool)
_POW2 = (np.uint64(1) << np.arange(32, dtype=np.uint64))


class SegmentConstraint:
    """State = (segment index, segment-local state); `done` once the last segment completes, after
    which only EOS is allowed."""

    def __init__(self, segments: List[Segment], eos_id: int):
        self.segments = segments
        self.eos_id = eos_id
        self.tries = {i: _trie(s.options) for i, s in enumerate(segments) if isinstance(s, Alt)}

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
                if b != -1:
                    allowed[b] = True
            if -1 in local:  # an option may end here
                nb, eos = self.allowed_bytes(self._normalize((i + 1, 0)))
                allowed |= nb
                return allowed, eos
        return allowed, False

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

    def mask(self, st, vocab_size: int) -> np.ndarray:
        """uint32 bitmask [vocab_size/32] for the sampler kernel."""
        allowed, eos = self.allowed_bytes(st)
        bits = np.zeros(vocab_size, dtype=bool)
        bits[:256] = allowed
        if eos and 0 <= self.eos_id < vocab_size:
            bits[self.eos_id] = True
        if not bits.any():  # dead end: allow EOS so the sequence can stop
            bits[self.eos_id] = True
        return (bits.reshape(-1, 32).astype(np.uint64) @ _POW2).astype(np.uint32)


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
            segs += [_lit('"'), Str(), _lit('"')]
        elif p.get("type") == "boolean":
            segs.append(Alt([b"true", b"false"]))
        else:
            return None
    segs.append(_lit("}"))
    return segs


def constraint_for_schema(schema: Any, eos_id: int) -> Optional[SegmentConstraint]:
    segs = compile_json_schema(schema)
    return SegmentConstraint(segs, eos_id) if segs is not None else None
