"""Varlen packing of token-id lists for the encoders (BERT-style and decoder embedders).

Thousands of candidates per consensus batch must not cost per-token Python work: the bench packs
4096 x 128 generated ids while the GPU waits for the encoder's first kernel.  The engine keeps each
sequence's generated tokens in an ``array('i')`` (``engine.Sequence.tokens``), so the common case is a
zero-copy ``np.frombuffer`` view per candidate and one concatenation; plain lists of equal length go
through one flat iterator, anything else row by row.
"""
from __future__ import annotations

import itertools
from array import array
from typing import Sequence, Tuple

import numpy as np


def _row(tl, cap: int, tail: bool) -> np.ndarray:
    if isinstance(tl, array) and tl.typecode == "i":
        a = np.frombuffer(tl, dtype=np.int32) if len(tl) else np.zeros(0, dtype=np.int32)
    else:
        a = np.asarray(list(tl), dtype=np.int64)
    a = a[-cap:] if tail else a[:cap]
    return a if len(a) else np.zeros(1, dtype=a.dtype)


def pack_ids(token_lists: Sequence[Sequence[int]], cap: int, vocab: int,
             tail: bool = False) -> Tuple[np.ndarray, np.ndarray, np.ndarray, int]:
    """-> (ids int32 [T], positions int32 [T], cu_seqlens int32 [n+1], max_len).  Each list is truncated to
    ``cap`` tokens (its first ``cap``, or its last with ``tail`` — last-token pooling keeps the end), an
    empty list becomes [0], ids are folded into ``vocab``."""
    n = len(token_lists)
    if n == 0:
        z = np.zeros(0, dtype=np.int32)
        return z, z, np.zeros(1, dtype=np.int32), 0
    if all(isinstance(tl, array) and tl.typecode == "i" for tl in token_lists):
        lens = np.fromiter((len(tl) for tl in token_lists), dtype=np.int64, count=n)
        if int(lens.min()) >= 1 and int(lens.max()) <= cap:
            # nothing to truncate or pad: the arrays' bytes joined in C, one copy
            ids = np.frombuffer(b"".join(token_lists), dtype=np.int32)
        else:
            rows = [_row(tl, cap, tail) for tl in token_lists]
            lens = np.fromiter((len(r) for r in rows), dtype=np.int64, count=n)
            ids = np.concatenate(rows).astype(np.int32)
    else:
        lens = np.fromiter((max(1, min(len(tl), cap)) for tl in token_lists), dtype=np.int64, count=n)
        n0 = int(lens[0])
        if (lens == n0).all() and all(len(tl) >= n0 for tl in token_lists):
            # one flat iterator straight into the array (half the host time of a nested-list asarray)
            if all(len(tl) == n0 for tl in token_lists):
                src = token_lists
            else:
                src = (list(tl)[-n0:] if tail else list(tl)[:n0] for tl in token_lists)
            ids = np.fromiter(itertools.chain.from_iterable(src), dtype=np.int64, count=n0 * n)
        else:
            ids = np.concatenate([_row(tl, cap, tail).astype(np.int64) for tl in token_lists])
        ids = ids.astype(np.int32)
    ids = np.remainder(ids, np.int32(vocab), dtype=np.int32)
    cu = np.zeros(n + 1, dtype=np.int32)
    np.cumsum(lens, out=cu[1:])
    n0 = int(lens[0])
    if (lens == n0).all():
        pos = np.tile(np.arange(n0, dtype=np.int32), n)
    else:
        pos = np.arange(int(cu[-1]), dtype=np.int32) - np.repeat(cu[:-1], lens)
    return ids, pos.astype(np.int32, copy=False), cu, int(lens.max())
