"""HBM-resident embedding archive: a per-GPU, content-addressed store of encoder embeddings.

The north star keeps the completions archive "resident in 288 GB HBM".  The JSON side of the archive
(`store.py`) holds the completions themselves; this module holds what is expensive to recompute from
them — the unit embedding of every text the encoder has seen — as rows of ONE preallocated device slab
(no per-entry allocations, no fragmentation, gathers are a single index_select).

Keys are content hashes (xxh3-128 of the encoder's token ids + the truncation length), so an archived
completion that comes back as a choice or candidate (`{"type": "chat_completion", "id", "choice_index"}`
resolved by `archive/resolve.py`), the same choice text seen by many voters / requests, or a training-
table request repeated verbatim is embedded once per GPU.  Eviction is LRU over whole rows under a byte
budget (``LWC_EMBED_CACHE_MB``; 288 GB of HBM holds ~70 M 1024-d fp32 rows, so the default budget of
4 GiB — ~1 M rows of bge-large — is a rounding error next to the decoder's KV cache).

The reference has no embedding storage at all (its archive is a panicking trait stub,
src/completions_archive/fetcher.rs:31-65).
"""
from __future__ import annotations

import threading
from collections import OrderedDict
from typing import List, Optional, Sequence, Tuple

import numpy as np
import torch
import xxhash


def content_key(token_ids: Sequence[int], max_tokens: int) -> bytes:
    """16-byte key of an encoder input: xxh3-128 over the (truncation-aware) int32 token ids."""
    a = np.asarray(token_ids[:max_tokens], dtype=np.int32)
    return xxhash.xxh3_128_digest(a.tobytes(), seed=max_tokens)


class ResidentEmbeddings:
    def __init__(self, dim: int, device, budget_bytes: int, dtype=torch.float32):
        self.dim = dim
        self.device = torch.device(device)
        self.dtype = dtype
        row = dim * torch.empty((), dtype=dtype).element_size()
        self.capacity = max(0, int(budget_bytes) // row)
        self.slab = torch.empty(self.capacity, dim, dtype=dtype, device=self.device)
        self._slots: "OrderedDict[bytes, int]" = OrderedDict()
        self._free = list(range(self.capacity - 1, -1, -1))
        self._lock = threading.Lock()
        self.hits = self.misses = self.evictions = 0

    def __len__(self) -> int:
        return len(self._slots)

    @property
    def bytes_used(self) -> int:
        return len(self._slots) * self.dim * self.slab.element_size()

    def lookup(self, keys: Sequence[bytes]) -> List[Optional[int]]:
        """Slot of each key (None = miss); hits are refreshed in the LRU order."""
        out: List[Optional[int]] = []
        with self._lock:
            for k in keys:
                s = self._slots.get(k)
                if s is not None:
                    self._slots.move_to_end(k)
                    self.hits += 1
                else:
                    self.misses += 1
                out.append(s)
        return out

    def gather(self, slots: Sequence[int]) -> torch.Tensor:
        idx = torch.as_tensor(list(slots), dtype=torch.int64).to(self.device, non_blocking=True)
        return self.slab.index_select(0, idx)

    def put(self, keys: Sequence[bytes], emb: torch.Tensor) -> None:
        """Insert rows (evicting least-recently-used rows when the slab is full).  Keys already present are
        refreshed, not duplicated.  At most ``capacity`` NEW keys are stored per call (the excess is skipped):
        otherwise a key inserted earlier in the same call could be evicted and its slot handed to a later
        key, leaving two rows of one index_copy_ aimed at one slot."""
        if self.capacity == 0 or not keys:
            return
        rows, slots = [], []
        with self._lock:
            for i, k in enumerate(keys):
                if k in self._slots:
                    self._slots.move_to_end(k)
                    continue
                if len(rows) >= self.capacity:
                    continue
                if not self._free:
                    if not self._slots:
                        break
                    _, s = self._slots.popitem(last=False)
                    self._free.append(s)
                    self.evictions += 1
                s = self._free.pop()
                self._slots[k] = s
                rows.append(i)
                slots.append(s)
        if rows:
            src = emb.index_select(0, torch.as_tensor(rows, dtype=torch.int64, device=emb.device))
            self.slab.index_copy_(0, torch.as_tensor(slots, dtype=torch.int64, device=self.device),
                                  src.to(device=self.device, dtype=self.dtype))

    def embed_through(self, token_lists: Sequence[Sequence[int]], max_tokens: int,
                      embed_fn) -> Tuple[torch.Tensor, int]:
        """Embeddings [n, d] for ``token_lists``, running ``embed_fn(missing_lists) -> [m, d]`` only on the
        cache misses (deduplicated: a text repeated inside one call is embedded once).  Returns the rows
        and the number of texts actually encoded."""
        keys = [content_key(t, max_tokens) for t in token_lists]
        slots = self.lookup(keys)
        miss_first: "OrderedDict[bytes, int]" = OrderedDict()
        for i, (k, s) in enumerate(zip(keys, slots)):
            if s is None and k not in miss_first:
                miss_first[k] = i
        out = torch.empty(len(keys), self.dim, dtype=self.dtype, device=self.device)
        hit_rows = [i for i, s in enumerate(slots) if s is not None]
        if hit_rows:
            out[torch.as_tensor(hit_rows, device=self.device)] = self.gather([slots[i] for i in hit_rows])
        if miss_first:
            fresh = embed_fn([token_lists[i] for i in miss_first.values()]).to(device=self.device, dtype=self.dtype)
            pos = {k: j for j, k in enumerate(miss_first)}
            miss_rows = [i for i, s in enumerate(slots) if s is None]
            out[torch.as_tensor(miss_rows, device=self.device)] = fresh[
                torch.as_tensor([pos[keys[i]] for i in miss_rows], device=self.device)]
            self.put(list(miss_first), fresh)
        return out, len(miss_first)

    def stats(self) -> dict:
        return {"entries": len(self._slots), "capacity": self.capacity, "bytes": self.bytes_used,
                "hits": self.hits, "misses": self.misses, "evictions": self.evictions}
