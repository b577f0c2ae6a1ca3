"""Completions archive: every completion the server produces, resolvable by id.

The reference only defines the trait (src/completions_archive/fetcher.rs:3-29) with a panicking OSS
stub (:31-65); the hosted product supplies storage.  This is the framework's own implementation:
an in-memory LRU of unary completions (chat / score / multichat) with an optional append-only JSONL
log for durability (replayed on start-up), i.e. checkpoint/resume for the serving state.  Lookups
return deep copies so callers can mutate freely.
"""
from __future__ import annotations

import json
import os
import threading
from collections import OrderedDict
from typing import Any, Optional, Tuple

from ..errors import ArchiveError
from ..schema.chat import ChatCompletion
from ..schema.score import MultichatCompletion, ScoreCompletion

KINDS = {"chat": ChatCompletion, "score": ScoreCompletion, "multichat": MultichatCompletion}


class CompletionsArchive:
    def __init__(self, capacity: int = 100_000, path: Optional[str] = None):
        self.capacity = capacity
        self.path = path
        self._d: "OrderedDict[str, Tuple[str, Any]]" = OrderedDict()
        self._lock = threading.Lock()
        if path and os.path.exists(path):
            self._replay(path)

    def _replay(self, path: str) -> None:
        with open(path, "r", encoding="utf-8") as f:
            for line in f:
                line = line.strip()
                if not line:
                    continue
                try:
                    rec = json.loads(line)
                    kind = rec["kind"]
                    obj = KINDS[kind].model_validate(rec["completion"])
                except Exception:
                    continue  # torn tail line after a crash
                self._put(kind, obj, persist=False)

    def _put(self, kind: str, obj: Any, persist: bool = True) -> None:
        with self._lock:
            self._d[obj.id] = (kind, obj)
            self._d.move_to_end(obj.id)
            while len(self._d) > self.capacity:
                self._d.popitem(last=False)
            if persist and self.path:
                with open(self.path, "a", encoding="utf-8") as f:
                    f.write(json.dumps({"kind": kind, "completion": obj.to_obj()}, ensure_ascii=False) + "\n")

    def store_chat(self, c: ChatCompletion) -> None:
        self._put("chat", c)

    def store_score(self, c: ScoreCompletion) -> None:
        self._put("score", c)

    def store_multichat(self, c: MultichatCompletion) -> None:
        self._put("multichat", c)

    def _get(self, kind: str, cid: str):
        with self._lock:
            v = self._d.get(cid)
        if v is None or v[0] != kind:
            raise ArchiveError.not_found(kind, cid)
        return v[1].model_copy(deep=True)

    # the reference trait (fetcher.rs:3-29)
    async def fetch_chat_completion(self, ctx: Any, cid: str) -> ChatCompletion:
        return self._get("chat", cid)

    async def fetch_score_completion(self, ctx: Any, cid: str) -> ScoreCompletion:
        return self._get("score", cid)

    async def fetch_multichat_completion(self, ctx: Any, cid: str) -> MultichatCompletion:
        return self._get("multichat", cid)

    def __len__(self) -> int:
        return len(self._d)
