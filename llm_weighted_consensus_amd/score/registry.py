"""Score-model registry: validated `Model`s by content-addressed id.

Implements the reference's `score::model::Fetcher` seam (src/score/model/fetcher.rs:3-23, panicking in
the OSS build; dispatched for 22-char ids or `author/<22-char>` at src/score/completions/client.rs:
911-950).  Every inline model a request validates is registered so it can be referenced by id later;
an optional JSON file persists the registry across restarts.
"""
from __future__ import annotations

import json
import os
import threading
from typing import Any, Dict, Optional

from ..errors import ResponseError, ResponseErrorException
from ..utils import json as sjson
from .model import Model, ModelBase


class ModelRegistry:
    def __init__(self, path: Optional[str] = None):
        self.path = path
        self._models: Dict[str, Model] = {}
        self._lock = threading.Lock()
        if path and os.path.exists(path):
            with open(path, "r", encoding="utf-8") as f:
                for o in json.load(f):
                    m = Model.from_obj(o)
                    self._models[m.id] = m

    def register(self, m: Model) -> Model:
        with self._lock:
            new = m.id not in self._models
            self._models[m.id] = m
            if new and self.path:
                tmp = self.path + ".tmp"
                with open(tmp, "w", encoding="utf-8") as f:
                    f.write("[" + ",".join(sjson.dumps(x.to_obj()) for x in self._models.values()) + "]")
                os.replace(tmp, self.path)
        return m

    def register_base(self, base: ModelBase) -> Model:
        return self.register(base.into_model_validate())

    async def fetch(self, ctx: Any, model_id: str) -> Model:
        with self._lock:
            m = self._models.get(model_id)
        if m is None:
            raise ResponseErrorException(ResponseError(code=404, message={
                "kind": "model_not_found", "error": f"score model not found: {model_id}"}))
        return m

    def get(self, model_id: str) -> Optional[Model]:
        return self._models.get(model_id)

    def __len__(self) -> int:
        return len(self._models)
