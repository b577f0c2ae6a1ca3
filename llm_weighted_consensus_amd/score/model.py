"""Score model identity: `ModelBase` (1..=128 voters + a weight mode) -> validated `Model`.

Contract: reference src/score/model/mod.rs:37-199 —
  prepare -> 1..=128 llms -> weight.validate -> per llm: id / training_table_id / multichat_id and
  `into_llm` validation -> sort llms by id -> model id = xxh3(weight JSON ‖ sorted llm ids);
  training-table id = xxh3(embeddings JSON ‖ llm training-table ids); multichat id =
  xxh3(multichat ids in llm order ‖ multichat ids sorted); indices assigned as the reference does
  (multichat_index = position in the sorted id list + duplicates seen so far).
"""
from __future__ import annotations

from typing import List, Literal, Optional, Union

from pydantic import Field

from ..schema.base import Wire
from ..schema.chat import ProviderPreferences
from ..utils import json as sjson
from .llm import I32_MAX, Hasher, Llm, LlmBase, prepare_provider, validate_provider, weight_type


class ModelWeightStatic(Wire):
    type: Literal["static"] = "static"


class TrainingTableEmbeddings(Wire):
    model: str
    max_tokens: int
    provider: Optional[ProviderPreferences] = None

    def prepare(self) -> None:
        self.provider = prepare_provider(self.provider)

    def validate_emb(self) -> None:
        if self.model == "":
            raise ValueError("`embeddings.model` cannot be empty")
        if self.max_tokens > I32_MAX:
            raise ValueError(f"`embeddings.max_tokens` must be at most {I32_MAX}: got {self.max_tokens}")
        validate_provider(self.provider)


class ModelWeightTrainingTable(Wire):
    type: Literal["training_table"] = "training_table"
    embeddings: TrainingTableEmbeddings
    top: int

    def validate_weight(self) -> None:
        if self.top < 1:
            raise ValueError(f"training table weight `top` must be at least 1: `top`={self.top}")
        if self.top > I32_MAX:
            raise ValueError(f"training table weight `top` must be at most {I32_MAX}: `top`={self.top}")


ModelWeight = Union[ModelWeightStatic, ModelWeightTrainingTable]


class ModelBase(Wire):
    llms: List[LlmBase]
    weight: ModelWeight = Field(default_factory=ModelWeightStatic, union_mode="left_to_right")

    def into_model_validate(self) -> "Model":
        """Raises ValueError (-> ScoreError.invalid_model)."""
        mb = self.model_copy(deep=True)
        if isinstance(mb.weight, ModelWeightTrainingTable):
            mb.weight.embeddings.prepare()
        for l in mb.llms:
            l.prepare()
        if len(mb.llms) < 1:
            raise ValueError("query model must have at least 1 llm")
        if len(mb.llms) > 128:
            raise ValueError(f"query model must have at most 128 llms: llms_len={len(mb.llms)}")
        wtype = "static" if isinstance(mb.weight, ModelWeightStatic) else "training_table"
        if wtype == "training_table":
            mb.weight.validate_weight()
        tt_ids: Optional[List[str]] = [] if wtype == "training_table" else None
        mc_ids: List[str] = []
        llms: List[Llm] = []
        for base in mb.llms:
            lid = base.id_string()
            ttid = base.training_table_id_string()
            mcid = base.multichat_id_string()
            if tt_ids is not None and ttid is not None and ttid not in tt_ids:
                tt_ids.append(ttid)
            mc_ids.append(mcid)
            base.validate_llm(wtype)
            llms.append(Llm(base, lid, 0, mcid, -1, ttid, None))
        llms.sort(key=lambda x: x.id)
        if tt_ids is not None:
            tt_ids.sort()
        mc_ids.sort()
        h = Hasher()
        h.write(sjson.dumps(mb.weight.to_obj()))
        tth = None
        if tt_ids is not None:
            tth = Hasher()
            tth.write(sjson.dumps(mb.weight.embeddings.to_obj()))
        mch = Hasher()
        seen = {}
        for i, l in enumerate(llms):
            h.write(l.id)
            l.index = i
            if tth is not None:
                tth.write(l.training_table_id)
                l.training_table_index = tt_ids.index(l.training_table_id)
            seen[l.multichat_id] = seen.get(l.multichat_id, 0) + 1
            mch.write(l.multichat_id)
            l.multichat_index = mc_ids.index(l.multichat_id) + seen[l.multichat_id] - 1
        for mi, mcid in enumerate(mc_ids):
            mch.write(mcid)
            for l in llms:
                if l.multichat_id == mcid and l.multichat_index < 0:
                    l.multichat_index = mi
        return Model(id=h.finish_id(), multichat_id=mch.finish_id(),
                     training_table_id=tth.finish_id() if tth is not None else None, llms=llms, weight=mb.weight)


class Model:
    """A validated score model (reference Model, model/mod.rs:202-211)."""

    def __init__(self, id: str, multichat_id: str, training_table_id: Optional[str], llms: List[Llm], weight):
        self.id, self.multichat_id, self.training_table_id = id, multichat_id, training_table_id
        self.llms, self.weight = llms, weight

    @property
    def weight_type(self) -> str:
        return "static" if isinstance(self.weight, ModelWeightStatic) else "training_table"

    def to_obj(self) -> dict:
        o = {"id": self.id, "multichat_id": self.multichat_id}
        if self.training_table_id is not None:
            o["training_table_id"] = self.training_table_id
        o["llms"] = [l.to_obj() for l in self.llms]
        o["weight"] = self.weight.to_obj()
        return o

    def to_json(self) -> str:
        return sjson.dumps(self.to_obj())

    @classmethod
    def from_obj(cls, o: dict) -> "Model":
        w = o.get("weight") or {"type": "static"}
        weight = ModelWeightStatic.model_validate(w) if w.get("type") == "static" else \
            ModelWeightTrainingTable.model_validate(w)
        return cls(o["id"], o["multichat_id"], o.get("training_table_id"), [Llm.from_obj(x) for x in o["llms"]],
                   weight)
