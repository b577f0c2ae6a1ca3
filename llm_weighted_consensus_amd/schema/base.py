"""Wire-type base: pydantic v2 models that serialise like the reference's serde derives.

* Field order = declaration order (serde derive order; serde_json `preserve_order`).
* ``Optional`` fields are omitted when ``None`` (serde ``skip_serializing_if = "Option::is_none"``)
  unless listed in ``__keep_none__`` (plain ``Option`` fields without the attribute serialise ``null``).
* Internally tagged enums (``#[serde(tag = "role")]`` / ``tag = "type"``) are modelled as a ``Literal``
  tag declared FIRST, which is where serde emits the tag.
* Unknown input fields are ignored (serde default), untagged unions try variants left to right.
"""
from __future__ import annotations

from typing import Any, ClassVar, FrozenSet

from pydantic import BaseModel, ConfigDict

from ..utils import json as sjson


def to_obj(v: Any) -> Any:
    if isinstance(v, Wire):
        return v.to_obj()
    if isinstance(v, list):
        return [to_obj(x) for x in v]
    if isinstance(v, tuple):
        return [to_obj(x) for x in v]
    if isinstance(v, dict):
        return {k: to_obj(x) for k, x in v.items()}
    return v


class Wire(BaseModel):
    model_config = ConfigDict(extra="ignore", populate_by_name=True, validate_assignment=False,
                              protected_namespaces=())
    __keep_none__: ClassVar[FrozenSet[str]] = frozenset()
    __flatten__: ClassVar[FrozenSet[str]] = frozenset()

    def to_obj(self) -> dict:
        out: dict = {}
        keep = type(self).__keep_none__
        flat = type(self).__flatten__
        for name, field in type(self).model_fields.items():
            v = getattr(self, name)
            if v is None and name not in keep:
                continue
            if name in flat and isinstance(v, Wire):
                out.update(v.to_obj())
                continue
            out[field.alias or name] = to_obj(v)
        extra = getattr(self, "__pydantic_extra__", None)
        if extra:
            out.update({k: to_obj(x) for k, x in extra.items()})
        return out

    def to_json(self) -> str:
        return sjson.dumps(self.to_obj())

    def clone(self):
        return self.model_copy(deep=True)

    @classmethod
    def parse(cls, obj: Any):
        return cls.model_validate(obj)


# --- merge helpers (reference chat/completions/response.rs:812-872) -------------------------------

def push_opt_str(a, b):
    if b is None:
        return a
    return b if a is None else a + b


def push_opt_num(a, b):
    if b is None:
        return a
    return b if a is None else a + b


def push_opt_list(a, b):
    if b is None:
        return a
    return list(b) if a is None else a + list(b)


def first_some(a, b):
    return b if a is None else a
