"""Wire-type base: pydantic v2 models that serialise like the reference's serde derives.

* Field order = declaration order (serde derive order; serde_json `preserve_order`).
* ``Optional`` fields are omitted when ``None`` (serde ``skip_serializing_if = "Option::is_none"``)
  unless listed in ``__keep_none__`` (plain ``Option`` fields without the attribute serialise ``null``).
* Internally tagged enums (``#[serde(tag = "role")]`` / ``tag = "type"``) are modelled as a ``Literal``
  tag declared FIRST, which is where serde emits the tag.
* Unknown input fields are ignored (serde default), untagged unions try variants left to right.
"""
from __future__ import annotations

import copy
from typing import Any, ClassVar, FrozenSet

from pydantic import BaseModel, ConfigDict

from ..utils import json as sjson


def to_obj(v: Any) -> Any:
    if isinstance(v, Wire):
        return v.to_obj()
    if isinstance(v, (list, tuple)):  # scalars inline (token byte lists): no call per element
        return [x if isinstance(x, _IMMUTABLE) else to_obj(x) for x in v]
    if isinstance(v, dict):
        return {k: x if isinstance(x, _IMMUTABLE) else to_obj(x) for k, x in v.items()}
    return v


_IMMUTABLE = (str, int, float, bool, bytes, type(None))


def _clone(v: Any) -> Any:
    if isinstance(v, _IMMUTABLE):
        return v
    if isinstance(v, Wire):
        return v.clone()
    if isinstance(v, list):
        return [_clone(x) for x in v]
    if isinstance(v, dict):
        return {k: _clone(x) for k, x in v.items()}
    if isinstance(v, tuple):
        return tuple(_clone(x) for x in v)
    return copy.deepcopy(v)


_PLANS: dict = {}


def _plan(cls) -> list:
    """Per class: (field name, wire key, keep None, flatten) in declaration order (cached)."""
    p = _PLANS.get(cls)
    if p is None:
        keep, flat = cls.__keep_none__, cls.__flatten__
        p = [(n, f.alias or n, n in keep, n in flat) for n, f in cls.model_fields.items()]
        _PLANS[cls] = p
    return p


class Wire(BaseModel):
    model_config = ConfigDict(extra="ignore", populate_by_name=True, validate_assignment=False,
                              protected_namespaces=())
    __keep_none__: ClassVar[FrozenSet[str]] = frozenset()
    __flatten__: ClassVar[FrozenSet[str]] = frozenset()

    def to_obj(self) -> dict:
        out: dict = {}
        d = self.__dict__
        for name, key, keep, flat in _plan(type(self)):
            v = d[name]
            if v is None:
                if keep:
                    out[key] = None
                continue
            if isinstance(v, _IMMUTABLE):
                out[key] = v
            elif isinstance(v, Wire):
                if flat:
                    out.update(v.to_obj())
                else:
                    out[key] = v.to_obj()
            else:
                out[key] = to_obj(v)
        extra = self.__pydantic_extra__
        if extra:
            out.update({k: to_obj(x) for k, x in extra.items()})
        return out

    def to_json(self) -> str:
        return sjson.dumps(self.to_obj())

    def clone(self):
        """Deep copy.  Field-wise construction without validation — pydantic's generic deep copy
        (``model_copy(deep=True)``: copy.deepcopy with its memo) was ~10 % of the serving front end's
        time, cloning every voter chunk as the score aggregate merges it."""
        cls = type(self)
        new = cls.__new__(cls)
        _set = object.__setattr__
        _set(new, "__dict__", {k: _clone(v) for k, v in self.__dict__.items()})
        _set(new, "__pydantic_fields_set__", set(self.__pydantic_fields_set__))
        extra = self.__pydantic_extra__
        _set(new, "__pydantic_extra__", None if extra is None else {k: _clone(v) for k, v in extra.items()})
        priv = self.__pydantic_private__
        _set(new, "__pydantic_private__", None if priv is None else copy.deepcopy(priv))
        return new

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
