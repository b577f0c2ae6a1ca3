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
import typing
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


def _list_kind(ann) -> str:
    """'scalars' for a (optional) list of str/int/float/bool (token byte lists), 'wires' for a list of one
    Wire class, '' otherwise."""
    args = [a for a in typing.get_args(ann) if a is not type(None)] if typing.get_origin(ann) is typing.Union else [ann]
    if len(args) != 1 or typing.get_origin(args[0]) not in (list, typing.List):
        return ""
    el = typing.get_args(args[0])
    if len(el) != 1:
        return ""
    if el[0] in (str, int, float, bool):
        return "scalars"
    return "wires" if isinstance(el[0], type) and issubclass(el[0], Wire) else ""


_SCALARS = frozenset(_IMMUTABLE)
_GEN: dict = {}


def _compile_to_obj(cls):
    """Straight-line ``to_obj`` for one class, generated from its field plan: no loop over the plan and
    no per-field flag tests at run time (the serving front end turns ~800 objects into dicts per scored
    response).  Scalars are recognised by exact class; anything else (str enums included) goes through
    the generic :func:`to_obj`, which returns scalars unchanged."""
    src = ["def _to_obj(self):", " d = self.__dict__", " out = {}"]
    fields = cls.model_fields
    for name, key, keep, flat in _plan(cls):
        src += [f" v = d[{name!r}]",
                " if v is None:" + (f" out[{key!r}] = None" if keep else " pass"),
                f" elif v.__class__ in _SCALARS: out[{key!r}] = v",
                " elif isinstance(v, Wire): " + ("out.update(v.to_obj())" if flat else f"out[{key!r}] = v.to_obj()")]
        kind = _list_kind(fields[name].annotation)
        if kind == "scalars":  # still checked per element: a list field may be assigned anything
            src.append(f" elif v.__class__ is list: out[{key!r}] = [x if x.__class__ in _SCALARS else _any(x) for x in v]")
        elif kind == "wires":
            src.append(f" elif v.__class__ is list: out[{key!r}] = [x.to_obj() if isinstance(x, Wire) else _any(x) for x in v]")
        src.append(f" else: out[{key!r}] = _any(v)")
    src += [" extra = self.__pydantic_extra__",
            " if extra: out.update({k: _any(x) for k, x in extra.items()})",
            " return out"]
    ns = {"_SCALARS": _SCALARS, "Wire": Wire, "_any": to_obj}
    exec("\n".join(src), ns)  # noqa: S102 - source built above from the class's own field names
    f = ns["_to_obj"]
    f.__qualname__ = f"{cls.__qualname__}.to_obj"
    f._lwc_generated = True
    return f


class Wire(BaseModel):
    model_config = ConfigDict(extra="ignore", populate_by_name=True, validate_assignment=False,
                              protected_namespaces=())
    __keep_none__: ClassVar[FrozenSet[str]] = frozenset()
    __flatten__: ClassVar[FrozenSet[str]] = frozenset()

    @classmethod
    def __pydantic_init_subclass__(cls, **kw):
        super().__pydantic_init_subclass__(**kw)
        # classes that do not override to_obj get their generated one as the method itself; overrides
        # reach it through super().to_obj() -> Wire.to_obj
        # (compiled on first use: the field annotations of classes with forward references resolve later)
        cur = cls.to_obj
        if cur is Wire.to_obj or getattr(cur, "_lwc_generated", False):
            def first_use(self, cls=cls):
                f = _GEN.get(cls)
                if f is None:
                    f = _GEN[cls] = _compile_to_obj(cls)
                cls.to_obj = f
                return f(self)
            first_use._lwc_generated = True
            cls.to_obj = first_use

    def to_obj(self) -> dict:
        cls = type(self)
        f = _GEN.get(cls)
        if f is None:
            f = _GEN[cls] = _compile_to_obj(cls)
        return f(self)

    def to_json(self) -> str:
        return sjson.dumps(self)

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

    @classmethod
    def trusted(cls, **fields):
        """An instance from values the caller guarantees are already valid and complete (every field given,
        engine-produced token data): no validation pass — the per-token logprob objects of the local chat
        client are the serving front end's most numerous allocation."""
        new = cls.__new__(cls)
        _set = object.__setattr__
        _set(new, "__dict__", fields)
        _set(new, "__pydantic_fields_set__", set(fields))
        _set(new, "__pydantic_extra__", None)
        _set(new, "__pydantic_private__", None)
        return new


def _native_plan(cls):
    """The native JSON encoder's view of a type (csrc/runtime/json_encode.cpp): a Wire class whose to_obj
    is the generated field walk -> ((name, key, keep_none), ...); one with its own to_obj or flattened
    fields -> None (the encoder writes its to_obj()); anything else -> False."""
    if not (isinstance(cls, type) and issubclass(cls, Wire)):
        return False
    cur = cls.to_obj
    if not (cur is Wire.to_obj or getattr(cur, "_lwc_generated", False)) or cls.__flatten__:
        return None
    return tuple((name, key, bool(keep)) for name, key, keep, _flat in _plan(cls))


sjson.PLAN_OF = _native_plan


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
