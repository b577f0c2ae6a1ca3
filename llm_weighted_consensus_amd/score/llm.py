"""LLM voter configuration: canonicalisation, validation and content-addressed ids.

Contract: reference src/score/llm/mod.rs —
  * `LlmBase` fields and serde order (:7-73); `weight` and `output_mode` always serialise;
  * `prepare()` (:76-258) maps defaults to "unset" so equivalent configs hash identically;
  * `validate()` (:260-511) ranges and messages;
  * ids (:513-549): xxh3-128 (seed 0) of the compact serde JSON, base62, left-padded with '0' to 22;
    training-table id = id with weight reset to the default; multichat id additionally resets
    output_mode / synthetic_reasoning / top_logprobs.
The JSON text is produced by utils.json (ryu float formatting), see that module.
"""
from __future__ import annotations

import copy
from typing import Dict, List, Literal, Optional, Union

import xxhash
from pydantic import Field

from ..schema.base import Wire
from ..schema.chat import Message, ProviderPreferences, Reasoning, Stop, Verbosity
from ..utils import json as sjson

_B62 = "0123456789ABCDEFGHIJKLMNOPQRSTUVWXYZabcdefghijklmnopqrstuvwxyz"
I32_MAX = 2 ** 31 - 1


def base62(n: int) -> str:
    if n == 0:
        return "0"
    s = []
    while n:
        n, r = divmod(n, 62)
        s.append(_B62[r])
    return "".join(reversed(s))


def id_from_text(text: str) -> str:
    return base62(xxhash.xxh3_128_intdigest(text.encode("utf-8"), seed=0)).rjust(22, "0")


class Hasher:
    """Streaming xxh3-128 (seed 0) — `update` chunks == hashing their concatenation."""

    def __init__(self):
        self._h = xxhash.xxh3_128(seed=0)

    def write(self, s: str) -> None:
        self._h.update(s.encode("utf-8"))

    def finish_id(self) -> str:
        return base62(self._h.intdigest()).rjust(22, "0")


OutputMode = Literal["instruction", "json_schema", "tool_call"]
WeightType = Literal["static", "training_table"]


class WeightStatic(Wire):
    type: Literal["static"] = "static"
    weight: float = 1.0

    def validate_weight(self) -> Optional[str]:
        if not (self.weight > 0.0):
            return f"`weight` must be a normal positive number: `weight`={_dec(self.weight)}"
        return None


class WeightTrainingTable(Wire):
    type: Literal["training_table"] = "training_table"
    base_weight: float
    min_weight: float
    max_weight: float

    def validate_weight(self) -> Optional[str]:
        b, lo, hi = self.base_weight, self.min_weight, self.max_weight
        if b < lo or b > hi or lo > hi or b <= 0 or lo <= 0 or hi <= 0:
            return ("LLM must have normal positive base, min, and max weights for training table weights mode: "
                    f"`base_weight={_dec(b)}`, `min_weight={_dec(lo)}`, `max_weight={_dec(hi)}`")
        return None


def _dec(x: float) -> str:
    """rust_decimal Display of a value parsed from f64 (plain decimal, no exponent)."""
    s = format(x, "f") if abs(x) >= 1e-6 else repr(x)
    if "." in s:
        s = s.rstrip("0").rstrip(".")
    return s


LlmWeight = Union[WeightStatic, WeightTrainingTable]


def weight_type(w) -> WeightType:
    return "static" if isinstance(w, WeightStatic) else "training_table"


class LlmBase(Wire):
    model: str
    weight: LlmWeight = Field(default_factory=WeightStatic, union_mode="left_to_right")
    output_mode: OutputMode = "instruction"
    synthetic_reasoning: Optional[bool] = None
    top_logprobs: Optional[int] = None
    prefix_messages: Optional[List[Message]] = None
    suffix_messages: Optional[List[Message]] = None
    frequency_penalty: Optional[float] = None
    logit_bias: Optional[Dict[str, int]] = None
    max_completion_tokens: Optional[int] = None
    presence_penalty: Optional[float] = None
    stop: Optional[Stop] = None
    temperature: Optional[float] = None
    top_p: Optional[float] = None
    max_tokens: Optional[int] = None
    min_p: Optional[float] = None
    provider: Optional[ProviderPreferences] = None
    reasoning: Optional[Reasoning] = None
    repetition_penalty: Optional[float] = None
    top_a: Optional[float] = None
    top_k: Optional[int] = None
    verbosity: Optional[Verbosity] = None
    models: Optional[List[str]] = None

    # ------------------------------------------------------------------ prepare (canonicalise)
    def prepare(self) -> None:
        def f64(name, default):
            if getattr(self, name) is not None and getattr(self, name) == default:
                setattr(self, name, None)

        if self.synthetic_reasoning is False:
            self.synthetic_reasoning = None
        if self.top_logprobs == 0:
            self.top_logprobs = None
        if self.prefix_messages is not None and len(self.prefix_messages) == 0:
            self.prefix_messages = None
        if self.suffix_messages is not None and len(self.suffix_messages) == 0:
            self.suffix_messages = None
        f64("frequency_penalty", 0.0)
        if self.logit_bias is not None and len(self.logit_bias) == 0:
            self.logit_bias = None
        f64("max_completion_tokens", 0)
        f64("presence_penalty", 0.0)
        if isinstance(self.stop, list):
            if len(self.stop) == 0:
                self.stop = None
            elif len(self.stop) == 1:
                self.stop = self.stop[0]
            else:
                self.stop = sorted(self.stop)
        f64("temperature", 1.0)
        f64("top_p", 1.0)
        f64("max_tokens", 0)
        f64("min_p", 0.0)
        self.provider = prepare_provider(self.provider)
        r = self.reasoning
        if r is not None:
            if r.max_tokens == 0:
                r.max_tokens = None
            if r.enabled is True and (r.effort is not None or r.max_tokens is not None):
                r.enabled = None
            elif r.enabled is False and r.effort is None and r.max_tokens is None:
                r.enabled = None
            if r.max_tokens is None and r.enabled is None and r.effort is None:
                self.reasoning = None
        f64("repetition_penalty", 1.0)
        f64("top_a", 0.0)
        f64("top_k", 0)
        if self.verbosity == "medium":
            self.verbosity = None
        if self.models is not None and len(self.models) == 0:
            self.models = None

    # ------------------------------------------------------------------ validate
    def validate_llm(self, expect: WeightType) -> None:
        """Raises ValueError with the reference's messages."""
        def f64(v, name, lo, hi):
            if v is not None:
                if v != v or v in (float("inf"), float("-inf")):
                    raise ValueError(f"`{name}` must be a finite number: `{name}`={v}")
                if v < lo or v > hi:
                    raise ValueError(f"`{name}` must be between {_num(lo)} and {_num(hi)}: `{name}`={_num(v)}")

        def u64(v, name, lo, hi):
            if v is not None and (v < lo or v > hi):
                raise ValueError(f"`{name}` must be between {lo} and {hi}: `{name}`={v}")

        def strings(vals, name):
            if vals is not None:
                seen = set()
                for s in vals:
                    if s == "":
                        raise ValueError(f"`{name}` cannot contain empty strings")
                    if s in seen:
                        raise ValueError(f"`{name}` cannot contain duplicate strings: `{s}`")
                    seen.add(s)

        if self.model == "":
            raise ValueError("`model` cannot be empty")
        wt = weight_type(self.weight)
        if wt != expect:
            raise ValueError(f"expected weight of type `{expect}`, found `{wt}`")
        err = self.weight.validate_weight()
        if err:
            raise ValueError(err)
        if self.synthetic_reasoning and self.output_mode == "instruction":
            raise ValueError("`synthetic_reasoning` cannot be true when `output_mode` is `instruction`")
        if self.top_logprobs is not None and self.top_logprobs > 20:
            raise ValueError(f"`top_logprobs` must be between 0 and 20: `top_logprobs`={self.top_logprobs}")
        f64(self.frequency_penalty, "frequency_penalty", -2.0, 2.0)
        if self.logit_bias is not None:
            for tok, w in self.logit_bias.items():
                if tok == "":
                    raise ValueError("`logit_bias` keys cannot be empty")
                if not tok.isascii() or not tok.isdigit():
                    raise ValueError(f"`logit_bias` keys must be numeric: `logit_bias`={tok}")
                if tok[0] == "0" and len(tok) > 1:
                    raise ValueError(f"`logit_bias` keys cannot have leading zeroes: `logit_bias`={tok}")
                if w > 100 or w < -100:
                    raise ValueError(f"`logit_bias` values must be between -100 and 100: `logit_bias[{tok}]`={w}")
        u64(self.max_completion_tokens, "max_completion_tokens", 0, I32_MAX)
        f64(self.presence_penalty, "presence_penalty", -2.0, 2.0)
        if isinstance(self.stop, list):
            strings(self.stop, "stop")
        elif isinstance(self.stop, str) and self.stop == "":
            raise ValueError("`stop` cannot be an empty string")
        f64(self.temperature, "temperature", 0.0, 2.0)
        f64(self.top_p, "top_p", 0.0, 1.0)
        u64(self.max_tokens, "max_tokens", 0, I32_MAX)
        f64(self.min_p, "min_p", 0.0, 1.0)
        validate_provider(self.provider)
        r = self.reasoning
        if r is not None:
            if r.max_tokens is not None and r.max_tokens > I32_MAX:
                raise ValueError(f"`reasoning.max_tokens` must be at most {I32_MAX}: "
                                 f"`reasoning.max_tokens`={r.max_tokens}")
            if r.effort is not None and r.max_tokens is not None:
                raise ValueError("`reasoning.max_tokens` and `reasoning.effort` cannot be set at the same time")
            if r.enabled is False and r.max_tokens is not None and r.effort is None:
                raise ValueError("`reasoning.enabled` cannot be false when `reasoning.max_tokens` is set")
            if r.enabled is False and r.max_tokens is None and r.effort is not None:
                raise ValueError("`reasoning.enabled` cannot be false when `reasoning.effort` is set")
        f64(self.repetition_penalty, "repetition_penalty", 0.0, 2.0)
        f64(self.top_a, "top_a", 0.0, 1.0)
        u64(self.top_k, "top_k", 0, I32_MAX)
        if self.models is not None:
            seen = set()
            for m in self.models:
                if m == "":
                    raise ValueError("models cannot contain empty strings")
                if m == self.model or m in seen:
                    raise ValueError(f"models cannot contain duplicate strings: `models`={m}")
                seen.add(m)

    # ------------------------------------------------------------------ ids
    def id_text(self) -> str:
        return sjson.dumps(self.to_obj())

    def id_string(self) -> str:
        return id_from_text(self.id_text())

    def training_table_id_string(self) -> Optional[str]:
        if weight_type(self.weight) != "training_table":
            return None
        c = self.model_copy(deep=True)
        c.weight = WeightStatic()
        return c.id_string()

    def multichat_id_string(self) -> str:
        c = self.model_copy(deep=True)
        c.weight = WeightStatic()
        c.output_mode = "instruction"
        c.synthetic_reasoning = None
        c.top_logprobs = None
        return c.id_string()


def _num(v) -> str:
    """Rust Display for f64 (no trailing `.0` for integral values)."""
    if isinstance(v, float) and v.is_integer():
        return str(int(v))
    return repr(v) if isinstance(v, float) else str(v)


def prepare_provider(p: Optional[ProviderPreferences]) -> Optional[ProviderPreferences]:
    if p is None:
        return None
    if p.is_empty():
        return None
    if p.order is not None and len(p.order) == 0:
        p.order = None
    if p.allow_fallbacks is True:
        p.allow_fallbacks = None
    if p.require_parameters is False:
        p.require_parameters = None
    if p.data_collection == "allow":
        p.data_collection = None
    for f in ("only", "ignore", "quantizations"):
        v = getattr(p, f)
        if v is not None:
            v = sorted(v)
            setattr(p, f, v if v else None)
    return None if p.is_empty() else p


def validate_provider(p: Optional[ProviderPreferences]) -> None:
    if p is None:
        return
    for f in ("order", "only", "ignore", "quantizations"):
        vals = getattr(p, f)
        if vals is not None:
            seen = set()
            for s in vals:
                if s == "":
                    raise ValueError(f"`provider.{f}` cannot contain empty strings")
                if s in seen:
                    raise ValueError(f"`provider.{f}` cannot contain duplicate strings: `{s}`")
                seen.add(s)
    if p.sort is not None and p.sort == "":
        raise ValueError("`provider.sort` cannot be empty")


class Llm:
    """A validated voter inside a score model (reference Llm, llm/mod.rs:720-745)."""

    __slots__ = ("base", "id", "index", "multichat_id", "multichat_index", "training_table_id",
                 "training_table_index")

    def __init__(self, base: LlmBase, id: str, index: int, multichat_id: str, multichat_index: int,
                 training_table_id: Optional[str], training_table_index: Optional[int]):
        self.base, self.id, self.index = base, id, index
        self.multichat_id, self.multichat_index = multichat_id, multichat_index
        self.training_table_id, self.training_table_index = training_table_id, training_table_index

    def to_obj(self) -> dict:
        o = {"id": self.id, "index": self.index, "multichat_id": self.multichat_id,
             "multichat_index": self.multichat_index}
        if self.training_table_id is not None:
            o["training_table_id"] = self.training_table_id
        if self.training_table_index is not None:
            o["training_table_index"] = self.training_table_index
        o.update(self.base.to_obj())
        return o

    @classmethod
    def from_obj(cls, o: dict) -> "Llm":
        base = LlmBase.model_validate(o)
        return cls(base, o["id"], o["index"], o["multichat_id"], o["multichat_index"], o.get("training_table_id"),
                   o.get("training_table_index"))
