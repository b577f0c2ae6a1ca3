"""serde_json-compatible JSON text.

The reference serialises with serde_json (`preserve_order`, compact by default, `to_string_pretty` for
the choice map shown to voters: src/score/completions/client.rs:1580-1603) and formats f64 with ryu
(rust_decimal `serde-float` goes through f64 too, Cargo.toml:28).  Python's json differs only in float
text (``1e-07`` vs ``1e-7``, ``1e+16`` vs ``1e16``, ``1e-05`` vs ``0.00001``) — which matters because
model ids are hashes of the JSON text (src/score/llm/mod.rs:513-522).  String escaping of
``json.dumps(ensure_ascii=False)`` already equals serde_json's (``\\"``, ``\\\\``, ``\\b\\f\\n\\r\\t``,
other C0 controls as lowercase ``\\u00xx``).
"""
from __future__ import annotations

import json as _json
import math
import re
from typing import Any

_enc_str = _json.encoder.py_encode_basestring  # ensure_ascii=False escaping (== serde_json)
try:  # the C accelerator has identical output
    from _json import encode_basestring as _enc_str  # type: ignore  # noqa: F811
except Exception:  # pragma: no cover
    pass


def ryu_f64(x: float) -> str:
    """Format an f64 exactly like serde_json/ryu (shortest round-trip digits, ryu layout)."""
    if math.isnan(x) or math.isinf(x):
        return "null"  # serde_json writes non-finite floats as null
    if x == 0.0:
        return "-0.0" if math.copysign(1.0, x) < 0 else "0.0"
    r = repr(x)
    sign = ""
    if r[0] == "-":
        sign, r = "-", r[1:]
    if "e" in r:
        mant, e = r.split("e")
        e = int(e)
    else:
        mant, e = r, 0
    if "." in mant:
        ip, fp = mant.split(".")
    else:
        ip, fp = mant, ""
    if fp == "0":
        fp = ""
    digits = (ip + fp).lstrip("0")
    k = e - len(fp)  # value = int(ip+fp) * 10^k
    # strip trailing zeros into the exponent (shortest digits)
    stripped = digits.rstrip("0")
    k += len(digits) - len(stripped)
    d = stripped or "0"
    length = len(d)
    kk = length + k
    if 0 <= k and kk <= 16:
        s = d + "0" * k + ".0"
    elif 0 < kk <= 16:
        s = d[:kk] + "." + d[kk:]
    elif -5 < kk <= 0:
        s = "0." + "0" * (-kk) + d
    elif length == 1:
        s = d + "e" + str(kk - 1)
    else:
        s = d[0] + "." + d[1:] + "e" + str(kk - 1)
    return sign + s


def _enc(v: Any, out: list) -> None:
    if v is None:
        out.append("null")
    elif v is True:
        out.append("true")
    elif v is False:
        out.append("false")
    elif isinstance(v, str):
        out.append(_enc_str(v))
    elif isinstance(v, int):
        out.append(str(v))
    elif isinstance(v, float):
        out.append(ryu_f64(v))
    elif isinstance(v, dict):
        out.append("{")
        first = True
        for k, x in v.items():
            if not first:
                out.append(",")
            first = False
            out.append(_enc_str(str(k)))
            out.append(":")
            _enc(x, out)
        out.append("}")
    elif isinstance(v, (list, tuple)):
        out.append("[")
        for i, x in enumerate(v):
            if i:
                out.append(",")
            _enc(x, out)
        out.append("]")
    elif hasattr(v, "to_obj"):
        _enc(v.to_obj(), out)
    else:
        raise TypeError(f"not JSON serialisable: {type(v)!r}")


_C_DUMPS = _json.JSONEncoder(ensure_ascii=False, separators=(",", ":"), allow_nan=True).encode
# a number in exponent form or a non-finite float: the only places Python's float repr and ryu differ
# (as a whole value: after ':' ',' '[' and before ',' ']' '}'; a string that contains such text only costs
# the exact path)
_NEEDS_RYU = re.compile(r"[:,\[]-?(?:\d+(?:\.\d+)?e[-+]?\d+|NaN|Infinity)[,\]}]")


def _plain(v: Any) -> Any:
    return v.to_obj() if hasattr(v, "to_obj") else v


# a JSON string literal (skipped as a whole) or a number in exponent form / a non-finite float
_FIX_FLOATS = re.compile(r'"(?:[^"\\]|\\.)*"|(-?\d+(?:\.\d+)?e[-+]?\d+|NaN|-?Infinity)')


def _fix_float(m: "re.Match") -> str:
    t = m.group(1)
    if t is None:
        return m.group(0)  # a string literal, unchanged
    if t in ("NaN", "Infinity", "-Infinity"):
        return "null"
    return ryu_f64(float(t))


try:  # the native encoder (csrc/runtime/json_encode.cpp): one C++ walk, ryu floats, no rewrite pass
    from .._runtime import json_dumps as _native_dumps  # type: ignore
except Exception:  # pragma: no cover - runtime not built
    _native_dumps = None
# schema/base.py installs the wire types' field plans here: the native encoder then writes Wire objects
# straight from their fields (no to_obj dict tree)
PLAN_OF = None


def _maybe_exp(s: str) -> bool:
    """Whether ``s`` may hold a number in exponent form: some "e-" / "e+" between two digits (str.find runs
    in C; ids such as "fake-..." contain "e-" without digits around it)."""
    for pat in ("e-", "e+"):
        i = s.find(pat)
        while i != -1:
            if 0 < i and s[i - 1].isdigit() and i + 2 < len(s) and s[i + 2].isdigit():
                return True
            i = s.find(pat, i + 2)
    return False


def dumps(v: Any) -> str:
    """Compact serde_json text (serde_json::to_string).  The native encoder (C++, _runtime) writes it
    directly.  Without it: Python's C encoder, whose output equals serde_json's except for floats in exponent
    form (Python ``1e-05``, ryu ``1e-5``) and non-finite floats (serde_json: null); those are rewritten in one
    C-regex pass that skips string literals.  Values neither C encoder takes use the exact Python encoder."""
    if _native_dumps is not None and (PLAN_OF is not None or isinstance(v, (dict, list))):
        try:
            return _native_dumps(v, PLAN_OF)
        except (TypeError, ValueError, UnicodeError):
            pass
    s = None
    p = _plain(v)
    if isinstance(p, (dict, list)):  # (a bare scalar: the exact encoder)
        try:
            s = _C_DUMPS(p)
        except (TypeError, ValueError):
            s = None
    if s is not None:
        if not _maybe_exp(s) and "NaN" not in s and "Infinity" not in s:
            return s  # (Python writes every exponent with a sign): nothing anywhere to rewrite
        return _FIX_FLOATS.sub(_fix_float, s) if _NEEDS_RYU.search(s) else s
    out: list = []
    _enc(v, out)
    return "".join(out)


def _enc_pretty(v: Any, out: list, ind: int) -> None:
    if isinstance(v, dict):
        if not v:
            out.append("{}")
            return
        out.append("{\n")
        items = list(v.items())
        for i, (k, x) in enumerate(items):
            out.append("  " * (ind + 1))
            out.append(_enc_str(str(k)))
            out.append(": ")
            _enc_pretty(x, out, ind + 1)
            out.append(",\n" if i + 1 < len(items) else "\n")
        out.append("  " * ind + "}")
    elif isinstance(v, (list, tuple)):
        if not v:
            out.append("[]")
            return
        out.append("[\n")
        for i, x in enumerate(v):
            out.append("  " * (ind + 1))
            _enc_pretty(x, out, ind + 1)
            out.append(",\n" if i + 1 < len(v) else "\n")
        out.append("  " * ind + "]")
    elif hasattr(v, "to_obj"):
        _enc_pretty(v.to_obj(), out, ind)
    else:
        _enc(v, out)


def dumps_pretty(v: Any) -> str:
    """serde_json::to_string_pretty (two-space indent, ": " separators)."""
    out: list = []
    _enc_pretty(v, out, 0)
    return "".join(out)


def loads(s: str) -> Any:
    return _json.loads(s)
