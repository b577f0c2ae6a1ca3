"""The serde-compatible JSON text: the native (C++) encoder and the C-encoder fallback of ``utils.json.dumps`` equal the exact
(pure-Python, ryu float) encoder on arbitrary nested values, including floats whose Python repr uses an
exponent, non-finite floats and strings that merely look like numbers; Wire clone / to_obj keep the
wire shape and never alias the source."""
import math

from hypothesis import given, settings
from hypothesis import strategies as st

from llm_weighted_consensus_amd.schema import chat as C
from llm_weighted_consensus_amd.utils import json as J


def _exact(v):
    out: list = []
    J._enc(v, out)
    return "".join(out)


scalars = st.one_of(st.none(), st.booleans(), st.integers(-10**20, 10**20),
                    st.floats(allow_nan=True, allow_infinity=True),
                    st.sampled_from([1e-5, -1.5e-9, 1e16, 1e300, 0.0001, -0.0, 390e4, 1e-7]),
                    st.text(max_size=12), st.sampled_from(["390e4fe4", ",1e5,", "NaN", "x\u0001\"y", "é"]))
values = st.recursive(scalars, lambda ch: st.one_of(st.lists(ch, max_size=5),
                                                    st.dictionaries(st.text(max_size=6), ch, max_size=5)),
                      max_leaves=25)


@settings(max_examples=400, deadline=None)
@given(values)
def test_fast_path_equals_exact_encoder(v):
    assert J.dumps(v) == _exact(v)


def test_exponent_floats_take_the_exact_path():
    assert J.dumps({"a": [1e-5, 1e16, math.inf]}) == '{"a":[0.00001,1e16,null]}'
    assert J.dumps({"id": "chatcmpl-390e4fe4", "x": 0.5}) == '{"id":"chatcmpl-390e4fe4","x":0.5}'


def test_clone_is_deep_and_keeps_fields_set():
    lp = C.Logprobs(content=[C.Logprob(token="a", bytes=[97], logprob=-0.1,
                                       top_logprobs=[C.TopLogprob(token="b", bytes=[98], logprob=-1.0)])])
    ch = C.StreamChoice(delta=C.Delta(content="hi"), index=0, logprobs=lp)
    cl = ch.clone()
    assert cl.to_obj() == ch.to_obj() and cl.model_fields_set == ch.model_fields_set
    cl.logprobs.content[0].top_logprobs[0].logprob = 3.0
    cl.logprobs.content.append(cl.logprobs.content[0])
    cl.delta.content += "!"
    assert ch.logprobs.content[0].top_logprobs[0].logprob == -1.0 and len(ch.logprobs.content) == 1
    assert ch.delta.content == "hi"


def test_merge_extends_logprobs_in_place_without_aliasing_the_source():
    a = C.StreamChoice(delta=C.Delta(content="a"), index=0,
                       logprobs=C.Logprobs(content=[C.Logprob(token="a", bytes=[97], logprob=-0.1, top_logprobs=[])]))
    b = C.StreamChoice(delta=C.Delta(content="b"), index=0,
                       logprobs=C.Logprobs(content=[C.Logprob(token="b", bytes=[98], logprob=-0.2, top_logprobs=[])]))
    agg = a.clone()
    agg.push(b)
    agg.push(b.clone())
    assert agg.delta.content == "abb" and [x.token for x in agg.logprobs.content] == ["a", "b", "b"]
    assert [x.token for x in a.logprobs.content] == ["a"] and [x.token for x in b.logprobs.content] == ["b"]


def _loop_to_obj(v):
    """The plain field-plan walk the generated per-class to_obj replaces (same output required)."""
    from llm_weighted_consensus_amd.schema.base import _IMMUTABLE, Wire, _plan
    if isinstance(v, Wire):
        out = {}
        for name, key, keep, flat in _plan(type(v)):
            x = v.__dict__[name]
            if x is None:
                if keep:
                    out[key] = None
            elif isinstance(x, Wire) and flat:
                out.update(_loop_to_obj(x))
            else:
                out[key] = x if isinstance(x, _IMMUTABLE) else _loop_to_obj(x)
        return out
    if isinstance(v, (list, tuple)):
        return [_loop_to_obj(x) for x in v]
    if isinstance(v, dict):
        return {k: _loop_to_obj(x) for k, x in v.items()}
    return v


def test_generated_to_obj_matches_the_field_walk():
    from llm_weighted_consensus_amd.schema import score as S
    from llm_weighted_consensus_amd.schema.base import Wire
    lp = C.Logprobs(content=[C.Logprob(token="a", bytes=[97], logprob=-0.1,
                                       top_logprobs=[C.TopLogprob(token="b", bytes=None, logprob=-1.0)])])
    chunk = C.ChatCompletionChunk(id="x", created=1, model="m", choices=[
        C.StreamChoice(delta=C.Delta(content="hi", role="assistant"), index=0, logprobs=lp, finish_reason="stop")])
    assert chunk.to_obj() == _loop_to_obj(chunk)
    sc = S.ScoreStreamChoice(delta=S.ScoreDelta(content="k"), index=2, weight=1.5, model="v", model_index=0)
    got = sc.to_obj()
    assert got["finish_reason"] is None and "error" not in got  # keep-none and the override still apply
    # a list field assigned a tuple after validation, and a subclass with its own extra field
    lp.content[0].bytes = (97,)
    assert lp.to_obj()["content"][0]["bytes"] == [97]

    class Extended(C.Delta):
        extra_note: str = "n"
    assert Extended(content="c").to_obj() == dict(_loop_to_obj(Extended(content="c")), extra_note="n")
    assert isinstance(Extended(content="c"), Wire) and "extra_note" not in C.Delta(content="c").to_obj()


def test_native_float_text_equals_ryu_layout():
    """csrc/runtime/json_encode.cpp formats f64 with std::to_chars' shortest digits in ryu's layout: the
    same text as the Python ryu_f64 on random bit patterns, the layout's boundaries and the specials."""
    import random
    import struct

    from llm_weighted_consensus_amd import _runtime as RT

    rng = random.Random(7)
    xs = [struct.unpack("<d", struct.pack("<Q", rng.getrandbits(64)))[0] for _ in range(20000)]
    xs += [rng.uniform(-1, 1) * 10.0 ** rng.randint(-30, 30) for _ in range(20000)]
    xs += [1e-5, 1e-4, 9.999e-5, 1e15, 1e16, 1e17, 123456789012345680.0, 0.1, 5e-324, 1.7976931348623157e308,
           -0.0, 0.0, 1.0, 100.0, 0.3, 2.5e-7, math.inf, -math.inf, math.nan]
    for x in xs:
        assert RT.json_f64(x) == J.ryu_f64(x), repr(x)


@settings(max_examples=300, deadline=None)
@given(values)
def test_python_fallback_equals_exact_encoder(v):
    """Without the native encoder: the C json encoder + exponent rewrite path."""
    native, J._native_dumps = J._native_dumps, None
    try:
        assert J.dumps(v) == _exact(v)
    finally:
        J._native_dumps = native


def test_native_encoder_refuses_unknown_types_and_falls_back():
    class Obj:
        def to_obj(self):
            return {"k": [1, 2.5e-7]}

    assert J.dumps({"a": Obj()}) == '{"a":{"k":[1,2.5e-7]}}'
    assert J.dumps({"s": "\u0000\u001f\u007f é \"q\" \\ \t"}) == _exact({"s": "\u0000\u001f\u007f é \"q\" \\ \t"})
    assert J.dumps([10 ** 30, -10 ** 30, True, None]) == "[1000000000000000000000000000000,-1000000000000000000000000000000,true,null]"


def test_native_wire_walk_equals_to_obj_text():
    """The native encoder writes Wire objects from their field plans (no to_obj dict tree): the text equals
    dumps(to_obj()) for generated-plan classes, classes with their own to_obj (score choices), instances
    carrying extra fields, aliases and kept Nones."""
    from llm_weighted_consensus_amd.schema import score as S

    lp = C.Logprobs(content=[C.Logprob(token="a\\n", bytes=[97, 10], logprob=-1e-7,
                                       top_logprobs=[C.TopLogprob(token="b", bytes=None, logprob=-1.5e-5)])])
    chunk = C.ChatCompletionChunk(id="x", created=1, model="m", choices=[
        C.StreamChoice(delta=C.Delta(content="hi", role="assistant"), index=0, logprobs=lp, finish_reason="stop")])
    sc = S.ScoreStreamChoice(delta=S.ScoreDelta(content="k"), index=2, weight=1.5, model="v", model_index=0)
    extra = C.Delta.model_validate({"content": "c"})
    object.__setattr__(extra, "__pydantic_extra__", {"note": 1e-9})
    for obj in (chunk, sc, lp, extra, [chunk, {"k": sc}]):
        want = J.dumps(_obj(obj))
        assert J.dumps(obj) == want == _exact(_obj(obj))


def _obj(v):
    from llm_weighted_consensus_amd.schema.base import to_obj
    return to_obj(v)
