"""The serde-compatible JSON text: the C-encoder fast path of ``utils.json.dumps`` equals the exact
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
