"""Score orchestrator end-to-end on the FakeChatClient (CPU): every voter branch of the reference
(src/score/completions/client.rs:93-908), tally/confidence, error unification, archive references."""
import asyncio
import math

import pytest

from llm_weighted_consensus_amd.archive.store import CompletionsArchive
from llm_weighted_consensus_amd.chat.fake import Failure, FakeChatClient, Scripted, select_keys
from llm_weighted_consensus_amd.errors import ChatError, ScoreError
from llm_weighted_consensus_amd.schema import chat as C
from llm_weighted_consensus_amd.schema import score as S
from llm_weighted_consensus_amd.score.orchestrator import ScoreClient


def run(coro):
    return asyncio.run(coro)


def pick_paris(req):
    keys = select_keys(req)
    return next(k for k, v in keys if "Paris" in v), [k for k, v in keys if "Paris" not in v]


def policy(req):
    if req.model.startswith("fail"):
        code = int(req.model.split("-")[1])
        return Failure(ChatError.bad_status(code, {"code": code}))
    if req.model == "midfail":
        return Failure(ChatError.stream_timeout(), after_chunks=2)
    if req.model == "garbage":
        return [Scripted("no key at all")]
    good, bad = pick_paris(req)
    if req.model == "tool":
        return [Scripted('{"response_key":"%s"}' % good, tool_call=True)]
    if req.model == "json":
        assert isinstance(req.response_format, C.ResponseFormatJsonSchema)
        return [Scripted('{"response_key":"%s"}' % good)]
    if req.top_logprobs:
        lp = [("`", [("`", 0.0)]),
              (good[1], [(good[1], math.log(0.6)), (bad[0][1], math.log(0.3)), ("zz", math.log(0.1))]),
              ("`", [("`", 0.0)])]
        return [Scripted(good, logprobs=lp)]
    if req.model == "wrong":
        return [Scripted(f"clearly {bad[0]}")]
    return [Scripted(f"The answer is {good}.")]


def make_req(llms, choices=("Paris", "London", "Berlin"), stream=True, **kw):
    return S.ScoreCompletionCreateParams.model_validate(dict(
        messages=[{"role": "user", "content": "What is the capital of France?"}],
        model={"llms": llms}, choices=list(choices), stream=stream, **kw))


async def collect(client, req):
    out = []
    async for item in await client.create_streaming(None, req):
        out.append(item)
    return out


def test_weighted_tally_and_confidence():
    sc = ScoreClient(FakeChatClient(policy), rng_seed=3)
    req = make_req([{"model": "a", "weight": {"type": "static", "weight": 3}}, {"model": "wrong"},
                    {"model": "lp", "top_logprobs": 5}])
    items = run(collect(sc, req))
    final = items[-1]
    assert isinstance(final, S.ScoreCompletionChunk)
    by_idx = {c.index: c for c in final.choices}
    # voter a: one-hot Paris x3; wrong: one-hot on a non-Paris choice x1; lp: 0.6/0.9 Paris, 0.3/0.9 other
    w_paris = 3 + 0.6 / 0.9
    assert by_idx[0].weight == pytest.approx(w_paris)
    total = sum(by_idx[i].weight for i in range(3))
    assert total == pytest.approx(5.0)
    assert by_idx[0].confidence == pytest.approx(w_paris / 5.0)
    assert sum(by_idx[i].confidence for i in range(3)) == pytest.approx(1.0)
    # voter confidences = sum_i conf_i * vote_i; final chunk carries no deltas / finish reasons
    for c in final.choices:
        assert c.delta.content is None and c.delta.vote is None and c.finish_reason is None
    assert final.usage is not None and final.usage.prompt_tokens == 30 and final.usage.total_cost == pytest.approx(0.003)
    assert final.weight_data.type == "static"
    # first yielded item is the initial chunk of provided choices
    first = items[0]
    assert [c.index for c in first.choices] == [0, 1, 2] and all(c.finish_reason == "stop" for c in first.choices)


def test_unary_equals_stream_fold():
    sc = ScoreClient(FakeChatClient(policy), rng_seed=5)
    req = make_req([{"model": "a"}, {"model": "lp", "top_logprobs": 3}], stream=False)
    u = run(sc.create_unary(None, req))
    assert u.object == "chat.completion"
    assert len(u.choices) == 5
    votes = [c.message.vote for c in u.choices[3:]]
    assert all(v is not None and sum(v) == pytest.approx(1.0) for v in votes)
    # voter a: one-hot Paris; voter lp: 0.6/0.9 on Paris (top-logprob probabilities renormalised)
    assert u.choices[0].confidence == pytest.approx((1 + 0.6 / 0.9) / 2)
    obj = u.to_obj()
    assert obj["weight_data"] == {"type": "static"}
    assert "vote" in obj["choices"][0]["message"] and obj["choices"][0]["message"]["vote"] is None


def test_voter_errors_and_all_votes_failed_code_unification():
    sc = ScoreClient(FakeChatClient(policy), rng_seed=1)
    items = run(collect(sc, make_req([{"model": "fail-429"}, {"model": "fail-404"}])))
    assert isinstance(items[-1], ScoreError)
    assert items[-1].status() == 400 and items[-1].message()["error"]["kind"] == "all_votes_failed"
    items = run(collect(sc, make_req([{"model": "fail-429"}, {"model": "fail-503"}])))
    assert items[-1].status() == 500
    items = run(collect(sc, make_req([{"model": "fail-429"}, {"model": "fail-429"}])))
    assert items[-1].status() == 429
    # one healthy voter: no AllVotesFailed, the failed voter is an error choice
    items = run(collect(sc, make_req([{"model": "fail-429"}, {"model": "a"}])))
    assert not isinstance(items[-1], ScoreError)
    errs = [c for it in items[:-1] for c in it.choices if c.error is not None]
    assert errs and errs[0].finish_reason == "error" and errs[0].error.code == 429


def test_mid_stream_error_and_invalid_content():
    sc = ScoreClient(FakeChatClient(policy), rng_seed=2)
    items = run(collect(sc, make_req([{"model": "midfail"}, {"model": "garbage"}, {"model": "a"}])))
    agg = None
    for it in items[:-1]:
        if agg is None:
            agg = it.clone()
        else:
            agg.push(it)
    mid = [c for c in agg.choices if c.model_index is not None and c.error is not None]
    kinds = sorted(c.error.message["error"]["kind"] if "error" in c.error.message else "" for c in mid)
    assert "invalid_content" in str([c.error.message for c in mid])
    assert "stream_timeout" in str([c.error.message for c in mid])


def test_output_modes_json_schema_and_tool_call():
    fake = FakeChatClient(policy)
    sc = ScoreClient(fake, rng_seed=9)
    req = make_req([{"model": "json", "output_mode": "json_schema", "synthetic_reasoning": True},
                    {"model": "tool", "output_mode": "tool_call"}], stream=False)
    u = run(sc.create_unary(None, req))
    assert u.choices[0].confidence == pytest.approx(1.0)
    reqs = {r.model: r for r in fake.requests}
    js = reqs["json"].response_format.json_schema
    assert js.name == "response_key" and js.strict is True
    assert list(js.schema_["properties"]) == ["_think", "response_key"]
    tr = reqs["tool"]
    assert tr.tool_choice.function.name == "response_key" and tr.tools[-1].function.name == "response_key"
    # tool arguments became content and tool_calls finish became stop
    tool_choice = next(c for c in u.choices if c.model_index is not None and c.message.content
                       and "response_key" in c.message.content and c.finish_reason == "stop")
    assert tool_choice.message.tool_calls is None
    # the prompt: structured modes omit the key list instruction
    sysmsg = reqs["json"].messages[-1]
    assert sysmsg.role == "system" and "Output exactly one response key" not in sysmsg.content


def test_prompt_appends_to_trailing_system_message_and_prefix_suffix():
    fake = FakeChatClient(policy)
    sc = ScoreClient(fake, rng_seed=4)
    req = S.ScoreCompletionCreateParams.model_validate(dict(
        messages=[{"role": "user", "content": "Q?"}, {"role": "system", "content": "be brief"}],
        model={"llms": [{"model": "a", "prefix_messages": [{"role": "system", "content": "PFX"}],
                         "suffix_messages": [{"role": "user", "content": "SFX"}]}]},
        choices=["Paris", "Rome"], stream=False))
    run(sc.create_unary(None, req))
    msgs = fake.requests[0].messages
    assert msgs[0].content == "PFX" and msgs[-2].role == "user"
    # suffix ends with a user message -> a NEW trailing system message carries the selection prompt
    assert msgs[-1].role == "system" and msgs[-1].content.startswith("Select the response:\n\n{\n  \"`")
    req2 = S.ScoreCompletionCreateParams.model_validate(dict(
        messages=[{"role": "user", "content": "Q?"}, {"role": "system", "content": "be brief"}],
        model={"llms": [{"model": "a"}]}, choices=["Paris", "Rome"], stream=False))
    fake.requests.clear()
    run(sc.create_unary(None, req2))
    last = fake.requests[0].messages[-1]
    assert last.content.startswith("be brief\n\nSelect the response:")
    assert "Output exactly one response key including backticks, nothing else:\n- `" in last.content


def test_validation_errors():
    sc = ScoreClient(FakeChatClient(policy))
    with pytest.raises(ScoreError) as e:
        run(sc.create_streaming(None, make_req([{"model": "a"}], choices=["only"])))
    assert e.value.status() == 400 and e.value.message()["error"]["kind"] == "expected_two_or_more_choices"
    with pytest.raises(ScoreError) as e:
        run(sc.create_streaming(None, make_req([{"model": "a", "temperature": 3}])))
    assert e.value.status() == 400 and "temperature" in e.value.message()["error"]["error"]
    with pytest.raises(ScoreError) as e:
        run(sc.create_streaming(None, make_req([])))
    assert "at least 1 llm" in e.value.message()["error"]["error"]
    bad = S.ScoreCompletionCreateParams.model_validate(dict(messages=[], model="not json{", choices=["a", "b"]))
    with pytest.raises(ScoreError) as e:
        run(sc.create_streaming(None, bad))
    assert e.value.message()["error"] == {"kind": "invalid_model", "error": "not json{"}
    missing = S.ScoreCompletionCreateParams.model_validate(dict(messages=[], model="A" * 22, choices=["a", "b"]))
    with pytest.raises(ScoreError) as e:
        run(sc.create_streaming(None, missing))
    assert e.value.status() == 404


def test_model_by_id_and_json_string():
    sc = ScoreClient(FakeChatClient(policy), rng_seed=0)
    u = run(sc.create_unary(None, make_req([{"model": "a"}], stream=False)))
    mid = u.model
    assert len(mid) == 22
    for ref in (mid, f"someone/{mid}"):
        u2 = run(sc.create_unary(None, S.ScoreCompletionCreateParams.model_validate(dict(
            messages=[{"role": "user", "content": "x"}], model=ref, choices=["Paris", "Rome"], stream=False))))
        assert u2.model == mid
    import json as _j
    u3 = run(sc.create_unary(None, S.ScoreCompletionCreateParams.model_validate(dict(
        messages=[{"role": "user", "content": "x"}], model=_j.dumps({"llms": [{"model": "a"}]}),
        choices=["Paris", "Rome"], stream=False))))
    assert u3.model == mid


def test_archive_references_in_choices_and_messages():
    archive = CompletionsArchive()
    chat = C.ChatCompletion(id="chatcmpl-1", created=1, model="m", choices=[C.UnaryChoice(
        message=C.UnaryMessage(content="Paris", reasoning="thinking"), finish_reason="stop", index=0)])
    archive.store_chat(chat)
    sc = ScoreClient(FakeChatClient(policy), archive=archive, rng_seed=8)
    prev = run(sc.create_unary(None, make_req([{"model": "a"}], stream=False)))
    req = S.ScoreCompletionCreateParams.model_validate(dict(
        messages=[{"role": "user", "content": "q"}, {"role": "chat_completion", "id": "chatcmpl-1"}],
        model={"llms": [{"model": "a"}]},
        choices=[{"type": "chat_completion", "id": "chatcmpl-1", "choice_index": 0},
                 {"type": "score_completion", "id": prev.id, "choice_index": 1}, "Berlin"], stream=False))
    u = run(sc.create_unary(None, req))
    c0 = u.choices[0]
    assert c0.message.content == "Paris" and c0.completion_metadata.id == "chatcmpl-1"
    assert u.choices[1].message.content == "London"
    assert u.choices[0].confidence == pytest.approx(1.0)  # choice text was "thinking\n\nParis"
    bad = S.ScoreCompletionCreateParams.model_validate(dict(
        messages=[{"role": "user", "content": "q"}], model={"llms": [{"model": "a"}]},
        choices=[{"type": "chat_completion", "id": "chatcmpl-1", "choice_index": 7}, "x"]))
    with pytest.raises(ScoreError) as e:
        run(sc.create_streaming(None, bad))
    assert e.value.status() == 400 and e.value.message()["error"]["kind"] == "invalid_completion_choice_index"
    bad2 = S.ScoreCompletionCreateParams.model_validate(dict(
        messages=[{"role": "chat_completion", "id": "chatcmpl-1", "choice_index": 3}], model={"llms": [{"model": "a"}]},
        choices=["a", "b"]))
    with pytest.raises(ScoreError) as e:
        run(sc.create_streaming(None, bad2))
    assert e.value.status() == 400 and e.value.message()["error"]["kind"] == "chat"
    nf = S.ScoreCompletionCreateParams.model_validate(dict(
        messages=[], model={"llms": [{"model": "a"}]}, choices=[{"type": "chat_completion", "id": "nope"}, "b"]))
    with pytest.raises(ScoreError) as e:
        run(sc.create_streaming(None, nf))
    assert e.value.status() == 404


def test_choice_union_parsing_order():
    req = S.ScoreCompletionCreateParams.model_validate(dict(
        messages=[], model="x", choices=["text", {"type": "chat_completion", "id": "a"},
                                         {"type": "multichat_completion", "id": "b", "choice_index": 2},
                                         {"content": "raw", "refusal": None}, {"foo": 1}]))
    kinds = [type(c).__name__ for c in req.choices]
    assert kinds == ["str", "ChatCompletionChoiceRef", "MultichatCompletionChoiceRef", "UnaryMessage", "UnaryMessage"]
    assert req.choices[1].choice_index == 0
