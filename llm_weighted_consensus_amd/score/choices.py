"""Score-choice conversions (reference src/score/completions/client.rs:1165-1289)."""
from __future__ import annotations

from typing import Optional

from ..schema import chat as C
from ..schema import score as S
from ..utils import json as sjson


def message_to_text(m: C.UnaryMessage) -> str:
    """`convert_completion_message_to_text`: reasoning, content, refusal and pretty-JSON tool calls
    joined by blank lines."""
    tc_text: Optional[str] = None
    if m.tool_calls:
        items = []
        for tc in m.tool_calls:
            try:
                args = sjson.loads(tc.function.arguments)
            except Exception:
                args = tc.function.arguments
            items.append({"type": "tool_call", "name": tc.function.name, "arguments": args})
        tc_text = sjson.dumps_pretty(items)
    text = m.reasoning if m.reasoning is not None else ""
    for part in (m.content, m.refusal, tc_text):
        if part is None:
            continue
        if text:
            text += "\n\n"
        text += part
    return text


def message_to_delta(m: C.UnaryMessage) -> S.ScoreDelta:
    """`convert_chat_completion_choice_message_to_delta` (+ tool calls -> delta tool calls)."""
    tcs = None
    if m.tool_calls is not None:
        tcs = [C.StreamToolCall(index=i, id=t.id, function=C.StreamToolCallFunction(name=t.function.name,
                                                                                   arguments=t.function.arguments),
                                type=t.type) for i, t in enumerate(m.tool_calls)]
    return S.ScoreDelta(content=m.content, refusal=m.refusal, role="assistant", tool_calls=tcs, reasoning=m.reasoning,
                        images=m.images)


def unary_message_of(choice) -> C.UnaryMessage:
    """The chat-level message of any archived choice (score choices carry `vote` on top)."""
    m = choice.message
    if isinstance(m, S.ScoreUnaryMessage):
        return C.UnaryMessage(**{k: getattr(m, k) for k in C.UnaryMessage.model_fields})
    return m
