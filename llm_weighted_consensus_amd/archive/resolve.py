"""Resolution of archived-completion references in messages and score choices.

Contract: reference src/chat/completions/client.rs:437-645 (dedup ids -> concurrent fetch -> id map;
replace `chat_completion` / `score_completion` / `multichat_completion` messages with assistant
messages: content + generated images as `image_url` parts, refusal, tool calls; reasoning dropped;
400 on a bad `choice_index`) and src/score/completions/client.rs:952-1163 (the same for score choices,
then `convert_choices_to_internal_choices`).
"""
from __future__ import annotations

import asyncio
from typing import Any, Dict, List, Tuple

from ..errors import ChatError, ScoreError
from ..schema import chat as C
from ..schema import score as S

# completion kind by reference-message role / choice type
_KIND = {"chat_completion": "chat", "score_completion": "score", "multichat_completion": "multichat"}


async def _fetch_all(archive, ctx, refs: List[Tuple[str, str]]) -> Dict[str, Tuple[str, Any]]:
    seen, todo = set(), []
    for kind, cid in refs:
        if cid in seen:
            continue
        seen.add(cid)
        todo.append((kind, cid))
    if not todo:
        return {}

    async def one(kind, cid):
        f = {"chat": archive.fetch_chat_completion, "score": archive.fetch_score_completion,
             "multichat": archive.fetch_multichat_completion}[kind]
        return kind, await f(ctx, cid)

    res = await asyncio.gather(*(one(k, c) for k, c in todo))
    return {obj.id: (kind, obj) for kind, obj in res}


async def fetch_completions_from_messages(archive, ctx, messages) -> Dict[str, Tuple[str, Any]]:
    refs = [(_KIND[m.role], m.id) for m in messages if isinstance(m, C.COMPLETION_REF_MESSAGES)]
    return await _fetch_all(archive, ctx, refs)


async def fetch_completions_from_choices_and_messages(archive, ctx, choices, messages):
    refs = []
    for ch in choices:
        if isinstance(ch, (S.ChatCompletionChoiceRef, S.ScoreCompletionChoiceRef, S.MultichatCompletionChoiceRef)):
            refs.append((_KIND[ch.type], ch.id))
    refs += [(_KIND[m.role], m.id) for m in messages if isinstance(m, C.COMPLETION_REF_MESSAGES)]
    return await _fetch_all(archive, ctx, refs)


def _choice_message(kind: str, comp, index: int):
    for ch in comp.choices:
        if ch.index == index:
            if kind == "score":
                m = ch.message
                return C.UnaryMessage(**{k: getattr(m, k) for k in C.UnaryMessage.model_fields}), ch
            return ch.message, ch
    return None, None


def convert_completion_choice_message_to_assistant_message(msg: C.UnaryMessage, name) -> C.AssistantMessage:
    images = [C.ImageUrlPart(image_url=C.ImageUrl(url=i.image_url.url)) for i in (msg.images or [])]
    if msg.content is not None and images:
        content = [C.TextPart(text=msg.content)] + images
    elif msg.content is not None:
        content = msg.content
    elif images:
        content = images
    else:
        content = None
    tool_calls = None
    if msg.tool_calls is not None:
        tool_calls = [C.AssistantToolCall(id=t.id, function=C.AssistantToolCallFunction(
            name=t.function.name, arguments=t.function.arguments)) for t in msg.tool_calls]
    return C.AssistantMessage(content=content, name=name, refusal=msg.refusal, tool_calls=tool_calls, reasoning=None)


def replace_completion_messages(completions: Dict[str, Tuple[str, Any]], messages: list,
                                error_cls=ChatError) -> None:
    if not completions:
        return
    for i, m in enumerate(messages):
        if not isinstance(m, C.COMPLETION_REF_MESSAGES):
            continue
        kind, comp = completions[m.id]
        msg, _ = _choice_message(kind, comp, m.choice_index)
        if msg is None:
            raise error_cls.invalid_completion_choice_index(m.id, m.choice_index)
        messages[i] = convert_completion_choice_message_to_assistant_message(msg, m.name)


class InternalChoice:
    """Resolved score choice (reference request.rs:93-110)."""

    __slots__ = ("kind", "text", "message", "completion", "choice")

    def __init__(self, kind: str, text=None, message=None, completion=None, choice=None):
        self.kind, self.text, self.message, self.completion, self.choice = kind, text, message, completion, choice


def convert_choices_to_internal_choices(completions, choices) -> List[InternalChoice]:
    out = []
    for ch in choices:
        if isinstance(ch, str):
            out.append(InternalChoice("text", text=ch))
        elif isinstance(ch, C.UnaryMessage):
            out.append(InternalChoice("message", message=ch))
        else:
            kind, comp = completions[ch.id]
            found = next((c for c in comp.choices if c.index == ch.choice_index), None)
            if found is None:
                raise ScoreError.invalid_completion_choice_index(ch.id, ch.choice_index)
            out.append(InternalChoice(kind, completion=comp, choice=found.model_copy(deep=True)))
    return out
