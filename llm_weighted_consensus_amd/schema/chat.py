"""Chat completions wire types (OpenAI + OpenRouter fields) and the streaming merge algebra.

Behavioural contract: reference src/chat/completions/request.rs (request side, incl. the three
completion-reference message roles and `template_content`) and src/chat/completions/response.rs
(streaming chunk/choice/delta/tool-call `push`, unary `From<chunk>`, `Usage::push` /
`with_total_cost`, `Logprobs::push`).  Field order and omission rules follow the serde derives.
"""
from __future__ import annotations

from typing import Annotated, Any, Dict, List, Literal, Optional, Union

from pydantic import Field

from .base import Wire, push_opt_list, push_opt_num

# ============================================================================ request side

ServiceTier = Literal["auto", "default", "flex"]
ReasoningEffort = Literal["minimal", "low", "medium", "high"]
Verbosity = Literal["low", "medium", "high"]


class SimpleContentPart(Wire):
    text: str
    type: Literal["text"] = "text"


SimpleContent = Union[str, List[SimpleContentPart]]


def simple_content_text(c: SimpleContent) -> str:
    return c if isinstance(c, str) else "".join(p.text for p in c)


class ImageUrl(Wire):
    url: str
    detail: Optional[Literal["auto", "low", "high"]] = None


class InputAudio(Wire):
    data: str
    format: Literal["wav", "mp3"]


class VideoUrl(Wire):
    url: str


class File(Wire):
    file_data: Optional[str] = None
    file_id: Optional[str] = None
    filename: Optional[str] = None


class TextPart(Wire):
    type: Literal["text"] = "text"
    text: str


class ImageUrlPart(Wire):
    type: Literal["image_url"] = "image_url"
    image_url: ImageUrl


class InputAudioPart(Wire):
    type: Literal["input_audio"] = "input_audio"
    input_audio: InputAudio


class InputVideoPart(Wire):
    type: Literal["input_video"] = "input_video"
    video_url: VideoUrl


class FilePart(Wire):
    type: Literal["file"] = "file"
    file: File


RichContentPart = Annotated[Union[TextPart, ImageUrlPart, InputAudioPart, InputVideoPart, FilePart],
                           Field(discriminator="type")]
RichContent = Union[str, List[RichContentPart]]


def rich_content_text(c: RichContent) -> str:
    if isinstance(c, str):
        return c
    return "".join(p.text for p in c if isinstance(p, TextPart))


class AssistantToolCallFunction(Wire):
    name: str
    arguments: str


class AssistantToolCall(Wire):
    id: str
    function: AssistantToolCallFunction
    type: Literal["function"] = "function"

    def template(self) -> str:
        return "<tool_call>" + self.to_json() + "</tool_call>"


def _role_prefix(role: str, name: Optional[str]) -> str:
    return role + (f" ({name})" if name is not None else "") + ": "


class DeveloperMessage(Wire):
    role: Literal["developer"] = "developer"
    content: SimpleContent
    name: Optional[str] = None

    def template(self) -> str:
        return _role_prefix("developer", self.name) + simple_content_text(self.content)


class SystemMessage(Wire):
    role: Literal["system"] = "system"
    content: SimpleContent
    name: Optional[str] = None

    def template(self) -> str:
        return _role_prefix("system", self.name) + simple_content_text(self.content)


class UserMessage(Wire):
    role: Literal["user"] = "user"
    content: RichContent
    name: Optional[str] = None

    def template(self) -> str:
        return _role_prefix("user", self.name) + rich_content_text(self.content)


class AssistantMessage(Wire):
    role: Literal["assistant"] = "assistant"
    content: Optional[RichContent] = None
    name: Optional[str] = None
    refusal: Optional[str] = None
    tool_calls: Optional[List[AssistantToolCall]] = None
    reasoning: Optional[str] = None

    def template(self) -> str:
        # reference request.rs:443-478
        s, wrote = "", False
        pre = _role_prefix("assistant", self.name)
        if self.content is not None:
            s += pre + rich_content_text(self.content)
            wrote = True
        if self.refusal is not None:
            if wrote:
                s += "\n"
            s += pre + self.refusal
            wrote = True
        if self.tool_calls is not None:
            if wrote:
                s += "\n"
            s += pre + "".join(tc.template() for tc in self.tool_calls)
        return s


class ToolMessage(Wire):
    role: Literal["tool"] = "tool"
    content: RichContent
    tool_call_id: str

    def template(self) -> str:
        return f"tool ({self.tool_call_id}): " + rich_content_text(self.content)


class ChatCompletionMessage(Wire):
    role: Literal["chat_completion"] = "chat_completion"
    id: str
    choice_index: int = 0
    name: Optional[str] = None

    def template(self) -> str:
        return ""


class ScoreCompletionMessage(Wire):
    role: Literal["score_completion"] = "score_completion"
    id: str
    choice_index: int = 0
    name: Optional[str] = None

    def template(self) -> str:
        return ""


class MultichatCompletionMessage(Wire):
    role: Literal["multichat_completion"] = "multichat_completion"
    id: str
    choice_index: int = 0
    name: Optional[str] = None

    def template(self) -> str:
        return ""


COMPLETION_REF_MESSAGES = (ChatCompletionMessage, ScoreCompletionMessage, MultichatCompletionMessage)


Message = Annotated[Union[DeveloperMessage, SystemMessage, UserMessage, AssistantMessage, ToolMessage,
                          ChatCompletionMessage, ScoreCompletionMessage, MultichatCompletionMessage],
                    Field(discriminator="role")]


def template_content(messages: List[Message]) -> str:
    """`ChatCompletionCreateParams::template_content` (reference request.rs:78-91)."""
    return "\n".join(m.template() for m in messages)


class JsonSchema(Wire):
    name: str
    description: Optional[str] = None
    schema_: Optional[Any] = Field(default=None, alias="schema")
    strict: Optional[bool] = None


class ResponseFormatText(Wire):
    type: Literal["text"] = "text"


class ResponseFormatJsonObject(Wire):
    type: Literal["json_object"] = "json_object"


class ResponseFormatJsonSchema(Wire):
    type: Literal["json_schema"] = "json_schema"
    json_schema: JsonSchema


ResponseFormat = Annotated[Union[ResponseFormatText, ResponseFormatJsonObject, ResponseFormatJsonSchema],
                          Field(discriminator="type")]


class StreamOptions(Wire):
    include_usage: Optional[bool] = None


class ToolChoiceFunctionFunction(Wire):
    name: str


class ToolChoiceFunction(Wire):
    type: Literal["function"] = "function"
    function: ToolChoiceFunctionFunction


ToolChoice = Union[Literal["none", "auto", "required"], ToolChoiceFunction]


class FunctionDefinition(Wire):
    name: str
    description: Optional[str] = None
    parameters: Optional[Any] = None
    strict: Optional[bool] = None


class Tool(Wire):
    function: FunctionDefinition
    type: Literal["function"] = "function"


class PredictionContentPart(Wire):
    text: str
    type: Literal["text"] = "text"


class Prediction(Wire):
    content: Union[str, List[PredictionContentPart]]
    type: Literal["content"] = "content"


class UserLocationApproximate(Wire):
    city: Optional[str] = None
    country: Optional[str] = None
    region: Optional[str] = None
    timezone: Optional[str] = None


class UserLocation(Wire):
    approximate: UserLocationApproximate
    type: Literal["approximate"] = "approximate"


class WebSearchOptions(Wire):
    search_context_size: Optional[Literal["low", "medium", "high"]] = None
    user_location: Optional[UserLocation] = None


class ProviderPreferences(Wire):
    order: Optional[List[str]] = None
    allow_fallbacks: Optional[bool] = None
    require_parameters: Optional[bool] = None
    data_collection: Optional[Literal["allow", "deny"]] = None
    only: Optional[List[str]] = None
    ignore: Optional[List[str]] = None
    quantizations: Optional[List[str]] = None
    sort: Optional[str] = None

    def is_empty(self) -> bool:
        return all(getattr(self, f) is None for f in type(self).model_fields)


class Plugin(Wire):
    model_config = dict(Wire.model_config, extra="allow")
    id: str


class Reasoning(Wire):
    max_tokens: Optional[int] = None
    effort: Optional[ReasoningEffort] = None
    enabled: Optional[bool] = None


class UsageRequest(Wire):
    include: bool


Stop = Union[str, List[str]]


class ChatCompletionCreateParams(Wire):
    messages: List[Message]
    model: str
    frequency_penalty: Optional[float] = None
    logit_bias: Optional[Dict[str, int]] = None
    logprobs: Optional[bool] = None
    max_completion_tokens: Optional[int] = None
    modalities: Optional[List[str]] = None
    n: Optional[int] = None
    parallel_tool_calls: Optional[bool] = None
    prediction: Optional[Prediction] = None
    presence_penalty: Optional[float] = None
    reasoning_effort: Optional[ReasoningEffort] = None
    response_format: Optional[ResponseFormat] = None
    seed: Optional[int] = None
    service_tier: Optional[ServiceTier] = None
    stop: Optional[Stop] = None
    stream: Optional[bool] = None
    stream_options: Optional[StreamOptions] = None
    temperature: Optional[float] = None
    tool_choice: Optional[ToolChoice] = None
    tools: Optional[List[Tool]] = None
    top_logprobs: Optional[int] = None
    top_p: Optional[float] = None
    web_search_options: Optional[WebSearchOptions] = None
    # openrouter fields
    max_tokens: Optional[int] = None
    min_p: Optional[float] = None
    plugins: Optional[List[Plugin]] = None
    provider: Optional[ProviderPreferences] = None
    reasoning: Optional[Reasoning] = None
    repetition_penalty: Optional[float] = None
    top_a: Optional[float] = None
    top_k: Optional[int] = None
    usage: Optional[UsageRequest] = None
    verbosity: Optional[Verbosity] = None
    models: Optional[List[str]] = None

    def template_content(self) -> str:
        return template_content(self.messages)




# ============================================================================ response side

FinishReason = Literal["stop", "length", "tool_calls", "content_filter", "error"]


class CompletionTokensDetails(Wire):
    accepted_prediction_tokens: Optional[int] = None
    audio_tokens: Optional[int] = None
    reasoning_tokens: Optional[int] = None
    rejected_prediction_tokens: Optional[int] = None

    def push(self, o: "CompletionTokensDetails") -> None:
        for f in type(self).model_fields:
            setattr(self, f, push_opt_num(getattr(self, f), getattr(o, f)))


class PromptTokensDetails(Wire):
    audio_tokens: Optional[int] = None
    cached_tokens: Optional[int] = None

    def push(self, o: "PromptTokensDetails") -> None:
        for f in type(self).model_fields:
            setattr(self, f, push_opt_num(getattr(self, f), getattr(o, f)))


class CostDetails(Wire):
    upstream_inference_cost: Optional[float] = None
    upstream_upstream_inference_cost: Optional[float] = None

    def push(self, o: "CostDetails") -> None:
        for f in type(self).model_fields:
            setattr(self, f, push_opt_num(getattr(self, f), getattr(o, f)))

    def is_empty(self) -> bool:
        return self.upstream_inference_cost is None and self.upstream_upstream_inference_cost is None

    def total_cost(self) -> float:
        return (self.upstream_inference_cost or 0.0) + (self.upstream_upstream_inference_cost or 0.0)


class Usage(Wire):
    completion_tokens: int = 0
    prompt_tokens: int = 0
    total_tokens: int = 0
    completion_tokens_details: Optional[CompletionTokensDetails] = None
    prompt_tokens_details: Optional[PromptTokensDetails] = None
    cost: Optional[float] = None
    cost_details: Optional[CostDetails] = None
    total_cost: Optional[float] = None

    def push(self, o: "Usage") -> None:
        """reference response.rs:587-625 (total_cost is NOT summed)."""
        self.completion_tokens += o.completion_tokens
        self.prompt_tokens += o.prompt_tokens
        self.total_tokens += o.total_tokens
        for f in ("completion_tokens_details", "prompt_tokens_details", "cost_details"):
            a, b = getattr(self, f), getattr(o, f)
            if a is not None and b is not None:
                a.push(b)
            elif a is None and b is not None:
                setattr(self, f, b.clone())
        self.cost = push_opt_num(self.cost, o.cost)

    def is_empty(self) -> bool:
        return (self.completion_tokens == 0 and self.prompt_tokens == 0 and self.total_tokens == 0
                and self.completion_tokens_details is None and self.prompt_tokens_details is None)

    def with_total_cost(self) -> None:
        """reference response.rs:635-649."""
        if self.total_cost is None and (self.cost is not None or
                                        (self.cost_details is not None and not self.cost_details.is_empty())):
            t = 0.0
            if self.cost is not None:
                t += self.cost
            if self.cost_details is not None:
                t += self.cost_details.total_cost()
            self.total_cost = t


class TopLogprob(Wire):
    __keep_none__ = frozenset({"bytes", "logprob"})
    token: str
    bytes: Optional[List[int]] = None
    logprob: Optional[float] = None


class Logprob(Wire):
    __keep_none__ = frozenset({"bytes"})
    token: str
    bytes: Optional[List[int]] = None
    logprob: float
    top_logprobs: List[TopLogprob] = []


class Logprobs(Wire):
    __keep_none__ = frozenset({"content", "refusal"})
    content: Optional[List[Logprob]] = None
    refusal: Optional[List[Logprob]] = None

    def push(self, o: "Logprobs") -> None:
        if o.content is not None:
            if self.content is None:
                self.content = list(o.content)
            else:
                self.content.extend(o.content)  # owned by the aggregate: no O(n^2) re-concatenation
        if o.refusal is not None:
            if self.refusal is None:
                self.refusal = list(o.refusal)
            else:
                self.refusal.extend(o.refusal)  # owned by the aggregate: no O(n^2) re-concatenation


class ImageUrlOut(Wire):
    url: str


class Image(Wire):
    type: Literal["image_url"] = "image_url"
    image_url: ImageUrlOut


class StreamToolCallFunction(Wire):
    name: Optional[str] = None
    arguments: Optional[str] = None

    def push(self, o: "StreamToolCallFunction") -> None:
        if o.name is not None and self.name is None:
            self.name = o.name
        if o.arguments is not None:
            self.arguments = o.arguments if self.arguments is None else self.arguments + o.arguments


class StreamToolCall(Wire):
    index: int
    id: Optional[str] = None
    function: Optional[StreamToolCallFunction] = None
    type: Optional[Literal["function"]] = None

    def push(self, o: "StreamToolCall") -> None:
        if o.id is not None and self.id is None:
            self.id = o.id
        if self.function is not None and o.function is not None:
            self.function.push(o.function)
        elif self.function is None and o.function is not None:
            self.function = o.function.clone()
        if o.type is not None and self.type is None:
            self.type = o.type


class Delta(Wire):
    content: Optional[str] = None
    refusal: Optional[str] = None
    role: Optional[Literal["assistant"]] = None
    tool_calls: Optional[List[StreamToolCall]] = None
    reasoning: Optional[str] = None
    images: Optional[List[Image]] = None

    def push(self, o: "Delta") -> None:
        if o.content is not None:
            self.content = o.content if self.content is None else self.content + o.content
        if o.refusal is not None:
            self.refusal = o.refusal if self.refusal is None else self.refusal + o.refusal
        if o.role is not None and self.role is None:
            self.role = o.role
        if o.tool_calls is not None:
            if self.tool_calls is None:
                self.tool_calls = [t.clone() for t in o.tool_calls]
            else:
                for t in o.tool_calls:
                    mine = next((x for x in self.tool_calls if x.index == t.index), None)
                    if mine is not None:
                        mine.push(t)
                    else:
                        self.tool_calls.append(t.clone())
        if o.reasoning is not None:
            self.reasoning = o.reasoning if self.reasoning is None else self.reasoning + o.reasoning
        self.images = push_opt_list(self.images, [i.clone() for i in o.images] if o.images is not None else None)

    def tool_as_content(self) -> None:
        """reference response.rs:161-177: move tool-call arguments into content."""
        tcs, self.tool_calls = self.tool_calls, None
        for tc in tcs or []:
            if tc.function is not None and tc.function.arguments is not None:
                if self.content is not None:
                    self.content += tc.function.arguments
                else:
                    self.content = tc.function.arguments


class StreamChoice(Wire):
    __keep_none__ = frozenset({"finish_reason"})
    delta: Delta
    finish_reason: Optional[FinishReason] = None
    index: int
    logprobs: Optional[Logprobs] = None

    def push(self, o: "StreamChoice") -> None:
        self.delta.push(o.delta)
        if o.finish_reason is not None and self.finish_reason is None:
            self.finish_reason = o.finish_reason
        if self.logprobs is not None and o.logprobs is not None:
            self.logprobs.push(o.logprobs)
        elif self.logprobs is None and o.logprobs is not None:
            self.logprobs = o.logprobs.clone()


def push_choices(mine: list, others: list, owned: bool = False) -> None:
    """O(C) find-by-index merge used by every chunk type (reference response.rs:56-78).  ``owned``: the
    caller hands ``others`` over (nothing else holds them): a new choice is taken as is, not deep-copied."""
    for oc in others:
        tgt = next((c for c in mine if c.index == oc.index), None)
        if tgt is not None:
            tgt.push(oc)
        else:
            mine.append(oc if owned else oc.clone())


class ChatCompletionChunk(Wire):
    id: str
    choices: List[StreamChoice]
    created: int
    model: str
    object: Literal["chat.completion.chunk"] = "chat.completion.chunk"
    service_tier: Optional[ServiceTier] = None
    system_fingerprint: Optional[str] = None
    usage: Optional[Usage] = None
    provider: Optional[str] = None

    def push(self, o: "ChatCompletionChunk") -> None:
        push_choices(self.choices, o.choices)
        if o.service_tier is not None and self.service_tier is None:
            self.service_tier = o.service_tier
        if o.system_fingerprint is not None and self.system_fingerprint is None:
            self.system_fingerprint = o.system_fingerprint
        if self.usage is not None and o.usage is not None:
            self.usage.push(o.usage)
        elif self.usage is None and o.usage is not None:
            self.usage = o.usage.clone()
        if o.provider is not None and self.provider is None:
            self.provider = o.provider

    def with_total_cost(self) -> None:
        if self.usage is not None:
            self.usage.with_total_cost()


# ---- unary ----------------------------------------------------------------------------------------

class UnaryToolCallFunction(Wire):
    name: str = ""
    arguments: str = ""


class UnaryToolCall(Wire):
    id: str = ""
    function: UnaryToolCallFunction = UnaryToolCallFunction()
    type: Literal["function"] = "function"

    @classmethod
    def from_stream(cls, t: StreamToolCall) -> "UnaryToolCall":
        f = t.function
        return cls(id=t.id or "", function=UnaryToolCallFunction(name=(f.name if f else None) or "",
                                                                  arguments=(f.arguments if f else None) or ""),
                   type=t.type or "function")


class AnnotationUrlCitation(Wire):
    end_index: int
    start_index: int
    title: str
    url: str


class Annotation(Wire):
    type: Literal["url_citation"] = "url_citation"
    url_citation: AnnotationUrlCitation


class Audio(Wire):
    id: str
    data: str
    expires_at: int
    transcript: str


class UnaryMessage(Wire):
    __keep_none__ = frozenset({"content", "refusal"})
    content: Optional[str] = None
    refusal: Optional[str] = None
    role: Literal["assistant"] = "assistant"
    annotations: Optional[List[Annotation]] = None
    audio: Optional[Audio] = None
    tool_calls: Optional[List[UnaryToolCall]] = None
    reasoning: Optional[str] = None
    images: Optional[List[Image]] = None

    @classmethod
    def from_delta(cls, d: Delta) -> "UnaryMessage":
        return cls(content=d.content, refusal=d.refusal, role="assistant",
                   tool_calls=[UnaryToolCall.from_stream(t) for t in d.tool_calls] if d.tool_calls is not None
                   else None, reasoning=d.reasoning, images=d.images)


class UnaryChoice(Wire):
    __keep_none__ = frozenset({"logprobs"})
    message: UnaryMessage
    finish_reason: FinishReason = "error"
    index: int
    logprobs: Optional[Logprobs] = None

    @classmethod
    def from_stream(cls, c: StreamChoice) -> "UnaryChoice":
        return cls(message=UnaryMessage.from_delta(c.delta), finish_reason=c.finish_reason or "error", index=c.index,
                   logprobs=c.logprobs)


class ChatCompletion(Wire):
    id: str = ""
    choices: List[UnaryChoice] = []
    created: int = 0
    model: str = ""
    object: Literal["chat.completion"] = "chat.completion"
    service_tier: Optional[ServiceTier] = None
    system_fingerprint: Optional[str] = None
    usage: Optional[Usage] = None
    provider: Optional[str] = None

    @classmethod
    def from_chunk(cls, c: ChatCompletionChunk) -> "ChatCompletion":
        return cls(id=c.id, choices=[UnaryChoice.from_stream(x) for x in c.choices], created=c.created, model=c.model,
                   service_tier=c.service_tier, system_fingerprint=c.system_fingerprint, usage=c.usage,
                   provider=c.provider)


def fold_chunks(chunks) -> Optional[ChatCompletionChunk]:
    agg = None
    for c in chunks:
        if agg is None:
            agg = c.clone()
        else:
            agg.push(c)
    return agg
