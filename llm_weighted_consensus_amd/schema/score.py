"""Score completions wire types (request, streaming/unary response, merge algebra) and the
multichat / embeddings response types.

Contracts: reference src/score/completions/request.rs (choices: text | archived completion ref |
raw assistant message, >= 2), src/score/completions/response.rs (chunk + `weight_data`; choice adds
weight/confidence/error/model/model_index/completion_metadata; delta adds `vote`),
src/score/completions/weight.rs:5-18 (weight data), src/multichat/completions/response.rs and
src/embeddings/response.rs.
"""
from __future__ import annotations

from typing import Annotated, Any, List, Literal, Optional, Union

from pydantic import Field

from ..errors import ResponseError
from .base import Wire
from .chat import (Delta, FinishReason, Logprobs, Message, ServiceTier, StreamOptions, Tool,
                   UnaryChoice, UnaryMessage, UsageRequest, Usage, push_choices)

# ============================================================================ request

class ChatCompletionChoiceRef(Wire):
    type: Literal["chat_completion"]
    id: str
    choice_index: int = 0


class ScoreCompletionChoiceRef(Wire):
    type: Literal["score_completion"]
    id: str
    choice_index: int = 0


class MultichatCompletionChoiceRef(Wire):
    type: Literal["multichat_completion"]
    id: str
    choice_index: int = 0


# untagged, tried left to right exactly like serde (request.rs:68-91)
Choice = Union[str, ChatCompletionChoiceRef, ScoreCompletionChoiceRef, MultichatCompletionChoiceRef, UnaryMessage]
ChoiceField = Annotated[Choice, Field(union_mode="left_to_right")]


class ScoreCompletionCreateParams(Wire):
    messages: List[Message]
    model: Any  # str id | JSON-string model | inline ModelBase (validated by score.model)
    seed: Optional[int] = None
    service_tier: Optional[ServiceTier] = None
    stream: Optional[bool] = None
    stream_options: Optional[StreamOptions] = None
    tools: Optional[List[Tool]] = None  # read-only tools shown to voters
    usage: Optional[UsageRequest] = None
    choices: List[ChoiceField]

    def template_content(self) -> str:
        from .chat import template_content

        return template_content(self.messages)


# ============================================================================ response

class CompletionMetadata(Wire):
    id: str = ""
    created: int = 0
    model: str = ""
    service_tier: Optional[ServiceTier] = None
    system_fingerprint: Optional[str] = None
    usage: Optional[Usage] = None
    provider: Optional[str] = None

    def push(self, o: "CompletionMetadata") -> None:
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


class ScoreDelta(Delta):
    """chat Delta flattened + vote (serde(flatten))."""
    vote: Optional[List[float]] = None

    def push(self, o: "ScoreDelta") -> None:
        Delta.push(self, o)
        if o.vote is not None and self.vote is None:
            self.vote = list(o.vote)


class ScoreStreamChoice(Wire):
    __keep_none__ = frozenset({"finish_reason"})
    delta: ScoreDelta
    finish_reason: Optional[FinishReason] = None
    index: int
    logprobs: Optional[Logprobs] = None
    weight: Optional[float] = None
    confidence: Optional[float] = None
    error: Optional[ResponseError] = None
    model: Optional[str] = None
    model_index: Optional[int] = None
    completion_metadata: Optional[CompletionMetadata] = None

    def to_obj(self) -> dict:
        o = super().to_obj()
        if self.error is not None:
            o["error"] = self.error.to_obj()
        return o

    def push(self, o: "ScoreStreamChoice") -> None:
        self.delta.push(o.delta)
        if o.finish_reason is not None and self.finish_reason is None:
            self.finish_reason = o.finish_reason
        if self.logprobs is not None and o.logprobs is not None:
            self.logprobs.push(o.logprobs)
        elif self.logprobs is None and o.logprobs is not None:
            self.logprobs = o.logprobs.clone()
        if o.weight is not None and self.weight is None:
            self.weight = o.weight
        if o.confidence is not None and self.confidence is None:
            self.confidence = o.confidence
        if o.error is not None and self.error is None:
            self.error = o.error
        if o.model is not None and self.model is None:
            self.model = o.model
        if o.model_index is not None and self.model_index is None:
            self.model_index = o.model_index
        if self.completion_metadata is not None and o.completion_metadata is not None:
            self.completion_metadata.push(o.completion_metadata)
        elif self.completion_metadata is None and o.completion_metadata is not None:
            self.completion_metadata = o.completion_metadata.clone()

    def tool_as_content(self) -> None:
        if self.finish_reason == "tool_calls":
            self.finish_reason = "stop"
        self.delta.tool_as_content()

    def has_finish_reason_or_usage(self) -> bool:
        return self.finish_reason is not None or (self.completion_metadata is not None
                                                  and self.completion_metadata.usage is not None)


class WeightDataStatic(Wire):
    type: Literal["static"] = "static"


class EmbeddingItem(Wire):
    embedding: List[float]
    index: int
    object: Literal["embedding"] = "embedding"


class CreateEmbeddingResponse(Wire):
    data: List[EmbeddingItem]
    model: str
    object: Literal["list"] = "list"
    usage: Optional[Usage] = None


class WeightDataTrainingTable(Wire):
    type: Literal["training_table"] = "training_table"
    embeddings_response: CreateEmbeddingResponse


WeightData = Annotated[Union[WeightDataStatic, WeightDataTrainingTable], Field(discriminator="type")]


class ScoreCompletionChunk(Wire):
    id: str
    choices: List[ScoreStreamChoice]
    created: int
    model: str
    object: Literal["chat.completion.chunk"] = "chat.completion.chunk"
    usage: Optional[Usage] = None
    weight_data: Optional[WeightData] = None

    def push(self, o: "ScoreCompletionChunk", owned: bool = False) -> None:
        push_choices(self.choices, o.choices, owned)
        if self.usage is not None and o.usage is not None:
            self.usage.push(o.usage)
        elif self.usage is None and o.usage is not None:
            self.usage = o.usage.clone()
        if o.weight_data is not None and self.weight_data is None:
            self.weight_data = o.weight_data

    def tool_as_content(self) -> None:
        for c in self.choices:
            c.tool_as_content()

    def clone_without_choices(self) -> "ScoreCompletionChunk":
        return ScoreCompletionChunk(id=self.id, choices=[], created=self.created, model=self.model,
                                    usage=self.usage.clone() if self.usage else None, weight_data=self.weight_data)


class ScoreUnaryMessage(UnaryMessage):
    __keep_none__ = frozenset({"content", "refusal", "vote"})
    vote: Optional[List[float]] = None


class ScoreUnaryChoice(Wire):
    __keep_none__ = frozenset({"logprobs", "weight", "confidence", "error", "model", "model_index",
                               "completion_metadata"})
    message: ScoreUnaryMessage
    finish_reason: FinishReason = "error"
    index: int
    logprobs: Optional[Logprobs] = None
    weight: Optional[float] = None
    confidence: Optional[float] = None
    error: Optional[ResponseError] = None
    model: Optional[str] = None
    model_index: Optional[int] = None
    completion_metadata: Optional[CompletionMetadata] = None

    def to_obj(self) -> dict:
        o = super().to_obj()
        o["error"] = self.error.to_obj() if self.error is not None else None
        return o

    @classmethod
    def from_stream(cls, c: ScoreStreamChoice) -> "ScoreUnaryChoice":
        m = UnaryMessage.from_delta(c.delta)
        return cls(message=ScoreUnaryMessage(**{k: getattr(m, k) for k in UnaryMessage.model_fields}, vote=c.delta.vote),
                   finish_reason=c.finish_reason or "error", index=c.index, logprobs=c.logprobs, weight=c.weight,
                   confidence=c.confidence, error=c.error, model=c.model, model_index=c.model_index,
                   completion_metadata=c.completion_metadata)


class ScoreCompletion(Wire):
    __keep_none__ = frozenset({"weight_data"})
    id: str
    choices: List[ScoreUnaryChoice]
    created: int
    model: str
    object: Literal["chat.completion"] = "chat.completion"
    usage: Optional[Usage] = None
    weight_data: Optional[WeightData] = None

    @classmethod
    def from_chunk(cls, c: ScoreCompletionChunk) -> "ScoreCompletion":
        return cls(id=c.id, choices=[ScoreUnaryChoice.from_stream(x) for x in c.choices], created=c.created,
                   model=c.model, usage=c.usage, weight_data=c.weight_data)


# ============================================================================ multichat

class MultichatStreamChoice(Wire):
    __keep_none__ = frozenset({"finish_reason"})
    delta: Delta
    finish_reason: Optional[FinishReason] = None
    index: int
    logprobs: Optional[Logprobs] = None
    error: Optional[ResponseError] = None
    model: Optional[str] = None
    model_index: Optional[int] = None
    completion_metadata: Optional[CompletionMetadata] = None

    def to_obj(self) -> dict:
        o = super().to_obj()
        if self.error is not None:
            o["error"] = self.error.to_obj()
        return o

    def push(self, o: "MultichatStreamChoice") -> None:
        self.delta.push(o.delta)
        if o.finish_reason is not None and self.finish_reason is None:
            self.finish_reason = o.finish_reason
        if self.logprobs is not None and o.logprobs is not None:
            self.logprobs.push(o.logprobs)
        elif self.logprobs is None and o.logprobs is not None:
            self.logprobs = o.logprobs.clone()
        if o.error is not None and self.error is None:
            self.error = o.error
        if o.model is not None and self.model is None:
            self.model = o.model
        if o.model_index is not None and self.model_index is None:
            self.model_index = o.model_index
        if self.completion_metadata is not None and o.completion_metadata is not None:
            self.completion_metadata.push(o.completion_metadata)
        elif self.completion_metadata is None and o.completion_metadata is not None:
            self.completion_metadata = o.completion_metadata.clone()

    def has_finish_reason_or_usage(self) -> bool:
        return self.finish_reason is not None or (self.completion_metadata is not None
                                                  and self.completion_metadata.usage is not None)


class MultichatCompletionChunk(Wire):
    id: str
    choices: List[MultichatStreamChoice]
    created: int
    model: str
    object: Literal["chat.completion.chunk"] = "chat.completion.chunk"
    usage: Optional[Usage] = None

    def push(self, o: "MultichatCompletionChunk") -> None:
        push_choices(self.choices, o.choices)
        if self.usage is not None and o.usage is not None:
            self.usage.push(o.usage)
        elif self.usage is None and o.usage is not None:
            self.usage = o.usage.clone()

    def clone_without_choices(self) -> "MultichatCompletionChunk":
        return MultichatCompletionChunk(id=self.id, choices=[], created=self.created, model=self.model,
                                        usage=self.usage.clone() if self.usage else None)


class MultichatUnaryChoice(Wire):
    __keep_none__ = frozenset({"logprobs", "error", "model", "model_index", "completion_metadata"})
    message: UnaryMessage
    finish_reason: FinishReason = "error"
    index: int
    logprobs: Optional[Logprobs] = None
    error: Optional[ResponseError] = None
    model: Optional[str] = None
    model_index: Optional[int] = None
    completion_metadata: Optional[CompletionMetadata] = None

    def to_obj(self) -> dict:
        o = super().to_obj()
        o["error"] = self.error.to_obj() if self.error is not None else None
        return o

    @classmethod
    def from_stream(cls, c: MultichatStreamChoice) -> "MultichatUnaryChoice":
        return cls(message=UnaryMessage.from_delta(c.delta), finish_reason=c.finish_reason or "error", index=c.index,
                   logprobs=c.logprobs, error=c.error, model=c.model, model_index=c.model_index,
                   completion_metadata=c.completion_metadata)


class MultichatCompletion(Wire):
    id: str
    choices: List[MultichatUnaryChoice]
    created: int
    model: str
    object: Literal["chat.completion"] = "chat.completion"
    usage: Optional[Usage] = None

    @classmethod
    def from_chunk(cls, c: MultichatCompletionChunk) -> "MultichatCompletion":
        return cls(id=c.id, choices=[MultichatUnaryChoice.from_stream(x) for x in c.choices], created=c.created,
                   model=c.model, usage=c.usage)
