"""Error taxonomy with the reference's HTTP statuses and JSON shapes.

* ``ResponseError{code, message}`` — the error carried inside choices and streamed as an SSE event
  (reference src/error.rs:8-40; `From<&T: StatusError>` falls back to the HTTP reason phrase).
* ``ChatError`` kinds → ``{"kind":"chat","error":{...}}`` (src/chat/completions/error.rs:4-96), plus
  engine-side kinds of the local backend (overloaded, bad request, engine failure).
* ``ScoreError`` kinds → ``{"kind":"score","error":{...}}`` (src/score/completions/error.rs:3-73).
"""
from __future__ import annotations

from http import HTTPStatus
from typing import Any, Optional

from pydantic import BaseModel

from .utils import json as sjson


def reason_phrase(code: int) -> str:
    try:
        s = HTTPStatus(code)
        return f"{s.value} {s.phrase}"
    except ValueError:
        return "unknown"


class StatusError(Exception):
    """Base: every framework error knows its HTTP status and JSON message."""

    def status(self) -> int:
        return 500

    def message(self) -> Optional[Any]:
        return None

    def to_response_error(self) -> "ResponseError":
        return ResponseError.from_status_error(self)


class ResponseError(BaseModel):
    code: int
    message: Any = None

    @classmethod
    def from_status_error(cls, e: "StatusError") -> "ResponseError":
        m = e.message()
        return cls(code=e.status(), message=m if m is not None else reason_phrase(e.status()))

    def to_obj(self) -> dict:
        return {"code": self.code, "message": self.message}

    def to_json(self) -> str:
        return sjson.dumps(self.to_obj())

    def status(self) -> int:
        return self.code


class ResponseErrorException(StatusError):
    def __init__(self, err: ResponseError):
        super().__init__(str(err.to_obj()))
        self.err = err

    def status(self) -> int:
        return self.err.code

    def message(self):
        return self.err.message


# ------------------------------------------------------------------------------------------- chat

class ChatError(StatusError):
    kind = "chat"

    def __init__(self, code: int, detail: Any, text: str = ""):
        super().__init__(text or str(detail))
        self.code, self.detail = code, detail

    def status(self) -> int:
        return self.code

    def message(self):
        return {"kind": "chat", "error": self.detail}

    # constructors mirroring the reference variants
    @classmethod
    def empty_stream(cls):
        return cls(500, {"kind": "empty_stream", "error": "received an empty stream"})

    @classmethod
    def deserialization(cls, err: str):
        return cls(500, {"kind": "deserialization", "error": err})

    @classmethod
    def bad_status(cls, code: int, body: Any):
        return cls(code, {"kind": "bad_status", "error": body})

    @classmethod
    def stream_error(cls, err: str, code: int = 500):
        return cls(code, {"kind": "stream_error", "error": err})

    @classmethod
    def stream_timeout(cls):
        return cls(500, {"kind": "stream_timeout", "error": "error fetching stream: timeout"})

    @classmethod
    def transport(cls, err: str, code: int = 500):
        return cls(code, {"kind": "reqwest", "error": err})

    @classmethod
    def provider(cls, code: Optional[int], message: Any, metadata: Any):
        return cls(code or 500, {"kind": "provider", "message": message, "metadata": metadata})

    @classmethod
    def invalid_completion_choice_index(cls, cid: str, index: int):
        return cls(400, {"kind": "invalid_completion_choice_index",
                         "error": f"invalid choice_index for completion {cid}: {index}"})

    # local-engine kinds
    @classmethod
    def invalid_request(cls, err: str):
        return cls(400, {"kind": "invalid_request", "error": err})

    @classmethod
    def model_not_found(cls, model: str):
        return cls(404, {"kind": "model_not_found", "error": f"model not served: {model}"})

    @classmethod
    def overloaded(cls, err: str = "engine overloaded"):
        return cls(503, {"kind": "overloaded", "error": err})

    @classmethod
    def engine(cls, err: str):
        return cls(500, {"kind": "engine", "error": err})


class CtxError(StatusError):
    def __init__(self, err: ResponseError):
        super().__init__(str(err.to_obj()))
        self.err = err

    def status(self):
        return self.err.code

    def message(self):
        return {"kind": "chat", "error": self.err.message if self.err.message is not None else "ctx error"}


class ArchiveError(StatusError):
    """Completions-archive failure (fetch by id)."""

    def __init__(self, code: int, message: Any):
        super().__init__(str(message))
        self.code, self.msg = code, message

    def status(self):
        return self.code

    def message(self):
        return self.msg

    @classmethod
    def not_found(cls, kind: str, cid: str):
        return cls(404, {"kind": "completion_not_found", "error": f"{kind} completion not found: {cid}"})


# ------------------------------------------------------------------------------------------ score

class ScoreError(StatusError):
    def __init__(self, code: int, detail: Any, text: str = ""):
        super().__init__(text or str(detail))
        self.code, self.detail = code, detail

    def status(self) -> int:
        return self.code

    def message(self):
        return {"kind": "score", "error": self.detail}

    @classmethod
    def wrap(cls, e: StatusError) -> "ScoreError":
        """FetchModel / FetchModelWeights / Chat / archive errors keep their status and inner message."""
        return cls(e.status(), e.message())

    @classmethod
    def invalid_model(cls, err: str):
        return cls(400, {"kind": "invalid_model", "error": err})

    @classmethod
    def expected_two_or_more_choices(cls, n: int):
        return cls(400, {"kind": "expected_two_or_more_choices",
                         "error": f"expected 2 or more provided choices but got {n}"})

    @classmethod
    def invalid_content(cls):
        return cls(500, {"kind": "invalid_content", "error": "expected a valid response key"})

    @classmethod
    def all_votes_failed(cls, code: Optional[int]):
        return cls(code if code is not None else 500,
                   {"kind": "all_votes_failed", "error": "all votes failed, see choices for further details"})

    @classmethod
    def invalid_completion_choice_index(cls, cid: str, index: int):
        return cls(400, {"kind": "invalid_completion_choice_index",
                         "error": f"invalid choice_index for completion {cid}: {index}"})

    @classmethod
    def not_implemented(cls, what: str):
        return cls(501, {"kind": "not_implemented", "error": what})
