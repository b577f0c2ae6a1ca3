"""Per-sequence sampling parameters of the local engine.

Mirrors the generation knobs a voter (`LlmBase`, reference src/score/llm/mod.rs:7-73) or a chat
request (src/chat/completions/request.rs:4-76) can set, with the reference's defaults (the
`prepare()` canonicalisation treats temperature 1, top_p 1, penalties 0, repetition 1, top_k 0,
min_p 0, top_a 0 as "unset").
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional


@dataclass
class SamplingParams:
    temperature: float = 1.0
    top_p: float = 1.0
    top_k: int = 0
    min_p: float = 0.0
    top_a: float = 0.0
    frequency_penalty: float = 0.0
    presence_penalty: float = 0.0
    repetition_penalty: float = 1.0
    max_tokens: int = 256
    stop: List[str] = field(default_factory=list)
    stop_token_ids: List[int] = field(default_factory=list)
    ignore_eos: bool = False
    logprobs: bool = False
    top_logprobs: int = 0
    seed: Optional[int] = None
    # index of this request's first candidate when its n candidates are split across engines
    # (EngineGroup): candidate i draws with seed*1000003 + seed_offset + i on whichever GPU runs it
    seed_offset: int = 0
    logit_bias: Optional[Dict[int, float]] = None
    # constrained decoding (engine/constraints.py TokenConstraint): .start() / .advance(state, token) /
    # .is_done(state) / .mask_entry(state)
    constraint: Optional[object] = None

    @property
    def uses_penalties(self) -> bool:
        return self.frequency_penalty != 0.0 or self.presence_penalty != 0.0 or self.repetition_penalty != 1.0

    def validate(self, vocab_size: int) -> None:
        if not (0.0 <= self.temperature <= 2.0):
            raise ValueError(f"temperature must be between 0 and 2: {self.temperature}")
        if not (0.0 <= self.top_p <= 1.0):
            raise ValueError(f"top_p must be between 0 and 1: {self.top_p}")
        if not (0 <= self.top_logprobs <= 20):
            raise ValueError(f"top_logprobs must be between 0 and 20: {self.top_logprobs}")
        if self.logit_bias:
            for k, v in self.logit_bias.items():
                if not (0 <= int(k) < vocab_size):
                    raise ValueError(f"logit_bias token out of range: {k}")
                if not (-100 <= v <= 100):
                    raise ValueError(f"logit_bias values must be between -100 and 100: {v}")
