"""Model architecture configs (public shapes, random-init or safetensors weights).

Shapes come from the public model configs named in SURVEY.md §2.3 (not from the reference, which
runs no model): Llama-3-8B, Mixtral-8x7B, Mistral-7B/e5-mistral-7b and the bge-* BERT encoders.
Small variants exist for tests.
"""
from __future__ import annotations

from dataclasses import dataclass, replace
from typing import Optional


@dataclass(frozen=True)
class DecoderConfig:
    name: str
    vocab_size: int
    hidden: int
    layers: int
    heads: int
    kv_heads: int
    head_dim: int
    ffn: int
    rope_theta: float = 500000.0
    rms_eps: float = 1e-5
    max_position: int = 8192
    # llama-3 style rope scaling (factor, low_freq_factor, high_freq_factor, original_max_position)
    rope_scaling: Optional[tuple] = None
    # mixture of experts (Mixtral): experts per layer and experts per token; 0 = dense
    num_experts: int = 0
    experts_per_token: int = 0
    tie_embeddings: bool = False
    bos_token_id: int = 1
    eos_token_id: int = 2

    @property
    def qkv_dim(self) -> int:
        return (self.heads + 2 * self.kv_heads) * self.head_dim

    def params(self) -> int:
        d, f = self.hidden, self.ffn
        attn = d * self.qkv_dim + self.heads * self.head_dim * d
        mlp = 3 * d * f * max(1, self.num_experts) + (d * self.num_experts if self.num_experts else 0)
        emb = self.vocab_size * d * (1 if self.tie_embeddings else 2)
        return self.layers * (attn + mlp + 2 * d) + emb + d


@dataclass(frozen=True)
class EncoderConfig:
    name: str
    vocab_size: int
    hidden: int
    layers: int
    heads: int
    ffn: int
    max_position: int = 512
    type_vocab: int = 2
    ln_eps: float = 1e-12
    pooling: str = "cls"  # cls | mean | last

    @property
    def head_dim(self) -> int:
        return self.hidden // self.heads


DECODERS = {
    "llama-3-8b": DecoderConfig("llama-3-8b", 128256, 4096, 32, 32, 8, 128, 14336, rope_theta=500000.0,
                                rms_eps=1e-5, max_position=8192, rope_scaling=(8.0, 1.0, 4.0, 8192),
                                bos_token_id=128000, eos_token_id=128001),
    "mistral-7b": DecoderConfig("mistral-7b", 32000, 4096, 32, 32, 8, 128, 14336, rope_theta=10000.0, rms_eps=1e-5,
                                max_position=32768),
    "mixtral-8x7b": DecoderConfig("mixtral-8x7b", 32000, 4096, 32, 32, 8, 128, 14336, rope_theta=1e6, rms_eps=1e-5,
                                  max_position=32768, num_experts=8, experts_per_token=2),
    # e5-mistral-7b-instruct: Mistral-7B decoder used as an embedder (last-token pooling, 4096-d)
    "e5-mistral-7b": DecoderConfig("e5-mistral-7b", 32000, 4096, 32, 32, 8, 128, 14336, rope_theta=10000.0,
                                   rms_eps=1e-5, max_position=32768),
    # tests / smoke: same code paths, tiny sizes
    "llama-tiny": DecoderConfig("llama-tiny", 4096, 512, 2, 8, 2, 128, 1024, rope_theta=500000.0, max_position=2048,
                                bos_token_id=1, eos_token_id=2),
    "mixtral-tiny": DecoderConfig("mixtral-tiny", 4096, 512, 2, 8, 2, 128, 512, rope_theta=1e6, max_position=2048,
                                  num_experts=4, experts_per_token=2),
}

ENCODERS = {
    "bge-small-en-v1.5": EncoderConfig("bge-small-en-v1.5", 30522, 384, 12, 12, 1536),
    "bge-base-en-v1.5": EncoderConfig("bge-base-en-v1.5", 30522, 768, 12, 12, 3072),
    "bge-large-en-v1.5": EncoderConfig("bge-large-en-v1.5", 30522, 1024, 24, 16, 4096),
    "bert-tiny": EncoderConfig("bert-tiny", 30522, 256, 2, 4, 1024),
}


def decoder_config(name: str, **overrides) -> DecoderConfig:
    cfg = DECODERS[name]
    return replace(cfg, **overrides) if overrides else cfg


def encoder_config(name: str, **overrides) -> EncoderConfig:
    key = name.split("/")[-1].lower()
    if key.startswith("bge-") and not key.endswith("-v1.5") and key + "-en-v1.5" in ENCODERS:
        key = key + "-en-v1.5"
    cfg = ENCODERS[key]
    return replace(cfg, **overrides) if overrides else cfg
