"""Embeddings service: OpenAI-compatible `/embeddings` on the local BGE encoder.

Produces the reference's `CreateEmbeddingResponse` (src/embeddings/response.rs:4-30).  Texts are
byte-tokenized into the encoder vocabulary (no tokenizer downloads here), packed varlen (no padding
FLOPs) and run through the gfx950 encoder kernels on a dedicated HIP stream so embedding work can
overlap the decode engine on the same GPU.
"""
from __future__ import annotations

import threading
from typing import List, Sequence, Tuple, Union

import torch

from ..schema import chat as C
from ..schema import score as S


class EmbeddingService:
    def __init__(self, encoder, name: str):
        self.encoder = encoder
        self.name = name
        self.lock = threading.Lock()
        self.stream = torch.cuda.Stream(device=encoder.device) if encoder.device.type == "cuda" else None

    def tokenize(self, text: str) -> List[int]:
        V = self.encoder.cfg.vocab_size
        return [101] + [(b % (V - 1000)) + 1000 for b in text.encode("utf-8")] + [102]  # [CLS] ... [SEP]

    def embed_token_lists(self, lists: Sequence[Sequence[int]], max_tokens: int = 512) -> Tuple[torch.Tensor, int]:
        with self.lock:
            if self.stream is not None:
                with torch.cuda.stream(self.stream):
                    f32, _ = self.encoder.embed(lists, max_tokens)
                self.stream.synchronize()
            else:
                f32, _ = self.encoder.embed(lists, max_tokens)
        ntok = sum(min(len(l), max_tokens, self.encoder.cfg.max_position) for l in lists)
        return f32, ntok

    def embed_texts(self, texts: Sequence[str], max_tokens: int = 512) -> Tuple[torch.Tensor, int]:
        return self.embed_token_lists([self.tokenize(t) for t in texts], max_tokens)

    def create(self, inputs: Union[str, List[str], List[int], List[List[int]]], max_tokens: int = 512) -> S.CreateEmbeddingResponse:
        if isinstance(inputs, str):
            f32, ntok = self.embed_texts([inputs], max_tokens)
        elif inputs and isinstance(inputs[0], int):
            f32, ntok = self.embed_token_lists([inputs], max_tokens)
        elif inputs and isinstance(inputs[0], list):
            f32, ntok = self.embed_token_lists(inputs, max_tokens)
        else:
            f32, ntok = self.embed_texts(list(inputs), max_tokens)
        rows = f32.double().cpu().tolist()
        return S.CreateEmbeddingResponse(data=[S.EmbeddingItem(embedding=r, index=i) for i, r in enumerate(rows)],
                                         model=self.name, usage=C.Usage(prompt_tokens=ntok, total_tokens=ntok))
