"""Embeddings service: OpenAI-compatible `/embeddings` on the local BGE encoder.

Produces the reference's `CreateEmbeddingResponse` (src/embeddings/response.rs:4-30).  Texts are
tokenized with the model's own tokenizer.json when the spec names one (WordPiece [CLS] ... [SEP]), else
byte-tokenized into the encoder vocabulary (no tokenizer downloads here), packed varlen (no padding
FLOPs) and run through the gfx950 encoder kernels on a dedicated HIP stream so embedding work can
overlap the decode engine on the same GPU.  Embeddings are kept in an HBM-resident, content-addressed
archive (`archive/hbm.py`, ``LWC_EMBED_CACHE_MB``): a text the encoder has already seen on this GPU is
gathered from the slab instead of re-encoded.
"""
from __future__ import annotations

import os
import threading
from typing import List, Optional, Sequence, Tuple, Union

import torch

from ..archive.hbm import ResidentEmbeddings
from ..schema import chat as C
from ..schema import score as S


class EmbeddingService:
    def __init__(self, encoder, name: str, cache_mb: Optional[float] = None, tokenizer=None):
        self.encoder = encoder
        self.name = name
        self.tokenizer = tokenizer
        self.lock = threading.Lock()
        self.stream = torch.cuda.Stream(device=encoder.device) if encoder.device.type == "cuda" else None
        if cache_mb is None:
            cache_mb = float(os.environ.get("LWC_EMBED_CACHE_MB", "4096" if self.stream is not None else "64"))
        self.cache = (ResidentEmbeddings(encoder.cfg.hidden, encoder.device, int(cache_mb * 2**20))
                      if cache_mb > 0 else None)

    def _encode(self, lists: Sequence[Sequence[int]], max_tokens: int) -> torch.Tensor:
        if self.stream is not None:
            with torch.cuda.stream(self.stream):
                f32, _ = self.encoder.embed(lists, max_tokens)
            self.stream.synchronize()
            return f32
        return self.encoder.embed(lists, max_tokens)[0]

    def tokenize(self, text: str) -> List[int]:
        dec = getattr(self.encoder, "model", None)  # decoder-as-embedder: the pooled last token is EOS
        if dec is not None:
            bos, eos = dec.cfg.bos_token_id, dec.cfg.eos_token_id
            V = dec.cfg.vocab_size
            body = (self.tokenizer.encode_with_specials(text) if self.tokenizer is not None
                    else ([bos if bos is not None else V - 2] + list(text.encode("utf-8"))))
            return body + [eos if eos is not None else V - 1]
        if self.tokenizer is not None:
            return self.tokenizer.encode_with_specials(text)
        V = self.encoder.cfg.vocab_size
        return [101] + [(b % (V - 1000)) + 1000 for b in text.encode("utf-8")] + [102]  # [CLS] ... [SEP]

    def embed_token_lists(self, lists: Sequence[Sequence[int]], max_tokens: int = 512) -> Tuple[torch.Tensor, int]:
        with self.lock:
            if self.cache is not None:
                f32, _ = self.cache.embed_through(lists, max_tokens, lambda miss: self._encode(miss, max_tokens))
            else:
                f32 = self._encode(lists, max_tokens)
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


def build_embedding_service(name: str, spec: dict, dev) -> "EmbeddingService":
    """An embedding model from a server spec ({"arch", "weights": "random:<seed>" | path, "tokenizer",
    "max_tokens", "fp8"}) on ``dev``: BERT/BGE encoders, or a decoder arch as a last-token-pooling embedder
    (e5-mistral).  Used by the server front end and by EngineGroup workers (candidates embedded on the
    GPU that generated them)."""
    import torch

    from ..engine.tokenizer import HFTokenizer
    from ..models.bert import BertEncoder
    from ..models.config import DECODERS, decoder_config, encoder_config

    w = spec.get("weights", "random:0")
    path, seed = (None, int(w.split(":", 1)[1])) if str(w).startswith("random:") else (w, 0)
    dev = torch.device(dev)
    if spec["arch"] in DECODERS:  # decoder-as-embedder (e5-mistral): last-token pooling
        if dev.type == "cpu":
            raise ValueError(f"embedding model {name}: decoder embedders need an MI355X")
        from ..models.embedder import DecoderEmbedder
        from ..models.llama import LlamaModel

        dcfg = decoder_config(spec["arch"])
        mtok = int(spec.get("max_tokens", 4096))
        enc = DecoderEmbedder(LlamaModel(dcfg, device=dev, seed=seed, weights_path=path, max_position=mtok + 64,
                                         fp8_dense=bool(spec.get("fp8", False)), fold_norms=False),
                              max_tokens=mtok)
    else:
        enc = BertEncoder(encoder_config(spec["arch"]), device=dev, seed=seed, weights_path=path,
                          dtype=torch.float32 if dev.type == "cpu" else torch.bfloat16)
    tok = HFTokenizer(spec["tokenizer"]) if spec.get("tokenizer") else None
    return EmbeddingService(enc, name, tokenizer=tok)
