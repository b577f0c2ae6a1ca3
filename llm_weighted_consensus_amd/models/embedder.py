"""Decoder-as-embedder (e5-mistral-7b style, BASELINE config 5's embedder): the last token's final hidden
state of a causal decoder, L2-normalised (4096-d for Mistral-7B shapes).

Runs the same gfx950 kernel set as generation (`LlamaModel.encode`: cache-less prefill path, varlen
causal flash attention, fused RMSNorm/RoPE/SwiGLU) and pools with the K9d pool_l2norm kernel in LAST
mode.  It exposes the `embed(token_lists, max_tokens)` interface of `BertEncoder`, so the embeddings
service, the consensus scorer and the training-table weights use either encoder family.
"""
from __future__ import annotations

from typing import Optional, Sequence

import torch

from .. import ops
from .config import DecoderConfig
from .packing import pack_ids


class DecoderEmbedder:
    def __init__(self, model, max_tokens: int = 4096):
        self.model = model
        self.device = model.device
        self.max_tokens = max_tokens
        cfg: DecoderConfig = model.cfg
        # the embeddings service reads these like an EncoderConfig
        self.cfg = type("EmbedCfg", (), {"vocab_size": cfg.vocab_size, "max_position": max_tokens,
                                         "hidden": cfg.hidden, "pooling": "last", "name": cfg.name})()

    def pack(self, token_lists: Sequence[Sequence[int]], max_tokens: Optional[int] = None):
        """Varlen packing keeping each sequence's END (the last token is pooled), numpy-vectorised
        (models/packing.py)."""
        cap = min(max_tokens or self.max_tokens, self.max_tokens)
        ids, pos, cu, max_len = pack_ids(token_lists, cap, self.cfg.vocab_size, tail=True)
        dev = self.device
        return (torch.from_numpy(ids).to(dev), torch.from_numpy(pos).to(dev), torch.from_numpy(cu).to(dev), max_len)

    def embed(self, token_lists: Sequence[Sequence[int]], max_tokens: Optional[int] = None):
        """-> (unit f32 [n, d], unit bf16 [n, d])"""
        ids, pos, cu, max_len = self.pack(token_lists, max_tokens)
        # only each sequence's last token is pooled: the last layer's o projection, MLP and the final norm run
        # on those rows alone (LlamaModel._layers ``keep``)
        last = (cu[1:] - 1).long()
        h = self.model.encode(ids, pos, cu, max_len, keep=last)
        rows = torch.arange(h.shape[0] + 1, dtype=cu.dtype, device=cu.device)
        return ops.pool_l2norm(h, rows, ops.POOL_LAST)
