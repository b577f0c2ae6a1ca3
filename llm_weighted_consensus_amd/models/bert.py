"""BERT/BGE-style encoder (bge-small/base/large shapes) for embeddings on the gfx950 kernel set.

Serves the reference's embeddings capability (`CreateEmbeddingResponse`, src/embeddings/response.rs:1-30,
carried in training-table weight data src/score/completions/weight.rs:15-18) and the embedding
consensus scorer.  Sequences are packed (cu_seqlens) — no padding FLOPs:

    x   = LN(word[ids] + (pos + type0)[pos])          K7 gathers + K9a LN (+residual)
    per layer (post-norm):
      qkv = x Wqkv^T + b                               hipBLASLt (fused q|k|v)
      a   = varlen bidirectional flash attention       K9c (MFMA, LDS-tiled QK^T)
      x   = LN(x + a Wo^T + bo)                         K9a fused residual
      h   = gelu(x W1^T + b1)                          GEMM with the bias + GELU in its epilogue (K9b)
      x   = LN(x + h W2^T + b2)
    e   = L2norm(pool(x))                               K9d (CLS for bge)

On a CPU device the same weights run through :meth:`BertEncoder.forward_reference` (plain fp32
PyTorch): that is BASELINE config 1 ("bge-small embeddings + cosine score on CPU, plumbing, no GPU")
and the numerics oracle of the GPU tests — it is selected by the device, never as a fallback for a
GPU whose kernels failed to load.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass
from typing import Optional, Sequence

import torch
import torch.nn.functional as F

from .. import ops
from ..ops import gemm_plan
from .config import EncoderConfig
from .packing import pack_ids

POOL_MODES = {"cls": ops.POOL_CLS, "mean": ops.POOL_MEAN, "last": ops.POOL_LAST}


@dataclass
class EncLayer:
    wqkv: torch.Tensor
    bqkv: torch.Tensor
    wo: torch.Tensor
    bo: torch.Tensor
    ln1_g: torch.Tensor
    ln1_b: torch.Tensor
    w1: torch.Tensor
    b1: torch.Tensor
    w2: torch.Tensor
    b2: torch.Tensor
    ln2_g: torch.Tensor
    ln2_b: torch.Tensor


class BertEncoder:
    def __init__(self, cfg: EncoderConfig, device="cuda", dtype=torch.bfloat16, seed: int = 0,
                 weights_path: Optional[str] = None):
        if cfg.head_dim not in (32, 64, 128):
            raise NotImplementedError(f"encoder head_dim {cfg.head_dim} (attention kernel supports 32/64/128)")
        self.cfg, self.device, self.dtype = cfg, torch.device(device), dtype
        if weights_path:
            self._load(weights_path)
        else:
            self._random_init(seed)
        self.scale = 1.0 / math.sqrt(cfg.head_dim)
        self.fused_residual = os.environ.get("LWC_ENC_FUSED_RESIDUAL", "ffn2")

    def _random_init(self, seed: int) -> None:
        c, dev, dt = self.cfg, self.device, self.dtype
        g = torch.Generator(device=dev)
        g.manual_seed(seed + 7)

        def rnd(*shape, s=0.02):
            return (torch.randn(*shape, generator=g, device=dev) * s).to(dt)
        # NOTE: the same seed gives different weights on CPU and GPU generators; tests that compare
        # the two paths build one model and move it with :meth:`to`.

        zeros = lambda *s: torch.zeros(*s, device=dev, dtype=dt)
        ones = lambda *s: torch.ones(*s, device=dev, dtype=dt)
        d, f = c.hidden, c.ffn
        self.word = rnd(c.vocab_size, d)
        pos = rnd(c.max_position, d)
        typ = rnd(c.type_vocab, d)
        self.pos_type = (pos.float() + typ[0].float()).to(dt).contiguous()
        self.emb_ln_g, self.emb_ln_b = ones(d), zeros(d)
        self.layers = [EncLayer(rnd(3 * d, d), zeros(3 * d), rnd(d, d), zeros(d), ones(d), zeros(d), rnd(f, d),
                                zeros(f), rnd(d, f), zeros(d), ones(d), zeros(d)) for _ in range(c.layers)]

    def _load(self, path: str) -> None:  # HF BertModel safetensors layout
        from safetensors.torch import load_file

        sd = load_file(path, device="cpu")
        dev, dt = self.device, self.dtype
        pre = "bert." if any(k.startswith("bert.") for k in sd) else ""
        t = lambda n: sd[pre + n].to(device=dev, dtype=dt).contiguous()
        self.word = t("embeddings.word_embeddings.weight")
        self.pos_type = (t("embeddings.position_embeddings.weight").float()
                         + t("embeddings.token_type_embeddings.weight")[0].float()).to(dt).contiguous()
        self.emb_ln_g, self.emb_ln_b = t("embeddings.LayerNorm.weight"), t("embeddings.LayerNorm.bias")
        self.layers = []
        for i in range(self.cfg.layers):
            p = f"encoder.layer.{i}."
            qkv_w = torch.cat([t(p + f"attention.self.{n}.weight") for n in ("query", "key", "value")])
            qkv_b = torch.cat([t(p + f"attention.self.{n}.bias") for n in ("query", "key", "value")])
            self.layers.append(EncLayer(
                qkv_w.contiguous(), qkv_b.contiguous(), t(p + "attention.output.dense.weight"),
                t(p + "attention.output.dense.bias"), t(p + "attention.output.LayerNorm.weight"),
                t(p + "attention.output.LayerNorm.bias"), t(p + "intermediate.dense.weight"),
                t(p + "intermediate.dense.bias"), t(p + "output.dense.weight"), t(p + "output.dense.bias"),
                t(p + "output.LayerNorm.weight"), t(p + "output.LayerNorm.bias")))

    def forward_reference(self, ids: torch.Tensor, positions: torch.Tensor, cu: torch.Tensor) -> torch.Tensor:
        """Plain fp32 PyTorch forward of the same packed batch -> hidden [T, d] f32 (CPU path / oracle)."""
        c = self.cfg
        H, Dh, d = c.heads, c.head_dim, c.hidden
        f32 = lambda t: t.float()
        x = F.layer_norm(f32(self.word)[ids.long()] + f32(self.pos_type)[positions.long()], (d,),
                         f32(self.emb_ln_g), f32(self.emb_ln_b), c.ln_eps)
        bounds = cu.tolist()
        for L in self.layers:
            qkv = x @ f32(L.wqkv).t() + f32(L.bqkv)
            a = torch.empty(x.shape[0], d, dtype=torch.float32, device=x.device)
            for i in range(len(bounds) - 1):
                s0, s1 = bounds[i], bounds[i + 1]
                q = qkv[s0:s1, :d].view(-1, H, Dh)
                k = qkv[s0:s1, d:2 * d].view(-1, H, Dh)
                v = qkv[s0:s1, 2 * d:].view(-1, H, Dh)
                p = (torch.einsum("qhd,khd->hqk", q, k) * self.scale).softmax(-1)
                a[s0:s1] = torch.einsum("hqk,khd->qhd", p, v).reshape(-1, d)
            x = F.layer_norm(x + a @ f32(L.wo).t() + f32(L.bo), (d,), f32(L.ln1_g), f32(L.ln1_b), c.ln_eps)
            h = F.gelu(x @ f32(L.w1).t() + f32(L.b1))
            x = F.layer_norm(x + h @ f32(L.w2).t() + f32(L.b2), (d,), f32(L.ln2_g), f32(L.ln2_b), c.ln_eps)
        return x

    @staticmethod
    def pool_reference(h: torch.Tensor, cu: torch.Tensor, mode: str) -> torch.Tensor:
        b = cu.tolist()
        rows = []
        for i in range(len(b) - 1):
            seg = h[b[i]:b[i + 1]].float()
            rows.append(seg[0] if mode == "cls" else seg[-1] if mode == "last" else seg.mean(0))
        return F.normalize(torch.stack(rows), dim=-1)

    def forward_packed(self, ids: torch.Tensor, positions: torch.Tensor, cu: torch.Tensor, max_len: int) -> torch.Tensor:
        """ids/positions [T] int32, cu [n+1] int32 -> hidden [T, d] bf16 (HIP kernels; CPU device:
        the fp32 reference)."""
        if self.device.type == "cpu":
            return self.forward_reference(ids, positions, cu)
        c = self.cfg
        H, Dh, d = c.heads, c.head_dim, c.hidden
        T = ids.shape[0]
        x = ops.layernorm(ops.embedding(self.word, ids), self.emb_ln_g, self.emb_ln_b, c.ln_eps,
                          residual=ops.embedding(self.pos_type, positions))
        lin = gemm_plan.linear_bias  # bias (+ GELU) in the GEMM epilogue (gemm8p) or hipBLASLt, per shape
        # post-LN residual: a projection whose GEMM adds its product into the stream x (residual epilogue) hands
        # its bias to the LayerNorm that follows as a pre-norm bias, in place: the norm reads one [T, d] tensor
        # instead of the projection output and the stream.  LWC_ENC_FUSED_RESIDUAL: "ffn2" (default) for FFN2
        # only, "all" for o too, "0" for neither.  Measured (bge-base, 0.5 M tokens): hipBLASLt's beta = 1 GEMM
        # reads the stream under FFN2's K = 3072 loop almost free (+29 us vs the bias GEMM, the norm -134 us)
        # but not under o's K = 768 (+119 us): profiles/round6_ab.md
        mode = self.fused_residual if d <= 1024 else "0"
        fuse_o, fuse_f = mode == "all", mode in ("all", "ffn2")
        for L in self.layers:
            qkv = lin(x, L.wqkv, L.bqkv)
            a = ops.prefill_attention(qkv[:, :d], qkv[:, d:2 * d], qkv[:, 2 * d:], cu, max_len, H, H, Dh, self.scale,
                                      causal=False)
            if fuse_o:
                gemm_plan.linear_residual_(a, L.wo, x)
                ops.layernorm(x, L.ln1_g, L.ln1_b, c.ln_eps, out=x, pre_bias=L.bo)
            else:
                x = ops.layernorm(lin(a, L.wo, L.bo), L.ln1_g, L.ln1_b, c.ln_eps, residual=x)
            h = lin(x, L.w1, L.b1, gelu=True)
            if fuse_f:
                gemm_plan.linear_residual_(h, L.w2, x)
                ops.layernorm(x, L.ln2_g, L.ln2_b, c.ln_eps, out=x, pre_bias=L.b2)
            else:
                x = ops.layernorm(lin(h, L.w2, L.b2), L.ln2_g, L.ln2_b, c.ln_eps, residual=x)
        return x

    def to(self, device, dtype=None) -> "BertEncoder":
        """Copy of this encoder on another device (e.g. a GPU model's weights on CPU for the oracle)."""
        out = BertEncoder.__new__(BertEncoder)
        out.cfg, out.device, out.scale = self.cfg, torch.device(device), self.scale
        out.fused_residual = self.fused_residual
        out.dtype = dtype or self.dtype
        mv = lambda t: t.to(device=device, dtype=out.dtype)
        out.word, out.pos_type, out.emb_ln_g, out.emb_ln_b = (mv(self.word), mv(self.pos_type), mv(self.emb_ln_g),
                                                             mv(self.emb_ln_b))
        out.layers = [EncLayer(*[mv(getattr(L, f)) for f in EncLayer.__dataclass_fields__]) for L in self.layers]
        return out

    def pack(self, token_lists: Sequence[Sequence[int]], max_tokens: Optional[int] = None):
        """Varlen packing (ids folded into the vocab, truncated at max_tokens, empty -> [0]) with numpy
        (models/packing.py): thousands of candidates per consensus batch must not cost per-token Python work."""
        cap = min(max_tokens or self.cfg.max_position, self.cfg.max_position)
        ids, pos, cu, max_len = pack_ids(token_lists, cap, self.cfg.vocab_size)
        dev = self.device
        return (torch.from_numpy(ids).to(dev), torch.from_numpy(pos).to(dev), torch.from_numpy(cu).to(dev), max_len)

    def embed(self, token_lists: Sequence[Sequence[int]], max_tokens: Optional[int] = None):
        """Embed sequences (token ids in this encoder's vocab; ids are folded into range) ->
        (unit f32 [n, d], unit bf16 [n, d])."""
        ids, pos, cu, max_len = self.pack(token_lists, max_tokens)
        return self.embed_packed(ids, pos, cu, max_len)

    def embed_packed(self, ids, pos, cu, max_len):
        h = self.forward_packed(ids, pos, cu, max_len)
        if self.device.type == "cpu":
            e = self.pool_reference(h, cu, self.cfg.pooling)
            return e, e.to(torch.bfloat16)
        return ops.pool_l2norm(h, cu, POOL_MODES[self.cfg.pooling])
