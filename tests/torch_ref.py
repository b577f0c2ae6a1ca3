"""Plain-PyTorch fp32 references for the HIP kernels (numerics oracles for the GPU tests)."""
from __future__ import annotations

import math

import torch
import torch.nn.functional as F


def rmsnorm(x, w, eps):
    x = x.float()
    return x * torch.rsqrt(x.pow(2).mean(-1, keepdim=True) + eps) * w.float()


def layernorm(x, g, b, eps):
    return F.layer_norm(x.float(), (x.shape[-1],), g.float(), b.float(), eps)


def rope(x, pos, cos, sin):
    """rotate-half RoPE; x [T, H, D]; cos/sin [maxpos, D/2]."""
    x = x.float()
    half = x.shape[-1] // 2
    c = cos[pos.long()].unsqueeze(1)
    s = sin[pos.long()].unsqueeze(1)
    x1, x2 = x[..., :half], x[..., half:]
    return torch.cat([x1 * c - x2 * s, x2 * c + x1 * s], dim=-1)


def attention(q, k, v, causal, scale):
    """q [Tq, Hq, D], k/v [Tk, Hkv, D] fp32 single sequence; GQA by repeat."""
    Hq, Hkv = q.shape[1], k.shape[1]
    k = k.repeat_interleave(Hq // Hkv, dim=1)
    v = v.repeat_interleave(Hq // Hkv, dim=1)
    s = torch.einsum("qhd,khd->hqk", q.float(), k.float()) * scale
    if causal:
        Tq, Tk = q.shape[0], k.shape[0]
        mask = torch.ones(Tq, Tk, dtype=torch.bool, device=q.device).tril(Tk - Tq)
        s = s.masked_fill(~mask, float("-inf"))
    p = s.softmax(-1)
    return torch.einsum("hqk,khd->qhd", p, v.float())


def llama_forward(model, tokens):
    """Full-sequence fp32 forward of a models.llama.LlamaModel (single sequence) -> logits [T, V]."""
    cfg = model.cfg
    T = tokens.shape[0]
    Hq, Hkv, D = cfg.heads, cfg.kv_heads, cfg.head_dim
    pos = torch.arange(T, device=tokens.device)
    x = model.embed[tokens.long()].float()
    for L in model.layers:
        h = rmsnorm(x, L.attn_norm, cfg.rms_eps)
        qkv = h @ L.wqkv.float().t()
        q = qkv[:, : Hq * D].view(T, Hq, D)
        k = qkv[:, Hq * D:(Hq + Hkv) * D].view(T, Hkv, D)
        v = qkv[:, (Hq + Hkv) * D:].view(T, Hkv, D)
        q = rope(q, pos, model.cos, model.sin)
        k = rope(k, pos, model.cos, model.sin)
        a = attention(q, k, v, True, 1.0 / math.sqrt(D)).reshape(T, Hq * D)
        x = x + a @ L.wo.float().t()
        h = rmsnorm(x, L.mlp_norm, cfg.rms_eps)
        gu = h @ L.w_gate_up.float().t()
        g, u = gu.chunk(2, dim=-1)
        x = x + (F.silu(g) * u) @ L.w_down.float().t()
    h = rmsnorm(x, model.final_norm, cfg.rms_eps)
    return h @ model.lm_head.float().t()
