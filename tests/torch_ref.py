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


def dense(w):
    """fp32 view of a projection weight (bf16 tensor, or an ops.Fp8Weight dequantised: q * s)."""
    if hasattr(w, "q") and hasattr(w, "s"):
        return w.q.float() * w.s.view(-1, 1)
    return w.float()


def llama_forward(model, tokens, hidden_only=False):
    """Full-sequence fp32 forward of a models.llama.LlamaModel (single sequence) -> logits [T, V]."""
    cfg = model.cfg
    T = tokens.shape[0]
    Hq, Hkv, D = cfg.heads, cfg.kv_heads, cfg.head_dim
    pos = torch.arange(T, device=tokens.device)
    x = model.embed[tokens.long()].float()
    for L in model.layers:
        h = rmsnorm(x, L.attn_norm, cfg.rms_eps)
        qkv = h @ dense(L.wqkv).t()
        q = qkv[:, : Hq * D].view(T, Hq, D)
        k = qkv[:, Hq * D:(Hq + Hkv) * D].view(T, Hkv, D)
        v = qkv[:, (Hq + Hkv) * D:].view(T, Hkv, D)
        q = rope(q, pos, model.cos, model.sin)
        k = rope(k, pos, model.cos, model.sin)
        a = attention(q, k, v, True, 1.0 / math.sqrt(D)).reshape(T, Hq * D)
        x = x + a @ dense(L.wo).t()
        h = rmsnorm(x, L.mlp_norm, cfg.rms_eps)
        if hasattr(L, "router"):
            x = x + moe_mlp(model, L, h)
        else:
            gu = h @ dense(L.w_gate_up).t()
            if getattr(L, "gu_block", 0):  # gate/up rows interleaved in blocks (ops.swiglu_interleave)
                gu = gu.view(gu.shape[0], -1, 2, L.gu_block)
                g, u = gu[:, :, 0].reshape(gu.shape[0], -1), gu[:, :, 1].reshape(gu.shape[0], -1)
            else:
                g, u = gu.chunk(2, dim=-1)
            x = x + (F.silu(g) * u) @ dense(L.w_down).t()
    h = rmsnorm(x, model.final_norm, cfg.rms_eps)
    if hidden_only:
        return h
    return h @ model.lm_head.float().t()


def llama_hidden(model, tokens):
    """Final RMS-normed hidden states [T, d] (fp32) of the reference forward."""
    return llama_forward(model, tokens, hidden_only=True)


def moe_mlp(model, L, h):
    """fp32 Mixtral MoE MLP (TP=1 weights; fp8 experts dequantised with their per-channel scales)."""
    k = model.full_cfg.experts_per_token
    logits = h @ L.router.float().t()
    top, ids = logits.topk(k, dim=-1)
    w = top.softmax(-1)
    w13 = L.w13.float() * (L.s13.unsqueeze(-1) if L.s13 is not None else 1.0)
    w2 = L.w2.float() * (L.s2.unsqueeze(-1) if L.s2 is not None else 1.0)
    out = torch.zeros_like(h)
    for t in range(h.shape[0]):
        for j in range(k):
            e = int(ids[t, j])
            gu = h[t] @ w13[e].t()
            if getattr(L, "gu_block", 0):
                gu = gu.view(-1, 2, L.gu_block)
                g, u = gu[:, 0].reshape(-1), gu[:, 1].reshape(-1)
            else:
                g, u = gu.chunk(2)
            out[t] += w[t, j] * ((F.silu(g) * u) @ w2[e].t())
    return out
