"""Llama-family decoder (Llama-3 / Mistral shapes) on the gfx950 kernel set.

This is the local generation backend that replaces the reference's upstream providers
(reference: every voter is an OpenAI-compatible chat call, src/chat/completions/client.rs:308-332).

Per layer (decode, B sequences):
    rmsnorm                       K1
    qkv  = x @ Wqkv^T             K6 (fused q|k|v weight)
    rope + paged KV write         K2 (in place, one pass)
    attn = paged GQA decode       K3 (cascade for forked candidates, else split-K)
    x   += attn @ Wo^T            K6 with the residual add in its epilogue, then K1
    act  = silu(x Wg^T) (x Wu^T)  K6 with SwiGLU in its epilogue (fused gate|up weight), or GEMM + K5
    x   += act @ Wd^T             K6 + residual, then K1
K6 is chosen per shape by ops/gemm_plan.py among hipBLASLt and the hand-written cores (gemm4w, gemm8p),
timed on the device.

Folded RMSNorm (decode chain, dense bf16 on the GPU): every norm weight is folded into the projection that
reads it at load (W_qkv diag(g_attn), W_gate_up diag(g_mlp), W_lm_head diag(g_final); the norm weights become
ones, so the unfolded path computes the same function), and a decode step where the chain was timed faster
(:meth:`LlamaModel.tune_gemms`) runs NO norm kernel: the o / down projections' residual epilogues emit the
partial row sums of squares of the new residual stream, from which the next projection (qkv, gate|up,
lm_head) scales its accumulator rows by 1/rms (gemm4w RS modes, csrc/kernels/gemm4w.hip):
    ss = rms_rowsumsq(embedding)                  (once)
    qkv = gemm4w(x, W_qkv', ss)   ...   x += gemm4w(attn, W_o) -> ss
    act = gemm4w(x, W_gu', ss, SwiGLU)   x += gemm4w(act, W_d) -> ss     ...   logits = gemm4w(x, W_lm', ss)  Prefill uses the same layer with the varlen causal flash-attention kernel (K4) over
the fresh k/v of the qkv buffer; mixed chunked-prefill steps (forward_mixed) send decode rows to K3 and
prompt-chunk rows to K4's paged-KV mode; the k/v are scattered into the paged cache in the RoPE pass.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass
from pathlib import Path
from typing import Optional

import torch
import torch.nn.functional as F

from .. import ops
from ..ops import blas_tuning, gemm_plan
from .config import DecoderConfig


def rope_tables(cfg: DecoderConfig, device, max_pos: Optional[int] = None):
    """Host-built cos/sin tables [max_pos, D/2] f32 (Appendix B: no on-device trig), with the
    Llama-3 frequency scaling when configured."""
    D = cfg.head_dim
    max_pos = max_pos or cfg.max_position
    inv = 1.0 / (cfg.rope_theta ** (torch.arange(0, D, 2, dtype=torch.float64) / D))
    if cfg.rope_scaling is not None:
        factor, lo_f, hi_f, orig = cfg.rope_scaling
        lo_wl, hi_wl = orig / lo_f, orig / hi_f
        wl = 2 * math.pi / inv
        smooth = (orig / wl - lo_f) / (hi_f - lo_f)
        scaled = torch.where(wl > lo_wl, inv / factor, inv)
        mid = (wl <= lo_wl) & (wl >= hi_wl)
        scaled = torch.where(mid, (1 - smooth) * inv / factor + smooth * inv, scaled)
        inv = scaled
    t = torch.arange(max_pos, dtype=torch.float64)
    ang = torch.outer(t, inv)
    return ang.cos().float().to(device).contiguous(), ang.sin().float().to(device).contiguous()


@dataclass
class LayerWeights:
    attn_norm: torch.Tensor
    wqkv: torch.Tensor      # [(Hq+2Hkv)*D, d]
    wo: torch.Tensor        # [d, Hq*D]
    mlp_norm: torch.Tensor
    w_gate_up: torch.Tensor  # [2F, d]  rows: gate then up (gu_block 0) or interleaved in blocks of gu_block
    w_down: torch.Tensor    # [d, F]
    gu_block: int = 0


class KVCache:
    """One flat bf16 pool for all layers: [L, 2, num_blocks, Hkv*BS*D]; per-layer K view
    [NB, Hkv, BS, D] and 4-token-interleaved V view [NB, Hkv, BS/4, D, 4] (see attention_decode.hip)."""

    def __init__(self, cfg: DecoderConfig, num_blocks: int, block_size: int, device, dtype=torch.bfloat16):
        self.cfg, self.num_blocks, self.block_size = cfg, num_blocks, block_size
        self.block_elems = cfg.kv_heads * block_size * cfg.head_dim
        self.pool = torch.zeros(cfg.layers, 2, num_blocks, self.block_elems, dtype=dtype, device=device)
        Hkv, D = cfg.kv_heads, cfg.head_dim
        self.k = [self.pool[l, 0].view(num_blocks, Hkv, block_size, D) for l in range(cfg.layers)]
        self.v = [self.pool[l, 1].view(num_blocks, Hkv, block_size // 4, D, 4) for l in range(cfg.layers)]

    @staticmethod
    def bytes_per_block(cfg: DecoderConfig, block_size: int) -> int:
        return cfg.layers * 2 * cfg.kv_heads * block_size * cfg.head_dim * 2

    def copy_blocks(self, pairs: torch.Tensor) -> None:
        """Copy-on-write block copies (K12) for every layer, K and V."""
        if pairs.numel():
            ops.kv_block_copy(self.pool.view(self.cfg.layers * 2, self.num_blocks, self.block_elems), pairs)


class _NullCache:
    """Shape-only stand-in for KVCache when no KV is written (encode): one shared 1-block buffer."""

    def __init__(self, cfg: DecoderConfig, device):
        buf = torch.zeros(2, 1, cfg.kv_heads, 16, cfg.head_dim, dtype=torch.bfloat16, device=device)
        self.k = [buf[0]] * cfg.layers
        self.v = [buf[1].view(1, cfg.kv_heads, 4, cfg.head_dim, 4)] * cfg.layers


class LlamaModel:
    def __init__(self, cfg: DecoderConfig, device="cuda", dtype=torch.bfloat16, seed: int = 0,
                 weights_path: Optional[str] = None, max_position: Optional[int] = None, fp8_dense: bool = False,
                 fold_norms: bool = True):
        if cfg.num_experts and type(self) is LlamaModel:
            raise NotImplementedError("MoE decoders use models.mixtral.MixtralModel")
        self.cfg, self.device, self.dtype = cfg, torch.device(device), dtype
        self.cos, self.sin = rope_tables(cfg, self.device, max_position)
        if weights_path:
            self._load(weights_path)
        else:
            self._random_init(seed)
        self.scale = 1.0 / math.sqrt(cfg.head_dim)
        self.g8_ws = None
        # fp8 configurations (BASELINE config 5: the e5-mistral embedder): the qkv / o / gate|up / down
        # projections in e4m3 with per-channel scales, activations quantised per row; lm_head stays bf16
        self.fp8_dense = bool(fp8_dense) and self.device.type == "cuda"
        if self.fp8_dense:
            for L in self.layers:
                if isinstance(L, LayerWeights):
                    L.wqkv, L.wo = ops.Fp8Weight(L.wqkv), ops.Fp8Weight(L.wo)
                    if L.gu_block == 0 and L.w_gate_up.shape[0] % 64 == 0:
                        # gate|up interleaved in blocks of 32: gemm8g's epilogue applies the SwiGLU
                        L.w_gate_up, L.gu_block = ops.swiglu_interleave(L.w_gate_up), 32
                    L.w_gate_up, L.w_down = ops.Fp8Weight(L.w_gate_up), ops.Fp8Weight(L.w_down)
            torch.cuda.empty_cache()
        if self.device.type == "cuda":
            # gemm8p (ops/gemm_plan.py): the gate|up rows interleaved in blocks of 32 so its epilogue can
            # apply SwiGLU; a stream-K workspace owned by the model (never allocated inside a capture)
            for L in self.layers:
                if (isinstance(L, LayerWeights) and not self.fp8_dense and L.gu_block == 0
                        and L.w_gate_up.shape[0] % 64 == 0):
                    L.w_gate_up = ops.swiglu_interleave(L.w_gate_up)
                    L.gu_block = 32
            self.g8_ws = ops.new_gemm8p_workspace(self.device)
            blas_tuning.enable()  # offline-tuned library solutions: only with LWC_TUNED_BLAS=1 (off by default)
        # folded RMSNorm (module docstring): the plain dense bf16 decoder on the GPU
        self.norm_folded = False
        self.extra_bytes = 0  # device bytes the folded norms add (a tied lm_head's own copy)
        self.final_norm_weight: Optional[torch.Tensor] = None  # the final norm's weight once lm_head holds it
        self.chain: Optional[ops.NormChain] = None
        self.chain_m: dict = {}  # decode batch M -> (use the chain, qkv tile width)
        # ``fold_norms=False``: models that never decode through lm_head (the decoder-as-embedder) skip it
        if (fold_norms and self.device.type == "cuda" and not self.fp8_dense and type(self) is LlamaModel
                and os.environ.get("LWC_NORM_FOLD", "1") != "0" and isinstance(self.layers[0], LayerWeights)):
            self._fold_norms()

    def _fold_norms(self) -> None:
        """W diag(g) for every projection that reads a normalised row, then g = 1 (the unfolded path computes the
        same function).  One bf16 rounding of each folded weight (exact for the random-init unit norm weights).

        The final norm's weight is folded into lm_head only; :meth:`encode` (hidden states, no lm_head) keeps
        applying it (``final_norm_weight``).  A tied lm_head becomes its own vocab x hidden copy (W_emb diag(g)):
        ~1 GB more at Llama-3-8B shapes, reported by ``extra_bytes``."""
        def fold(w: torch.Tensor, g: torch.Tensor) -> torch.Tensor:
            out = torch.empty_like(w)
            gf = g.float()
            for r in range(0, w.shape[0], 8192):
                out[r:r + 8192] = (w[r:r + 8192].float() * gf).to(w.dtype)
            return out

        for L in self.layers:
            L.wqkv, L.attn_norm = fold(L.wqkv, L.attn_norm), torch.ones_like(L.attn_norm)
            L.w_gate_up, L.mlp_norm = fold(L.w_gate_up, L.mlp_norm), torch.ones_like(L.mlp_norm)
        tied = self.lm_head is self.embed
        self.lm_head = fold(self.lm_head, self.final_norm)  # (a tied embedding table keeps its own copy)
        self.extra_bytes = self.lm_head.numel() * self.lm_head.element_size() if tied else 0
        self.final_norm_weight = self.final_norm  # what encode() applies
        self.final_norm = torch.ones_like(self.final_norm)
        self.norm_folded = True
        torch.cuda.empty_cache()

    # ------------------------------------------------------------------ weights
    def _random_init(self, seed: int) -> None:
        cfg, dev, dt = self.cfg, self.device, self.dtype
        g = torch.Generator(device=dev)
        g.manual_seed(seed)
        std = 0.02

        def rnd(*shape, s=std):
            return (torch.randn(*shape, generator=g, device=dev, dtype=torch.float32) * s).to(dt)

        d, qkv, F_ = cfg.hidden, cfg.qkv_dim, cfg.ffn
        self.embed = rnd(cfg.vocab_size, d)
        self.layers = []
        out_std = std / math.sqrt(2 * cfg.layers)
        for _ in range(cfg.layers):
            self.layers.append(LayerWeights(
                attn_norm=torch.ones(d, device=dev, dtype=dt),
                wqkv=rnd(qkv, d),
                wo=rnd(d, cfg.heads * cfg.head_dim, s=out_std),
                mlp_norm=torch.ones(d, device=dev, dtype=dt),
                w_gate_up=rnd(2 * F_, d),
                w_down=rnd(d, F_, s=out_std),
            ))
        self.final_norm = torch.ones(d, device=dev, dtype=dt)
        self.lm_head = self.embed if cfg.tie_embeddings else rnd(cfg.vocab_size, d)

    def _load(self, path: str) -> None:
        """Load HF-layout safetensors (model.layers.N.self_attn.q_proj.weight ...) and fuse q|k|v and
        gate|up into the engine's layout."""
        from safetensors.torch import load_file

        files = sorted(Path(path).glob("*.safetensors")) if Path(path).is_dir() else [Path(path)]
        sd = {}
        for f in files:
            sd.update(load_file(str(f), device="cpu"))
        dev, dt = self.device, self.dtype

        def t(name):
            return sd[name].to(device=dev, dtype=dt).contiguous()

        self.embed = t("model.embed_tokens.weight")
        self.layers = []
        for i in range(self.cfg.layers):
            p = f"model.layers.{i}."
            self.layers.append(LayerWeights(
                attn_norm=t(p + "input_layernorm.weight"),
                wqkv=torch.cat([t(p + "self_attn.q_proj.weight"), t(p + "self_attn.k_proj.weight"),
                                t(p + "self_attn.v_proj.weight")]).contiguous(),
                wo=t(p + "self_attn.o_proj.weight"),
                mlp_norm=t(p + "post_attention_layernorm.weight"),
                w_gate_up=torch.cat([t(p + "mlp.gate_proj.weight"), t(p + "mlp.up_proj.weight")]).contiguous(),
                w_down=t(p + "mlp.down_proj.weight"),
            ))
        self.final_norm = t("model.norm.weight")
        self.lm_head = t("lm_head.weight") if "lm_head.weight" in sd else self.embed

    # ------------------------------------------------------------------ forward
    def _residual_into(self, inp: torch.Tensor, w: torch.Tensor, x_res: torch.Tensor, mode: str) -> None:
        """x_res += inp . w^T, leaving the partial row sums of squares of the new x_res in ``self.chain`` per
        ``mode``: "own32" / "own64" — gemm4w's residual epilogue writes them (RS 2, schedule 32 / 64);
        "sumsq" — the planner's residual GEMM, then one rms_rowsumsq pass; "plain" — no partials (the next
        consumer normalises with the norm kernel)."""
        if mode in ("own32", "own64"):
            ops.gemm4w(inp, w, residual=x_res, out=x_res, chain=self.chain, var=32 if mode == "own32" else 64)
            return
        gemm_plan.linear_add_(inp, w, x_res, ws=self.g8_ws)
        if mode == "sumsq":
            ops.rms_rowsumsq(x_res, self.chain)

    def _chain_layers(self, x_res: torch.Tensor, cache: KVCache, positions, slots, attn_fn, rope_q: bool,
                      plan: dict) -> torch.Tensor:
        """Decode layers + lm_head with the folded norms per ``plan`` (:meth:`_tune_chain`): at each norm point
        ("attn": qkv, "mlp": gate|up, "final": lm_head) either the consumer scales its rows from the chain's
        partials ("fold") or the norm kernel (weights ones: the norms are in the projections) runs first;
        the producers of folded points leave partials by ``plan["o"]`` / ``plan["down"]``.  Returns logits."""
        cfg, ch = self.cfg, self.chain
        T = x_res.shape[0]
        Hq, Hkv, D = cfg.heads, cfg.kv_heads, cfg.head_dim
        ones, eps = self.final_norm, cfg.rms_eps  # (every norm weight is ones after folding)
        if plan["attn"]:
            ops.rms_rowsumsq(x_res, ch)
        nl = len(self.layers)
        qv, gv, lv = plan.get("qkv_var", 32), plan.get("gu_var", 32), plan.get("lm_var", 32)
        for li, L in enumerate(self.layers):
            if plan["attn"]:
                qkv = ops.gemm4w(x_res, L.wqkv, bn=plan["qkv_bn"], chain=ch, var=qv)
            else:
                qkv = self._proj(ops.rmsnorm(x_res, ones, eps), L.wqkv)
            ops.rope_kv_write(qkv, positions, self.cos, self.sin, cache.k[li], cache.v[li], Hq, Hkv, D, slots=slots,
                              rope_q=rope_q)
            attn = attn_fn(qkv, li).reshape(T, Hq * D)
            self._residual_into(attn, L.wo, x_res, plan["o"] if plan["mlp"] else "plain")
            if plan["mlp"]:
                act = ops.gemm4w(x_res, L.w_gate_up, swiglu=True, chain=ch, var=gv)
            else:
                act = gemm_plan.swiglu(ops.rmsnorm(x_res, ones, eps), L.w_gate_up, L.gu_block, ws=self.g8_ws)
            nxt = plan["attn"] if li + 1 < nl else plan["final"]
            self._residual_into(act, L.w_down, x_res, plan["down"] if nxt else "plain")
        if plan["final"]:
            sk = ops.split_plan(T, self.lm_head.shape[0], cfg.hidden) if plan.get("lm_split") and lv == 64 else (1, 0)
            return ops.gemm4w(x_res, self.lm_head, chain=ch, var=lv, splits=sk[0], split_from=sk[1])
        return self._proj(ops.rmsnorm(x_res, ones, eps), self.lm_head)

    def chain_ok(self, M: int) -> bool:
        """Whether a decode step of M rows folds at least one norm (timed faster at M, before capture)."""
        c = self.chain_m.get(M)
        return bool(c and (c["attn"] or c["mlp"] or c["final"])) and self.chain is not None and M <= self.chain.max_rows

    def _layers(self, x_res: torch.Tensor, cache: KVCache, positions, slots, attn_fn, rope_q: bool = True,
                keep: Optional[torch.Tensor] = None, final_norm: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Runs every layer; x_res is the residual stream (updated in place); returns the final
        normalised hidden state.  ``rope_q=False``: q leaves the qkv projection un-rotated and ``attn_fn``
        rotates it (the decode kernels' load-time RoPE).  ``keep`` (row indices): only those rows' final
        states are wanted (a prefill's last tokens, an embedder's pooled token) — the last layer still runs
        qkv / RoPE / the cache write / attention over every row (later tokens' keys and values), then its
        o projection, MLP and the final norm over the kept rows only; returns [len(keep), d].  ``final_norm``:
        the weight of the last norm (default ``self.final_norm``; ones once it is folded into lm_head)."""
        cfg = self.cfg
        T = x_res.shape[0]
        Hq, Hkv, D = cfg.heads, cfg.kv_heads, cfg.head_dim
        # Dense single-rank layers add the o / down projections into the residual stream inside the GEMM
        # (gemm_plan.linear_add_), so the norms that follow only read x_res and write h.  Subclasses that
        # reduce the projections across ranks or route them through experts use the separate
        # residual-add + norm kernel.
        fused = self._dense_residual and self.g8_ws is not None
        # fp8 projections: the norms feeding them also emit the per-row e4m3 activation (ops.QAct) in the
        # same pass, so no separate quantisation kernel re-reads the normalised rows
        qn = isinstance(self.layers[0].wqkv, ops.Fp8Weight)
        if qn:
            h = ops.rmsnorm_quant_fp8(x_res, self.layers[0].attn_norm, cfg.rms_eps)
        else:
            h = ops.rmsnorm(x_res, self.layers[0].attn_norm, cfg.rms_eps)
        for li, L in enumerate(self.layers):
            qkv = self._proj(h, L.wqkv)
            ops.rope_kv_write(qkv, positions, self.cos, self.sin, cache.k[li], cache.v[li], Hq, Hkv, D, slots=slots,
                              rope_q=rope_q)
            attn = attn_fn(qkv, li)
            if keep is not None and li + 1 == len(self.layers):
                attn = attn.index_select(keep) if isinstance(attn, ops.MXAct) else \
                    attn.reshape(T, Hq * D).index_select(0, keep)
                x_res = x_res.index_select(0, keep)
                T = x_res.shape[0]
            nxt = (self.layers[li + 1].attn_norm if li + 1 < len(self.layers) else
                   self.final_norm if final_norm is None else final_norm)
            if fused:
                gemm_plan.linear_add_(attn.view(T, Hq * D), L.wo, x_res, ws=self.g8_ws)
                h = ops.rmsnorm(x_res, L.mlp_norm, cfg.rms_eps)
                gemm_plan.linear_add_(self._act(h, L), L.w_down, x_res, ws=self.g8_ws)
                h = ops.rmsnorm(x_res, nxt, cfg.rms_eps)
            elif qn:
                o = self._attn_out(attn if isinstance(attn, ops.MXAct) else attn.view(T, Hq * D), L)
                h = ops.rmsnorm_quant_fp8(o, L.mlp_norm, cfg.rms_eps, residual=x_res, keep_bf16=self._mlp_reads_bf16)
                down = self._mlp(h, L)
                if li + 1 < len(self.layers):
                    h = ops.rmsnorm_quant_fp8(down, nxt, cfg.rms_eps, residual=x_res)
                else:  # the final norm feeds the bf16 lm_head / pooling
                    h = ops.rmsnorm(down, nxt, cfg.rms_eps, residual=x_res)
            else:
                o = self._attn_out(attn.view(T, Hq * D), L)
                h = ops.rmsnorm(o, L.mlp_norm, cfg.rms_eps, residual=x_res)
                down = self._mlp(h, L)
                h = ops.rmsnorm(down, nxt, cfg.rms_eps, residual=x_res)
        return h

    # whether _mlp reads the bf16 rows of its (fp8-quantised) input too (the MoE router does)
    _mlp_reads_bf16 = False

    def _attn_mx(self) -> bool:
        """Whether the attention kernels (decode cascade, prefill) hand the o projection an MX activation: fp8 o weights on gemm8g
        (head_dim 128, every head one 128-wide K slice); LWC_ATTN_MX=0 keeps bf16 + the row quantisation."""
        L = self.layers[0]
        return (os.environ.get("LWC_ATTN_MX", "1") != "0" and isinstance(L.wo, ops.Fp8Weight)
                and self.cfg.head_dim == 128 and ops.FP8_GEMM != "blas" and L.wo.q.shape[0] % 8 == 0)

    @property
    def _dense_residual(self) -> bool:
        cls = type(self)
        return (cls._attn_out is LlamaModel._attn_out and cls._mlp is LlamaModel._mlp
                and not getattr(self, "fp8_dense", False))

    def _proj(self, x, w: torch.Tensor) -> torch.Tensor:
        """Dense projection on the per-shape backend (ops/gemm_plan.py: hipBLASLt, gemm4w or gemm8p); e4m3
        weights: row-quantised activations (an ops.QAct from the producing norm, or quantised here) into the
        fp8 GEMM (gemm8g dense or the library, ops.linear_fp8_q)."""
        if isinstance(w, ops.Fp8Weight):
            return ops.linear_fp8(x, w)
        if self.g8_ws is None:
            return F.linear(x, w)
        return gemm_plan.linear(x, w, ws=self.g8_ws)

    def _attn_out(self, attn: torch.Tensor, L) -> torch.Tensor:
        """Output projection (row-parallel + all-reduce in tensor-parallel subclasses)."""
        return self._proj(attn, L.wo)

    def _mlp(self, h: torch.Tensor, L) -> torch.Tensor:
        """Dense SwiGLU MLP: gate|up GEMM with SwiGLU (fused in gemm8p's epilogue, or hipBLASLt + K5
        silu_mul), down GEMM.  fp8: gate|up fp8 GEMM, SwiGLU fused with the down projection's row
        quantisation (K11e), down fp8 GEMM."""
        if isinstance(L.w_down, ops.Fp8Weight):
            if ops.dense_mx_ok(h, L.w_gate_up, L.w_down, L.gu_block):
                # large batches (the embedder's prefill): the activation in MX form, no quantisation pass
                aq, amx = ops.linear_fp8_swiglu_mx(h, L.w_gate_up)
                return ops.linear_fp8_mx(aq, amx, L.w_down)
            aq, as_ = ops.linear_fp8_swiglu(h, L.w_gate_up, L.gu_block)
            return ops.linear_fp8_q(aq, as_, L.w_down)
        return self._proj(self._act(h, L), L.w_down)

    def _act(self, h: torch.Tensor, L) -> torch.Tensor:
        """silu(h Wg^T) * (h Wu^T): the gate|up GEMM with its SwiGLU."""
        if self.g8_ws is None:
            return ops.silu_mul(F.linear(h, L.w_gate_up), block=L.gu_block)
        return gemm_plan.swiglu(h, L.w_gate_up, L.gu_block, ws=self.g8_ws)

    def comm_arm(self) -> None:
        """Tensor-parallel subclasses queue the readback of their collective's error word here."""

    def comm_poll(self) -> None:
        """Tensor-parallel subclasses raise here once a failed collective is visible on the host."""

    def tune_gemms(self, M: int, bucket: bool = False, lm_head: bool = True, only=None) -> None:
        """Pick the GEMM backend of every decode projection at batch M by timing both (before the
        bucket's hipGraph is captured; see ops/gemm_plan.py).  ``bucket``: M is a row-count bucket of the
        mixed chunked-prefill steps (their M varies step to step); ``lm_head``: tune the vocabulary
        projection too (mixed steps only project the decode rows and completed prompts' last tokens);
        ``only``: the epilogues to tune (e.g. ("swiglu",): the gate|up projection alone)."""
        if self.g8_ws is None or not isinstance(self.layers[0], LayerWeights) or self.fp8_dense:
            return
        cfg, L = self.cfg, self.layers[0]
        if only is not None:
            if "swiglu" in only:
                x = torch.randn(M, cfg.hidden, device=self.device).to(self.dtype)
                gemm_plan.tune(x, L.w_gate_up, "swiglu", L.gu_block, ws=self.g8_ws, bucket=bucket)
            return
        x = torch.randn(M, cfg.hidden, device=self.device).to(self.dtype)
        xa = torch.randn(M, cfg.heads * cfg.head_dim, device=self.device).to(self.dtype)
        xf = torch.randn(M, cfg.ffn, device=self.device).to(self.dtype)
        gemm_plan.tune(x, L.wqkv, ws=self.g8_ws, bucket=bucket)
        epi = "residual" if self._dense_residual else "plain"
        gemm_plan.tune(xa, L.wo, epi, ws=self.g8_ws, bucket=bucket)
        gemm_plan.tune(x, L.w_gate_up, "swiglu", L.gu_block, ws=self.g8_ws, bucket=bucket)
        gemm_plan.tune(xf, L.w_down, epi, ws=self.g8_ws, bucket=bucket)
        if lm_head:
            gemm_plan.tune(x, self.lm_head, ws=self.g8_ws, bucket=bucket)
        if self.norm_folded and not bucket and lm_head:
            self._tune_chain(M, x, xa, xf)

    def _tune_chain(self, M: int, x, xa, xf) -> None:
        """Decode batch M: decide, per norm point, between the norm kernel + the best projection backend and the
        folded norm (the consumer's row-scaled gemm4w, the producer leaving partial row sums of squares by its
        own residual epilogue or by one rms_rowsumsq pass after the planner's GEMM).  Every candidate is
        timed alone (interleaved rounds, median), the plan is the cheaper side at each point and is recorded
        in ``chain_m`` (``LWC_NORM_CHAIN=0|1`` forces all-unfolded / all-folded)."""
        if M in self.chain_m or torch.cuda.is_current_stream_capturing():
            return
        cfg, L = self.cfg, self.layers[0]
        none = {"attn": False, "mlp": False, "final": False, "qkv_bn": 192, "o": "plain", "down": "plain"}
        # below 256 rows the chain's 256-row tiles run mostly empty and the weight-streaming cores win every
        # projection: not timed (a serving engine meets many such buckets)
        if (cfg.hidden + 255) // 256 > 16 or M < 256:
            self.chain_m[M] = none
            return
        if self.chain is None:  # once, for every decode bucket (captured graphs keep these addresses)
            self.chain = ops.NormChain(max(M, 8192), cfg.hidden, cfg.rms_eps, self.device)
        if M > self.chain.max_rows:
            self.chain_m[M] = none
            return
        ch, eps = self.chain, cfg.rms_eps
        x_res = x.clone()
        ones = self.final_norm
        ops.rms_rowsumsq(x_res, ch)  # valid partials for the row-scaled candidates
        P0 = ch.P
        w = {"qkv": L.wqkv, "o": L.wo, "gu": L.w_gate_up, "down": L.w_down, "lm": self.lm_head}

        def fold(name, **kw):
            def run():
                ch.P = P0
                ops.gemm4w(x, w[name], chain=ch, **kw)
            return run

        # the row-scaled consumers at both schedules (VAR 32: block-staged epilogue; 64: wave-local, next tile
        # prefetched) and, for qkv, both tile widths
        cons = {"qkv": {f"qkv_rs{bn}v{v}": (bn, v) for bn in (192, 256) for v in (32, 64)},
                "gu": {f"gu_rsv{v}": (256, v) for v in (32, 64)},
                "lm": {f"lm_rsv{v}": (256, v) for v in (32, 64)}}
        lm_sk = ops.split_plan(M, self.lm_head.shape[0], cfg.hidden)  # lm_head's ragged last round, split

        def res(name, inp, var):
            return lambda: ops.gemm4w(inp, w[name], residual=x_res, out=x_res, chain=ch, var=var)

        runs = {
            "norm": lambda: ops.rmsnorm(x_res, ones, eps),
            "sumsq": lambda: ops.rms_rowsumsq(x_res, ch),
            "qkv": lambda: self._proj(x, L.wqkv),
            "o": lambda: gemm_plan.linear_add_(xa, L.wo, x_res, ws=self.g8_ws),
            "o_own32": res("o", xa, 32), "o_own64": res("o", xa, 64),
            "gu": lambda: gemm_plan.swiglu(x, L.w_gate_up, L.gu_block, ws=self.g8_ws),
            "down": lambda: gemm_plan.linear_add_(xf, L.w_down, x_res, ws=self.g8_ws),
            "down_own32": res("down", xf, 32), "down_own64": res("down", xf, 64),
            "lm": lambda: self._proj(x, self.lm_head),
        }
        for pt, cands in cons.items():
            for k, (bn, v) in cands.items():
                runs[k] = fold(pt, bn=bn, var=v, swiglu=pt == "gu")
        if lm_sk[0] > 1:
            runs["lm_rsv64s"] = fold("lm", bn=256, var=64, splits=lm_sk[0], split_from=lm_sk[1])
        ts = {k: [] for k in runs}
        for _ in range(3):  # interleaved rounds (one process, one device: matched clocks and caches)
            for k, fn in runs.items():
                ts[k].append(gemm_plan._time(fn, iters=3, rounds=1))
        t = {k: sorted(v)[len(v) // 2] for k, v in ts.items()}
        ch.P = P0

        def producer(name):  # the cheapest way to leave partials, and its cost over the plain residual GEMM
            # (isolated timings; the engine's in-step A/B of whole captured decode steps then decides between
            # this plan, the all-library one and the all-own one: LlamaModel.step_plans)
            opts = {"own32": t[f"{name}_own32"], "own64": t[f"{name}_own64"], "sumsq": t[name] + t["sumsq"]}
            best = min(opts, key=opts.get)
            return best, opts[best] - t[name]

        def consumer(pt):
            k = min(cons[pt], key=lambda c: t[c])
            return k, cons[pt][k]

        lm_split = "lm_rsv64s" in t and t["lm_rsv64s"] < min(t["lm_rsv32"], t["lm_rsv64"])

        o_mode, o_extra = producer("o")
        d_mode, d_extra = producer("down")
        (qk, (qkv_bn, qv)), (gk, (_, gv)), (lk, (_, lv)) = consumer("qkv"), consumer("gu"), consumer("lm")
        # each point: folded (consumer + producer's extra) vs the norm kernel + the consumer's best backend
        attn = t[qk] + d_extra < t["norm"] + t["qkv"]
        mlp = t[gk] + o_extra < t["norm"] + t["gu"]
        if lm_split:
            lk, lv = "lm_rsv64s", 64
        final = t[lk] + d_extra < t["norm"] + t["lm"]
        force = os.environ.get("LWC_NORM_CHAIN")
        if force is not None:
            attn = mlp = final = force == "1"
        plan = {"attn": attn, "mlp": mlp, "final": final, "qkv_bn": qkv_bn, "qkv_var": qv, "gu_var": gv,
                "lm_var": lv, "lm_split": lm_split, "o": o_mode, "down": d_mode}
        self.chain_m[M] = plan
        key = (M, cfg.hidden, 0, "norm_chain")
        gemm_plan.TIMINGS[key] = t
        gemm_plan._CHOICE[key] = ",".join(f"{k}={v}" for k, v in plan.items())

    # ------------------------------------------------------------------ whole-step plans (engine in-step A/B)
    def _plan_keys(self, M: int) -> dict:
        cfg = self.cfg
        epi = "residual" if self._dense_residual else "plain"
        return {"qkv": (M, cfg.qkv_dim, cfg.hidden, "plain"), "o": (M, cfg.hidden, cfg.heads * cfg.head_dim, epi),
                "gu": (M, 2 * cfg.ffn, cfg.hidden, "swiglu"), "down": (M, cfg.hidden, cfg.ffn, epi),
                "lm": (M, cfg.vocab_size, cfg.hidden, "plain")}

    def step_plans(self, M: int) -> dict:
        """Candidate plans for a decode step of M rows, for the engine's in-step A/B (it captures the decode
        graph under each and times replays: isolated per-GEMM timings misjudge the step's clock and cache
        state, ``profiles/gemm4w_stamps_r5.md``).  ``planner``: the per-shape and norm-chain choices of
        :meth:`tune_gemms`; ``library``: every projection on hipBLASLt, no folded norm; ``own``: every
        projection on its fastest hand-written core with the whole norm chain folded.  {} when nothing was
        tuned at M."""
        keys = self._plan_keys(M)
        if self.g8_ws is None or not any(k in gemm_plan._CHOICE for k in keys.values()):
            return {}
        plans = {"planner": {"choices": {n: gemm_plan._CHOICE.get(k) for n, k in keys.items()},
                             "chain": self.chain_m.get(M)}}
        none = {"attn": False, "mlp": False, "final": False, "qkv_bn": 192, "o": "plain", "down": "plain"}
        plans["library"] = {"choices": {n: "blas" for n in keys}, "chain": none if M in self.chain_m else None}
        own = {}
        for n, k in keys.items():
            t = {b: v for b, v in gemm_plan.TIMINGS.get(k, {}).items() if b != "blas" and isinstance(v, float)}
            own[n] = min(t, key=t.get) if t else gemm_plan._CHOICE.get(k)
        chain = self.chain_m.get(M)
        t = gemm_plan.TIMINGS.get((M, self.cfg.hidden, 0, "norm_chain"))
        if chain is not None and t:
            def best(cands):
                return min(cands, key=lambda c: t.get(c, float("inf")))
            q = best([f"qkv_rs{bn}v{v}" for bn in (192, 256) for v in (32, 64)])
            lm = best(["lm_rsv32", "lm_rsv64", "lm_rsv64s"])
            chain = {"attn": True, "mlp": True, "final": True, "qkv_bn": int(q[6:9]), "qkv_var": int(q[10:]),
                     "gu_var": int(best(["gu_rsv32", "gu_rsv64"])[6:]), "lm_var": int(lm[6:8]),
                     "lm_split": lm.endswith("s"), "o": best(["o_own32", "o_own64"])[2:],
                     "down": best(["down_own32", "down_own64"])[5:]}
        plans["own"] = {"choices": own, "chain": chain}
        return plans

    def step_moves(self, M: int, plan: dict) -> list:
        """Single-decision changes of ``plan`` (the engine's coordinate-descent A/B, after the whole-plan
        round): each projection's backend (hipBLASLt <-> its fastest hand-written core) where the norm chain
        does not own it, each norm point folded or not, the consumers' schedule / tile width, the producers'
        mode.  [(label, delta)]: ``with_move(plan, delta)`` applies one."""
        keys = self._plan_keys(M)
        own = {}
        for n, k in keys.items():
            t = {b: v for b, v in gemm_plan.TIMINGS.get(k, {}).items() if b != "blas" and isinstance(v, float)}
            own[n] = min(t, key=t.get) if t else None
        ch = plan.get("chain")
        owned = set()
        if ch is not None and self.chain is not None and M <= self.chain.max_rows:
            owned = {n for n, pt in (("qkv", "attn"), ("gu", "mlp"), ("lm", "final")) if ch.get(pt)}
            if ch.get("mlp") and ch.get("o") in ("own32", "own64"):
                owned.add("o")
            if (ch.get("attn") or ch.get("final")) and ch.get("down") in ("own32", "own64"):
                owned.add("down")
        moves = []

        def variant(label, choices=None, chain=None):
            moves.append((label, {"choices": dict(choices or {}), "chain": dict(chain or {})}))

        for n in keys:
            c = plan["choices"].get(n)
            if n in owned or own[n] is None:
                continue
            variant(f"{n}={'blas' if c != 'blas' else own[n]}", {n: "blas" if c != "blas" else own[n]})
        if ch is not None and self.chain is not None and M <= self.chain.max_rows:
            for pt in ("attn", "mlp", "final"):
                variant(f"{pt}_fold={not ch.get(pt)}", chain={pt: not ch.get(pt)})
            # (only moves that change the step: a consumer's schedule / tile width where its norm point is
            # folded, a producer's mode where a folded point reads it — plan_summary's rules.  A no-op move
            # once "won" by 0.3 % of replay noise)
            if ch.get("final"):
                variant(f"lm_split={not ch.get('lm_split', False)}", chain={"lm_split": not ch.get("lm_split", False),
                                                                            "lm_var": 64})
            for key, pt, alts in (("qkv_var", "attn", (32, 64)), ("gu_var", "mlp", (32, 64)),
                                  ("lm_var", "final", (32, 64)), ("qkv_bn", "attn", (192, 256))):
                cur = ch.get(key, alts[0])
                for v in alts:
                    if v != cur and ch.get(pt):
                        variant(f"{key}={v}", chain={key: v})
            for key, live in (("o", ch.get("mlp")), ("down", ch.get("attn") or ch.get("final"))):
                for v in ("own32", "own64", "sumsq"):
                    if v != ch.get(key) and live:
                        variant(f"{key}_producer={v}", chain={key: v})
        return moves

    @staticmethod
    def with_move(plan: dict, delta: dict) -> dict:
        """``plan`` with one :meth:`step_moves` delta applied (choices and chain entries overridden)."""
        ch = plan.get("chain")
        return {"choices": dict(plan["choices"], **delta.get("choices", {})),
                "chain": dict(ch, **delta.get("chain", {})) if ch is not None else None}

    def apply_step_plan(self, M: int, plan: dict) -> None:
        """Make ``plan`` (one of :meth:`step_plans`) the choice of every projection at M (and of the norm chain)."""
        keys = self._plan_keys(M)
        for n, c in plan["choices"].items():
            if c is not None:
                gemm_plan._CHOICE[keys[n]] = c
        if plan.get("chain") is not None:
            self.chain_m[M] = dict(plan["chain"])

    def plan_summary(self, M: int) -> dict:
        """The kernels a decode step of M rows runs, compactly (bench JSON / logs)."""
        keys = self._plan_keys(M)
        out = {n: gemm_plan._CHOICE.get(k, "blas") for n, k in keys.items()}
        c = self.chain_m.get(M)
        if c and self.chain_ok(M):
            if c["attn"]:
                out["qkv"] = f"g4 rs{c['qkv_bn']} v{c.get('qkv_var', 32)}"
            if c["mlp"]:
                out["gu"] = f"g4 rs v{c.get('gu_var', 32)}"
            if c["final"]:
                out["lm"] = f"g4 rs v{c.get('lm_var', 32)}" + (" split-K tail" if c.get("lm_split") else "")
            if c["mlp"] and c["o"] != "plain":
                out["o"] = out["o"] + "+sumsq" if c["o"] == "sumsq" else f"g4 rs2 v{c['o'][3:]}"
            if (c["attn"] or c["final"]) and c["down"] != "plain":
                out["down"] = out["down"] + "+sumsq" if c["down"] == "sumsq" else f"g4 rs2 v{c['down'][3:]}"
        return out

    def decode(self, tokens: torch.Tensor, positions: torch.Tensor, slots: torch.Tensor, block_tables: torch.Tensor,
               ctx_lens: torch.Tensor, cache: KVCache, num_splits: int = 1,
               cascade_tiles: Optional[torch.Tensor] = None) -> torch.Tensor:
        """One decode step for B sequences -> logits [B, V] bf16.  All inputs are device tensors
        (int32), so the whole call can be captured in a hipGraph.  Attention: ``cascade_tiles`` [T, 3] —
        the one-launch cascade kernel (shared prompt blocks read once per super-tile; the engine's
        large-batch path); otherwise split-K paged decode."""
        cfg = self.cfg
        x = ops.embedding(self.embed, tokens)
        B = tokens.shape[0]
        # q is rotated inside the attention kernels as they load it (rope_kv_write rotates and caches k
        # only): q's round trip through HBM in rope_kv_write (2/3 of its bytes at GQA 4) is gone.
        # LWC_DECODE_QROPE=0: the previous split (rope_kv_write rotates q in place), an A/B knob
        q_at_load = os.environ.get("LWC_DECODE_QROPE", "1") != "0"
        rope = (self.cos, self.sin, positions) if q_at_load else None
        if cascade_tiles is not None:
            # fp8 o projection (config 5): the attention output leaves the kernel in MX form (ops.MXAct)
            mx = self._attn_mx()

            def attn_fn(qkv, li):
                return ops.paged_decode_cascade(qkv, cache.k[li], cache.v[li], block_tables, ctx_lens, cascade_tiles,
                                                cfg.heads, self.scale, rope=rope, mx=mx)
        else:
            part_o = part_lse = None
            if num_splits > 1:
                part_o = torch.empty(B * cfg.heads * num_splits * cfg.head_dim, dtype=torch.float32, device=x.device)
                part_lse = torch.empty(B * cfg.heads * num_splits, dtype=torch.float32, device=x.device)

            def attn_fn(qkv, li):
                return ops.paged_decode(qkv, cache.k[li], cache.v[li], block_tables, ctx_lens, cfg.heads, self.scale,
                                        num_splits=num_splits, part_o=part_o, part_lse=part_lse, rope=rope)

        if self.chain_ok(B):
            return self._chain_layers(x, cache, positions, slots, attn_fn, not q_at_load, self.chain_m[B])
        h = self._layers(x, cache, positions, slots, attn_fn, rope_q=not q_at_load)
        return self._proj(h, self.lm_head)

    def encode(self, tokens: torch.Tensor, positions: torch.Tensor, cu_seqlens: torch.Tensor,
               max_seqlen: int, keep: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Cache-less causal forward of packed sequences -> final-normed hidden states [T, d] (decoder used
        as an embedder, e.g. e5-mistral: the caller pools the last token).  RoPE runs without a cache
        write (slots=None), attention is the varlen prefill kernel over the fresh k/v."""
        cfg = self.cfg
        Hq, Hkv, D = cfg.heads, cfg.kv_heads, cfg.head_dim
        null = _NullCache(cfg, self.device)
        x = ops.embedding(self.embed, tokens)

        mx = self._attn_mx()  # fp8 o projection: the attention epilogue writes its MX operand

        def attn_fn(qkv, li):
            q, k, v = qkv[:, : Hq * D], qkv[:, Hq * D:(Hq + Hkv) * D], qkv[:, (Hq + Hkv) * D:]
            if mx:
                return ops.prefill_attention_mx(q, k, v, cu_seqlens, max_seqlen, Hq, Hkv, self.scale, causal=True)
            return ops.prefill_attention(q, k, v, cu_seqlens, max_seqlen, Hq, Hkv, D, self.scale, causal=True)

        # the hidden states themselves are the output: the real final norm weight, also when it is folded
        # into lm_head for decoding
        return self._layers(x, null, positions, None, attn_fn, keep=keep,
                            final_norm=self.final_norm_weight)

    def prefill(self, tokens: torch.Tensor, positions: torch.Tensor, slots: torch.Tensor, cu_seqlens: torch.Tensor,
                max_seqlen: int, last_idx: torch.Tensor, cache: KVCache, ctx: Optional[dict] = None) -> torch.Tensor:
        """Prefill packed prompts (cu_seqlens) -> logits of each sequence's last token [nseq, V].

        ``ctx`` (cross-request prefix cache): the packed tokens are only each prompt's UNCACHED tail and
        attention also needs the cached head.  ctx = {k_slots [sum klen] int64: cache slots of every
        position of each prompt (cached + new), cu_k [nseq+1] int32, q_lens, k_lens (host lists)}; per
        layer, after the new rows are written, the whole key range is gathered from the paged cache and
        the varlen kernel runs with queries at the end of each key range."""
        cfg = self.cfg
        Hq, Hkv, D = cfg.heads, cfg.kv_heads, cfg.head_dim
        x = ops.embedding(self.embed, tokens)
        mx = self._attn_mx()  # fp8 o projection: the attention epilogue writes its MX operand

        def attn_fn(qkv, li):
            q = qkv[:, : Hq * D]
            if ctx is not None:
                kf, vf = ops.kv_gather(cache.k[li], cache.v[li], ctx["k_slots"])
                return ops.prefill_attention(q, kf, vf, cu_seqlens, max_seqlen, Hq, Hkv, D, self.scale, causal=True,
                                             cu_seqlens_k=ctx["cu_k"], lens=(ctx["q_lens"], ctx["k_lens"]))
            k = qkv[:, Hq * D:(Hq + Hkv) * D]
            v = qkv[:, (Hq + Hkv) * D:]
            if mx:
                return ops.prefill_attention_mx(q, k, v, cu_seqlens, max_seqlen, Hq, Hkv, self.scale, causal=True)
            return ops.prefill_attention(q, k, v, cu_seqlens, max_seqlen, Hq, Hkv, D, self.scale, causal=True)

        h = self._layers(x, cache, positions, slots, attn_fn, keep=last_idx)  # last layer: o / MLP on these rows
        return F.linear(h, self.lm_head)

    def forward_mixed(self, tokens: torch.Tensor, positions: torch.Tensor, slots: torch.Tensor, cache: KVCache,
                      n_dec: int, dec: Optional[dict], chunk: dict, logit_rows: torch.Tensor) -> torch.Tensor:
        """ONE forward over [n_dec decode rows || prompt-chunk rows] (mixed chunked prefill): every projection
        is one GEMM over both; per layer the decode rows go to the paged decode kernel (``dec``: block_tables,
        ctx_lens and either cascade ``tiles`` or ``splits``) and the chunk rows to the paged-KV prefill kernel
        (``chunk``: cu_q, block_tables, k_lens device tensors, max_q, host lens) — earlier chunks of a prompt
        are read straight from the paged cache.  Returns logits of ``logit_rows`` [R, V]."""
        cfg = self.cfg
        Hq, D = cfg.heads, cfg.head_dim
        x = ops.embedding(self.embed, tokens)
        T = tokens.shape[0]
        part_o = part_lse = None
        splits = 1 if dec is None else int(dec.get("splits", 1))
        if n_dec and "tiles" not in dec and splits > 1:
            part_o = torch.empty(n_dec * Hq * splits * D, dtype=torch.float32, device=x.device)
            part_lse = torch.empty(n_dec * Hq * splits, dtype=torch.float32, device=x.device)

        def attn_fn(qkv, li):
            out = torch.empty(T, Hq * D, dtype=qkv.dtype, device=qkv.device)
            if n_dec:
                o = out[:n_dec].view(n_dec, Hq, D)
                if "tiles" in dec:
                    ops.paged_decode_cascade(qkv[:n_dec], cache.k[li], cache.v[li], dec["block_tables"],
                                             dec["ctx_lens"], dec["tiles"], Hq, self.scale, out=o)
                else:
                    ops.paged_decode(qkv[:n_dec], cache.k[li], cache.v[li], dec["block_tables"], dec["ctx_lens"], Hq,
                                     self.scale, num_splits=splits, out=o, part_o=part_o, part_lse=part_lse)
            ops.prefill_attention_paged(qkv[n_dec:], cache.k[li], cache.v[li], chunk["cu_q"], chunk["block_tables"],
                                        chunk["k_lens"], chunk["max_q"], Hq, self.scale, out=out[n_dec:],
                                        lens=chunk.get("lens") if li == 0 else None)
            return out

        h = self._layers(x, cache, positions, slots, attn_fn)
        return self._proj(h.index_select(0, logit_rows), self.lm_head)
