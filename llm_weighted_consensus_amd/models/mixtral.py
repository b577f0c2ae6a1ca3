"""Mixtral-style sparse mixture-of-experts decoder (BASELINE config 5: Mixtral-8x7B sampler, fp8 MFMA,
tensor-parallel degree 2).

Attention, KV cache, prefill/decode/cascade paths are the Llama ones (`LlamaModel`); only the MLP
changes.  Per layer, for the T tokens of a step:

    route  = h Wr^T, top-k softmax       K11a moe_router: the router GEMV fused with the top-k (many
             segments + permutation         workgroups), then one workgroup for segments / permutation
    gu     = grouped GEMM over experts   K6g, A rows gathered through src_row (no permute copy)
    act    = silu(g) * u                 K5
    y      = grouped GEMM over experts   K6g
    out    = sum_j w[t,j] y[inv[t,j]]    K11d moe_combine
With ``fp8=True`` the expert weights are OCP e4m3 with per-output-channel scales (quantised at load)
and activations are quantised per row on the fly (K11e), feeding the fp8 MFMA path of the grouped
GEMM: half the weight bytes — what bounds a MoE decode step, which touches every expert's weights.

Tensor parallelism (``tp_group``): attention heads and every expert's FFN columns are split across
the ranks (Megatron layout: q/k/v and gate|up column-parallel, o and down row-parallel); the two
row-parallel outputs are summed with one all-reduce each (C3) before the residual norm — the
IPC one-shot kernel of `parallel/allreduce.py` when ``tp_comm`` is given (graph-capturable), else the
process group's.  The shard is
taken from the full random-init / loaded weights so any TP degree computes the same function.

Expert parallelism (``ep_group``, C4, `parallel/expert.py`): the alternative to TP for the MoE layers.
Rank r of the EP group keeps experts [r*E/W, (r+1)*E/W) with their FULL FFN width (grouped-GEMM tiles
stay 2x wider than under TP=2) and replicated attention; each rank decodes its own sequences and the
(token, slot) rows travel to the expert owners and back with two all-to-alls per layer (fp8 mode
dispatches the e4m3 rows + per-row scales: half the bytes).  Ranks must step in lockstep (every rank
calls every layer, with zero tokens if idle); the padded exchange with a fixed ``ep_capacity`` (the
most tokens any rank feeds a layer in one step, e.g. the largest decode bucket) keeps the decode step
free of host synchronisation.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Optional

import torch

from .. import ops
from ..ops import gemm_plan
from .config import DecoderConfig
from .llama import LlamaModel


@dataclass
class MoELayerWeights:
    attn_norm: torch.Tensor
    wqkv: torch.Tensor
    wo: torch.Tensor
    mlp_norm: torch.Tensor
    router: torch.Tensor          # [E, d]
    w13: torch.Tensor             # [E, 2F_local, d]  (bf16 or e4m3fn)
    w2: torch.Tensor              # [E, d, F_local]
    s13: Optional[torch.Tensor]   # fp8 per-channel scales [E, 2F_local]
    s2: Optional[torch.Tensor]    # [E, d]
    gu_block: int = 0             # >0: w13 rows interleave gate|up in blocks of this size (fp8 path)


class MixtralModel(LlamaModel):
    def __init__(self, cfg: DecoderConfig, device="cuda", dtype=torch.bfloat16, seed: int = 0,
                 weights_path: Optional[str] = None, max_position: Optional[int] = None, fp8: bool = False,
                 tp_rank: int = 0, tp_size: int = 1, tp_group=None, ep_rank: int = 0, ep_size: int = 1,
                 ep_group=None, ep_mode: str = "padded", ep_capacity: Optional[int] = None, tp_comm=None,
                 ep_comm=None):
        if not cfg.num_experts:
            raise ValueError(f"{cfg.name} is dense; use LlamaModel")
        if ep_size > 1 and tp_size > 1:
            raise ValueError("choose TP or EP for the MoE decoder, not both")
        if cfg.num_experts % ep_size:
            raise ValueError(f"ep_size {ep_size} must divide num_experts {cfg.num_experts}")
        self.ep_rank, self.ep_size, self.ep_capacity = ep_rank, ep_size, ep_capacity
        self.ep = None
        if ep_size > 1:
            from ..parallel.expert import ExpertParallel

            self.ep = ExpertParallel(cfg.num_experts, group=ep_group, mode=ep_mode, comm=ep_comm)
            if self.ep.W != ep_size:
                raise ValueError(f"ep_group has {self.ep.W} ranks, ep_size is {ep_size}")
        if cfg.heads % tp_size or cfg.kv_heads % tp_size or cfg.ffn % tp_size:
            raise ValueError(f"tp_size {tp_size} must divide heads, kv_heads and ffn")
        self.fp8, self.tp_rank, self.tp_size, self.tp_group = fp8, tp_rank, tp_size, tp_group
        # C3 transport: a parallel.allreduce.CustomAllReduce (IPC peer buffers, one graph-capturable kernel)
        # or None for the process group's all-reduce (RCCL / gloo; not capturable)
        self.tp_comm = tp_comm
        self.full_cfg = cfg
        super().__init__(cfg, device=device, dtype=dtype, seed=seed, weights_path=weights_path,
                         max_position=max_position)
        # the attention kernels see the per-rank head counts
        if tp_size > 1:
            from dataclasses import replace

            self.cfg = replace(cfg, heads=cfg.heads // tp_size, kv_heads=cfg.kv_heads // tp_size)
        self.scale = 1.0 / math.sqrt(cfg.head_dim)

    def tune_gemms(self, M: int, bucket: bool = False, lm_head: bool = True, only=None) -> None:
        """The bf16 vocabulary projection is the MoE decoder's one dense bf16 GEMM (attention projections and
        experts are fp8, planned per shape in ops.linear_fp8_q): time the library against the hand-written
        cores at decode batch M before the bucket's graph is captured (ops/gemm_plan.py)."""
        if lm_head and only is None and self.g8_ws is not None and not isinstance(self.lm_head, ops.Fp8Weight):
            x = torch.randn(M, self.cfg.hidden, device=self.device).to(self.dtype)
            gemm_plan.tune(x, self.lm_head, ws=self.g8_ws, bucket=bucket)

    # ------------------------------------------------------------------ weights
    def _shard_layer(self, attn_norm, wq, wk, wv, wo, mlp_norm, router, w1, w3, w2) -> MoELayerWeights:
        """Full per-layer tensors -> this rank's shard (+ fp8 quantisation of the experts)."""
        r, n = self.tp_rank, self.tp_size
        cfg = self.full_cfg
        D, F_ = cfg.head_dim, cfg.ffn
        hq, hk, fl = cfg.heads // n, cfg.kv_heads // n, F_ // n
        q = wq[r * hq * D:(r + 1) * hq * D]
        k = wk[r * hk * D:(r + 1) * hk * D]
        v = wv[r * hk * D:(r + 1) * hk * D]
        wqkv = torch.cat([q, k, v]).contiguous()
        wo_s = wo[:, r * hq * D:(r + 1) * hq * D].contiguous()
        if self.ep_size > 1:  # this EP rank's experts, full FFN width
            el = cfg.num_experts // self.ep_size
            e0 = self.ep_rank * el
            w1, w3, w2 = w1[e0:e0 + el], w3[e0:e0 + el], w2[e0:e0 + el]
        w13 = torch.cat([w1[:, r * fl:(r + 1) * fl], w3[:, r * fl:(r + 1) * fl]], dim=1).contiguous()  # [E,2fl,d]
        w2_s = w2[:, :, r * fl:(r + 1) * fl].contiguous()                                             # [E,d,fl]
        s13 = s2 = None
        if self.fp8:
            # gate / up rows interleaved in blocks of 32 per expert: the grouped fp8 GEMM applies the SwiGLU
            # in its epilogue (no [rows, 2F] intermediate), then one per-row e4m3 pass feeds the down GEMM
            w13 = torch.stack([ops.swiglu_interleave(w13[e]) for e in range(w13.shape[0])])
            w13, s13 = ops.quant_fp8_weight(w13)
            w2_s, s2 = ops.quant_fp8_weight(w2_s)
            # the attention projections are fp8 too (config 5: fp8 MFMA throughout; router and lm_head bf16)
            wqkv, wo_s = ops.Fp8Weight(wqkv), ops.Fp8Weight(wo_s)
        return MoELayerWeights(attn_norm, wqkv, wo_s, mlp_norm, router.contiguous(), w13, w2_s, s13, s2,
                               32 if self.fp8 else 0)

    def _random_init(self, seed: int) -> None:
        cfg, dev, dt = self.full_cfg, self.device, self.dtype
        g = torch.Generator(device=dev)
        g.manual_seed(seed)
        std = 0.02

        def rnd(*shape, s=std):
            return (torch.randn(*shape, generator=g, device=dev, dtype=torch.float32) * s).to(dt)

        d, F_, E, D = cfg.hidden, cfg.ffn, cfg.num_experts, cfg.head_dim
        self.embed = rnd(cfg.vocab_size, d)
        out_std = std / math.sqrt(2 * cfg.layers)
        self.layers = []
        for _ in range(cfg.layers):
            wq, wk, wv = rnd(cfg.heads * D, d), rnd(cfg.kv_heads * D, d), rnd(cfg.kv_heads * D, d)
            wo = rnd(d, cfg.heads * D, s=out_std)
            router = rnd(E, d, s=0.1)
            w1, w3 = rnd(E, F_, d), rnd(E, F_, d)
            w2 = rnd(E, d, F_, s=out_std)
            ones = torch.ones(d, device=dev, dtype=dt)
            self.layers.append(self._shard_layer(ones, wq, wk, wv, wo, ones.clone(), router, w1, w3, w2))
            del w1, w3, w2
        self.final_norm = torch.ones(d, device=dev, dtype=dt)
        self.lm_head = self.embed if cfg.tie_embeddings else rnd(cfg.vocab_size, d)

    def _load(self, path: str) -> None:
        """HF Mixtral safetensors (model.layers.N.block_sparse_moe.{gate,experts.e.w1/w2/w3})."""
        from pathlib import Path

        from safetensors.torch import load_file

        files = sorted(Path(path).glob("*.safetensors")) if Path(path).is_dir() else [Path(path)]
        sd = {}
        for f in files:
            sd.update(load_file(str(f), device="cpu"))
        dev, dt = self.device, self.dtype
        t = lambda n: sd[n].to(device=dev, dtype=dt).contiguous()  # noqa: E731
        cfg = self.full_cfg
        self.embed = t("model.embed_tokens.weight")
        self.layers = []
        for i in range(cfg.layers):
            p = f"model.layers.{i}."
            m = p + "block_sparse_moe."
            ex = lambda w: torch.stack([t(f"{m}experts.{e}.{w}.weight") for e in range(cfg.num_experts)])  # noqa
            self.layers.append(self._shard_layer(
                t(p + "input_layernorm.weight"), t(p + "self_attn.q_proj.weight"), t(p + "self_attn.k_proj.weight"),
                t(p + "self_attn.v_proj.weight"), t(p + "self_attn.o_proj.weight"),
                t(p + "post_attention_layernorm.weight"), t(m + "gate.weight"), ex("w1"), ex("w3"), ex("w2")))
        self.final_norm = t("model.norm.weight")
        self.lm_head = t("lm_head.weight") if "lm_head.weight" in sd else self.embed

    # ------------------------------------------------------------------ forward pieces
    def _all_reduce(self, x: torch.Tensor) -> torch.Tensor:
        if self.tp_size > 1:
            if self.tp_comm is not None:
                return self.tp_comm.all_reduce_(x)
            from ..parallel import dist as pdist

            pdist.all_reduce_(x, group=self.tp_group)
        return x

    def _comms(self):
        return [c for c in (self.tp_comm, self.ep.comm if self.ep is not None else None)
                if c is not None and hasattr(c, "arm")]

    def comm_arm(self) -> None:
        """Queue the asynchronous readback of the TP all-reduce's / EP all-to-all's error word (after a
        step's launch)."""
        for c in self._comms():
            c.arm()

    def comm_poll(self) -> None:
        """Raise parallel.allreduce.CommFailure if a completed readback shows a peer never arrived."""
        for c in self._comms():
            c.poll()

    @property
    def graph_safe(self) -> bool:
        """Whether a decode step may be captured in a hipGraph: every collective inside it must be a
        stream kernel (the IPC all-reduce), not a host-driven process-group call."""
        if self.tp_size == 1 and self.ep_size == 1:
            return True
        if self.tp_size > 1:
            return self.tp_comm is not None
        # EP: the padded exchange with a fixed capacity over the IPC all-to-all has no host step
        return (self.ep is not None and self.ep.comm is not None and self.ep.mode == "padded"
                and self.ep_capacity is not None)

    def _attn_out(self, attn: torch.Tensor, L) -> torch.Tensor:
        return self._all_reduce(self._proj(attn, L.wo))

    def _experts(self, x: torch.Tensor, row_off: torch.Tensor, L: MoELayerWeights,
                 scale: Optional[torch.Tensor] = None, a_rows: Optional[torch.Tensor] = None,
                 rows: Optional[int] = None) -> torch.Tensor:
        """Grouped expert FFN over expert-major rows (optionally gathered through ``a_rows``)."""
        if self.fp8:
            n = rows if rows is not None else (a_rows.numel() if a_rows is not None else x.shape[0])
            if L.gu_block == 32 and ops.moe_mx_ok(x, L.w13, L.w2, n):
                # MX middle: e4m3 + e8m0 block scales straight from the gate|up epilogue into the down MFMAs
                aq, amx = ops.grouped_gemm_swiglu_mx(x, L.w13, row_off, scale, L.s13, a_rows=a_rows, rows=rows)
                return ops.grouped_gemm(aq, L.w2, row_off, w_scale=L.s2, a_mx=amx)
            act = ops.grouped_gemm(x, L.w13, row_off, a_rows=a_rows, rows=rows, a_scale=scale, w_scale=L.s13,
                                   swiglu=True)
            aq, as_ = ops.quant_fp8_rows(act)
            return ops.grouped_gemm(aq, L.w2, row_off, a_scale=as_, w_scale=L.s2)
        gu = ops.grouped_gemm(x, L.w13, row_off, a_rows=a_rows, rows=rows)
        return ops.grouped_gemm(ops.silu_mul(gu), L.w2, row_off)

    _mlp_reads_bf16 = True  # the router projects the bf16 rows

    @staticmethod
    def _split_act(h):
        """(bf16 rows, e4m3 rows | None, row scales | None) of an MLP input (ops.QAct from a fused norm)."""
        if isinstance(h, ops.QAct):
            return h.bf16, h.q, h.s
        return h, None, None

    def _mlp_ep(self, h, L: MoELayerWeights) -> torch.Tensor:
        """EP MoE layer: route locally, dispatch rows to the expert owners, combine locally.  Padded mode on
        the GPU runs the exchange as the ep.hip kernels (pack through the dispatch permutation, unpack,
        back, combine: ExpertParallel.run_combined); the torch glue stays for CPU process groups and the
        exact (prefill) mode."""
        k = self.full_cfg.experts_per_token
        h, hq, hs = self._split_act(h)
        _ids, w, row_off, src, inv = ops.route(h, L.router, k)
        cap = None if self.ep_capacity is None else self.ep_capacity * k
        if h.is_cuda and self.ep.mode == "padded":
            if self.fp8 and hq is None:
                hq, hs = ops.quant_fp8_rows(h)
            return self.ep.run_combined(hq if self.fp8 else h, row_off, src, inv, w, k,
                                        lambda xl, ro, sl: self._experts(xl, ro, L, sl),
                                        x_scale=hs if self.fp8 else None, capacity=cap)
        idx = src.long()
        if self.fp8:
            if hq is None:
                hq, hs = ops.quant_fp8_rows(h)
            xs = hq.view(torch.uint8)[idx].view(torch.float8_e4m3fn)  # e4m3 rows gathered as bytes
            ss = hs[idx]
        else:
            xs, ss = h[idx], None
        y = self.ep.run(xs, row_off, lambda xl, ro, sl: self._experts(xl, ro, L, sl), x_scale=ss, capacity=cap)
        return ops.moe_combine(y.contiguous(), inv, w, k)

    def _mlp(self, h, L: MoELayerWeights) -> torch.Tensor:
        if self.ep is not None:
            return self._mlp_ep(h, L)
        k = self.full_cfg.experts_per_token
        h, hq, hs = self._split_act(h)
        _ids, w, row_off, src, inv = ops.route(h, L.router, k)
        rows = h.shape[0] * k
        if self.fp8:
            if hq is None:
                hq, hs = ops.quant_fp8_rows(h)
            y = self._experts(hq, row_off, L, hs, a_rows=src, rows=rows)
        else:
            y = self._experts(h, row_off, L, a_rows=src, rows=rows)
        return self._all_reduce(ops.moe_combine(y, inv, w, k))
