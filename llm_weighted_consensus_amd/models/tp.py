"""Tensor parallelism (C3) for the decoders: the Megatron layout over a TP group of ranks.

q/k/v and gate|up are column-parallel (each rank keeps Hq/T query heads, Hkv/T KV heads and F/T FFN
columns), o and down row-parallel; the two row-parallel outputs of a layer are summed with one all-reduce
each before the residual norm — the IPC one-shot kernel of `parallel/allreduce.py` when ``tp_comm`` is
given (one graph-capturable launch: the decode step stays one hipGraph), else the process group's
all-reduce.  Embedding, final norm and lm_head are replicated: every rank holds the full hidden state after
each all-reduce, computes the same logits and samples the same tokens, so the engines of a TP replica step
in lockstep with no logits exchange.  The shard of every weight is cut from the full random-init / loaded
tensor, so any TP degree computes the same function as TP=1 (up to the all-reduce's summation order).

Used by the dense decoders (:class:`TPLlamaModel`: Llama-3 / Mistral voters and the e5-mistral embedder
at "tp": 2, BASELINE config 5's "TP=2 each") and by `models/mixtral.py` (experts column-split too).
"""
from __future__ import annotations

from typing import Optional

import torch

from .config import DecoderConfig
from .llama import LayerWeights, LlamaModel


class TensorParallel:
    """All-reduce + error-word plumbing shared by the TP decoders (mixin; needs tp_size / tp_comm /
    tp_group attributes)."""

    tp_size: int = 1
    tp_comm = None
    tp_group = None

    def _all_reduce(self, x: torch.Tensor) -> torch.Tensor:
        if self.tp_size > 1:
            if self.tp_comm is not None:
                return self.tp_comm.all_reduce_(x)
            from ..parallel import dist as pdist

            pdist.all_reduce_(x, group=self.tp_group)
        return x

    def _comms(self):
        return [c for c in (self.tp_comm,) if c is not None and hasattr(c, "arm")]

    def comm_arm(self) -> None:
        """Queue the asynchronous readback of the collectives' error word (after a step's launch)."""
        for c in self._comms():
            c.arm()

    def comm_poll(self) -> None:
        """Raise parallel.allreduce.CommFailure if a completed readback shows a peer never arrived."""
        for c in self._comms():
            c.poll()


def shard_dense_layer(L: LayerWeights, cfg: DecoderConfig, rank: int, size: int) -> LayerWeights:
    """The rank's Megatron shard of one dense layer (full ``cfg`` head / FFN counts; gate|up not yet
    interleaved)."""
    D, F_ = cfg.head_dim, cfg.ffn
    hq, hk, fl = cfg.heads // size, cfg.kv_heads // size, F_ // size
    Q, K = cfg.heads * D, cfg.kv_heads * D
    w = L.wqkv
    q = w[rank * hq * D:(rank + 1) * hq * D]
    k = w[Q + rank * hk * D:Q + (rank + 1) * hk * D]
    v = w[Q + K + rank * hk * D:Q + K + (rank + 1) * hk * D]
    gu = L.w_gate_up
    if L.gu_block:
        raise ValueError("shard before the gate|up interleave")
    gate, up = gu[rank * fl:(rank + 1) * fl], gu[F_ + rank * fl:F_ + (rank + 1) * fl]
    return LayerWeights(attn_norm=L.attn_norm, wqkv=torch.cat([q, k, v]).contiguous(),
                        wo=L.wo[:, rank * hq * D:(rank + 1) * hq * D].contiguous(), mlp_norm=L.mlp_norm,
                        w_gate_up=torch.cat([gate, up]).contiguous(),
                        w_down=L.w_down[:, rank * fl:(rank + 1) * fl].contiguous())


class TPLlamaModel(TensorParallel, LlamaModel):
    """Dense decoder (Llama-3 / Mistral) over ``tp_size`` ranks: this rank's attention heads and FFN
    columns, an all-reduce after o and after down (see the module docstring)."""

    def __init__(self, cfg: DecoderConfig, device="cuda", dtype=torch.bfloat16, seed: int = 0,
                 weights_path: Optional[str] = None, max_position: Optional[int] = None, fp8_dense: bool = False,
                 tp_rank: int = 0, tp_size: int = 1, tp_group=None, tp_comm=None):
        if cfg.num_experts:
            raise ValueError(f"{cfg.name} is a MoE decoder; use MixtralModel")
        if cfg.heads % tp_size or cfg.kv_heads % tp_size or cfg.ffn % tp_size:
            raise ValueError(f"tp_size {tp_size} must divide heads, kv_heads and ffn")
        self.tp_rank, self.tp_size, self.tp_group, self.tp_comm = tp_rank, tp_size, tp_group, tp_comm
        self.full_cfg = cfg
        super().__init__(cfg, device=device, dtype=dtype, seed=seed, weights_path=weights_path,
                         max_position=max_position, fp8_dense=fp8_dense)
        if tp_size > 1:  # the attention kernels and the KV cache see the per-rank head counts
            from dataclasses import replace

            self.cfg = replace(cfg, heads=cfg.heads // tp_size, kv_heads=cfg.kv_heads // tp_size,
                               ffn=cfg.ffn // tp_size)

    def _shard_all(self) -> None:
        if self.tp_size > 1:
            self.layers = [shard_dense_layer(L, self.full_cfg, self.tp_rank, self.tp_size) for L in self.layers]
            if self.device.type == "cuda":
                torch.cuda.empty_cache()

    def _random_init(self, seed: int) -> None:
        LlamaModel._random_init(self, seed)  # the full model's tensors (same generator order as TP=1)
        self._shard_all()

    def _load(self, path: str) -> None:
        LlamaModel._load(self, path)
        self._shard_all()

    def _attn_out(self, attn: torch.Tensor, L) -> torch.Tensor:
        return self._all_reduce(self._proj(attn, L.wo))

    def _mlp(self, h: torch.Tensor, L) -> torch.Tensor:
        return self._all_reduce(LlamaModel._mlp(self, h, L))

    @property
    def graph_safe(self) -> bool:
        """A decode step captures into a hipGraph only when its all-reduces are stream kernels (the IPC
        one-shot all-reduce), not host-driven process-group calls."""
        return self.tp_size == 1 or self.tp_comm is not None
