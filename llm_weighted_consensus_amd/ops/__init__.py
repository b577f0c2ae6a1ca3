"""Python face of the hand-written gfx950 HIP kernels (``csrc/kernels``).

Every function here allocates its outputs (unless ``out=`` is given) and calls straight into
``_kernels.so``; there is no eager-PyTorch fallback.  If the extension is missing the first call
raises: on a GPU box a silent fallback would hide that the native path is not the one running.

Layout conventions shared with the engine:
  * fused qkv rows  : [T, (Hq + 2*Hkv) * D]
  * K cache (layer) : [num_blocks, Hkv, block_size, D]
  * V cache (layer) : [num_blocks, Hkv, block_size/4, D, 4]   (4-token interleaved, see attention_decode.hip)
"""
from __future__ import annotations

import contextlib
import importlib
import os
import threading
from typing import Optional, Sequence, Tuple

import torch

_K = None
_ERR: Optional[BaseException] = None


def kernels():
    """Return the loaded ``_kernels`` extension, raising loudly if it is unavailable."""
    global _K, _ERR
    if _K is None:
        try:
            _K = importlib.import_module("llm_weighted_consensus_amd.ops._kernels")
        except BaseException as e:  # pragma: no cover - depends on the build
            _ERR = e
            raise RuntimeError(
                "llm_weighted_consensus_amd HIP kernels are not built: run "
                "`python -m llm_weighted_consensus_amd._build` (hipcc --offload-arch=gfx950)"
            ) from e
    return _K


def available() -> bool:
    try:
        kernels()
        return True
    except RuntimeError:
        return False


# ---------------------------------------------------------------------------------------------
# normalisation / element-wise


def rmsnorm(x: torch.Tensor, w: torch.Tensor, eps: float, residual: Optional[torch.Tensor] = None,
            out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """y = rmsnorm(x [+ residual]) * w.  With ``residual`` given, ``residual`` is updated in place to
    ``x + residual`` (the pre-norm residual stream) — the fused K1 kernel."""
    if out is None:
        out = torch.empty_like(x)
    kernels().rmsnorm(x, residual, w, out, float(eps))
    return out


class QAct:
    """A normalised activation handed to fp8 projections: per-row e4m3 rows ``q`` [M, d] with scales ``s`` [M]
    (``q * s[:, None]`` ~= the bf16 activation) and, when a consumer needs it, the bf16 rows ``bf16``."""

    __slots__ = ("bf16", "q", "s")

    def __init__(self, bf16: Optional[torch.Tensor], q: torch.Tensor, s: torch.Tensor):
        self.bf16, self.q, self.s = bf16, q, s


def rmsnorm_quant_fp8(x: torch.Tensor, w: torch.Tensor, eps: float, residual: Optional[torch.Tensor] = None,
                      keep_bf16: bool = False) -> QAct:
    """RMSNorm (+ in-place residual update, as :func:`rmsnorm`) with the per-row e4m3 quantisation of its
    output fused into the same pass (csrc/kernels/norm.hip, wave per row): equal to
    ``quant_fp8_rows(rmsnorm(x, ...))``.  Widths the fused kernel does not take run the two kernels."""
    d = x.shape[-1]
    if d not in (2048, 4096, 8192):
        y = rmsnorm(x, w, eps, residual=residual)
        q, s = quant_fp8_rows(y)
        return QAct(y if keep_bf16 else None, q, s)
    q = torch.empty(x.shape, dtype=torch.float8_e4m3fn, device=x.device)
    s = torch.empty(x.numel() // d, dtype=torch.float32, device=x.device)
    y = torch.empty_like(x) if keep_bf16 else None
    kernels().rmsnorm_quant_fp8(x, residual, w, y, q, s, float(eps))
    return QAct(y, q, s)


def layernorm(x: torch.Tensor, g: torch.Tensor, b: torch.Tensor, eps: float,
              residual: Optional[torch.Tensor] = None, out: Optional[torch.Tensor] = None,
              pre_bias: Optional[torch.Tensor] = None) -> torch.Tensor:
    """y = layernorm(x [+ residual] [+ pre_bias]) * g + b (K9a).  ``pre_bias`` [d]: the bias of a projection
    whose GEMM already added the residual stream into x (the encoder's fused o / FFN2 residual).  ``out`` may
    be x itself for rows of at most 1024 elements (one wave per row loads before it stores)."""
    if out is None:
        out = torch.empty_like(x)
    kernels().layernorm(x, residual, g, b, out, float(eps), pre_bias)
    return out


def silu_mul(gate_up: torch.Tensor, out: Optional[torch.Tensor] = None, block: int = 0) -> torch.Tensor:
    """SwiGLU over a fused [T, 2F] = [gate | up] buffer (K5); ``block`` > 0: columns interleaved
    gate/up in blocks of ``block`` (the :func:`swiglu_interleave` weight layout)."""
    F = gate_up.shape[-1] // 2
    if out is None:
        out = torch.empty(*gate_up.shape[:-1], F, dtype=gate_up.dtype, device=gate_up.device)
    kernels().silu_mul(gate_up, out, int(block))
    return out


def embedding(table: torch.Tensor, ids: torch.Tensor, out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Row gather table[ids] (K7); ids int32."""
    if out is None:
        out = torch.empty(ids.numel(), table.shape[1], dtype=table.dtype, device=table.device)
    kernels().embedding(table, ids, out)
    return out


def rope_kv_write(qkv: torch.Tensor, positions: torch.Tensor, cos: torch.Tensor, sin: torch.Tensor,
                  k_cache: torch.Tensor, v_cache: torch.Tensor, Hq: int, Hkv: int, D: int,
                  slots: Optional[torch.Tensor] = None, rope_q: bool = True) -> None:
    """In-place rotate-half RoPE on q and k inside ``qkv`` and scatter k, v into the paged cache at
    ``slots`` (K2).  ``slots=None`` only rotates (no cache write).  ``rope_q=False`` (pure decode steps)
    leaves q un-rotated: the decode attention kernels rotate it as they load it (``rope=`` of
    :func:`paged_decode` / :func:`paged_decode_cascade`), which saves q's read and write-back here."""
    kernels().rope_kv_write(qkv, positions, slots, cos, sin, k_cache, v_cache, int(Hq), int(Hkv), int(D), bool(rope_q))


def v_token(v_cache: torch.Tensor, block: int, t: int) -> torch.Tensor:
    """[Hkv, D] view of token `t` of block `block` in a 4-token-interleaved V cache."""
    return v_cache[block, :, t // 4, :, t % 4]


def v_gather(v_cache: torch.Tensor, blocks: torch.Tensor, toks: torch.Tensor) -> torch.Tensor:
    """V rows [L, Hkv, D] of (block, token-in-block) pairs from a 4-token-interleaved V cache."""
    return v_cache[blocks.long(), :, toks.long() // 4, :, toks.long() % 4]


def kv_block_copy(cache: torch.Tensor, pairs: torch.Tensor) -> None:
    """Copy whole KV blocks src->dst for every layer, K and V (K12, copy-on-write fork).
    ``cache`` is viewed as [L*2, num_blocks, ...]."""
    kernels().kv_block_copy(cache, pairs)


# ---------------------------------------------------------------------------------------------
# attention


def paged_decode(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor, block_tables: torch.Tensor,
                 ctx_lens: torch.Tensor, Hq: int, scale: float, num_splits: int = 1,
                 out: Optional[torch.Tensor] = None, part_o: Optional[torch.Tensor] = None,
                 part_lse: Optional[torch.Tensor] = None,
                 rope: Optional[Tuple[torch.Tensor, torch.Tensor, torch.Tensor]] = None) -> torch.Tensor:
    """One-token paged GQA split-K decode attention (K3).  q: [B, >=Hq*D] (row stride allowed).  The
    engine's large batches of forked candidates use :func:`paged_decode_cascade` instead.  ``rope`` =
    (cos, sin, positions [B] int32): q arrives un-rotated and is rotated at load."""
    B = q.shape[0]
    D = k_cache.shape[-1]
    if out is None:
        out = torch.empty(B, Hq, D, dtype=q.dtype, device=q.device)
    if num_splits > 1 and (part_o is None or part_lse is None):
        part_o = torch.empty(B * Hq * num_splits * D, dtype=torch.float32, device=q.device)
        part_lse = torch.empty(B * Hq * num_splits, dtype=torch.float32, device=q.device)
    rc, rs, rp = rope if rope is not None else (None, None, None)
    kernels().paged_decode(q, k_cache, v_cache, block_tables, ctx_lens, out, part_o, part_lse, int(num_splits),
                           float(scale), rc, rs, rp)
    return out


def set_decode_wave_min_items(n: int) -> int:
    """Batch threshold (B * Hkv * splits) above which decode uses the wave-per-item kernel instead of
    the 4-waves-per-sequence kernel; returns the previous value (tests force both paths)."""
    return int(kernels().set_decode_wave_min_items(int(n)))


def cascade_rows_per_tile(G: int) -> int:
    """Sequences per cascade super-tile (8 waves x 16/G sequences)."""
    return int(kernels().cascade_rows_per_tile(int(G)))


class MXAct:
    """An activation in MX form for a block-scaled fp8 GEMM: e4m3 rows ``q`` [M, K] and e8m0 scales ``mx``
    [K/128, M, 4] (one per 32 consecutive values; value = q * 2^(mx - 127)); :func:`linear_fp8` takes it."""

    __slots__ = ("q", "mx")

    def __init__(self, q: torch.Tensor, mx: torch.Tensor):
        self.q, self.mx = q, mx

    def index_select(self, rows: torch.Tensor) -> "MXAct":
        """The activation of ``rows`` only (a prefill's kept last tokens)."""
        q = self.q.view(torch.uint8).index_select(0, rows).view(self.q.dtype)
        return MXAct(q, self.mx.index_select(1, rows).contiguous())


def paged_decode_cascade(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor, block_tables: torch.Tensor,
                         ctx_lens: torch.Tensor, tiles: torch.Tensor, Hq: int, scale: float,
                         out: Optional[torch.Tensor] = None,
                         rope: Optional[Tuple[torch.Tensor, torch.Tensor, torch.Tensor]] = None, mx: bool = False):
    """Cascade decode attention in ONE launch (K3c): per super-tile (row_start, nseq, prefix_blocks) the
    tile's sequences read their shared first `prefix_blocks` blocks once through LDS, then each
    sequence's own blocks; softmax states merge in registers.  Every row < B must be covered by
    exactly one tile (prefix_blocks = 0 for sequences that share nothing).  ``mx=True`` (head_dim 128): the
    output leaves the kernel as an :class:`MXAct` [B, Hq*D] for an fp8 o projection — no bf16 rows, no
    separate quantisation pass."""
    B = q.shape[0]
    D = k_cache.shape[-1]
    rc, rs, rp = rope if rope is not None else (None, None, None)
    if mx:
        q8 = torch.empty(B, Hq * D, dtype=torch.float8_e4m3fn, device=q.device)
        sc = torch.empty(Hq * D // 128, B, 4, dtype=torch.uint8, device=q.device)
        kernels().paged_decode_cascade(q, k_cache, v_cache, block_tables, ctx_lens, tiles, None, int(Hq), float(scale),
                                       rc, rs, rp, q8, sc)
        return MXAct(q8, sc)
    if out is None:
        out = torch.empty(B, Hq, D, dtype=q.dtype, device=q.device)
    kernels().paged_decode_cascade(q, k_cache, v_cache, block_tables, ctx_lens, tiles, out, int(Hq), float(scale),
                                   rc, rs, rp, None, None)
    return out


def prefill_attention(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, cu_seqlens: torch.Tensor, max_seqlen: int,
                      Hq: int, Hkv: int, D: int, scale: float, causal: bool,
                      out: Optional[torch.Tensor] = None, cu_seqlens_k: Optional[torch.Tensor] = None,
                      lens: Optional[Tuple[Sequence[int], Sequence[int]]] = None) -> torch.Tensor:
    """Varlen flash attention forward (K4 causal / K9c bidirectional); q,k,v are [T, H*D] views.
    ``cu_seqlens_k``: k/v hold their own per-sequence ranges (cached-prefix prefill: each sequence's
    queries are the LAST rows of its key range, causal with that offset); ``lens`` = the host-side
    (q lengths, k lengths), checked here before the launch."""
    if out is None:
        out = torch.empty(q.shape[0], Hq * D, dtype=q.dtype, device=q.device)
    if cu_seqlens_k is not None:
        if lens is None:
            raise ValueError("prefill_attention: cu_seqlens_k needs the host-side lengths")
        ql, kl = lens
        if len(ql) != len(kl) or any(a > b for a, b in zip(ql, kl)) or sum(kl) > k.shape[0] or sum(ql) > q.shape[0]:
            raise ValueError("prefill_attention: key ranges must cover their queries and fit k/v")
    kernels().prefill_attention(q, k, v, out, cu_seqlens, int(max_seqlen), int(Hq), int(Hkv), int(D), float(scale),
                                bool(causal), cu_seqlens_k)
    return out


def prefill_attention_mx(q: torch.Tensor, k: torch.Tensor, v: torch.Tensor, cu_seqlens: torch.Tensor,
                         max_seqlen: int, Hq: int, Hkv: int, scale: float, causal: bool) -> "MXAct":
    """:func:`prefill_attention` (head_dim 128, keys = queries) with the output in MX form for the fp8 o
    projection: e4m3 rows [T, Hq*128] + e8m0 scales [Hq, T, 4] straight from the kernel's epilogue (the
    decode cascade kernel's format) — no bf16 output, no row quantisation pass."""
    T = q.shape[0]
    q8 = torch.empty(T, Hq * 128, dtype=torch.float8_e4m3fn, device=q.device)
    mx = torch.empty(Hq, T, 4, dtype=torch.uint8, device=q.device)
    kernels().prefill_attention_mx(q, k, v, q8.view(torch.uint8), mx, cu_seqlens, int(max_seqlen), int(Hq), int(Hkv),
                                   float(scale), bool(causal))
    return MXAct(q8, mx)


def prefill_attention_paged(q: torch.Tensor, k_cache: torch.Tensor, v_cache: torch.Tensor, cu_seqlens: torch.Tensor,
                            block_tables: torch.Tensor, k_lens: torch.Tensor, max_seqlen: int, Hq: int, scale: float,
                            out: Optional[torch.Tensor] = None, lens: Optional[Tuple[Sequence[int], Sequence[int]]] = None
                            ) -> torch.Tensor:
    """Causal attention of query chunks against the PAGED KV cache (K4, mixed chunked prefill): sequence s's
    queries (rows cu_seqlens[s]..cu_seqlens[s+1] of q) are its key positions [k_lens[s] - len_q, k_lens[s]),
    keys read through ``block_tables`` [nseq, W] (W even, >= 2 * ceil(max k_len / 32)) — no gather of the
    cached keys.  ``lens`` = host-side (q lengths, k lengths), checked here before the launch."""
    D = k_cache.shape[-1]
    if out is None:
        out = torch.empty(q.shape[0], Hq * D, dtype=q.dtype, device=q.device)
    if lens is not None:
        ql, kl = lens
        W = block_tables.shape[1]
        if (len(ql) != len(kl) or any(a > b for a, b in zip(ql, kl)) or sum(ql) > q.shape[0]
                or any(-(-k // 32) * 2 > W for k in kl)):
            raise ValueError("prefill_attention_paged: key lengths must cover the queries and fit the block tables")
    kernels().prefill_attention_paged(q, k_cache, v_cache, out, cu_seqlens, block_tables, k_lens, int(max_seqlen),
                                      int(Hq), float(scale))
    return out


def kv_gather(k_cache: torch.Tensor, v_cache: torch.Tensor, slots: torch.Tensor):
    """Token rows of one layer's paged cache -> contiguous (k [n, Hkv*D], v [n, Hkv*D]) bf16, for the
    cached-prefix prefill (the cached blocks' keys/values next to the freshly written ones).  ``slots``
    [n] int64 = block * BS + offset; k_cache [NB, Hkv, BS, D], v_cache [NB, Hkv, BS/4, D, 4]."""
    NB, Hkv, BS, D = k_cache.shape
    slots = slots.to(torch.int64).contiguous()  # < NB * BS: the caller checks on the host (no device sync here)
    k = torch.empty(slots.numel(), Hkv * D, dtype=k_cache.dtype, device=k_cache.device)
    v = torch.empty_like(k)
    kernels().kv_gather(k_cache, v_cache, slots, k, v)
    return k, v


# ---------------------------------------------------------------------------------------------
# GEMM


def grouped_gemm(A: torch.Tensor, W: torch.Tensor, row_off: torch.Tensor, max_slots: Optional[int] = None,
                 out: Optional[torch.Tensor] = None, a_scale: Optional[torch.Tensor] = None,
                 w_scale: Optional[torch.Tensor] = None, bias: Optional[torch.Tensor] = None,
                 a_rows: Optional[torch.Tensor] = None, rows: Optional[int] = None,
                 splits: Optional[int] = None, swiglu: bool = False,
                 a_mx: Optional[torch.Tensor] = None) -> torch.Tensor:
    """Grouped GEMM on MFMA (K6g): rows [row_off[g], row_off[g+1]) of A times W[g]^T -> C [rows, N] bf16.
    ``a_rows`` [rows] gathers A's row for each output row (MoE dispatch; then ``rows`` = len(a_rows)).
    ``row_off`` lives on the device (MoE expert segments: no host sync, graph-capturable).  fp8 e4m3fn
    A/W take per-row ``a_scale`` and per-channel ``w_scale`` (config 5).  ``max_slots`` bounds the m-tiles
    (default: ceil(rows/128) + G, enough for any split of the rows into G groups).  ``splits`` > 1 splits
    K over that many workgroups per tile (fp32 atomics into a workspace, then one bf16 pass); default:
    chosen so a small-M launch (MoE decode down projection: 8 experts x 32 column tiles) still puts
    ~4 workgroups on every CU.  ``swiglu=True``: W's rows are gate / up interleaved in blocks of 32
    (:func:`swiglu_interleave` per group) and the result is silu(gate) * up [rows, N/2] — from the 8-phase
    kernel's epilogue when it takes the batch, else GEMM + the SwiGLU pass.  ``a_mx`` [K/128, rows, 4] uint8:
    A carries MX block scales (from :func:`grouped_gemm_swiglu_mx`) instead of ``a_scale`` — 8-phase kernel
    only."""
    if rows is None:
        rows = a_rows.numel() if a_rows is not None else A.shape[0]
    G, N, K = W.shape[0], W.shape[1], W.shape[2]
    if a_mx is not None:
        if out is None:
            out = torch.empty(rows, N, dtype=torch.bfloat16, device=A.device)
        kernels().gemm8g_fp8(A, W, out, row_off, -(-rows // 256) + G, None, None, w_scale.contiguous(), 0, a_mx, None)
        return out
    if _use_gemm8g(A, W, rows, G, N, K, bias, splits, out) and (not swiglu or N % 64 == 0):
        # large fp8 expert batches (>= ~1 full 256-row tile per expert on average): the 8-phase kernel
        if out is None:
            out = torch.empty(rows, N // 2 if swiglu else N, dtype=torch.bfloat16, device=A.device)
        kernels().gemm8g_fp8(A, W, out, row_off, -(-rows // 256) + G, a_rows, a_scale, w_scale.contiguous(),
                             int(bool(swiglu)), None, None)
        return out
    if swiglu:
        return silu_mul(grouped_gemm(A, W, row_off, max_slots=max_slots, a_scale=a_scale, w_scale=w_scale,
                                     bias=bias, a_rows=a_rows, rows=rows, splits=splits), out=out, block=32)
    if max_slots is None:
        max_slots = -(-rows // 128) + G
    if out is None:
        out = torch.empty(rows, N, dtype=torch.bfloat16, device=A.device)
    if splits is None:
        k_tiles = K * W.element_size() // 128
        wgs = max(1, -(-rows // 128)) * -(-N // 128)  # lower bound on the live tiles
        splits = max(1, min(k_tiles // 8, -(-1024 // wgs))) if wgs < 512 else 1
    kernels().grouped_gemm(A, W, out, row_off, int(max_slots), a_scale, w_scale, bias, a_rows, int(splits))
    return out


MOE_GEMM = os.environ.get("LWC_MOE_GEMM", "auto")  # auto | g8 (8-phase grouped fp8) | classic (128x128)
# fp8 expert FFN middle in MX form (gate|up epilogue writes e4m3 + e8m0 block scales, the down GEMM's MFMAs
# apply them): "1" (default) where both GEMMs take the 8-phase kernel, "0" = SwiGLU epilogue + row quantisation
MOE_MX = os.environ.get("LWC_MOE_MX", "1") != "0"


def grouped_gemm_swiglu_mx(A: torch.Tensor, W: torch.Tensor, row_off: torch.Tensor, a_scale: torch.Tensor,
                           w_scale: torch.Tensor, a_rows: Optional[torch.Tensor] = None, rows: Optional[int] = None):
    """Grouped fp8 gate|up GEMM (W rows gate / up interleaved in blocks of 32) with SwiGLU in the epilogue and
    the activation written as MX e4m3: -> (q [rows, F] e4m3, mx [F/128, rows, 4] uint8 e8m0).  Block b of each
    128-column slice is its columns [32b, 32b + 32); value = q * 2^(mx - 127).  The down GEMM takes them through ``grouped_gemm(q, W2, row_off, a_mx=mx)``, so
    the activation never exists in bf16 in HBM and no separate quantisation pass runs."""
    if rows is None:
        rows = a_rows.numel() if a_rows is not None else A.shape[0]
    G, N, K = W.shape
    F_ = N // 2
    q = torch.empty(rows, F_, dtype=torch.float8_e4m3fn, device=A.device)
    mx = torch.empty(N // 256, rows, 4, dtype=torch.uint8, device=A.device)
    kernels().gemm8g_fp8(A, W, q, row_off, -(-rows // 256) + G, a_rows, a_scale, w_scale.contiguous(), 2, None, mx)
    return q, mx


def moe_mx_ok(A: torch.Tensor, W13: torch.Tensor, W2: torch.Tensor, rows: int) -> bool:
    """Whether the expert FFN runs its middle in MX form (both GEMMs on the 8-phase kernel)."""
    if not MOE_MX or A.dtype != torch.float8_e4m3fn or W2.dtype != torch.float8_e4m3fn:
        return False
    G, N, K = W13.shape
    if N % 256 or W2.shape[2] != N // 2 or not _use_gemm8g(A, W13, rows, G, N, K, None, None, None):
        return False
    return rows * (N // 2) < (1 << 31) and (N // 256) * rows * 4 < (1 << 31)


def _use_gemm8g(A, W, rows, G, N, K, bias, splits, out) -> bool:
    if MOE_GEMM == "classic" or A.dtype != torch.float8_e4m3fn or bias is not None or (splits or 1) > 1:
        return False
    if K % 128 or N % 8 or A.stride(0) % 16 or A.shape[0] * A.stride(0) >= (1 << 31) or 256 * K >= (1 << 31):
        return False
    if out is not None and (out.stride(1) != 1 or out.stride(0) % 8):
        return False
    return MOE_GEMM == "g8" or rows >= 32 * G


def gemm8p(A: torch.Tensor, W: torch.Tensor, residual: Optional[torch.Tensor] = None,
           out: Optional[torch.Tensor] = None, swiglu: bool = False, ws=None, bias: Optional[torch.Tensor] = None,
           gelu: bool = False) -> torch.Tensor:
    """8-phase 256x256-tile MFMA GEMM (K6, csrc/kernels/gemm8p.hip): A [M, K] . W[N, K]^T (+ residual)
    -> [M, N] bf16.  ``swiglu=True`` takes a gate/up weight laid out by :func:`swiglu_interleave` and
    returns silu(A Wg^T) * (A Wu^T) [M, N/2] from the GEMM epilogue (no [M, N] intermediate).
    ``ws`` = (partials, flags) stream-K workspace (:func:`gemm8p_workspace`); a model passes its own so
    a captured graph owns no allocation; default: one per (device, stream), created outside capture.
    ``bias`` [N] (+ ``gelu``: exact erf GELU) is applied to the fp32 accumulators in the epilogue (the
    encoder's projections; FFN1's bias+GELU needs no separate pass)."""
    N = W.shape[0] // 2 if swiglu else W.shape[0]
    if out is None:
        out = torch.empty(A.shape[0], N, dtype=torch.bfloat16, device=A.device)
    if bias is not None:
        if swiglu or residual is not None:
            raise ValueError("gemm8p: bias epilogue combines with neither swiglu nor residual")
        epi, residual = (4 if gelu else 3), bias
    else:
        if gelu:
            raise ValueError("gemm8p: gelu needs a bias")
        epi = 2 if swiglu else (1 if residual is not None else 0)
    part, flags = ws if ws is not None else gemm8p_workspace(A.device)
    kernels().gemm8p(A, W, out, residual, epi, part, flags)
    return out


def skinny_gemm(A: torch.Tensor, W: torch.Tensor, residual: Optional[torch.Tensor] = None,
                out: Optional[torch.Tensor] = None, swiglu: bool = False) -> torch.Tensor:
    """Decode-sized projection (K6, csrc/kernels/skinny.hip): ``A [M <= 64, K] . W[N, K]^T`` (+ ``residual``,
    in place with ``out=residual``; or ``swiglu`` over a 32-row gate/up interleaved W, output [M, N / 2]) as a
    weight stream — one workgroup per 16 output columns, its 8 waves splitting K, partials summed in LDS in a
    fixed order.  Needs K % 2048 == 0 and N % 16 == 0 (SwiGLU: N % 64 == 0) (:func:`skinny_ok`)."""
    if swiglu and residual is not None:
        raise ValueError("skinny_gemm: swiglu and residual do not combine")
    if out is None:
        out = torch.empty(A.shape[0], W.shape[0] // 2 if swiglu else W.shape[0], dtype=torch.bfloat16,
                          device=A.device)
    kernels().skinny_gemm(A, W, out, residual, 2 if swiglu else (1 if residual is not None else 0))
    return out


def skinny_ok(M: int, N: int, K: int, swiglu: bool = False) -> bool:
    return 0 < M <= 64 and K % 2048 == 0 and N % (64 if swiglu else 16) == 0


def gemm4w(A: torch.Tensor, W: torch.Tensor, residual: Optional[torch.Tensor] = None,
           out: Optional[torch.Tensor] = None, swiglu: bool = False, bias: Optional[torch.Tensor] = None,
           gelu: bool = False, bn: int = 256, chain: "Optional[NormChain]" = None, var: int = 0,
           gm: int = 0, splits: int = 1, split_from: int = 0) -> torch.Tensor:
    """4-wave interleaved MFMA GEMM (K6, csrc/kernels/gemm4w.hip): one wave per SIMD owns a 128 x bn/2 slice of
    a 256 x ``bn`` tile (bn 256 or 192) with its 256 (192) fp32 accumulators in AGPRs; data-parallel tiles, no
    workspace.  Same epilogues as :func:`gemm8p`: ``residual`` (in place with ``out=residual``), ``swiglu``
    (interleaved gate|up W, bn 256), ``bias`` (+ ``gelu``).

    Folded RMSNorm (the decode chain, :class:`NormChain`): with ``chain`` a plain / SwiGLU projection scales
    its accumulator rows by 1/rms of its input rows from the chain's partial row sums of squares (the norm
    weight folded into W: rmsnorm(x) . W^T), and a residual projection writes the partials of its output for
    the next one.  ``var``: schedule (64: wave-local epilogue + next-tile prefetch, else 32: block-staged
    epilogue); ``gm``: m-tiles per group of the grouped tile order (0: by shape, see gemm4w.hip).

    Split-K (``splits`` > 1, schedule 64): the output tiles from ``split_from`` on run as ``splits`` units over
    about K / splits each (even K tile counts: K / 64 even and >= 2 * splits); the first arrivers publish fp32 partials, the last adds them and runs the epilogue (no
    workgroup waits on one that has not started).  For shapes whose tile count leaves CUs idle (the serving
    path's mid-size row counts: :func:`split_plan`) and a ragged last round (``split_from`` = the whole
    rounds).  The workspace is this module's, sized before graph capture (:func:`split_workspace`)."""
    N = W.shape[0] // 2 if swiglu else W.shape[0]
    if out is None:
        out = torch.empty(A.shape[0], N, dtype=torch.bfloat16, device=A.device)
    if bias is not None:
        if swiglu or residual is not None:
            raise ValueError("gemm4w: bias epilogue combines with neither swiglu nor residual")
        epi, residual = (4 if gelu else 3), bias
    else:
        if gelu:
            raise ValueError("gemm4w: gelu needs a bias")
        epi = 2 if swiglu else (1 if residual is not None else 0)
    sk = (int(splits), int(split_from), None, None)
    if splits > 1:
        part, cnt = split_workspace(A.shape[0], W.shape[0], bn, splits, split_from, A.device)
        sk = (int(splits), int(split_from), part, cnt)
    if chain is None:
        # (one launch for any M: the kernel's A resource spans one tile's rows.  Config 2's FFN2 input, 3 GiB at
        # 0.5 M tokens, ran as two row blocks before — 16 + 9 rounds, the second's last round holding one tile)
        kernels().gemm4w(A, W, out, residual, epi, int(bn), None, 0, 0, 0.0, int(var), int(gm), *sk)
    elif epi == 1:
        kernels().gemm4w(A, W, out, residual, epi, int(bn), chain.ss, 2, 0, 0.0, int(var), int(gm), *sk)
        chain.P = (N + 255) // 256
    elif epi in (0, 2):
        kernels().gemm4w(A, W, out, residual, epi, int(bn), chain.ss, 1, chain.P, chain.eps, int(var), int(gm), *sk)
    else:
        raise ValueError("gemm4w: chain= goes with the plain, SwiGLU or residual epilogue")
    return out


# split-K workspace of gemm4w (per device and host thread: two engines on two threads never share counters):
# fp32 partial slabs + the per-tile ticket / done counters (zeroed once; each tile's last arriver resets its
# pair).  Grown only outside graph capture; a replaced workspace is kept alive (_SPLIT_WS_RETIRED), since
# graphs captured before the growth still address it.
_SPLIT_WS: dict = {}
_SPLIT_WS_RETIRED: list = []


def split_workspace(M: int, N: int, bn: int, splits: int, split_from: int, device):
    """(part, cnt) big enough for a split-K gemm4w call of this shape (W rows N: for SwiGLU the interleaved
    gate|up rows).  Allocated / grown here, never under graph capture (a capture then needs it pre-sized by an
    eager call of the same shape: the planners time every backend before capturing)."""
    tiles = ((M + 255) // 256) * ((N + bn - 1) // bn)
    need_p = max(0, tiles - max(0, min(split_from, tiles))) * (splits - 1) * 256 * bn
    need_c = 2 * tiles
    key = (str(device), threading.get_ident())
    ws = _SPLIT_WS.get(key)
    if ws is None or ws[0].numel() < need_p or ws[1].numel() < need_c:
        if ws is not None:
            _SPLIT_WS_RETIRED.append(ws)
        if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
            raise RuntimeError("gemm4w split-K workspace must be sized before graph capture")
        old_p = ws[0].numel() if ws is not None else 0
        old_c = ws[1].numel() if ws is not None else 0
        ws = (torch.empty(max(need_p, old_p, 1), dtype=torch.float32, device=device),
              torch.zeros(max(need_c, old_c), dtype=torch.int32, device=device))
        _SPLIT_WS[key] = ws
    return ws


def split_plan(M: int, N: int, K: int, bn: int = 256, cus: int = 256) -> tuple:
    """(splits, split_from) for gemm4w's split-K (VAR 64 units: an even K tile count each), or (1, 0):
    * at most half as many tiles as CUs (the serving path's mid-size row counts: o / down at M = 2048 are 128
      tiles): the whole call split 2 or 4 ways while the units fit one round (a second round of half-K units
      costs what one round of whole tiles does: M = 2304's 144 tiles measured 136 vs 86 us split);
    * a ragged last round of at most half the CUs (lm_head at M = 4096: 8016 tiles = 31 rounds + 80): only that
      round's tiles split, 2 or 4 ways, into at most one round of shorter units."""
    tiles = ((M + 255) // 256) * ((N + bn - 1) // bn)
    KT = K // 64

    def ok(s):
        return KT % s == 0 and (KT // s) % 2 == 0

    if tiles <= cus // 2:
        s = 1
        while s < 4 and tiles * s * 2 <= cus and ok(2 * s):
            s *= 2
        return (s, 0) if s > 1 else (1, 0)
    tail = tiles % cus
    if 0 < tail <= cus // 2:
        s = 4 if tail * 4 <= cus and ok(4) else (2 if ok(2) else 1)
        return (s, tiles - tail) if s > 1 else (1, 0)
    return (1, 0)


class NormChain:
    """Buffers of the folded-RMSNorm decode chain (csrc/kernels/gemm4w.hip head): ``ss`` [16, max_rows] fp32
    partial row sums of squares of the residual stream — written by a residual projection (``P`` = its
    N / 256 partials) or :func:`rms_rowsumsq` (P = 1), read by the next plain / SwiGLU projection, which scales
    its rows by rsqrt(sum / K + eps).  Allocated once, outside graph capture (captured graphs keep its address)."""

    def __init__(self, max_rows: int, d: int, eps: float, device):
        if torch.cuda.is_available() and torch.cuda.is_current_stream_capturing():
            raise RuntimeError("NormChain buffers must be allocated outside hipGraph capture")
        if (d + 255) // 256 > 16:
            raise ValueError("NormChain: at most 16 partials per row (d <= 4096)")
        self.max_rows, self.d, self.eps = int(max_rows), int(d), float(eps)
        # rows padded to a multiple of 64 floats: every partial's LDS-DMA source is 16-byte aligned
        self.ss = torch.zeros(16, (self.max_rows + 63) // 64 * 64, dtype=torch.float32, device=device)
        self.P = 1

    def scales(self, M: int) -> torch.Tensor:
        """The row scales the consumers apply, for tests: rsqrt(sum of the P partials / d + eps)."""
        return torch.rsqrt(self.ss[:self.P, :M].sum(0) / self.d + self.eps)


def rms_rowsumsq(x: torch.Tensor, chain: "NormChain") -> None:
    """Start a chain: chain.ss[0] = the row sums of squares of x (one partial, P = 1)."""
    kernels().rms_rowsumsq(x, chain.ss)
    chain.P = 1


_G8_WS: dict = {}


def new_gemm8p_workspace(device: torch.device):
    """(fp32 partials [slots * 65536], int32 flags [slots]) for gemm8p's stream-K tail.  GEMMs that may
    run concurrently (different streams) need different workspaces; the kernel leaves the flags zero."""
    if torch.cuda.is_current_stream_capturing():
        raise RuntimeError("gemm8p workspace must be allocated outside hipGraph capture")
    slots = kernels().gemm8p_slots()
    return (torch.empty(slots * 65536, dtype=torch.float32, device=device),
            torch.zeros(slots, dtype=torch.int32, device=device))


def gemm8p_workspace(device: torch.device):
    """Default gemm8p workspace of the current (device, stream)."""
    device = torch.device(device)
    key = (device.index, torch.cuda.current_stream(device).cuda_stream)
    ws = _G8_WS.get(key)
    if ws is None:
        ws = _G8_WS[key] = new_gemm8p_workspace(device)
    return ws


def swiglu_interleave(w_gate_up: torch.Tensor, block: int = 32) -> torch.Tensor:
    """[gate (F rows); up (F rows)] -> rows interleaved in blocks of ``block``: gate[0:32], up[0:32],
    gate[32:64], ... — the layout gemm8p's SwiGLU epilogue expects (each 64-row group of a tile holds a
    gate block and the matching up block)."""
    F2, K = w_gate_up.shape
    F = F2 // 2
    assert F % block == 0, "ffn size must be a multiple of the interleave block"
    g, u = w_gate_up[:F].view(F // block, block, K), w_gate_up[F:].view(F // block, block, K)
    return torch.stack([g, u], dim=1).reshape(F2, K).contiguous()


def moe_route(logits: torch.Tensor, k: int):
    """Router top-k + softmax over the selected logits, expert segments and dispatch permutation (K11a).
    logits [T, E] bf16 -> (topk_ids [T,k] i32, topk_w [T,k] f32, row_off [E+1] i32, src_row [T*k] i32,
    inv [T*k] i32): expert-sorted row p reads token src_row[p]; (t, j) landed at row inv[t*k+j]."""
    T, E = logits.shape
    dev = logits.device
    ids = torch.empty(T, k, dtype=torch.int32, device=dev)
    w = torch.empty(T, k, dtype=torch.float32, device=dev)
    row_off = torch.empty(E + 1, dtype=torch.int32, device=dev)
    src = torch.empty(T * k, dtype=torch.int32, device=dev)
    inv = torch.empty(T * k, dtype=torch.int32, device=dev)
    kernels().moe_route(logits.contiguous(), int(k), ids, w, row_off, src, inv)
    return ids, w, row_off, src, inv


def moe_router(h: torch.Tensor, router: torch.Tensor, k: int, want_logits: bool = False):
    """Router GEMV fused with :func:`moe_route` (K11a): h [T, d] bf16 . router [E, d]^T -> the same five
    tensors (plus the bf16 logits [T, E] with ``want_logits``).  The logits are rounded to bf16 inside the
    kernel as ``F.linear`` would hold them, so expert choices match the unfused path.  E <= 16."""
    T = h.shape[0]
    E = router.shape[0]
    dev = h.device
    ids = torch.empty(T, k, dtype=torch.int32, device=dev)
    w = torch.empty(T, k, dtype=torch.float32, device=dev)
    row_off = torch.empty(E + 1, dtype=torch.int32, device=dev)
    src = torch.empty(T * k, dtype=torch.int32, device=dev)
    inv = torch.empty(T * k, dtype=torch.int32, device=dev)
    logits = torch.empty(T, E, dtype=torch.bfloat16, device=dev) if want_logits else None
    kernels().moe_router(h, router.contiguous(), int(k), ids, w, row_off, src, inv, logits)
    out = (ids, w, row_off, src, inv)
    return out + (logits,) if want_logits else out


def route(h: torch.Tensor, router: torch.Tensor, k: int):
    """MoE routing of bf16 rows: the fused router kernel on the GPU (E <= 16, d % 8 == 0), else the
    router projection + :func:`moe_route`."""
    if h.is_cuda and router.shape[0] <= 16 and h.shape[1] % 8 == 0 and h.stride(1) == 1 and h.stride(0) % 8 == 0:
        return moe_router(h, router, k)
    return moe_route(torch.nn.functional.linear(h, router), k)


def moe_combine(Y: torch.Tensor, inv: torch.Tensor, w: torch.Tensor, k: int,
                out: Optional[torch.Tensor] = None) -> torch.Tensor:
    """out[t] = sum_j w[t, j] * Y[inv[t*k + j]] (K11d): expert outputs back to token order."""
    T = w.shape[0]
    if out is None:
        out = torch.empty(T, Y.shape[1], dtype=Y.dtype, device=Y.device)
    kernels().moe_combine(Y, inv, w, int(k), out)
    return out


def quant_fp8_rows(x: torch.Tensor):
    """Per-row dynamic OCP e4m3 quantisation: (q [.., d] float8_e4m3fn, scale [rows] f32), x ~= q * scale."""
    q = torch.empty(x.shape, dtype=torch.float8_e4m3fn, device=x.device)
    scale = torch.empty(x.numel() // x.shape[-1], dtype=torch.float32, device=x.device)
    kernels().quant_fp8_rows(x.contiguous(), q, scale)
    return q, scale


def silu_mul_quant_fp8(gate_up: torch.Tensor, block: int = 0):
    """SwiGLU + per-row e4m3 quantisation fused (MoE expert FFN between its fp8 GEMMs): [rows, 2F] bf16 ->
    (q [rows, F] float8_e4m3fn, scale [rows] f32) — equal to quant_fp8_rows(silu_mul(gate_up)) without the
    bf16 activation round trip through HBM."""
    rows, F = gate_up.shape[0], gate_up.shape[1] // 2
    q = torch.empty(rows, F, dtype=torch.float8_e4m3fn, device=gate_up.device)
    scale = torch.empty(rows, dtype=torch.float32, device=gate_up.device)
    kernels().silu_mul_quant_fp8(gate_up.contiguous(), q, scale, int(block))
    return q, scale


def quant_fp8_weight(w: torch.Tensor):
    """Per-output-channel OCP e4m3 weight quantisation (host-side torch, load time): w [..., N, K] ->
    (q e4m3fn, scale [..., N] f32)."""
    s = (w.float().abs().amax(-1).clamp(min=1e-12) / 448.0)
    q = (w.float() / s.unsqueeze(-1)).to(torch.float8_e4m3fn)
    return q.contiguous(), s.contiguous()


class Fp8Weight:
    """A dense projection weight in OCP e4m3 with per-output-channel scales (``w ~= q * s[:, None]``), for
    the fp8 configurations (BASELINE config 5).  Built once at load time."""

    __slots__ = ("q", "s", "shape")

    def __init__(self, w: torch.Tensor):
        q, s = quant_fp8_weight(w)
        self.q, self.s = q, s.view(1, -1).contiguous()
        self.shape = tuple(w.shape)


# dense fp8 projections (config 5): "auto" times the hand-written 8-phase fp8 core (gemm8g in dense mode)
# against hipBLASLt's row-scaled fp8 GEMM per (row bucket, N, K) on the first eager call and keeps the
# hand-written one unless the library is faster by more than FP8_OWN_MARGIN; "g8g" / "blas" force one.
FP8_GEMM = os.environ.get("LWC_FP8_GEMM", "auto")
FP8_OWN_MARGIN = float(os.environ.get("LWC_FP8_OWN_MARGIN", "0.01"))
FP8_CHOICE: dict = {}
FP8_TIMINGS: dict = {}


def _fp8_bucket(M: int) -> int:
    return min(1 << max(M - 1, 1).bit_length(), 1 << 16)


def _g8g_dense_ok(xq: torch.Tensor, w: "Fp8Weight") -> bool:
    N, K = w.q.shape
    M = xq.shape[0]
    return (xq.is_cuda and xq.stride(1) == 1 and xq.stride(0) % 16 == 0 and K % 128 == 0 and N % 8 == 0
            and M >= 0 and 256 * K < (1 << 31) and xq.dtype == torch.float8_e4m3fn)


G8G_SPAN = 1 << 31  # bytes of A one gemm8g launch may address (its buffer range is 32-bit)


def gemm8g_dense(xq: torch.Tensor, xs: torch.Tensor, w: "Fp8Weight", out: Optional[torch.Tensor] = None,
                 swiglu: bool = False):
    """Dense fp8 GEMM on the hand-written 8-phase core (csrc/kernels/gemm8g.hip, G = 1, no row table):
    (xq [M, K] e4m3 . w.q^T) * xs[row] * w.s[col] -> bf16 [M, N]; ``swiglu``: w's rows are gate|up interleaved
    in blocks of 32 (:func:`swiglu_interleave`) and the epilogue writes silu(gate) * up, bf16 [M, N / 2].
    The kernel addresses A through a 32-bit buffer range: row blocks of < 2 GiB of A go one launch each
    (the e5-mistral embedder's prefill is ~0.5 M rows)."""
    M = xq.shape[0]
    N, K = w.q.shape
    if out is None:
        out = torch.empty(M, N // 2 if swiglu else N, dtype=torch.bfloat16, device=xq.device)
    if M == 0:
        return out
    step = max(256, (G8G_SPAN - 1) // xq.stride(0) // 256 * 256)
    s, ws, wq = xs.reshape(-1).contiguous(), w.s.reshape(-1), w.q.view(1, N, K)
    for r0 in range(0, M, step):
        r1 = min(M, r0 + step)
        kernels().gemm8g_fp8(xq[r0:r1], wq, out[r0:r1], None, -(-(r1 - r0) // 256), None, s[r0:r1], ws,
                             int(bool(swiglu)), None, None)
    return out


def _fp8_blas(xq, xs, w):
    return torch._scaled_mm(xq, w.q.t(), scale_a=xs.view(-1, 1), scale_b=w.s, out_dtype=torch.bfloat16)


def linear_fp8_q(xq: torch.Tensor, xs: torch.Tensor, w: Fp8Weight) -> torch.Tensor:
    """(e4m3 rows xq [M, K], row scales xs [M]) . w^T -> bf16 [M, N] (K6 fp8).  The hand-written 8-phase fp8
    core (:func:`gemm8g_dense`) or hipBLASLt's row-scaled fp8 GEMM (``torch._scaled_mm``), chosen per
    (row bucket, N, K) by timing (see FP8_GEMM); shapes the hand-written core does not take use the library."""
    if not _g8g_dense_ok(xq, w) or FP8_GEMM == "blas":
        return _fp8_blas(xq, xs, w)
    if FP8_GEMM == "g8g":
        return gemm8g_dense(xq, xs, w)
    M = xq.shape[0]
    key = (_fp8_bucket(M), w.q.shape[0], w.q.shape[1])
    c = FP8_CHOICE.get(key)
    if c is None:
        if torch.cuda.is_current_stream_capturing():
            c = "g8g" if M >= 256 else "blas"  # untimed shape inside a capture: no timing possible
        else:
            from .gemm_plan import _time

            t_own = _time(lambda: gemm8g_dense(xq, xs, w), iters=3, rounds=3)
            t_blas = _time(lambda: _fp8_blas(xq, xs, w), iters=3, rounds=3)
            FP8_TIMINGS[key] = {"g8g": t_own, "blas": t_blas}
            c = FP8_CHOICE[key] = "g8g" if t_own <= t_blas * (1 + FP8_OWN_MARGIN) else "blas"
    return gemm8g_dense(xq, xs, w) if c == "g8g" else _fp8_blas(xq, xs, w)


def linear_fp8_swiglu(x, w: Fp8Weight, block: int):
    """fp8 gate|up projection + SwiGLU + per-row e4m3 quantisation of the activation (the dense fp8 MLP's
    middle, config 5's e5-mistral embedder): x (bf16 [M, d] or a :class:`QAct`) -> (q [M, F] e4m3,
    scale [M] f32) for the down projection.  Two pipelines, timed per (row bucket, N, K) like
    :func:`linear_fp8_q`: gemm8g with SwiGLU in its epilogue then one quantisation pass over [M, F] (needs
    ``block`` == 32, the interleave the epilogue reads), or hipBLASLt's fp8 GEMM writing [M, 2F] bf16 then
    the fused silu_mul_quant_fp8 pass — the first never writes the [M, 2F] intermediate."""
    xq, xs = (x.q, x.s) if isinstance(x, QAct) else quant_fp8_rows(x)

    def own():
        return quant_fp8_rows(gemm8g_dense(xq, xs, w, swiglu=True))

    def lib():
        return silu_mul_quant_fp8(_fp8_blas(xq, xs, w), block)

    N, K = w.q.shape
    if block != 32 or N % 64 or not _g8g_dense_ok(xq, w) or FP8_GEMM == "blas":
        return silu_mul_quant_fp8(linear_fp8_q(xq, xs, w), block)
    if FP8_GEMM == "g8g":
        return own()
    key = ("swiglu", _fp8_bucket(xq.shape[0]), N, K)
    c = FP8_CHOICE.get(key)
    if c is None:
        if torch.cuda.is_current_stream_capturing():
            c = "g8g" if xq.shape[0] >= 256 else "blas"
        else:
            from .gemm_plan import _time

            t_own = _time(own, iters=3, rounds=3)
            t_blas = _time(lib, iters=3, rounds=3)
            FP8_TIMINGS[key] = {"g8g": t_own, "blas": t_blas}
            c = FP8_CHOICE[key] = "g8g" if t_own <= t_blas * (1 + FP8_OWN_MARGIN) else "blas"
    return own() if c == "g8g" else lib()


# dense fp8 MLP middle in MX form (config 5's embedder prefill): gate|up on gemm8g with the SwiGLU epilogue
# writing e4m3 + e8m0 block scales, the down projection's MFMAs applying them.  Taken from DENSE_MX_MIN_ROWS
# rows, where gemm8g wins both projections (profiles/moe_round4.md); "LWC_DENSE_MX=0" keeps the row-scaled path
DENSE_MX = os.environ.get("LWC_DENSE_MX", "1") != "0"
DENSE_MX_MIN_ROWS = 16384


@contextlib.contextmanager
def dense_mx_min_rows(rows: int):
    """Temporarily take the MX dense-MLP path from ``rows`` rows on (the benches' self-check re-embeds one
    request's candidates — a few thousand rows — on the path the whole batch took, so it compares sharding,
    not the MX vs row-quantised fp8 numerics: ~0.026 apart in cosine at config 5)."""
    global DENSE_MX_MIN_ROWS
    old, DENSE_MX_MIN_ROWS = DENSE_MX_MIN_ROWS, int(rows)
    try:
        yield
    finally:
        DENSE_MX_MIN_ROWS = old


def dense_mx_ok(x, w_gu: Fp8Weight, w_down: Fp8Weight, block: int) -> bool:
    xq = x.q if isinstance(x, QAct) else x
    M = xq.shape[0]
    N, K = w_gu.q.shape
    return (DENSE_MX and FP8_GEMM != "blas" and block == 32 and M >= DENSE_MX_MIN_ROWS and xq.is_cuda
            and N % 256 == 0 and K % 128 == 0 and w_down.q.shape[1] == N // 2 and w_down.q.shape[0] % 8 == 0)


def _row_blocks(M: int, row_bytes: int):
    step = max(256, (G8G_SPAN - 1) // row_bytes // 256 * 256)
    return [(r0, min(M, r0 + step)) for r0 in range(0, M, step)]


def linear_fp8_swiglu_mx(x, w: Fp8Weight):
    """Dense fp8 gate|up (rows interleaved in blocks of 32) + SwiGLU with the activation written in MX form:
    -> (q [M, F] e4m3, mx [F/128, M, 4] uint8 e8m0) for :func:`linear_fp8_mx`.  Row blocks as in
    :func:`gemm8g_dense` (the scales are per row, so the down GEMM may block its rows differently)."""
    xq, xs = (x.q, x.s) if isinstance(x, QAct) else quant_fp8_rows(x)
    M = xq.shape[0]
    N, K = w.q.shape
    q = torch.empty(M, N // 2, dtype=torch.float8_e4m3fn, device=xq.device)
    mx = torch.empty(N // 256, M, 4, dtype=torch.uint8, device=xq.device)
    s, ws, wq = xs.reshape(-1).contiguous(), w.s.reshape(-1), w.q.view(1, N, K)
    for r0, r1 in _row_blocks(M, xq.stride(0)):
        kernels().gemm8g_fp8(xq[r0:r1], wq, q[r0:r1], None, -(-(r1 - r0) // 256), None, s[r0:r1], ws, 2, None,
                             mx[:, r0:r1])
    return q, mx


def linear_fp8_mx(aq: torch.Tensor, amx: torch.Tensor, w: Fp8Weight) -> torch.Tensor:
    """(e4m3 [M, K] with MX block scales [K/128, M, 4]) . w^T -> bf16 [M, N] on gemm8g (the scales applied by
    the block-scaled MFMA)."""
    M = aq.shape[0]
    N, K = w.q.shape
    out = torch.empty(M, N, dtype=torch.bfloat16, device=aq.device)
    ws, wq = w.s.reshape(-1), w.q.view(1, N, K)
    for r0, r1 in _row_blocks(M, aq.stride(0)):
        kernels().gemm8g_fp8(aq[r0:r1], wq, out[r0:r1], None, -(-(r1 - r0) // 256), None, None, ws, 0,
                             amx[:, r0:r1], None)
    return out


def linear_fp8(x, w: Fp8Weight) -> torch.Tensor:
    """bf16 x [M, K] -> per-row e4m3 quantisation (K11e) -> fp8 GEMM -> bf16 [M, N].  A :class:`QAct`
    (quantised by the producing norm) goes straight to the GEMM."""
    if isinstance(x, MXAct):
        return linear_fp8_mx(x.q, x.mx, w)
    if isinstance(x, QAct):
        return linear_fp8_q(x.q, x.s, w)
    xq, xs = quant_fp8_rows(x)
    return linear_fp8_q(xq, xs, w)


# ---------------------------------------------------------------------------------------------
# sampling / scoring


def sample(logits: torch.Tensor, temperature: torch.Tensor, top_p: torch.Tensor, top_k: torch.Tensor,
           min_p: torch.Tensor, top_a: torch.Tensor, seeds: torch.Tensor, offsets: torch.Tensor,
           num_logprobs: int = 0, freq_pen=None, pres_pen=None, rep_pen=None, counts=None, count_rows=None,
           bias=None, bias_rows=None, mask=None, mask_rows=None, out_token=None, out_logprob=None,
           out_topk_ids=None, out_topk_lp=None, mask_logprobs: bool = False, need_logprob: bool = True):
    """Fused sampler (K8a-d).  Returns (tokens[B] int32, token_logprob[B] f32, topk_ids[B,K], topk_lp[B,K]).
    Logprobs are over the raw model distribution (OpenAI semantics); with ``mask_logprobs`` rows that
    carry a grammar mask report them over the MASKED distribution instead — at a constrained key-letter
    step that is the exact restricted softmax over the sibling letters (the local vote fast path).
    ``need_logprob=False`` (and ``num_logprobs=0``): nobody reads the sampled token's logprob, so the raw
    log-sum-exp is skipped (one exp pass fewer per row) and ``token_logprob`` is NaN."""
    B = logits.shape[0]
    dev = logits.device
    K = int(num_logprobs)
    if out_token is None:
        out_token = torch.empty(B, dtype=torch.int32, device=dev)
    if out_logprob is None:
        out_logprob = torch.empty(B, dtype=torch.float32, device=dev)
    if out_topk_ids is None:
        out_topk_ids = torch.empty(B, max(K, 1), dtype=torch.int32, device=dev)
    if out_topk_lp is None:
        out_topk_lp = torch.empty(B, max(K, 1), dtype=torch.float32, device=dev)
    kernels().sample(logits, temperature, top_p, top_k, min_p, top_a, freq_pen, pres_pen, rep_pen, counts, count_rows,
                     bias, bias_rows, mask, mask_rows, seeds, offsets, K, out_token, out_logprob, out_topk_ids,
                     out_topk_lp, bool(mask_logprobs), bool(need_logprob))
    return out_token, out_logprob, out_topk_ids[:, :K], out_topk_lp[:, :K]


POOL_CLS, POOL_MEAN, POOL_LAST = 0, 1, 2


def pool_l2norm(hidden: torch.Tensor, cu_seqlens: torch.Tensor, mode: int, out_bf16: bool = True):
    """Pool packed encoder states per sequence and L2-normalise (K9d).  Returns (f32, bf16|None)."""
    n = cu_seqlens.numel() - 1
    d = hidden.shape[1]
    of = torch.empty(n, d, dtype=torch.float32, device=hidden.device)
    ob = torch.empty(n, d, dtype=torch.bfloat16, device=hidden.device) if out_bf16 else None
    kernels().pool_l2norm(hidden, cu_seqlens, int(mode), of, ob)
    return of, ob


def knn_topk(E: torch.Tensor, q: torch.Tensor, k: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """K10c: the ``k`` rows of ``E`` [n, d] f32 with the largest dot product with ``q`` [d] — (values [k] f32,
    rows [k] int64), best first, ties to the lower row (torch.topk's order up to ties).  k <= 64."""
    vals, rows = kernels().knn_topk(E.contiguous(), q.reshape(-1).contiguous().to(E.dtype), int(k))
    return vals, rows.long()


def vote_tally(V: torch.Tensor, w: torch.Tensor, valid: torch.Tensor):
    """K10b: the voter tally of R requests in one launch.  V [R, L, C] f64 (padded choices 0), w [R, L] f64,
    valid [R, L] u8 (0: no vote).  Returns (choice weight [R, C], confidence [R, C], voter confidence [R, L],
    NaN where !valid) — bitwise equal to the host tally (same fp64 summation order)."""
    return tuple(kernels().vote_tally(V.contiguous(), w.contiguous(), valid.contiguous()))


def cosine_consensus(E: torch.Tensor, tau: float = 0.05):
    """Embedding consensus over R requests x n candidates (K10a): S = E E^T on MFMA, then
    centrality_i = mean_{j!=i} S_ij and weights = softmax(centrality / tau).
    E: [R, n, d] bf16 unit rows.  Returns (S [R,n,n], centrality [R,n], weights [R,n], best [R])."""
    R, n, d = E.shape
    n_pad = (n + 15) // 16 * 16
    S = torch.empty(R, n_pad, n_pad, dtype=torch.float32, device=E.device)
    cen = torch.empty(R, n, dtype=torch.float32, device=E.device)
    w = torch.empty(R, n, dtype=torch.float32, device=E.device)
    best = torch.empty(R, dtype=torch.int32, device=E.device)
    kernels().cosine_consensus(E.contiguous(), S, 1.0 / float(tau), cen, w, best)
    return S[:, :n, :n], cen, w, best


