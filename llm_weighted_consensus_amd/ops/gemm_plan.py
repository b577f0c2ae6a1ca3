"""Per-shape GEMM backend choice for the decoder projections (K6).

Backends computing ``A . W^T`` for the dense projections:

* ``blas``   — hipBLASLt through ``torch.nn.functional.linear`` (its own stream-K kernels);
* ``g8``     — the hand-written 8-phase MFMA GEMM with a stream-K tail (``csrc/kernels/gemm8p.hip``);
* ``g4``     — the hand-written 4-wave interleaved MFMA GEMM, 256 x 256 tiles (``csrc/kernels/gemm4w.hip``);
* ``g4n192`` — the same core with 256 x 192 tiles (the qkv projection at decode batch 4096: 512 tiles =
  two whole rounds of 256 CUs, where 256 x 256 tiles leave half of the second round idle);
* ``g4p``    — gemm4w 256 x 256 with the VAR 64 schedule: each persistent workgroup DMAs its next tile's
  first two K tiles inside its last two main-loop iterations and runs the wave-local epilogue on the
  transposed accumulator layout (``profiles/gemm4w_stamps_r5.md``).
* ``gv``     — the skinny weight-stream GEMM for decode-sized row counts (M <= 64; plain, residual and
  SwiGLU epilogues; ``csrc/kernels/skinny.hip``): the serving path's small decode steps.
* ``g4s``    — gemm4w VAR 64 with split-K (``ops.split_plan``): shapes whose tiles leave CUs idle (the
  serving path's mid-size row counts: o / down at M = 2048 are 128 tiles for 256 CUs) run every tile as 2-4
  K-range units, a ragged last round (lm_head) splits only that round's tiles.

The hand-written cores also fuse the SwiGLU of the gate|up projection, or the residual add of the o /
down projections (:func:`linear_add_`), into their epilogue.  None wins everywhere
(``profiles/gemm4w.md``), so the choice is made per (M, N, K, epilogue) by timing every applicable
backend on the device, once, before a decode bucket's hipGraph is captured (:meth:`LlamaModel.tune_gemms`);
a hand-written core is taken when it is at least as fast as the library (``OWN_MARGIN``, 0); for a decode bucket
the engine then A/Bs whole captured steps (planner / all-library / all-own, ``LlamaModel.step_plans``).  Untuned shapes (prefill,
encode) use hipBLASLt.  ``LWC_GEMM=blas|g8|g4|g4n192`` forces one backend (``auto`` = measured, the default).
"""
from __future__ import annotations

import os
from typing import Dict, Optional, Tuple

import torch
import torch.nn.functional as F

from . import gemm4w, gemm8p, silu_mul, skinny_gemm, skinny_ok, split_plan

MODE = os.environ.get("LWC_GEMM", "auto")
BACKENDS = ("blas", "g8", "g4", "g4n192", "g4p", "gv", "g4s")
# a hand-written core is chosen when it is at least as fast as the library in the isolated timings (no
# bias either way: the decode step's plan is then settled by the engine's in-step A/B of whole captured steps,
# engine.LLMEngine._step_ab, which sees the step's clock and cache state)
OWN_MARGIN = float(os.environ.get("LWC_GEMM_OWN_MARGIN", "0"))
EXCLUDE = {b for b in os.environ.get("LWC_GEMM_NO", "").split(",") if b}
# LWC_GEMM_SKINNY=0 leaves the skinny decode GEMM out of the timing (A/B knob)
SKINNY = os.environ.get("LWC_GEMM_SKINNY", "1") != "0"
_CHOICE: Dict[Tuple[int, int, int, str], str] = {}
TIMINGS: Dict[Tuple[int, int, int, str], Dict[str, float]] = {}


# row-count buckets (mixed chunked-prefill steps: decode rows + prompt-chunk rows vary every step): per
# (N, K, epilogue) a sorted list of (M bucket, choice); a call takes the smallest tuned bucket >= its M
_BUCKETS: Dict[Tuple[int, int, str], list] = {}


def choice(M: int, N: int, K: int, epi: str) -> str:
    if MODE in BACKENDS:
        return MODE
    c = _CHOICE.get((M, N, K, epi))
    if c is not None:
        return c
    bl = _BUCKETS.get((N, K, epi))
    if bl:
        for mb, cb in bl:
            if M <= mb:
                return cb
        return bl[-1][1]
    return "blas"


def _g8_ok(N: int, K: int, epi: str) -> bool:
    return K % 64 == 0 and N % (64 if epi == "swiglu" else 8) == 0


def _own_ok(b: str, x: torch.Tensor, N: int, K: int, epi: str) -> bool:
    """Whether hand-written backend ``b`` takes this call (layout and the cores' shape rules; ``LWC_GEMM_NO``:
    a comma list of backends the planner leaves out, for A/B runs)."""
    if b == "blas" or not _g8_ok(N, K, epi) or x.stride(1) != 1 or b in EXCLUDE:
        return False
    if b == "gv":
        return SKINNY and skinny_ok(x.shape[0], N, K, swiglu=epi == "swiglu")
    if b == "g4s":  # VAR 64, split-K wherever split_plan splits this M (else unsplit: a bucket's M varies)
        return x.is_cuda
    return not (b == "g4n192" and epi == "swiglu")


def _own(b: str, x: torch.Tensor, w: torch.Tensor, ws=None, **kw) -> torch.Tensor:
    if b == "g8":
        return gemm8p(x, w, ws=ws, **kw)
    if b == "gv":
        return skinny_gemm(x, w, **kw)
    if b == "g4s":
        s_, f_ = split_plan(x.shape[0], w.shape[0], x.shape[1])
        return gemm4w(x, w, var=64, splits=s_, split_from=f_, **kw)
    return gemm4w(x, w, bn=192 if b == "g4n192" else 256, var=64 if b == "g4p" else 0, **kw)


def linear(x: torch.Tensor, w: torch.Tensor, ws=None) -> torch.Tensor:
    """x [M, K] . w[N, K]^T -> [M, N] bf16 on the chosen backend."""
    M, K = x.shape
    N = w.shape[0]
    b = choice(M, N, K, "plain")
    if _own_ok(b, x, N, K, "plain"):
        return _own(b, x, w, ws)
    return F.linear(x, w)


def linear_add_(x: torch.Tensor, w: torch.Tensor, acc: torch.Tensor, ws=None) -> torch.Tensor:
    """acc += x [M, K] . w[N, K]^T in place (the residual-stream update of the o / down projections):
    hipBLASLt with beta = 1 (C = D = acc, one fp32 sum and one rounding), or gemm8p's residual
    epilogue writing over its residual operand (every output element is read and written by the same
    lane).  Saves the separate residual add's read and write of the [M, N] projection output."""
    M, K = x.shape
    N = w.shape[0]
    b = choice(M, N, K, "residual")
    if _own_ok(b, x, N, K, "residual") and acc.is_contiguous():
        return _own(b, x, w, ws, residual=acc, out=acc)
    return acc.addmm_(x, w.t())


def swiglu(x: torch.Tensor, w_gu: torch.Tensor, block: int, ws=None) -> torch.Tensor:
    """silu(x Wg^T) * (x Wu^T) [M, F] for a fused gate|up weight [2F, K] whose rows are [gate; up]
    (block 0) or interleaved in blocks of ``block`` (ops.swiglu_interleave; required by g8)."""
    M, K = x.shape
    N = w_gu.shape[0]
    b = choice(M, N, K, "swiglu")
    if block == 32 and _own_ok(b, x, N, K, "swiglu"):
        return _own(b, x, w_gu, ws, swiglu=True)
    return silu_mul(F.linear(x, w_gu), block=block)


def _m_bucket(M: int) -> int:
    """Encoder token counts vary per call: tune per power-of-two bucket (everything >= 64k tokens is one)."""
    return min(1 << max(M - 1, 1).bit_length(), 1 << 16)


def linear_bias(x: torch.Tensor, w: torch.Tensor, b: torch.Tensor, gelu: bool = False, ws=None) -> torch.Tensor:
    """x . w^T + b (optionally GELU) — the encoder projections.  g8 applies the bias / exact-erf GELU in
    its epilogue on the fp32 accumulators; blas is hipBLASLt with the bias, and for GELU its bias+GELU
    epilogue (``torch._addmm_activation``: the tanh form of GELU on the fp32 accumulator, max 8.1e-3 from
    the fp32 erf-GELU at the bge-large FFN1 shape — the bf16 output's own rounding, 7.8e-3 for gemm8p's
    exact erf — where GEMM + the K9b bias_gelu pass rounds twice, 1.6e-2, and runs 657 vs 510 us at
    65536 tokens: scripts/gelu_epilogue_probe.py).  The backend is chosen per (token bucket, N, K,
    epilogue) by timing the library and the hand-written cores (gemm8p, gemm4w, gemm4w VAR 64) on the first
    call."""
    M, K = x.shape
    N = w.shape[0]
    epi = "bias_gelu" if gelu else "bias"
    key = (_m_bucket(M), N, K, epi)
    c = MODE if MODE in ("blas", "g8", "g4", "g4p") else _CHOICE.get(key)
    # gemm8p addresses A through one 32-bit buffer range (operands of 2 GiB or more take the other backends);
    # gemm4w runs such an A as row blocks
    ok = _g8_ok(N, K, epi) and x.stride(1) == 1 and x.is_cuda
    small_a = M * x.stride(0) * 2 < (1 << 31)
    runs = {"g4": lambda: gemm4w(x, w, bias=b, gelu=gelu),
            "g4p": lambda: gemm4w(x, w, bias=b, gelu=gelu, var=64),
            "blas": ((lambda: torch._addmm_activation(b, x, w.t(), use_gelu=True)) if gelu
                     else (lambda: F.linear(x, w, b)))}
    if small_a:
        runs["g8"] = lambda: gemm8p(x, w, bias=b, gelu=gelu, ws=ws)
    if c is None:
        if not ok or torch.cuda.is_current_stream_capturing():
            c = "blas"
        else:
            t = {name: _time(fn, iters=2, rounds=3) for name, fn in runs.items()}
            TIMINGS[key] = t
            own = min((n for n in ("g8", "g4", "g4p") if n in t), key=lambda n: t[n])
            c = own if t[own] <= t["blas"] * (1 + OWN_MARGIN) else "blas"
        _CHOICE[key] = c
    # (a choice made for the token bucket at a smaller A may name gemm8p, which a 2 GiB A cannot take)
    return runs[c]() if c != "blas" and ok and c in runs else runs["blas"]()


def linear_residual_(x: torch.Tensor, w: torch.Tensor, acc: torch.Tensor, ws=None) -> torch.Tensor:
    """acc += x . w^T in place — the post-LN encoder's o / FFN2 projections with the residual stream added in
    the GEMM epilogue (their bias then enters the LayerNorm that follows as its pre-norm bias, so that norm
    reads one [M, d] tensor instead of two).  Backend per (token bucket, N, K), timed on the first call on a
    copy of acc: hipBLASLt with beta = 1 (``addmm_``), gemm4w's residual epilogue (VAR 32 / 64) or gemm8p's."""
    M, K = x.shape
    N = w.shape[0]
    key = (_m_bucket(M), N, K, "enc_residual")
    c = MODE if MODE in ("blas", "g8", "g4", "g4p") else _CHOICE.get(key)
    ok = _g8_ok(N, K, "residual") and x.stride(1) == 1 and x.is_cuda and acc.is_contiguous()
    small_a = M * x.stride(0) * 2 < (1 << 31)

    def runs_on(a):
        r = {"g4": lambda: gemm4w(x, w, residual=a, out=a), "g4p": lambda: gemm4w(x, w, residual=a, out=a, var=64),
             "blas": lambda: a.addmm_(x, w.t())}
        if small_a:
            r["g8"] = lambda: gemm8p(x, w, residual=a, out=a, ws=ws)
        return r

    if c is None:
        if not ok or torch.cuda.is_current_stream_capturing():
            c = "blas"
        else:
            scratch = acc.clone()  # the timing runs add into a copy, never into the stream
            t = {name: _time(fn, iters=2, rounds=3) for name, fn in runs_on(scratch).items()}
            del scratch
            TIMINGS[key] = t
            own = min((n for n in ("g8", "g4", "g4p") if n in t), key=lambda n: t[n])
            c = own if t[own] <= t["blas"] * (1 + OWN_MARGIN) else "blas"
        _CHOICE[key] = c
    runs = runs_on(acc)
    runs[c if c != "blas" and ok and c in runs else "blas"]()
    return acc


def _time(fn, iters: int = 5, rounds: int = 3) -> float:
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(rounds):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e) / iters * 1e3)
    return sorted(ts)[len(ts) // 2]


def tune(x: torch.Tensor, w: torch.Tensor, epi: str = "plain", block: int = 0, ws=None,
         bucket: bool = False) -> Optional[str]:
    """Time every applicable backend for this (M, N, K, epi) and record the choice (no-op under graph
    capture, off the GPU, for an already tuned shape, or when a backend is forced).  Rounds interleave the
    backends (one process, one device: their clock and cache states match).  ``bucket``: also the choice of
    every row count up to M not tuned exactly (down to the next smaller bucket)."""
    M, K = x.shape
    N = w.shape[0]
    key = (M, N, K, epi)
    if MODE != "auto" or not x.is_cuda or torch.cuda.is_current_stream_capturing():
        return _CHOICE.get(key)
    if key in _CHOICE:
        if bucket:
            _add_bucket(M, N, K, epi, _CHOICE[key])
        return _CHOICE[key]
    lo = None
    if bucket:
        # a bucket's choice serves every row count down to the next smaller bucket: time at its top and at the
        # middle of its range (256-row-tile cores cost in whole m-tiles, the library more smoothly; a choice
        # timed at the top alone took a split-K core that lost at the bucket's smaller row counts)
        prev = max((mb for mb, _ in _BUCKETS.get((N, K, epi), []) if mb < M), default=M // 2)
        lo = max(1, (prev + M) // 2)
        lo = lo if lo < M else None
    c = _tune(x, w, epi, block, ws, M, N, K, key, lo)
    if bucket:
        _add_bucket(M, N, K, epi, c)
    return c


def _add_bucket(M: int, N: int, K: int, epi: str, c: str) -> None:
    bl = _BUCKETS.setdefault((N, K, epi), [])
    if all(mb != M for mb, _ in bl):
        bl.append((M, c))
        bl.sort()


def _tune(x, w, epi, block, ws, M, N, K, key, lo=None) -> str:
    """``lo``: also time every backend at that row count (the bucket's middle); the choice minimises the sum."""
    if not _g8_ok(N, K, epi) or (epi == "swiglu" and block != 32):
        _CHOICE[key] = "blas"
        return "blas"
    acc = torch.zeros(M, N, dtype=x.dtype, device=x.device) if epi == "residual" else None

    def run(b, xx):
        aa = acc[:xx.shape[0]] if acc is not None else None
        if epi == "swiglu":
            return (lambda: silu_mul(F.linear(xx, w), block=block)) if b == "blas" else \
                (lambda: _own(b, xx, w, ws, swiglu=True))
        if epi == "residual":
            return (lambda: aa.addmm_(xx, w.t())) if b == "blas" else \
                (lambda: _own(b, xx, w, ws, residual=aa, out=aa))
        return (lambda: F.linear(xx, w)) if b == "blas" else (lambda: _own(b, xx, w, ws))

    runs = {}
    for b in BACKENDS:
        if b != "blas" and not _own_ok(b, x, N, K, epi):
            continue
        if b == "g4s" and (M < 256 or split_plan(M, N, K)[0] == 1 or lo is not None):
            # (unsplit at the top it is g4p.)  Not for the mixed steps' row-count buckets: timed 3-7 % ahead of
            # g4p at the buckets' rows, it ran the serving load's mixed steps 0.6-2 % slower (profiles/round6_ab.md)
            continue
        fns = [run(b, x)]
        if lo is not None:
            if b != "blas" and not _own_ok(b, x[:lo], N, K, epi):
                continue  # a backend must take the whole bucket
            fns.append(run(b, x[:lo]))
        runs[b] = fns
    ts = {b: [] for b in runs}
    # 5 interleaved rounds of 5 calls: o and gate|up are within 1-3 % between backends, and 3 x 3 calls
    # flipped the choice from run to run (profiles/bench_r64_round3.md); runs before graph capture only
    for _ in range(5):
        for b, fns in runs.items():
            ts[b].append(sum(_time(fn, iters=5, rounds=1) for fn in fns))
    med = {b: sorted(t)[len(t) // 2] for b, t in ts.items()}
    TIMINGS[key] = med
    own = min((b for b in med if b != "blas"), key=lambda b: med[b], default=None)
    _CHOICE[key] = own if own is not None and med[own] <= med["blas"] * (1 + OWN_MARGIN) else "blas"
    return _CHOICE[key]


def table() -> Dict[str, Dict[str, float]]:
    """Measured shapes -> {backend: us, 'choice': ...} (for logs and /metrics)."""
    return {f"{M}x{N}x{K}:{e}": dict(TIMINGS.get((M, N, K, e), {}), choice=c)
            for (M, N, K, e), c in _CHOICE.items()}
