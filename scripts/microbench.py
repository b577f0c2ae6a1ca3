#!/usr/bin/env python3
"""Micro-benchmarks of the decode hot path on one MI355X: the Llama-3-8B projection GEMMs at decode
batch sizes (hipBLASLt default vs TunableOp-tuned), paged decode attention, the fused sampler and the
small fused kernels.  Prints one line per case: time, TFLOP/s, GB/s."""
import argparse
import math
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters=50, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3  # us


def gemms(dev, Ms, tuned):
    shapes = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336),
              "lm_head": (128256, 4096)}
    for M in Ms:
        for name, (N, K) in shapes.items():
            x = torch.randn(M, K, device=dev).to(torch.bfloat16)
            w = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
            us = timeit(lambda: F.linear(x, w), iters=20)
            fl = 2 * M * N * K / (us * 1e-6) / 1e12
            gb = (N * K * 2 + M * K * 2 + M * N * 2) / (us * 1e-6) / 1e9
            print(f"gemm{'-tuned' if tuned else ''} M={M:4d} {name:8s} N={N:6d} K={K:5d}: {us:8.1f} us "
                  f"{fl:7.1f} TF/s {gb:7.0f} GB/s", flush=True)


def gemm_layouts(dev, Ms):
    """Same products through different operand layouts: hipBLASLt picks different kernels."""
    shapes = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}
    for M in Ms:
        for name, (N, K) in shapes.items():
            x = torch.randn(M, K, device=dev).to(torch.bfloat16)
            w = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
            wt = w.t().contiguous()
            xt = x.t().contiguous()
            cases = {
                "NT  x@w^T": lambda: F.linear(x, w),
                "NN  x@wt": lambda: torch.mm(x, wt),
                "sw  w@x^T": lambda: torch.mm(w, xt),
                "sw2 w@xT(view)": lambda: torch.mm(w, x.t()),
            }
            for cname, fn in cases.items():
                us = timeit(fn, iters=20)
                fl = 2 * M * N * K / (us * 1e-6) / 1e12
                print(f"layout M={M:4d} {name:8s} {cname:16s}: {us:8.1f} us {fl:7.1f} TF/s", flush=True)
    for n in (4096, 8192):
        a = torch.randn(n, n, device=dev).to(torch.bfloat16)
        b = torch.randn(n, n, device=dev).to(torch.bfloat16)
        us = timeit(lambda: torch.mm(a, b), iters=10)
        print(f"square {n}: {us:8.1f} us {2 * n ** 3 / (us * 1e-6) / 1e12:7.1f} TF/s", flush=True)


def gemm_backends(dev, Ms):
    """The decode GEMM shapes through each BLAS backend torch can dispatch to on ROCm."""
    shapes = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336),
              "lm_head": (128256, 4096)}
    for lib in ("cublaslt", "cublas", "ck"):
        try:
            torch.backends.cuda.preferred_blas_library(lib)
        except Exception as e:  # noqa: BLE001
            print(f"backend {lib}: unavailable ({e})", flush=True)
            continue
        for M in Ms:
            for name, (N, K) in shapes.items():
                x = torch.randn(M, K, device=dev).to(torch.bfloat16)
                w = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
                try:
                    us = timeit(lambda: F.linear(x, w), iters=20)
                except Exception as e:  # noqa: BLE001
                    print(f"backend {lib} M={M} {name}: failed ({type(e).__name__})", flush=True)
                    continue
                fl = 2 * M * N * K / (us * 1e-6) / 1e12
                print(f"backend {lib:8s} M={M:4d} {name:8s}: {us:8.1f} us {fl:7.1f} TF/s", flush=True)
    torch.backends.cuda.preferred_blas_library("cublaslt")


def grouped(dev):
    """Hand-written grouped MFMA GEMM (K6g) vs hipBLASLt on plain shapes, and the MoE decode shape."""
    from llm_weighted_consensus_amd import ops

    shapes = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336),
              "lm_head": (128256, 4096)}
    for M in (1024, 3072):
        for name, (N, K) in shapes.items():
            x = torch.randn(M, K, device=dev).to(torch.bfloat16)
            w = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
            off = torch.tensor([0, M], dtype=torch.int32, device=dev)
            t_h = timeit(lambda: F.linear(x, w), iters=20)
            t_g = timeit(lambda: ops.grouped_gemm(x, w.unsqueeze(0), off), iters=20)
            xq = x.to(torch.float8_e4m3fn)
            wq = w.unsqueeze(0).to(torch.float8_e4m3fn)
            sa = torch.ones(M, device=dev)
            sw = torch.ones(1, N, device=dev)
            t_8 = timeit(lambda: ops.grouped_gemm(xq, wq, off, a_scale=sa, w_scale=sw), iters=20)
            t_2 = timeit(lambda: ops.gemm8p(x, w), iters=20)
            err = (ops.gemm8p(x, w).float() - F.linear(x, w).float()).abs().max().item()
            fl = 2 * M * N * K / 1e12
            print(f"ggemm M={M:4d} {name:8s}: hipblaslt {t_h:7.1f} us ({fl / t_h * 1e6:6.0f} TF/s)  "
                  f"gemm8p {t_2:7.1f} us ({fl / t_2 * 1e6:6.0f}, err {err:.3g})  "
                  f"grouped-bf16 {t_g:7.1f} us ({fl / t_g * 1e6:6.0f})  grouped-fp8 {t_8:7.1f} us ({fl / t_8 * 1e6:6.0f})",
                  flush=True)
    # Mixtral decode MoE: T tokens x top-2 over 8 experts, d=4096, ffn=14336 (gate_up fused 28672)
    E, d, f = 8, 4096, 14336
    w13 = (torch.randn(E, 2 * f, d, device=dev) * 0.02).to(torch.bfloat16)
    for T in (256, 1024):
        rows = 2 * T
        sizes = torch.full((E,), rows // E, dtype=torch.int64)
        off = torch.cat([torch.zeros(1, dtype=torch.int64), sizes.cumsum(0)]).to(torch.int32).to(dev)
        x = torch.randn(rows, d, device=dev).to(torch.bfloat16)
        t = timeit(lambda: ops.grouped_gemm(x, w13, off), iters=10)
        fl = 2 * rows * 2 * f * d / 1e12
        print(f"ggemm moe gate_up T={T}: {t:7.1f} us ({fl / t * 1e6:6.0f} TF/s)", flush=True)


def gemm8p_study(dev, Ms):
    """8-phase 256x256 GEMM (csrc/kernels/gemm8p.hip) vs hipBLASLt, interleaved
    rounds in one process (median of 3), random operands; plus the fused SwiGLU epilogue against
    hipBLASLt gate_up + silu_mul."""
    from llm_weighted_consensus_amd import ops

    shapes = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336),
              "lm_head": (128256, 4096)}
    cases = [(M, name, N, K) for M in Ms for name, (N, K) in shapes.items()]
    cases += [(4096, "sq4096", 4096, 4096), (8192, "sq8192", 8192, 8192)]
    for M, name, N, K in cases:
        x = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
        w = ((torch.rand(N, K, device=dev) * 2 - 1) / K ** 0.5).to(torch.bfloat16)
        o = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        fns = {"hipblaslt": lambda: torch.matmul(x, w.t(), out=o), "gemm8p": lambda: ops.gemm8p(x, w, out=o)}
        ref = F.linear(x, w).float()
        err = (ops.gemm8p(x, w).float() - ref).abs().max().item()
        res = {k: [] for k in fns}
        for _ in range(3):
            for k, fn in fns.items():
                res[k].append(timeit(fn, iters=10 if M * N * K > 1e11 else 30))
        fl = 2 * M * N * K / 1e12
        line = "  ".join(f"{k} {sorted(v)[1]:8.1f} us ({fl / sorted(v)[1] * 1e6:5.0f})" for k, v in res.items())
        print(f"g8 M={M:5d} {name:8s}: {line}  err {err:.3g}", flush=True)
    for M in Ms:
        N, K = 28672, 4096
        x = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
        w = ((torch.rand(N, K, device=dev) * 2 - 1) / K ** 0.5).to(torch.bfloat16)
        wi = ops.swiglu_interleave(w)
        gu = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        h = torch.empty(M, N // 2, dtype=torch.bfloat16, device=dev)

        def unfused():
            torch.matmul(x, w.t(), out=gu)
            ops.silu_mul(gu, out=h)

        ref = F.silu(F.linear(x, w).float()[:, :N // 2]) * F.linear(x, w).float()[:, N // 2:]
        err = (ops.gemm8p(x, wi, swiglu=True).float() - ref).abs().max().item()
        ta, tb = [], []
        for _ in range(3):
            ta.append(timeit(unfused, iters=10))
            tb.append(timeit(lambda: ops.gemm8p(x, wi, out=h, swiglu=True), iters=10))
        print(f"g8 swiglu M={M:5d}: hipblaslt+silu_mul {sorted(ta)[1]:8.1f} us  gemm8p-fused {sorted(tb)[1]:8.1f} us"
              f"  err {err:.3g}", flush=True)


def gemm8p_ab(dev):
    """A/B of gemm8p knobs (env LWC_G8_*, read at launch) in interleaved rounds, median of 5."""
    from llm_weighted_consensus_amd import ops

    variants = [v.split(":") for v in os.environ.get("G8_VARIANTS", "GM=1:STAGGER=1,GM=4:STAGGER=1,GM=8:STAGGER=1,"
                                                     "GM=4:STAGGER=0").split(",")]
    shapes = [(4096, 4096, 4096, False), (3072, 28672, 4096, True), (3072, 6144, 4096, False),
              (3072, 4096, 14336, False), (3072, 4096, 4096, False), (3072, 128256, 4096, False),
              (8192, 8192, 8192, False)]
    for M, N, K, sw in shapes:
        x = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
        w = ((torch.rand(N, K, device=dev) * 2 - 1) / K ** 0.5).to(torch.bfloat16)
        if sw:
            w = ops.swiglu_interleave(w)
        res = {",".join(v): [] for v in variants}
        for _ in range(5):
            for v in variants:
                for kv in v:
                    k, val = kv.split("=")
                    os.environ["LWC_G8_" + k] = val
                res[",".join(v)].append(timeit(lambda: ops.gemm8p(x, w, swiglu=sw), iters=10))
        fl = 2 * M * N * K / 1e12
        line = "  ".join(f"[{k}] {sorted(t)[2]:7.1f} us ({fl / sorted(t)[2] * 1e6:5.0f})" for k, t in res.items())
        print(f"g8ab {M}x{N}x{K}{' swiglu' if sw else ''}: {line}", flush=True)
    for k in ("LWC_G8_GM", "LWC_G8_STAGGER"):
        os.environ.pop(k, None)


def gemm4w_ab(dev):
    """hipBLASLt vs gemm8p vs gemm4w (bn 256 / 192) on the headline's decode shapes (M = 4096), prefill and
    encoder shapes; interleaved rounds in one process, median of 5, random [-1, 1) operands."""
    import torch.nn.functional as F

    from llm_weighted_consensus_amd import ops

    shapes = [(4096, 6144, 4096, "plain"), (4096, 4096, 4096, "res"), (4096, 28672, 4096, "swiglu"),
              (4096, 4096, 14336, "res"), (4096, 128256, 4096, "plain"), (16384, 6144, 4096, "plain"),
              (65536, 3072, 1024, "bias"), (65536, 4096, 1024, "gelu"), (65536, 1024, 4096, "bias"),
              (8192, 8192, 8192, "plain")]
    only = os.environ.get("G4_SHAPES")
    if only:
        shapes = [shapes[int(i)] for i in only.split(",")]
    ws = ops.new_gemm8p_workspace(dev)
    for M, N, K, epi in shapes:
        x = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
        w = ((torch.rand(N, K, device=dev) * 2 - 1) / K ** 0.5).to(torch.bfloat16)
        b = (torch.rand(N, device=dev) - 0.5).to(torch.bfloat16)
        acc = torch.zeros(M, N, device=dev, dtype=torch.bfloat16)
        # gemm4w at both schedules (32: block-staged epilogue, 64: wave-local epilogue + next-tile prefetch;
        # G4_VARS selects) and both tile widths
        vars_ = [int(v) for v in os.environ.get("G4_VARS", "32,64").split(",")]
        gms = [int(v) for v in os.environ.get("G4_GMS", "0").split(",")]  # 0: the kernel's choice by shape
        vg = [(v, gm) for v in vars_ for gm in gms]

        def nm(p, v, gm):
            return f"{p}v{v}" + (f"g{gm}" if len(gms) > 1 else "")
        no_g8 = os.environ.get("G4_NO_G8") == "1"
        if epi == "swiglu":
            wi = ops.swiglu_interleave(w)
            runs = {"blas": lambda: ops.silu_mul(F.linear(x, wi), block=32),
                    "g8": lambda: ops.gemm8p(x, wi, swiglu=True, ws=ws)}
            runs.update({nm("g4", v, gm): (lambda v=v, gm=gm: ops.gemm4w(x, wi, swiglu=True, var=v, gm=gm)) for v, gm in vg})
        elif epi == "res":
            runs = {"blas": lambda: acc.addmm_(x, w.t()), "g8": lambda: ops.gemm8p(x, w, residual=acc, out=acc, ws=ws)}
            runs.update({nm("g4", v, gm): (lambda v=v, gm=gm: ops.gemm4w(x, w, residual=acc, out=acc, var=v, gm=gm))
                         for v, gm in vg})
        elif epi in ("bias", "gelu"):
            g = epi == "gelu"
            runs = {"blas": (lambda: torch._addmm_activation(b, x, w.t(), use_gelu=True)) if g
                    else (lambda: F.linear(x, w, b)),
                    "g8": lambda: ops.gemm8p(x, w, bias=b, gelu=g, ws=ws)}
            runs.update({nm("g4", v, gm): (lambda v=v, gm=gm: ops.gemm4w(x, w, bias=b, gelu=g, var=v, gm=gm))
                         for v, gm in vg})
        else:
            runs = {"blas": lambda: F.linear(x, w), "g8": lambda: ops.gemm8p(x, w, ws=ws)}
            runs.update({nm("g4", v, gm): (lambda v=v, gm=gm: ops.gemm4w(x, w, var=v, gm=gm)) for v, gm in vg})
            runs.update({nm("g4n192", v, gm): (lambda v=v, gm=gm: ops.gemm4w(x, w, bn=192, var=v, gm=gm))
                         for v, gm in vg})
        if no_g8:
            runs.pop("g8", None)
        res = {k: [] for k in runs}
        for _ in range(5):
            for k, fn in runs.items():
                res[k].append(timeit(fn, iters=10, warm=2))
        fl = 2 * M * N * K / 1e12
        line = "  ".join(f"{k} {sorted(t)[2]:8.1f} us ({fl / sorted(t)[2] * 1e6:5.0f})" for k, t in res.items())
        print(f"g4ab {M}x{N}x{K} {epi}: {line}", flush=True)
        del x, w, acc


def attention(dev):
    from llm_weighted_consensus_amd import ops

    Hq, Hkv, D, BS = 32, 8, 128, 16
    for B, ctx_len in [(256, 320), (512, 320), (64, 2048), (8, 4096)]:
        nb = (ctx_len + BS - 1) // BS
        NB = B * nb + 8
        kc = torch.randn(NB, Hkv, BS, D, device=dev).to(torch.bfloat16)
        vc = torch.randn(NB, Hkv, BS // 4, D, 4, device=dev).to(torch.bfloat16)
        bt = torch.arange(B * nb, device=dev, dtype=torch.int32).view(B, nb)
        ctx = torch.full((B,), ctx_len, device=dev, dtype=torch.int32)
        q = torch.randn(B, (Hq + 2 * Hkv) * D, device=dev).to(torch.bfloat16)
        for splits in (1, 2, 4, 8):
            us = timeit(lambda: ops.paged_decode(q, kc, vc, bt, ctx, Hq, 1 / math.sqrt(D), num_splits=splits))
            gb = B * ctx_len * Hkv * D * 2 * 2 / (us * 1e-6) / 1e9
            print(f"paged_decode B={B:4d} ctx={ctx_len:5d} splits={splits}: {us:8.1f} us {gb:7.0f} GB/s", flush=True)


def attention_prefix(dev):
    """The bench's decode attention: R groups of N candidates sharing a 256-token prompt, suffix of
    `gen` tokens each — prefix (cascade) pass + suffix pass vs plain, both kernel paths."""
    from llm_weighted_consensus_amd import ops

    Hq, Hkv, D, BS = 32, 8, 128, 16
    cases = [(16, 64, 16, 64), (48, 64, 16, 64), (48, 64, 16, 120), (64, 64, 16, 64)]
    if os.environ.get("MICRO_PREFIX_QUICK"):
        cases = [(48, 64, 16, 64), (64, 64, 16, 64)]
    for (R, N, P, gen) in cases:
        B = R * N
        sblk = (gen + 1 + BS - 1) // BS
        NB = R * P + B * sblk + 8
        kc = torch.randn(NB, Hkv, BS, D, device=dev).to(torch.bfloat16)
        vc = torch.randn(NB, Hkv, BS // 4, D, 4, device=dev).to(torch.bfloat16)
        width = P + sblk
        bt = torch.zeros(B, width, dtype=torch.int32)
        for r in range(R):
            bt[r * N:(r + 1) * N, :P] = torch.arange(r * P, (r + 1) * P, dtype=torch.int32)
        bt[:, P:] = (R * P + torch.arange(B * sblk, dtype=torch.int32)).view(B, sblk)
        bt = bt.to(dev)
        ctx = torch.full((B,), P * BS + gen + 1, device=dev, dtype=torch.int32)
        q = torch.randn(B, (Hq + 2 * Hkv) * D, device=dev).to(torch.bfloat16)
        per = 16 // (Hq // Hkv)
        sc = 1 / math.sqrt(D)
        for path, thr in (() if os.environ.get("MICRO_PREFIX_QUICK") else (("wg4", 1 << 30), ("wave", 0))):
            old = ops.set_decode_wave_min_items(thr)
            t_plain = timeit(lambda: ops.paged_decode(q, kc, vc, bt, ctx, Hq, sc))
            ops.set_decode_wave_min_items(old)
            print(f"plain decode R={R} N={N} P={P * BS} gen={gen} [{path}]: {t_plain:7.1f} us", flush=True)
        from llm_weighted_consensus_amd.engine.engine import cascade_table_size, cascade_tiles
        import numpy as np

        per_t = ops.cascade_rows_per_tile(Hq // Hkv)
        ct = np.zeros((cascade_table_size(B, per_t), 3), dtype=np.int32)
        nt = cascade_tiles([(r * N, N, P) for r in range(R)], per_t, ct)
        ct_exact = torch.from_numpy(ct[:nt].copy()).to(dev)
        ct = torch.from_numpy(ct).to(dev)
        t_exact = timeit(lambda: ops.paged_decode_cascade(q, kc, vc, bt, ctx, ct_exact, Hq, sc))
        print(f"  cascade exact grid ({nt} tiles): {t_exact:7.1f} us", flush=True)
        t_c = timeit(lambda: ops.paged_decode_cascade(q, kc, vc, bt, ctx, ct, Hq, sc))
        for pairs in os.environ.get("CASCADE_PAIRS", "").split(","):
            if pairs:
                os.environ["LWC_CASCADE_PAIRS"] = pairs
                tp_ = [timeit(lambda: ops.paged_decode_cascade(q, kc, vc, bt, ctx, ct, Hq, sc)) for _ in range(3)]
                print(f"  cascade LDS pairs={pairs}: {sorted(tp_)[1]:7.1f} us", flush=True)
        os.environ.pop("LWC_CASCADE_PAIRS", None)
        ref_o = ops.paged_decode(q, kc, vc, bt, ctx, Hq, sc)
        got = ops.paged_decode_cascade(q, kc, vc, bt, ctx, ct, Hq, sc)
        err = (got.float() - ref_o.float()).abs().max().item()
        print(f"cascade-decode R={R} N={N} P={P * BS} gen={gen}: {t_c:7.1f} us  (max|diff| vs plain {err:.3g})",
              flush=True)
        # decomposition: prefix only (ctx = prompt), suffix only (own blocks moved to the front, no prefix)
        ctx_p = torch.full((B,), P * BS, device=dev, dtype=torch.int32)
        t_p = timeit(lambda: ops.paged_decode_cascade(q, kc, vc, bt, ctx_p, ct, Hq, sc))
        bt_s = torch.zeros_like(bt)
        bt_s[:, :sblk] = bt[:, P:]
        ctx_s = torch.full((B,), gen + 1, device=dev, dtype=torch.int32)
        ct_s = np.zeros((cascade_table_size(B, per_t), 3), dtype=np.int32)
        cascade_tiles([(0, B, 0)], per_t, ct_s)
        ct_s = torch.from_numpy(ct_s).to(dev)
        t_s = timeit(lambda: ops.paged_decode_cascade(q, kc, vc, bt_s, ctx_s, ct_s, Hq, sc))
        ctx_f = torch.full((B,), P * BS + gen + 1, device=dev, dtype=torch.int32)
        t_f = timeit(lambda: ops.paged_decode_cascade(q, kc, vc, bt, ctx_f, ct_s, Hq, sc))
        print(f"  cascade parts: prefix-only {t_p:7.1f} us  suffix-only {t_s:7.1f} us  "
              f"no-sharing full ctx {t_f:7.1f} us", flush=True)


def prefill_attn(dev):
    """Chunk-prefill attention: queries = the last q rows of a k-key range, keys contiguous (cached-prefix
    path, after kv_gather) vs paged (block tables, the mixed chunked-prefill path); + the gather itself."""
    from llm_weighted_consensus_amd import ops

    Hq, Hkv, D, BS = 32, 8, 128, 16
    sc = 1 / math.sqrt(D)
    for n, ql, kl in [(1, 512, 512), (1, 512, 2048), (1, 512, 4096), (4, 256, 512), (1, 2048, 2048)]:
        nbs = -(-kl // BS)
        NB = n * nbs + 8
        kc = torch.randn(NB, Hkv, BS, D, device=dev).to(torch.bfloat16)
        vc = torch.randn(NB, Hkv, BS // 4, D, 4, device=dev).to(torch.bfloat16)
        W = 2 * -(-kl // 32)
        bt = torch.zeros(n, W, dtype=torch.int32)
        perm = torch.randperm(NB - 8, dtype=torch.int32)
        for i in range(n):
            bt[i, :nbs] = perm[i * nbs:(i + 1) * nbs]
        bt = bt.to(dev)
        q = torch.randn(n * ql, (Hq + 2 * Hkv) * D, device=dev).to(torch.bfloat16)
        cu_q = torch.arange(n + 1, device=dev, dtype=torch.int32) * ql
        cu_k = torch.arange(n + 1, device=dev, dtype=torch.int32) * kl
        k_lens = torch.full((n,), kl, device=dev, dtype=torch.int32)
        toks = torch.arange(kl, device=dev)
        slots = torch.cat([bt[i, toks // BS].long() * BS + toks % BS for i in range(n)])
        kf, vf = ops.kv_gather(kc, vc, slots)
        t_g = timeit(lambda: ops.kv_gather(kc, vc, slots))
        t_c = timeit(lambda: ops.prefill_attention(q[:, : Hq * D], kf, vf, cu_q, ql, Hq, Hkv, D, sc, True,
                                                   cu_seqlens_k=cu_k, lens=([ql] * n, [kl] * n)))
        t_p = timeit(lambda: ops.prefill_attention_paged(q, kc, vc, cu_q, bt, k_lens, ql, Hq, sc))
        fl = n * 4 * Hq * D * ql * (kl - ql / 2) / 1e12
        print(f"pfattn {n} x q{ql} k{kl}: gather {t_g:7.1f} us  contiguous {t_c:7.1f} us ({fl / t_c * 1e6:4.0f} TF/s)  "
              f"paged {t_p:7.1f} us ({fl / t_p * 1e6:4.0f} TF/s)", flush=True)


def bandwidth(dev):
    """HBM calibration: streaming read (sum), copy (read + write), and 4 KiB-segment gathers in random order
    (the decode attention's access pattern) — bytes moved / time."""
    n = 1 << 30  # 2 GiB of bf16
    x = torch.empty(n, dtype=torch.bfloat16, device=dev).normal_()
    y = torch.empty_like(x)
    us = timeit(lambda: x.sum(), iters=10)
    print(f"bw read (sum)          : {2 * n / us / 1e3:7.0f} GB/s", flush=True)
    us = timeit(lambda: x.view(-1, 4096).amax(dim=1), iters=10)
    print(f"bw read (row amax)     : {2 * n / us / 1e3:7.0f} GB/s", flush=True)
    us = timeit(lambda: y.copy_(x), iters=10)
    print(f"bw copy (r + w)        : {4 * n / us / 1e3:7.0f} GB/s", flush=True)
    seg = x.view(-1, 2048)  # 4 KiB rows
    idx = torch.randperm(seg.shape[0], device=dev)[: seg.shape[0] // 2]
    us = timeit(lambda: seg.index_select(0, idx), iters=10)
    print(f"bw 4KiB gather (r + w) : {2 * idx.numel() * 4096 / us / 1e3:7.0f} GB/s", flush=True)
    lg = torch.randn(4096, 128256, device=dev).to(torch.bfloat16)
    us = timeit(lambda: lg.amax(dim=1), iters=10)
    print(f"logits [4096, 128256] row amax: {us:7.1f} us ({lg.numel() * 2 / us / 1e3:5.0f} GB/s)", flush=True)
    us = timeit(lambda: torch.softmax(lg, dim=1), iters=5)
    print(f"logits [4096, 128256] softmax (r + w): {us:7.1f} us", flush=True)


def moe_decode(dev):
    """Mixtral decode MoE at the config-5 batch: fp8 experts, T tokens x top-2 over 8 experts, balanced and
    router-driven (uneven) segments; time and the expert-weight bytes streamed per second."""
    from llm_weighted_consensus_amd import ops

    E, d, f = 8, 4096, 14336
    g = torch.Generator(device=dev).manual_seed(0)
    w13 = (torch.randn(E, 2 * f, d, device=dev, generator=g) * 0.02).to(torch.bfloat16)
    w2 = (torch.randn(E, d, f, device=dev, generator=g) * 0.02).to(torch.bfloat16)
    q13, s13 = ops.quant_fp8_weight(w13)
    q2, s2 = ops.quant_fp8_weight(w2)
    del w13, w2
    router = (torch.randn(E, d, device=dev, generator=g) * 0.1).to(torch.bfloat16)
    for T in [int(t) for t in os.environ.get("MICRO_MOE_T", "512,2048").split(",")]:
        rows = 2 * T
        h = torch.randn(T, d, device=dev, generator=g).to(torch.bfloat16)
        _ids, _w, off_r, src, _inv = ops.moe_route(torch.nn.functional.linear(h, router), 2)
        sizes = torch.full((E,), rows // E, dtype=torch.int64)
        off_b = torch.cat([torch.zeros(1, dtype=torch.int64), sizes.cumsum(0)]).to(torch.int32).to(dev)
        hq, hs = ops.quant_fp8_rows(h)
        act = torch.randn(rows, f, device=dev, generator=g).to(torch.bfloat16)
        aq, as_ = ops.quant_fp8_rows(act)
        for label, off in (("balanced", off_b), ("routed", off_r)):
            t13 = timeit(lambda: ops.grouped_gemm(hq, q13, off, a_rows=src, rows=rows, a_scale=hs, w_scale=s13), iters=20)
            t2 = timeit(lambda: ops.grouped_gemm(aq, q2, off, a_scale=as_, w_scale=s2), iters=20)
            mx = int((off[1:] - off[:-1]).max())
            print(f"moe fp8 T={T:5d} {label:8s} (max rows/expert {mx:4d}): w13 {t13:7.1f} us "
                  f"({q13.numel() / t13 / 1e3:5.0f} GB/s of weights)  w2 {t2:7.1f} us ({q2.numel() / t2 / 1e3:5.0f} GB/s)",
                  flush=True)


def sampler(dev):
    from llm_weighted_consensus_amd import ops

    V = 128256
    for B in (512, 4096):
        logits = (torch.randn(B, V, device=dev) * 2).to(torch.bfloat16)
        f = lambda v: torch.full((B,), float(v), device=dev)
        seeds = torch.arange(B, device=dev, dtype=torch.int64)
        offs = torch.zeros(B, device=dev, dtype=torch.int64)
        tk = torch.zeros(B, dtype=torch.int32, device=dev)
        for label, tp, K, T in [("greedy", 1.0, 0, 0.0), ("temp", 1.0, 0, 0.8), ("top_p", 0.95, 0, 0.8),
                                ("top_p+lp20", 0.95, 20, 0.8)]:
            us = timeit(lambda: ops.sample(logits, f(T), f(tp), tk, f(0), f(0), seeds, offs, num_logprobs=K),
                        iters=20)
            print(f"sample B={B} {label:10s}: {us:8.1f} us  {B * V * 2 / (us * 1e-6) / 1e9:7.0f} GB/s", flush=True)


def small(dev):
    from llm_weighted_consensus_amd import ops

    from llm_weighted_consensus_amd.models.config import decoder_config
    from llm_weighted_consensus_amd.models.llama import KVCache, rope_tables

    cfg = decoder_config("llama-3-8b")
    cos, sin = rope_tables(cfg, dev, 4096)
    for T in (512, 3072, 4096):
        cache = KVCache(cfg, T + 64, 16, dev)
        qkv = torch.randn(T, cfg.qkv_dim, device=dev).to(torch.bfloat16)
        pos = torch.randint(0, 4000, (T,), device=dev, dtype=torch.int32)
        slots = (torch.randperm(T, device=dev).to(torch.int32) * 16 + 5)
        us = timeit(lambda: ops.rope_kv_write(qkv, pos, cos, sin, cache.k[0], cache.v[0], 32, 8, 128, slots=slots))
        us_k = timeit(lambda: ops.rope_kv_write(qkv, pos, cos, sin, cache.k[0], cache.v[0], 32, 8, 128, slots=slots,
                                                rope_q=False))
        print(f"rope_kv_write T={T}: {us:6.1f} us   k only (q rotated in the decode kernels): {us_k:6.1f} us",
              flush=True)
    for T in (512, 3072):
        x = torch.randn(T, 4096, device=dev).to(torch.bfloat16)
        r = torch.randn(T, 4096, device=dev).to(torch.bfloat16)
        w = torch.ones(4096, device=dev, dtype=torch.bfloat16)
        us = timeit(lambda: ops.rmsnorm(x, w, 1e-5, residual=r))
        print(f"rmsnorm+res T={T}: {us:6.1f} us", flush=True)
        gu = torch.randn(T, 2 * 14336, device=dev).to(torch.bfloat16)
        us = timeit(lambda: ops.silu_mul(gu))
        print(f"silu_mul T={T}: {us:6.1f} us", flush=True)


def encoder_gemms(dev):
    """The encoders' small-K projections (config 2 bge-base: d = 768, FFN 3072; bge-large: 1024 / 4096) at
    ENC_M tokens: hipBLASLt (bias / bias+GELU epilogue) vs gemm8p, gemm4w (VAR 32) and gemm4w VAR 64 (next
    tile's prologue under the epilogue, polynomial GELU), g4p192 its 256 x 192 tiles.  Median of 5 interleaved
    rounds."""
    import torch.nn.functional as F

    from llm_weighted_consensus_amd import ops

    M = int(os.environ.get("ENC_M", "524288"))  # config 2: 64 requests x 64 candidates x 128 tokens
    d = int(os.environ.get("ENC_D", "768"))
    shapes = [(3 * d, d, False), (d, d, False), (4 * d, d, True), (d, 4 * d, False)]
    for N, K, gelu in shapes:
        x = (torch.randn(M, K, device=dev) * 0.5).to(torch.bfloat16)
        w = (torch.randn(N, K, device=dev) / K ** 0.5).to(torch.bfloat16)
        b = (torch.randn(N, device=dev) * 0.1).to(torch.bfloat16)
        runs = {
            "blas": (lambda: torch._addmm_activation(b, x, w.t(), use_gelu=True)) if gelu else (lambda: F.linear(x, w, b)),
            # (gemm8p addresses A through one 32-bit buffer range: no A of 2 GiB or more)
            **({"g8": lambda: ops.gemm8p(x, w, bias=b, gelu=gelu)} if x.numel() * 2 < (1 << 31) else {}),
            "g4": lambda: ops.gemm4w(x, w, bias=b, gelu=gelu),
            "g4p": lambda: ops.gemm4w(x, w, bias=b, gelu=gelu, var=64),
            "g4p192": lambda: ops.gemm4w(x, w, bias=b, gelu=gelu, var=64, bn=192),
        }
        res = {k: [] for k in runs}
        for _ in range(5):
            for k, fn in runs.items():
                res[k].append(timeit(fn, iters=5, warm=1))
        line = "  ".join(f"{k} {sorted(t)[2]:8.1f}" for k, t in res.items())
        print(f"enc M={M} {N}x{K}{' gelu' if gelu else ''}: {line} us", flush=True)
        del x, w


def skinny_ab(dev):
    """Decode-sized projections (serving decode buckets): hipBLASLt vs the skinny weight-stream GEMM
    (skinny.hip) for Llama-3-8B's projections, plain and residual, median of 5 interleaved rounds; TB/s = W
    bytes / time."""
    import torch.nn.functional as F

    from llm_weighted_consensus_amd import ops

    shapes = [(6144, 4096, False), (4096, 4096, True), (28672, 4096, False), (4096, 14336, True),
              (128256, 4096, False)]  # (28672: gate|up with SwiGLU)
    for M in [int(m) for m in os.environ.get("SKINNY_M", "2,8,16,32,64").split(",")]:
        for N, K, res in shapes:
            x = ((torch.rand(M, K, device=dev) * 2 - 1)).to(torch.bfloat16)
            # rotate over enough weight copies to exceed the 256 MB last-level cache (a decode step streams
            # 32 layers of different weights)
            nw = max(1, min(16, (768 << 20) // (N * K * 2)))
            ws = [((torch.rand(N, K, device=dev) * 2 - 1) / K ** 0.5).to(torch.bfloat16) for _ in range(nw)]
            it = [0]

            def nxt():
                it[0] = (it[0] + 1) % nw
                return ws[it[0]]
            acc = torch.zeros(M, N, device=dev, dtype=torch.bfloat16)
            if res:
                runs = {"blas": lambda: acc.addmm_(x, nxt().t()),
                        "gv": lambda: ops.skinny_gemm(x, nxt(), residual=acc, out=acc)}
            elif N == 28672:  # gate|up: library + silu_mul vs the skinny SwiGLU epilogue
                runs = {"blas": lambda: ops.silu_mul(F.linear(x, nxt()), block=32),
                        "gv": lambda: ops.skinny_gemm(x, nxt(), swiglu=True)}
            else:
                runs = {"blas": lambda: F.linear(x, nxt()), "gv": lambda: ops.skinny_gemm(x, nxt())}
            t = {k: [] for k in runs}
            for _ in range(5):
                for k, fn in runs.items():
                    t[k].append(timeit(fn, iters=20, warm=3))
            gb = N * K * 2 / 1e12
            line = "  ".join(f"{k} {sorted(v)[2]:7.1f} us ({gb / sorted(v)[2] * 1e6:4.1f} TB/s)" for k, v in t.items())
            print(f"skinny M={M} {N}x{K}{' res' if res else ''}: {line}", flush=True)
            del x, ws, acc


def serve_shapes(dev):
    """Llama-3-8B projections at the serving path's mixed chunked-prefill row counts (2048 prompt rows + the
    decode rows): every backend the planner times, median of 5 interleaved rounds (SERVE_M overrides)."""
    import torch.nn.functional as F

    from llm_weighted_consensus_amd import ops

    d, Fd, QKV = 4096, 14336, 6144
    r = lambda *s: ((torch.rand(*s, device=dev) * 2 - 1) / s[-1] ** 0.5).to(torch.bfloat16)  # noqa: E731
    wqkv, wo, wgu, wd = r(QKV, d), r(d, d), ops.swiglu_interleave(r(2 * Fd, d)), r(d, Fd)
    for M in [int(m) for m in os.environ.get("SERVE_M", "512,1024,2048,2304,2560,3072").split(",")]:
        x, xa, xf = r(M, d) * 8, r(M, d) * 8, r(M, Fd) * 8
        acc = torch.zeros(M, d, device=dev, dtype=torch.bfloat16)
        runs = {
            "qkv blas": lambda: F.linear(x, wqkv), "qkv g4": lambda: ops.gemm4w(x, wqkv),
            "qkv g4n192": lambda: ops.gemm4w(x, wqkv, bn=192), "qkv g8": lambda: ops.gemm8p(x, wqkv),
            "o blas": lambda: acc.addmm_(xa, wo.t()), "o g4": lambda: ops.gemm4w(xa, wo, residual=acc, out=acc),
            "o g8": lambda: ops.gemm8p(xa, wo, residual=acc, out=acc),
            "gu blas+silu": lambda: ops.silu_mul(F.linear(x, wgu), block=32),
            "gu g4": lambda: ops.gemm4w(x, wgu, swiglu=True), "gu g4p": lambda: ops.gemm4w(x, wgu, swiglu=True, var=64),
            "gu g8": lambda: ops.gemm8p(x, wgu, swiglu=True),
            "down blas": lambda: acc.addmm_(xf, wd.t()), "down g4": lambda: ops.gemm4w(xf, wd, residual=acc, out=acc),
            "down g8": lambda: ops.gemm8p(xf, wd, residual=acc, out=acc),
        }
        # split-K (VAR 64) where ops.split_plan splits the call or its ragged tail
        for k, (w, K, kw) in {"qkv": (wqkv, d, {}), "o": (wo, d, {"residual": acc, "out": acc}),
                              "gu": (wgu, d, {"swiglu": True}), "down": (wd, Fd, {"residual": acc, "out": acc})}.items():
            S, f = ops.split_plan(M, w.shape[0], K)
            if S > 1:
                a_ = xf if k == "down" else (xa if k == "o" else x)
                runs[f"{k} g4s{S}@{f}"] = (lambda a_=a_, w=w, kw=kw, S=S, f=f:
                                           ops.gemm4w(a_, w, var=64, splits=S, split_from=f, **kw))
            # SERVE_SPLITS: forced whole-call splits (any S: uneven K shares) for qkv / o / down
            for S in [int(v) for v in os.environ.get("SERVE_SPLITS", "").split(",") if v]:
                if k != "gu" and (K // 64) // 2 >= S:
                    a_ = xf if k == "down" else (xa if k == "o" else x)
                    runs[f"{k} g4s{S}"] = (lambda a_=a_, w=w, kw=kw, S=S:
                                           ops.gemm4w(a_, w, var=64, splits=S, split_from=0, **kw))
        if os.environ.get("SERVE_ONLY"):  # e.g. "o ,down ": arms whose name starts with one of these
            pre = tuple(os.environ["SERVE_ONLY"].split(","))
            runs = {k: v for k, v in runs.items() if k.startswith(pre)}
        res = {k: [] for k in runs}
        for _ in range(5):
            for k, fn in runs.items():
                res[k].append(timeit(fn, iters=10, warm=2))
        for k, t in res.items():
            print(f"serve M={M} {k}: {sorted(t)[2]:8.1f} us", flush=True)


def g48_ab(dev):
    """Dense fp8: gemm8g (dense mode) vs hipBLASLt's row-scaled fp8 GEMM at config 5's shapes (median of 5
    interleaved rounds; G48_SHAPES picks a subset).  (The 4-wave gemm4w8 arm was removed in round 6: 3-13 %
    behind gemm8g, profiles/fp8_4wave_r5.md, and its accumulators rotated through in-flight copies.)"""
    from llm_weighted_consensus_amd import ops

    shapes = [(4096, 6144, 4096), (4096, 4096, 4096), (4096, 4096, 14336), (16384, 6144, 4096), (8192, 4096, 14336),
              (65536, 6144, 4096)]
    only = os.environ.get("G48_SHAPES")
    if only:
        shapes = [shapes[int(i)] for i in only.split(",")]
    for M, N, K in shapes:
        x = torch.randn(M, K, device=dev).to(torch.bfloat16)
        xq, xs = ops.quant_fp8_rows(x)
        del x
        w = ops.Fp8Weight((torch.randn(N, K, device=dev) / K ** 0.5).to(torch.bfloat16))
        runs = {"blas": lambda: ops._fp8_blas(xq, xs, w), "g8g": lambda: ops.gemm8g_dense(xq, xs, w)}
        res = {k: [] for k in runs}
        for _ in range(5):
            for k, fn in runs.items():
                res[k].append(timeit(fn, iters=5, warm=1))
        fl = 2 * M * N * K / 1e12
        line = "  ".join(f"{k} {sorted(t)[2]:8.1f} us ({fl / sorted(t)[2] * 1e6:5.0f})" for k, t in res.items())
        print(f"g48 {M}x{N}x{K}: {line}", flush=True)
        del xq, xs, w


def route_ab(dev):
    """Config-5 MoE plumbing at the decode batch (T = 4096 tokens, Mixtral d = 4096, 8 experts, top-2):
    the router projection + route (unfused: F.linear then moe_route) vs the fused moe_router kernel, and
    the other small per-layer kernels around the experts.  Median of 5 interleaved rounds."""
    import torch.nn.functional as F

    from llm_weighted_consensus_amd import ops

    T, d, E = int(os.environ.get("ROUTE_T", "4096")), 4096, 8
    h = torch.randn(T, d, device=dev).to(torch.bfloat16)
    r = torch.randn(T, d, device=dev).to(torch.bfloat16)
    router = (torch.randn(E, d, device=dev) * 0.05).to(torch.bfloat16)
    ones = torch.ones(d, device=dev, dtype=torch.bfloat16)
    lg = F.linear(h, router)
    _ids, w, _ro, _src, inv = ops.moe_route(lg, 2)
    Y = torch.randn(2 * T, d, device=dev).to(torch.bfloat16)
    runs = {
        "router F.linear": lambda: F.linear(h, router),
        "moe_route (logits)": lambda: ops.moe_route(lg, 2),
        "unfused (linear + route)": lambda: ops.moe_route(F.linear(h, router), 2),
        "fused moe_router": lambda: ops.moe_router(h, router, 2),
        "rmsnorm+res+q (bf16 kept)": lambda: ops.rmsnorm_quant_fp8(h, ones, 1e-5, residual=r, keep_bf16=True),
        "rmsnorm+res": lambda: ops.rmsnorm(h, ones, 1e-5, residual=r),
        "quant_fp8_rows": lambda: ops.quant_fp8_rows(h),
        "moe_combine": lambda: ops.moe_combine(Y, inv, w, 2),
    }
    res = {k: [] for k in runs}
    for _ in range(5):
        for k, fn in runs.items():
            res[k].append(timeit(fn, iters=20, warm=3))
    for k, t in res.items():
        print(f"route T={T} {k}: {sorted(t)[2]:8.1f} us", flush=True)


def chain_ab(dev):
    """Folded-RMSNorm decode chain at the headline's decode batch (Llama-3-8B shapes, M = 4096; random
    operands): per projection the unfolded backends (hipBLASLt / gemm4w, + the norm kernel) vs the row-scaled
    gemm4w modes, then one whole layer + lm_head both ways.  Interleaved rounds, median of 5."""
    import torch.nn.functional as F

    from llm_weighted_consensus_amd import ops

    M, d, Fd, V, QKV = int(os.environ.get("CHAIN_M", "4096")), 4096, 14336, 128256, 6144
    r = lambda *s: ((torch.rand(*s, device=dev) * 2 - 1) / s[-1] ** 0.5).to(torch.bfloat16)  # noqa: E731
    x = (torch.rand(M, d, device=dev) * 2 - 1).to(torch.bfloat16)
    xa, xf = r(M, d) * 8, r(M, Fd) * 8
    wqkv, wo, wgu, wd, wl = r(QKV, d), r(d, d), ops.swiglu_interleave(r(2 * Fd, d)), r(d, Fd), r(V, d)
    ones = torch.ones(d, device=dev, dtype=torch.bfloat16)
    ch = ops.NormChain(M, d, 1e-5, dev)
    acc = x.clone()
    ops.rms_rowsumsq(acc, ch)
    runs = {
        "rmsnorm": lambda: ops.rmsnorm(acc, ones, 1e-5),
        "rowsumsq": lambda: ops.rms_rowsumsq(acc, ch),
        "qkv blas": lambda: F.linear(x, wqkv),
        "qkv g4n192": lambda: ops.gemm4w(x, wqkv, bn=192),
        "qkv g4n192 rs": lambda: ops.gemm4w(x, wqkv, bn=192, chain=ch),
        "qkv g4 rs": lambda: ops.gemm4w(x, wqkv, chain=ch),
        "o blas res": lambda: acc.addmm_(xa, wo.t()),
        "o g4 res": lambda: ops.gemm4w(xa, wo, residual=acc, out=acc),
        "o g4 res+ss": lambda: ops.gemm4w(xa, wo, residual=acc, out=acc, chain=ch),
        "o g4 res+ss v64": lambda: ops.gemm4w(xa, wo, residual=acc, out=acc, chain=ch, var=64),
        "gu g4": lambda: ops.gemm4w(x, wgu, swiglu=True),
        "gu g4 rs": lambda: ops.gemm4w(x, wgu, swiglu=True, chain=ch),
        "down blas res": lambda: acc.addmm_(xf, wd.t()),
        "down g4 res": lambda: ops.gemm4w(xf, wd, residual=acc, out=acc),
        "down g4 res+ss": lambda: ops.gemm4w(xf, wd, residual=acc, out=acc, chain=ch),
        "down g4 res+ss v64": lambda: ops.gemm4w(xf, wd, residual=acc, out=acc, chain=ch, var=64),
        "lm blas": lambda: F.linear(x, wl),
        "lm g4": lambda: ops.gemm4w(x, wl),
        "lm g4 v64": lambda: ops.gemm4w(x, wl, var=64),
        "lm g4 rs": lambda: ops.gemm4w(x, wl, chain=ch),
    }
    res = {k: [] for k in runs}
    for _ in range(5):
        for k, fn in runs.items():
            res[k].append(timeit(fn, iters=10, warm=2))
    for k, t in res.items():
        print(f"chain {M} {k}: {sorted(t)[2]:8.1f} us", flush=True)
    med = {k: sorted(t)[2] for k, t in res.items()}
    base = (2 * med["rmsnorm"] + min(med["qkv blas"], med["qkv g4n192"]) + med["o blas res"] + med["gu g4"]
            + med["down blas res"])
    chain = (med["qkv g4n192 rs"] + min(med["o g4 res+ss"], med["o g4 res+ss v64"]) + med["gu g4 rs"]
             + min(med["down g4 res+ss"], med["down g4 res+ss v64"]))
    print(f"chain {M} per layer: unfolded {base:.1f} us, chain {chain:.1f} us; lm_head: unfolded "
          f"{med['rmsnorm'] + med['lm blas']:.1f}, chain {med['lm g4 rs']:.1f}", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("what", nargs="*", default=["gemm", "attn", "sample", "small"])
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    if "gemm" in a.what:
        gemms(dev, [int(m) for m in os.environ.get("MICRO_M", "256,512").split(",")], tuned=os.environ.get("PYTORCH_TUNABLEOP_ENABLED") == "1")
    if "backends" in a.what:
        gemm_backends(dev, [1024, 1536])
    if "grouped" in a.what:
        grouped(dev)
    if "g4ab" in a.what:
        gemm4w_ab(dev)
    if "chain" in a.what:
        chain_ab(dev)
    if "route" in a.what:
        route_ab(dev)
    if "enc" in a.what:
        encoder_gemms(dev)
    if "serve" in a.what:
        serve_shapes(dev)
    if "skinny" in a.what:
        skinny_ab(dev)
    if "g48" in a.what:
        g48_ab(dev)
    if "g8ab" in a.what:
        gemm8p_ab(dev)
    if "g8" in a.what:
        gemm8p_study(dev, [int(m) for m in os.environ.get("MICRO_M", "3072,1024").split(",")])
    if "layout" in a.what:
        gemm_layouts(dev, [int(m) for m in os.environ.get("MICRO_M", "512,1024").split(",")])
    if "attn" in a.what:
        attention(dev)
    if "bw" in a.what:
        bandwidth(dev)
    if "pfattn" in a.what:
        prefill_attn(dev)
    if "prefix" in a.what:
        attention_prefix(dev)
    if "sample" in a.what:
        sampler(dev)
    if "moe" in a.what:
        moe_decode(dev)
    if "small" in a.what:
        small(dev)


if __name__ == "__main__":
    main()
