#!/usr/bin/env python3
"""A/B of the fp8 MoE expert GEMMs (Mixtral-8x7B shapes, top-2 of 8 experts, random routing, A rows gathered
like the model does): the 128x128 grouped kernel (gemm.hip) vs the 8-phase grouped kernel (gemm8g.hip),
interleaved rounds in one process, median of 3.  TF/s = 2 * rows * N * K / time."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters=10):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3


def main():
    from llm_weighted_consensus_amd import ops

    dev = torch.device("cuda", 0)
    E, d, f = 8, 4096, 14336
    g = torch.Generator(device=dev).manual_seed(0)
    q13, s13 = ops.quant_fp8_weight((torch.randn(E, 2 * f, d, device=dev, generator=g) * 0.02).to(torch.bfloat16))
    q2, s2 = ops.quant_fp8_weight((torch.randn(E, d, f, device=dev, generator=g) * 0.02).to(torch.bfloat16))
    for T in (int(t) for t in os.environ.get("MOE_T", "512,1024,2048").split(",")):
        h = torch.randn(T, d, device=dev, generator=g).to(torch.bfloat16)
        logits = torch.randn(T, E, device=dev, generator=g).to(torch.bfloat16)
        _ids, _w, row_off, src, _inv = ops.moe_route(logits, 2)
        rows = 2 * T
        hq, hs = ops.quant_fp8_rows(h)
        act = torch.randn(rows, f, device=dev, generator=g).to(torch.bfloat16)
        aq, as_ = ops.quant_fp8_rows(act)
        res = {}
        for mode in ("classic", "g8") * 3:
            ops.MOE_GEMM = mode
            t13 = timeit(lambda: ops.grouped_gemm(hq, q13, row_off, a_rows=src, rows=rows, a_scale=hs, w_scale=s13))
            t2 = timeit(lambda: ops.grouped_gemm(aq, q2, row_off, a_scale=as_, w_scale=s2))
            res.setdefault(mode, []).append((t13, t2))
        ops.MOE_GEMM = "classic"
        ref = ops.grouped_gemm(hq, q13, row_off, a_rows=src, rows=rows, a_scale=hs, w_scale=s13)
        ops.MOE_GEMM = "g8"
        got = ops.grouped_gemm(hq, q13, row_off, a_rows=src, rows=rows, a_scale=hs, w_scale=s13)
        err = ((got.float() - ref.float()).norm() / ref.float().norm()).item()
        for mode, v in res.items():
            t13 = sorted(x[0] for x in v)[1]
            t2 = sorted(x[1] for x in v)[1]
            f13 = 2 * rows * 2 * f * d / t13 / 1e6
            f2 = 2 * rows * d * f / t2 / 1e6
            print(f"T={T:5d} {mode:8s}: w13 {t13:8.1f} us ({f13:5.0f} TF/s)  w2 {t2:8.1f} us ({f2:5.0f} TF/s)"
                  + (f"  rel diff vs classic {err:.2e}" if mode == "g8" else ""), flush=True)


if __name__ == "__main__":
    main()
