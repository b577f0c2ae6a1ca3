#!/usr/bin/env python3
"""A/B of the fp8 MoE expert FFN's middle (Mixtral-8x7B shapes, top-2 of 8, random routing, A rows gathered
as the model does): gate|up GEMM -> fused SwiGLU + e4m3 row quantisation (silu_mul_quant_fp8) vs the SwiGLU in
gemm8g's epilogue (gate / up rows interleaved) -> quant_fp8_rows.  Interleaved rounds, median of 3."""
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
    E, d, f, k = 8, 4096, 14336, 2
    g = torch.Generator(device=dev).manual_seed(0)
    w13 = (torch.randn(E, 2 * f, d, device=dev, generator=g) * 0.02).to(torch.bfloat16)
    q13, s13 = ops.quant_fp8_weight(w13)
    w13i = torch.stack([ops.swiglu_interleave(w13[e]) for e in range(E)])
    q13i, s13i = ops.quant_fp8_weight(w13i)
    del w13, w13i
    for T in (1024, 2048):
        h = torch.randn(T, d, device=dev, generator=g).to(torch.bfloat16)
        router = (torch.randn(E, d, device=dev, generator=g) * 0.1).to(torch.bfloat16)
        _ids, _w, row_off, src, _inv = ops.moe_route(torch.nn.functional.linear(h, router), k)
        hq, hs = ops.quant_fp8_rows(h)
        rows = T * k

        def old():
            gu = ops.grouped_gemm(hq, q13, row_off, a_rows=src, rows=rows, a_scale=hs, w_scale=s13)
            return ops.silu_mul_quant_fp8(gu)

        def new():
            act = ops.grouped_gemm(hq, q13i, row_off, a_rows=src, rows=rows, a_scale=hs, w_scale=s13i, swiglu=True)
            return ops.quant_fp8_rows(act)

        res = {"old": [], "new": []}
        for _ in range(3):
            for name, fn in (("old", old), ("new", new)):
                res[name].append(timeit(fn))
        med = {n: sorted(v)[1] for n, v in res.items()}
        a, b = old(), new()
        ra = a[0].float() * a[1][:, None]
        rb = b[0].float() * b[1][:, None]
        rel = ((ra - rb).norm() / ra.norm()).item()
        print(f"T={T:5d}: gate|up + silu_mul_quant {med['old']:8.1f} us   gate|up+SwiGLU epilogue + quant_rows "
              f"{med['new']:8.1f} us   rel diff {rel:.2e}", flush=True)


if __name__ == "__main__":
    main()
