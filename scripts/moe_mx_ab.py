#!/usr/bin/env python3
"""A/B of the fp8 MoE expert FFN (Mixtral-8x7B shapes, top-2 of 8, random routing, A rows gathered as the
model does), gate|up through down, three forms of the middle:
  rowq : SwiGLU in gemm8g's epilogue -> bf16 [rows, F] -> quant_fp8_rows -> down (per-row scales);
  mx   : SwiGLU epilogue writes e4m3 + e8m0 block scales -> down with the scales in its MFMAs.
Interleaved rounds, median of 5; relative difference of the two outputs."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from moe_swiglu_ab import timeit  # noqa: E402


def main():
    from llm_weighted_consensus_amd import ops

    dev = torch.device("cuda", 0)
    E, d, f, k = 8, 4096, 14336, 2
    g = torch.Generator(device=dev).manual_seed(0)
    w13 = torch.stack([ops.swiglu_interleave((torch.randn(2 * f, d, device=dev, generator=g) * 0.02).to(torch.bfloat16))
                       for _ in range(E)])
    q13, s13 = ops.quant_fp8_weight(w13)
    del w13
    w2 = (torch.randn(E, d, f, device=dev, generator=g) * 0.02).to(torch.bfloat16)
    q2, s2 = ops.quant_fp8_weight(w2)
    del w2
    for T in (2048, 4096):
        h = torch.randn(T, d, device=dev, generator=g).to(torch.bfloat16)
        router = (torch.randn(E, d, device=dev, generator=g) * 0.1).to(torch.bfloat16)
        _ids, _w, row_off, src, _inv = ops.moe_route(torch.nn.functional.linear(h, router), k)
        hq, hs = ops.quant_fp8_rows(h)
        rows = T * k

        def rowq():
            act = ops.grouped_gemm(hq, q13, row_off, a_rows=src, rows=rows, a_scale=hs, w_scale=s13, swiglu=True)
            aq, as_ = ops.quant_fp8_rows(act)
            return ops.grouped_gemm(aq, q2, row_off, a_scale=as_, w_scale=s2)

        def mx():
            aq, amx = ops.grouped_gemm_swiglu_mx(hq, q13, row_off, hs, s13, a_rows=src, rows=rows)
            return ops.grouped_gemm(aq, q2, row_off, w_scale=s2, a_mx=amx)

        res = {"rowq": [], "mx": []}
        for _ in range(5):
            for name, fn in (("rowq", rowq), ("mx", mx)):
                res[name].append(timeit(fn))
        med = {n: sorted(v)[2] for n, v in res.items()}
        a, b = rowq().float(), mx().float()
        rel = ((a - b).norm() / a.norm()).item()
        print(f"T={T:5d}: row-quantised middle {med['rowq']:8.1f} us   MX middle {med['mx']:8.1f} us   "
              f"rel diff {rel:.2e}", flush=True)


if __name__ == "__main__":
    main()
