#!/usr/bin/env python3
"""A/B of gemm8g's grouped tile order (LWC_G8G_GN: n-tiles an XCD walks per m-slot) and of skipping the
MFMAs of empty 64-row blocks in ragged tiles (LWC_G8G_SKIP) at config 5's routed
expert shapes (Mixtral-8x7B, top-2 of 8, random routing): gate|up with the SwiGLU epilogue (N = 2F = 28672,
K = 4096) and down (N = 4096, K = 14336).  Interleaved rounds, median of 5; outputs must be bitwise equal
across orders (the order moves work between workgroups, not the arithmetic)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from moe_swiglu_ab import timeit  # noqa: E402

ARMS = (("gn1,noskip", {"LWC_G8G_GN": "1", "LWC_G8G_SKIP": "0"}), ("gn1+skip", {"LWC_G8G_GN": "1", "LWC_G8G_SKIP": "1"}),
        ("slot-major,noskip", {"LWC_G8G_GN": "64", "LWC_G8G_SKIP": "0"}),
        ("slot-major+skip", {"LWC_G8G_GN": "64", "LWC_G8G_SKIP": "1"}))
ROUNDS = 5


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
        aq, as_ = ops.quant_fp8_rows(torch.randn(rows, f, device=dev, generator=g).to(torch.bfloat16))

        def gate_up():
            return ops.grouped_gemm(hq, q13, row_off, a_rows=src, rows=rows, a_scale=hs, w_scale=s13, swiglu=True)

        def down():
            return ops.grouped_gemm(aq, q2, row_off, rows=rows, a_scale=as_, w_scale=s2)

        for name, fn, flop in (("gate|up+SwiGLU", gate_up, 2 * rows * 2 * f * d), ("down", down, 2 * rows * d * f)):
            res = {arm: [] for arm, _ in ARMS}
            outs = {}
            for _ in range(ROUNDS):
                for arm, env in ARMS:
                    os.environ.update(env)
                    res[arm].append(timeit(fn))
                    outs[arm] = fn()
            ref = outs[ARMS[0][0]]
            line = " ".join(f"{arm}: {sorted(v)[len(v) // 2]:7.1f} us ({flop / sorted(v)[len(v) // 2] / 1e6:5.0f} TF/s)"
                            for arm, v in res.items())
            same = all(torch.equal(ref, o) for o in outs.values())
            print(f"T={T:5d} {name:15s} {line}  bitwise-equal={same}", flush=True)
            if not same:
                sys.exit(1)


if __name__ == "__main__":
    main()
