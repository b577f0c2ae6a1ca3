#!/usr/bin/env python3
"""A/B: o / down projection + residual add + RMSNorm, separate (F.linear -> fused residual-add+norm
kernel) vs the residual add inside the GEMM (hipBLASLt beta = 1, or gemm8p's residual epilogue) followed
by a plain norm.  Same process, interleaved, median of rounds."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

from llm_weighted_consensus_amd import ops  # noqa: E402


def timeit(fn, iters=20, rounds=5):
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


def main():
    dev = torch.device("cuda:0")
    for M in (3072, 4096):
        for K in (4096, 14336):
            N = 4096
            x = torch.randn(M, K, device=dev).to(torch.bfloat16)
            w = (torch.randn(N, K, device=dev) / K ** 0.5).to(torch.bfloat16)
            g = torch.ones(N, device=dev, dtype=torch.bfloat16)
            res = torch.randn(M, N, device=dev).to(torch.bfloat16)
            o = torch.randn(M, N, device=dev).to(torch.bfloat16)

            def sep():
                return ops.rmsnorm(F.linear(x, w), g, 1e-5, residual=res)

            def blas_fused():
                res.addmm_(x, w.t())
                return ops.rmsnorm(res, g, 1e-5)

            def g8_fused():
                ops.gemm8p(x, w, residual=res, out=res)
                return ops.rmsnorm(res, g, 1e-5)

            r = {k: timeit(f) for k, f in [("linear", lambda: F.linear(x, w)), ("addmm_", lambda: res.addmm_(x, w.t())),
                                            ("norm+res", lambda: ops.rmsnorm(o, g, 1e-5, residual=res)),
                                            ("norm", lambda: ops.rmsnorm(res, g, 1e-5)),
                                            ("A sep", sep), ("B blas-fused", blas_fused), ("C g8-fused", g8_fused)]}
            print(f"M={M} K={K}: " + "  ".join(f"{k} {v:.1f}" for k, v in r.items()), flush=True)


if __name__ == "__main__":
    main()
