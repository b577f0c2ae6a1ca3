#!/usr/bin/env python3
"""Encoder FFN1 (x W1^T + b1, GELU) options at the bench's token counts: hipBLASLt GEMM + a separate GELU
pass (what the removed K9b bias_gelu kernel did), hipBLASLt with its bias+GELU epilogue
(torch._addmm_activation, the shipped library path), gemm8p's bias+GELU epilogue, and the plain biased GEMM
as the lower bound.  Prints time and error vs fp32 erf-GELU."""
import sys
import os

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_weighted_consensus_amd import ops  # noqa: E402
from llm_weighted_consensus_amd.ops.gemm_plan import _time  # noqa: E402


def main():
    dev = torch.device("cuda")
    torch.manual_seed(0)
    for M in (16384, 65536):
        d, f = 1024, 4096
        x = (torch.randn(M, d, device=dev) * 0.5).to(torch.bfloat16)
        w = (torch.randn(f, d, device=dev) / d ** 0.5).to(torch.bfloat16)
        b = (torch.randn(f, device=dev) * 0.1).to(torch.bfloat16)
        ref = F.gelu(x.float() @ w.float().t() + b.float())
        arms = {
            "blas + separate GELU pass": lambda: F.gelu(F.linear(x, w, b)),
            "blas epilogue (addmm_activation)": lambda: torch._addmm_activation(b, x, w.t(), use_gelu=True),
            "gemm8p bias_gelu": lambda: ops.gemm8p(x, w, bias=b, gelu=True),
            "blas bias only (bound)": lambda: F.linear(x, w, b),
        }
        for name, fn in arms.items():
            try:
                y = fn()
                t = _time(fn, iters=5, rounds=5)
                err = (y.float() - ref).abs().max().item() if "bound" not in name else float("nan")
                print(f"M={M:6d} {name:36s} {t:9.1f} us   max|err| vs erf-GELU {err:.4g}", flush=True)
            except Exception as e:  # an arm the library does not support here
                print(f"M={M:6d} {name:36s} failed: {e!r}", flush=True)


if __name__ == "__main__":
    main()
