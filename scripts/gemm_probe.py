#!/usr/bin/env python3
"""Run one projection GEMM shape repeatedly on one backend, for rocprofv3 kernel traces / PMC counters.

    python scripts/gemm_probe.py g8|blas|g8swiglu M N K [iters]
"""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from llm_weighted_consensus_amd import ops

    kind, M, N, K = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
    iters = int(sys.argv[5]) if len(sys.argv) > 5 else 20
    dev = torch.device("cuda:0")
    x = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
    w = ((torch.rand(N, K, device=dev) * 2 - 1) / K ** 0.5).to(torch.bfloat16)
    if kind == "g8swiglu":
        w = ops.swiglu_interleave(w)
        fn = lambda: ops.gemm8p(x, w, swiglu=True)  # noqa: E731
    elif kind == "g8":
        fn = lambda: ops.gemm8p(x, w)  # noqa: E731
    elif kind.startswith("g4"):  # g4 / g4n192 (bn 192)
        bn = 192 if kind == "g4n192" else 256
        fn = lambda: ops.gemm4w(x, w, bn=bn)  # noqa: E731
    else:
        fn = lambda: F.linear(x, w)  # noqa: E731
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) / iters * 1e3
    print(f"{kind} M={M} N={N} K={K}: {us:.1f} us {2 * M * N * K / us / 1e6:.0f} TF/s", flush=True)


if __name__ == "__main__":
    main()
