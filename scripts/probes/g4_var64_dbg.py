"""Debug: gemm4w VAR 64 / 96 vs fp32 on small shapes; which K tiles the result actually summed."""
import itertools
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from llm_weighted_consensus_amd import ops  # noqa: E402

dev = torch.device("cuda", 0)
for (M, N, K) in [(256, 256, 256)]:
    torch.manual_seed(0)
    A = torch.randn(M, K, device=dev).to(torch.bfloat16)
    W = (torch.randn(N, K, device=dev) / K ** 0.5).to(torch.bfloat16)
    KT = K // 64
    parts = [A[:, 64 * t:64 * t + 64].float() @ W[:, 64 * t:64 * t + 64].float().t() for t in range(KT)]
    ref = sum(parts)
    for var in (32, 64, 96):
        out = ops.gemm4w(A, W, var=var).float()
        err = (out - ref).abs().max().item()
        print(f"M={M} N={N} K={K} var={var}: max err {err:.3f}", flush=True)
        if err > 0.1:
            best = None
            for combo in itertools.product(range(KT), repeat=KT):
                e = (out - sum(parts[c] for c in combo)).abs().max().item()
                if best is None or e < best[0]:
                    best = (e, combo)
            print(f"   closest K-tile multiset: {best[1]} (err {best[0]:.3f})", flush=True)
