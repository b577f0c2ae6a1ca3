"""Where does gemm4w VAR 64's GELU epilogue go non-finite?  M = 1000, N = 1024, K = 512 (test_gemm8p_bias_gelu
shape) and the identity-W value sweep."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from llm_weighted_consensus_amd import ops  # noqa: E402

dev = torch.device("cuda")
torch.manual_seed(0)
for var in (32, 64):
    M, K = 512, 128
    x = torch.linspace(-10, 10, M * K, device=dev).view(M, K).to(torch.bfloat16)
    W = torch.eye(K, device=dev).to(torch.bfloat16)
    b = torch.zeros(K, device=dev).to(torch.bfloat16)
    y = ops.gemm4w(x, W, bias=b, gelu=True, var=var).float()
    ref = torch.nn.functional.gelu(x.float())
    bad = ~torch.isfinite(y)
    print(f"identity var {var}: nonfinite {int(bad.sum())}, max err {float((y - ref)[~bad].abs().max()):.3g}", flush=True)
    if bad.any():
        idx = bad.nonzero()[:8]
        for r, c in idx.tolist():
            print("   ", r, c, float(x[r, c]), float(y[r, c]), flush=True)
    M, N, K = 1000, 1024, 512
    A = torch.randn(M, K, device=dev).to(torch.bfloat16)
    W = (torch.randn(N, K, device=dev) / K ** 0.5).to(torch.bfloat16)
    b = (torch.randn(N, device=dev) * 0.1).to(torch.bfloat16)
    y = ops.gemm4w(A, W, bias=b, gelu=True, var=var).float()
    ref = torch.nn.functional.gelu(A.float() @ W.float().t() + b.float())
    bad = ~torch.isfinite(y)
    print(f"random var {var}: nonfinite {int(bad.sum())} at rows {bad.any(1).nonzero().flatten()[:10].tolist()} "
          f"cols {bad.any(0).nonzero().flatten()[:10].tolist()}, max err {float((y - ref)[~bad].abs().max()):.3g}",
          flush=True)
