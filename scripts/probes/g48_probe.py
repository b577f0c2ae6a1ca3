"""gemm4w8 bring-up probe: max error vs fp32 per shape (isolates K-tile count, persistent rounds, ragged tiles)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from llm_weighted_consensus_amd import ops  # noqa: E402

dev = torch.device("cuda", 0)
torch.manual_seed(0)
for M, N, K in [(256, 256, 128), (256, 256, 256), (256, 256, 384), (256, 256, 512), (256, 256, 1024),
                (256, 256, 4096), (512, 512, 256), (4133, 6144, 256), (256 * 33, 256 * 8, 256), (4133, 6144, 4096)]:
    x = torch.randn(M, K, device=dev).to(torch.bfloat16)
    xq, xs = ops.quant_fp8_rows(x)
    w = ops.Fp8Weight((torch.randn(N, K, device=dev) / K ** 0.5).to(torch.bfloat16))
    ref = (xq.float() * xs.view(-1, 1)) @ (w.q.float() * w.s.view(-1, 1)).t()
    out = ops.gemm4w8_dense(xq, xs, w).float()
    d = (out - ref).abs()
    bad = (d > 0.02 * ref.abs().max() + 1e-3)
    rows = bad.any(1).nonzero().flatten()
    cols = bad.any(0).nonzero().flatten()
    print(f"{M}x{N}x{K}: max err {d.max().item():.4f} (ref max {ref.abs().max().item():.3f}); bad rows {rows.numel()} "
          f"{rows[:8].tolist()} cols {cols.numel()} {cols[:8].tolist()}", flush=True)
