"""Run one dense fp8 GEMM backend ITERS times (for rocprofv3 --pmc passes): fp8_gemm_run.py {g8g|blas} M N K ITERS"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from llm_weighted_consensus_amd import ops  # noqa: E402

kind, M, N, K, iters = sys.argv[1], *map(int, sys.argv[2:6])
dev = torch.device("cuda", 0)
xq, xs = ops.quant_fp8_rows(torch.randn(M, K, device=dev).to(torch.bfloat16))
w = ops.Fp8Weight((torch.randn(N, K, device=dev) / K ** 0.5).to(torch.bfloat16))
fn = {"g8g": lambda: ops.gemm8g_dense(xq, xs, w),
      "blas": lambda: ops._fp8_blas(xq, xs, w)}[kind]
for _ in range(iters):
    fn()
torch.cuda.synchronize()
print("done", kind)
