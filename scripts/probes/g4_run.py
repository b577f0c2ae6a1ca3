"""Run gate|up + SwiGLU (M = 4096, N = 28672, K = 4096) on one backend ITERS times, for rocprofv3 --pmc passes:
g4_run.py {g4v64|g4v32|blas} ITERS  (blas = hipBLASLt + silu_mul)"""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from llm_weighted_consensus_amd import ops  # noqa: E402

kind, iters = sys.argv[1], int(sys.argv[2])
dev = torch.device("cuda", 0)
M, N, K = 4096, 28672, 4096
x = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
w = ops.swiglu_interleave(((torch.rand(N, K, device=dev) * 2 - 1) / K ** 0.5).to(torch.bfloat16))
if kind == "blas":
    fn = lambda: ops.silu_mul(F.linear(x, w), block=32)  # noqa: E731
else:
    var = int(kind[3:])
    fn = lambda: ops.gemm4w(x, w, swiglu=True, var=var)  # noqa: E731
for _ in range(iters):
    fn()
torch.cuda.synchronize()
print("done", kind)
