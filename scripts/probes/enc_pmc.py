"""One FFN2-shaped call each of gemm4w VAR 64 and hipBLASLt at config 2's M (A = 3 GB streamed from HBM), for
a rocprofv3 --pmc pass (FETCH_SIZE, TCC hit / miss per kernel)."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from llm_weighted_consensus_amd import ops  # noqa: E402

dev = torch.device("cuda")
M, N, K = int(os.environ.get("ENC_M", "524288")), 768, 3072
x = (torch.randn(M, K, device=dev) * 0.5).to(torch.bfloat16)
w = (torch.randn(N, K, device=dev) / K ** 0.5).to(torch.bfloat16)
b = (torch.randn(N, device=dev) * 0.1).to(torch.bfloat16)
for _ in range(3):
    ops.gemm4w(x, w, bias=b, var=64)
    F.linear(x, w, b)
torch.cuda.synchronize()
print("done", flush=True)
