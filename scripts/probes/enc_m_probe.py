"""Does gemm4w's K loop slow down when A streams from HBM?  Config 2's FFN2 (N 768, K 3072) and o (N 768,
K 768) projections on VAR 64 at growing M (A from 96 MB, inside the 256 MB Infinity Cache, to 3 GB), with
hipBLASLt beside each: us per call and per K tile of a round."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from llm_weighted_consensus_amd import ops  # noqa: E402


def t(fn, it=3):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it * 1e3


dev = torch.device("cuda")
for N, K in ((768, 3072), (768, 768)):
    w = (torch.randn(N, K, device=dev) / K ** 0.5).to(torch.bfloat16)
    b = (torch.randn(N, device=dev) * 0.1).to(torch.bfloat16)
    for M in (16384, 65536, 262144, 524288):
        x = (torch.randn(M, K, device=dev) * 0.5).to(torch.bfloat16)
        own, lib = [], []
        for _ in range(3):
            own.append(t(lambda: ops.gemm4w(x, w, bias=b, var=64)))
            lib.append(t(lambda: F.linear(x, w, b)))
        o, l = sorted(own)[1], sorted(lib)[1]
        rounds = -(-(M // 256) * (N // 256) // 256)
        print(f"N {N} K {K} M {M:6d} (A {M * K * 2 / 2**20:6.0f} MiB): gemm4w {o:8.1f} us "
              f"({o / rounds / (K // 64):.3f} us/K tile over {rounds} rounds)  hipBLASLt {l:8.1f} us", flush=True)
        del x
