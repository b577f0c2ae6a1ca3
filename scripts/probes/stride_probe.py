"""Why does the down projection's K tile cost more cycles than o's?  gemm4w (plain epilogue, VAR 64) on the
decode batch with A rows 8 KB apart (o), 28 KB apart (a K = 4096 slice of the [4096, 14336] activation) and
the full down shape, per K tile, interleaved rounds in one process; hipBLASLt beside each."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
from llm_weighted_consensus_amd import ops  # noqa: E402


def t(fn, it=10):
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
M = 4096
a4 = torch.randn(M, 4096, device=dev).bfloat16()
a14 = torch.randn(M, 14336, device=dev).bfloat16()
w4 = (torch.randn(4096, 4096, device=dev) * 0.02).bfloat16()
w14 = (torch.randn(4096, 14336, device=dev) * 0.02).bfloat16()
w14s = w14[:, :4096].contiguous()
cases = {
    "A 8K rows, K 4096": (lambda: ops.gemm4w(a4, w4, var=64), lambda: F.linear(a4, w4), 64),
    "A 28K rows, K 4096": (lambda: ops.gemm4w(a14[:, :4096], w4, var=64), lambda: F.linear(a14[:, :4096], w4), 64),
    "down K 14336": (lambda: ops.gemm4w(a14, w14, var=64), lambda: F.linear(a14, w14), 224),
    "down K 14336 var32": (lambda: ops.gemm4w(a14, w14, var=32), None, 224),
}
res = {k: ([], []) for k in cases}
for _ in range(5):
    for k, (own, lib, kt) in cases.items():
        res[k][0].append(t(own))
        if lib is not None:
            res[k][1].append(t(lib))
for k, (o, l) in res.items():
    kt = cases[k][2]
    om = sorted(o)[2]
    lm = sorted(l)[2] if l else float("nan")
    print(f"{k:22s} gemm4w {om:8.1f} us ({om / kt:.3f} us/K tile)   hipBLASLt {lm:8.1f} us ({lm / kt:.3f})", flush=True)
