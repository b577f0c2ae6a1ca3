"""Encoder small-K GEMMs on gemm4w VAR 64 by tile-group size gm (m-tiles per group of the grouped order):
config 2's qkv / o / FFN1 + GELU / FFN2 at 0.5 M tokens, median of 5 interleaved rounds, us."""
import os
import sys

import torch

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
M, d = int(os.environ.get("ENC_M", "524288")), 768
GMS = [int(g) for g in os.environ.get("GMS", "1,2,4,8,16,32").split(",")]
for N, K, gelu in ((3 * d, d, False), (d, d, False), (4 * d, d, True), (d, 4 * d, False)):
    x = (torch.randn(M, K, device=dev) * 0.5).to(torch.bfloat16)
    w = (torch.randn(N, K, device=dev) / K ** 0.5).to(torch.bfloat16)
    b = (torch.randn(N, device=dev) * 0.1).to(torch.bfloat16)
    runs = {gm: (lambda gm=gm: ops.gemm4w(x, w, bias=b, gelu=gelu, var=64, gm=gm)) for gm in GMS}
    res = {k: [] for k in runs}
    for _ in range(5):
        for k, fn in runs.items():
            res[k].append(t(fn))
    print(f"{N}x{K}{' gelu' if gelu else ''}: " + "  ".join(f"gm{k} {sorted(v)[2]:7.1f}" for k, v in res.items()),
          flush=True)
    del x, w
