#!/usr/bin/env python3
"""Micro-benchmarks of the decode hot path on one MI355X: the Llama-3-8B projection GEMMs at decode
batch sizes (hipBLASLt default vs TunableOp-tuned), paged decode attention, the fused sampler and the
small fused kernels.  Prints one line per case: time, TFLOP/s, GB/s."""
import argparse
import math
import os
import sys
import time

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters=50, warm=5):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1e3  # us


def gemms(dev, Ms, tuned):
    shapes = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336),
              "lm_head": (128256, 4096)}
    for M in Ms:
        for name, (N, K) in shapes.items():
            x = torch.randn(M, K, device=dev).to(torch.bfloat16)
            w = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
            us = timeit(lambda: F.linear(x, w), iters=20)
            fl = 2 * M * N * K / (us * 1e-6) / 1e12
            gb = (N * K * 2 + M * K * 2 + M * N * 2) / (us * 1e-6) / 1e9
            print(f"gemm{'-tuned' if tuned else ''} M={M:4d} {name:8s} N={N:6d} K={K:5d}: {us:8.1f} us "
                  f"{fl:7.1f} TF/s {gb:7.0f} GB/s", flush=True)


def gemm_layouts(dev, Ms):
    """Same products through different operand layouts: hipBLASLt picks different kernels."""
    shapes = {"qkv": (6144, 4096), "o": (4096, 4096), "gate_up": (28672, 4096), "down": (4096, 14336)}
    for M in Ms:
        for name, (N, K) in shapes.items():
            x = torch.randn(M, K, device=dev).to(torch.bfloat16)
            w = (torch.randn(N, K, device=dev) * 0.02).to(torch.bfloat16)
            wt = w.t().contiguous()
            xt = x.t().contiguous()
            cases = {
                "NT  x@w^T": lambda: F.linear(x, w),
                "NN  x@wt": lambda: torch.mm(x, wt),
                "sw  w@x^T": lambda: torch.mm(w, xt),
                "sw2 w@xT(view)": lambda: torch.mm(w, x.t()),
            }
            for cname, fn in cases.items():
                us = timeit(fn, iters=20)
                fl = 2 * M * N * K / (us * 1e-6) / 1e12
                print(f"layout M={M:4d} {name:8s} {cname:16s}: {us:8.1f} us {fl:7.1f} TF/s", flush=True)
    for n in (4096, 8192):
        a = torch.randn(n, n, device=dev).to(torch.bfloat16)
        b = torch.randn(n, n, device=dev).to(torch.bfloat16)
        us = timeit(lambda: torch.mm(a, b), iters=10)
        print(f"square {n}: {us:8.1f} us {2 * n ** 3 / (us * 1e-6) / 1e12:7.1f} TF/s", flush=True)


def attention(dev):
    from llm_weighted_consensus_amd import ops

    Hq, Hkv, D, BS = 32, 8, 128, 16
    for B, ctx_len in [(256, 320), (512, 320), (64, 2048), (8, 4096)]:
        nb = (ctx_len + BS - 1) // BS
        NB = B * nb + 8
        kc = torch.randn(NB, Hkv, BS, D, device=dev).to(torch.bfloat16)
        vc = torch.randn(NB, Hkv, D, BS, device=dev).to(torch.bfloat16)
        bt = torch.arange(B * nb, device=dev, dtype=torch.int32).view(B, nb)
        ctx = torch.full((B,), ctx_len, device=dev, dtype=torch.int32)
        q = torch.randn(B, (Hq + 2 * Hkv) * D, device=dev).to(torch.bfloat16)
        for splits in (1, 2, 4, 8):
            us = timeit(lambda: ops.paged_decode(q, kc, vc, bt, ctx, Hq, 1 / math.sqrt(D), num_splits=splits))
            gb = B * ctx_len * Hkv * D * 2 * 2 / (us * 1e-6) / 1e9
            print(f"paged_decode B={B:4d} ctx={ctx_len:5d} splits={splits}: {us:8.1f} us {gb:7.0f} GB/s", flush=True)


def sampler(dev):
    from llm_weighted_consensus_amd import ops

    V = 128256
    for B in (256, 512):
        logits = (torch.randn(B, V, device=dev) * 2).to(torch.bfloat16)
        f = lambda v: torch.full((B,), float(v), device=dev)
        seeds = torch.arange(B, device=dev, dtype=torch.int64)
        offs = torch.zeros(B, device=dev, dtype=torch.int64)
        tk = torch.zeros(B, dtype=torch.int32, device=dev)
        for label, tp, K, T in [("greedy", 1.0, 0, 0.0), ("temp", 1.0, 0, 0.8), ("top_p", 0.95, 0, 0.8),
                                ("top_p+lp20", 0.95, 20, 0.8)]:
            us = timeit(lambda: ops.sample(logits, f(T), f(tp), tk, f(0), f(0), seeds, offs, num_logprobs=K),
                        iters=20)
            print(f"sample B={B} {label:10s}: {us:8.1f} us  {B * V * 2 / (us * 1e-6) / 1e9:7.0f} GB/s", flush=True)


def small(dev):
    from llm_weighted_consensus_amd import ops

    for T in (256, 512):
        x = torch.randn(T, 4096, device=dev).to(torch.bfloat16)
        r = torch.randn(T, 4096, device=dev).to(torch.bfloat16)
        w = torch.ones(4096, device=dev, dtype=torch.bfloat16)
        us = timeit(lambda: ops.rmsnorm(x, w, 1e-5, residual=r))
        print(f"rmsnorm+res T={T}: {us:6.1f} us", flush=True)
        gu = torch.randn(T, 2 * 14336, device=dev).to(torch.bfloat16)
        us = timeit(lambda: ops.silu_mul(gu))
        print(f"silu_mul T={T}: {us:6.1f} us", flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("what", nargs="*", default=["gemm", "attn", "sample", "small"])
    a = ap.parse_args()
    dev = torch.device("cuda:0")
    if "gemm" in a.what:
        gemms(dev, [256, 512], tuned=os.environ.get("PYTORCH_TUNABLEOP_ENABLED") == "1")
    if "layout" in a.what:
        gemm_layouts(dev, [512, 1024])
    if "attn" in a.what:
        attention(dev)
    if "sample" in a.what:
        sampler(dev)
    if "small" in a.what:
        small(dev)


if __name__ == "__main__":
    main()
