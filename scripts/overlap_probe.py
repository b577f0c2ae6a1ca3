#!/usr/bin/env python3
"""Can the decode step's bandwidth-bound attention overlap its compute-bound GEMMs?  Splits the headline
decode batch (4096 sequences) into two halves and times, per half-batch: the cascade attention
(R=32 groups x 64 candidates), the gate|up GEMM (M=2048), both back to back on one stream, and both
on two streams, against the whole batch's attention + GEMM.  Prints microseconds per (attention + GEMM) pair.
Usage: overlap_probe.py [iters]"""
import math
import os
import sys

import numpy as np
import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_weighted_consensus_amd import ops  # noqa: E402
from llm_weighted_consensus_amd.engine.engine import cascade_table_size, cascade_tiles  # noqa: E402


def attention(R, dev):
    Hq, Hkv, D, BS, N, P, gen = 32, 8, 128, 16, 64, 16, 64
    B = R * N
    sblk = (gen + 1 + BS - 1) // BS
    NB = R * P + B * sblk + 8
    kc = torch.randn(NB, Hkv, BS, D, device=dev).to(torch.bfloat16)
    vc = torch.randn(NB, Hkv, BS // 4, D, 4, device=dev).to(torch.bfloat16)
    q = torch.randn(B, (Hq + 2 * Hkv) * D, device=dev).to(torch.bfloat16)
    per_t = ops.cascade_rows_per_tile(Hq // Hkv)
    ct = np.zeros((cascade_table_size(B, per_t), 3), dtype=np.int32)
    bt = torch.zeros(B, P + sblk, dtype=torch.int32)
    for r in range(R):
        bt[r * N:(r + 1) * N, :P] = torch.arange(r * P, (r + 1) * P, dtype=torch.int32)
    bt[:, P:] = (R * P + torch.arange(B * sblk, dtype=torch.int32)).view(B, sblk)
    bt = bt.to(dev)
    ctx = torch.full((B,), P * BS + gen + 1, device=dev, dtype=torch.int32)
    cascade_tiles([(r * N, N, P) for r in range(R)], per_t, ct)
    ct = torch.from_numpy(ct).to(dev)
    sc = 1 / math.sqrt(D)
    return lambda: ops.paged_decode_cascade(q, kc, vc, bt, ctx, ct, Hq, sc)


def gemm(M, w, dev):
    x = torch.randn(M, w.shape[1], device=dev).to(torch.bfloat16)
    return lambda: F.linear(x, w)


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(3):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e) * 1e3 / iters)
    return sorted(ts)[1]


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    dev = torch.device("cuda")
    torch.manual_seed(0)
    w = (torch.randn(28672, 4096, device=dev) / 64).to(torch.bfloat16)
    a_full, a0, a1 = attention(64, dev), attention(32, dev), attention(32, dev)
    g_full, g0, g1 = gemm(4096, w, dev), gemm(2048, w, dev), gemm(2048, w, dev)
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    cur = torch.cuda.current_stream()

    def two_streams():
        # half 0's GEMM runs beside half 1's attention, then half 1's GEMM beside half 0's attention
        s1.wait_stream(cur)
        s2.wait_stream(cur)
        with torch.cuda.stream(s1):
            a1()
            g1()
        with torch.cuda.stream(s2):
            g0()
            a0()
        cur.wait_stream(s1)
        cur.wait_stream(s2)

    rows = {
        "attention B=4096": a_full,
        "gate_up M=4096": g_full,
        "whole batch: attention + gate_up, one stream": lambda: (a_full(), g_full()),
        "attention B=2048": a0,
        "gate_up M=2048": g0,
        "two halves, one stream": lambda: (a0(), g0(), a1(), g1()),
        "two halves, two streams (eager)": two_streams,
    }
    for name, fn in rows.items():
        print(f"{name:48s} {timed(fn, iters):9.1f} us", flush=True)


if __name__ == "__main__":
    main()
