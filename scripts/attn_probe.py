#!/usr/bin/env python3
"""Launch the bench's cascade decode attention (R groups x N candidates, 256-token shared prompt, `gen`
generated tokens each) `iters` times — a short, single-kernel program for rocprofv3 --pmc passes.
Usage: attn_probe.py [R] [iters] [mode: full | suffix]"""
import math
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_weighted_consensus_amd import ops  # noqa: E402
from llm_weighted_consensus_amd.engine.engine import cascade_table_size, cascade_tiles  # noqa: E402


def main():
    R = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    mode = sys.argv[3] if len(sys.argv) > 3 else "full"
    dev = torch.device("cuda")
    Hq, Hkv, D, BS, N, P, gen = 32, 8, 128, 16, 64, 16, 64
    B = R * N
    sblk = (gen + 1 + BS - 1) // BS
    NB = R * P + B * sblk + 8
    kc = torch.randn(NB, Hkv, BS, D, device=dev).to(torch.bfloat16)
    vc = torch.randn(NB, Hkv, BS // 4, D, 4, device=dev).to(torch.bfloat16)
    q = torch.randn(B, (Hq + 2 * Hkv) * D, device=dev).to(torch.bfloat16)
    per_t = ops.cascade_rows_per_tile(Hq // Hkv)
    ct = np.zeros((cascade_table_size(B, per_t), 3), dtype=np.int32)
    if mode == "suffix":  # each sequence's own blocks only (no shared prompt)
        bt = (R * P + torch.arange(B * sblk, dtype=torch.int32)).view(B, sblk).to(dev)
        ctx = torch.full((B,), gen + 1, device=dev, dtype=torch.int32)
        cascade_tiles([(0, B, 0)], per_t, ct)
    else:
        bt = torch.zeros(B, P + sblk, dtype=torch.int32)
        for r in range(R):
            bt[r * N:(r + 1) * N, :P] = torch.arange(r * P, (r + 1) * P, dtype=torch.int32)
        bt[:, P:] = (R * P + torch.arange(B * sblk, dtype=torch.int32)).view(B, sblk)
        bt = bt.to(dev)
        ctx = torch.full((B,), P * BS + gen + 1, device=dev, dtype=torch.int32)
        cascade_tiles([(r * N, N, P) for r in range(R)], per_t, ct)
    ct = torch.from_numpy(ct).to(dev)
    sc = 1 / math.sqrt(D)
    for _ in range(iters):
        ops.paged_decode_cascade(q, kc, vc, bt, ctx, ct, Hq, sc)
    torch.cuda.synchronize()
    print("ok", flush=True)


if __name__ == "__main__":
    main()
