#!/usr/bin/env python3
"""Probe of the block-scaled MFMA's A-scale mapping inside gemm8g's MX-A mode: A = ones, W = identity over
one 128-wide K slice, so out[r, k] = the scale the MFMA applied to A element (r, k).  Scale bytes are unique
per (row % 16, block); prints the measured byte grid for rows 0..31 at each 16-column chunk next to the
byte the kernel's layout assumes (block of 16-column chunk c = c // 2)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from llm_weighted_consensus_amd import ops

    dev = torch.device("cuda", 0)
    R, K, N = 256, 128, 128
    A = torch.ones(R, K, device=dev).to(torch.float8_e4m3fn)
    W = torch.eye(N, K, device=dev).to(torch.float8_e4m3fn).view(1, N, K)
    ws = torch.ones(1, N, device=dev)
    r = torch.arange(R, device=dev)
    mx = torch.empty(1, R, 4, dtype=torch.uint8, device=dev)
    for b in range(4):
        mx[0, :, b] = (100 + (r % 16) + 16 * b + 64 * ((r // 16) % 2)).to(torch.uint8)
    off = torch.tensor([0, R], dtype=torch.int32, device=dev)
    out = ops.grouped_gemm(A, W, off, w_scale=ws, a_mx=mx).float()
    meas = (torch.log2(out.clamp(min=1e-30)).round() + 127).long().cpu()
    exp = mx[0].long().cpu()
    blk = [c // 2 for c in range(8)]  # block b = K [32b, 32b + 32)
    bad = 0
    for row in range(32):
        got = [int(meas[row, 16 * c]) for c in range(8)]
        want = [int(exp[row, blk[c]]) for c in range(8)]
        uniform = all(int(meas[row, 16 * c + j]) == got[c] for c in range(8) for j in range(16))
        bad += got != want
        print(f"row {row:3d}: measured {got}  assumed {want}  chunk-uniform={uniform}")
    print("rows with a mismatch (of 32):", bad)


def probe_slices():
    """The same readout for each 128-wide K slice of K = 1024, two groups (the second starting at row 37):
    mismatching (row, chunk) counts per slice (0 everywhere = the scale tiles of later K tiles land right)."""
    from llm_weighted_consensus_amd import ops

    dev = torch.device("cuda", 0)
    R, K, N = 256, 1024, 128
    A = torch.ones(R, K, device=dev).to(torch.float8_e4m3fn)
    g = torch.Generator(device=dev).manual_seed(3)
    mx = torch.randint(110, 145, (K // 128, R, 4), dtype=torch.uint8, device=dev, generator=g)
    off = torch.tensor([0, 37, R], dtype=torch.int32, device=dev)
    ws = torch.ones(2, N, device=dev)
    for t in range(K // 128):
        W = torch.zeros(N, K, device=dev)
        W[torch.arange(N), 128 * t + torch.arange(N)] = 1.0
        Wq = W.to(torch.float8_e4m3fn).view(1, N, K).expand(2, N, K).contiguous()
        out = ops.grouped_gemm(A, Wq, off, w_scale=ws, a_mx=mx).float()
        meas = (torch.log2(out.clamp(min=1e-30)).round() + 127).long()
        want = mx[t].long()[:, torch.arange(N, device=dev) // 32]
        bad = (meas != want)
        print(f"slice {t}: mismatches {int(bad.sum())} of {bad.numel()}; rows with any: "
              f"{bad.any(1).nonzero().flatten()[:12].tolist()}", flush=True)


if __name__ == "__main__":
    main()
    probe_slices()
