#!/usr/bin/env python3
"""PMC probe: the fp8 MoE gate_up grouped GEMM at a decode batch (T tokens x top-2, balanced), N launches."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from llm_weighted_consensus_amd import ops

    T = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    n = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    dev = torch.device("cuda:0")
    E, d, f = 8, 4096, 14336
    g = torch.Generator(device=dev).manual_seed(0)
    q13, s13 = ops.quant_fp8_weight((torch.randn(E, 2 * f, d, device=dev, generator=g) * 0.02).to(torch.bfloat16))
    rows = 2 * T
    off = torch.arange(0, rows + 1, rows // E, dtype=torch.int32, device=dev)
    hq, hs = ops.quant_fp8_rows(torch.randn(rows, d, device=dev, generator=g).to(torch.bfloat16))
    for _ in range(n):
        ops.grouped_gemm(hq, q13, off, a_scale=hs, w_scale=s13)
    torch.cuda.synchronize()
    print("done")


if __name__ == "__main__":
    main()
