#!/usr/bin/env python3
"""Dense fp8 (e4m3, row-wise scales) GEMM options on gfx950 vs bf16 hipBLASLt: torch._scaled_mm (hipBLASLt
fp8), the hand-written block-scaled grouped GEMM at G=1 (csrc/kernels/gemm.hip), random operands."""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def timeit(fn, iters=10):
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
        ts.append(s.elapsed_time(e) / iters * 1e3)
    return sorted(ts)[1]


def main():
    from llm_weighted_consensus_amd import ops

    dev = torch.device("cuda", 0)
    for M, N, K in [(65536, 6144, 4096), (65536, 4096, 4096), (65536, 28672, 4096), (65536, 4096, 14336),
                    (4096, 6144, 4096), (2048, 4096, 4096)]:
        x = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
        w = ((torch.rand(N, K, device=dev) * 2 - 1) / K ** 0.5).to(torch.bfloat16)
        fl = 2 * M * N * K / 1e12
        t_bf = timeit(lambda: F.linear(x, w))
        xq, xs = ops.quant_fp8_rows(x)
        wq3, ws3 = ops.quant_fp8_weight(w.unsqueeze(0))
        wq, ws = wq3[0], ws3[0]
        line = f"M={M:6d} N={N:6d} K={K:6d}: bf16 {t_bf:8.1f} us ({fl / t_bf * 1e6:5.0f} TF)"
        try:
            sa = xs.view(M, 1).float()
            sb = ws.view(1, N).float()
            f = lambda: torch._scaled_mm(xq, wq.t(), scale_a=sa, scale_b=sb, out_dtype=torch.bfloat16)  # noqa
            ref = F.linear(x.float(), w.float())
            err = ((f().float() - ref).norm() / ref.norm()).item()
            t = timeit(f)
            line += f"  _scaled_mm {t:8.1f} us ({fl / t * 1e6:5.0f} TF, rel err {err:.3g})"
        except Exception as e:  # noqa: BLE001
            line += f"  _scaled_mm n/a ({str(e)[:80]})"
        off = torch.tensor([0, M], dtype=torch.int32, device=dev)
        g = lambda: ops.grouped_gemm(xq, wq3, off, a_scale=xs, w_scale=ws3)  # noqa: E731
        t = timeit(g)
        line += f"  grouped-fp8 {t:8.1f} us ({fl / t * 1e6:5.0f} TF)"
        tq = timeit(lambda: ops.quant_fp8_rows(x))
        line += f"  act-quant {tq:6.1f} us"
        print(line, flush=True)


if __name__ == "__main__":
    main()
