#!/usr/bin/env python3
"""hipBLASLt default heuristic vs PyTorch TunableOp (exhaustive hipBLASLt/rocBLAS solution search) on the
projection shapes the headline bench runs through ``F.linear``.

    python scripts/tunableop_probe.py [results.csv] [M,M,...|all]

Phase 1 times every shape with TunableOp off (torch's default hipBLASLt heuristic), phase 2 enables
tuning (results written to the CSV), phase 3 re-times with the tuned solutions.
"""
import sys
import time

import torch
import torch.nn.functional as F

PROJ = [(4096, 4096), (4096, 14336), (128256, 4096), (6144, 4096), (28672, 4096)]  # o, down, lm_head, qkv, gate_up
OTHER = [(12288, 6144, 4096), (12288, 4096, 4096), (12288, 28672, 4096), (12288, 4096, 14336),  # prefill 48 x 256
         (393216, 3072, 1024), (393216, 1024, 1024), (393216, 4096, 1024), (393216, 1024, 4096)]  # bge-large encode


def timeit(fn, iters=10, rounds=3):
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(rounds):
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record()
        for _ in range(iters):
            fn()
        e.record()
        torch.cuda.synchronize()
        ts.append(s.elapsed_time(e) / iters * 1e3)
    return sorted(ts)[len(ts) // 2]


def main():
    out = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/tunableop_results.csv"
    arg = sys.argv[2] if len(sys.argv) > 2 else "3072,4096"
    Ms = [3072, 4096] if arg == "all" else [int(m) for m in arg.split(",")]
    shapes = [(M, N, K) for M in Ms for N, K in PROJ] + (OTHER if arg == "all" else [])
    dev = torch.device("cuda:0")
    tun = torch.cuda.tunable
    ops = []
    for M, N, K in shapes:
        x = (torch.rand(M, K, device=dev) * 2 - 1).to(torch.bfloat16)
        w = ((torch.rand(N, K, device=dev) * 2 - 1) / K ** 0.5).to(torch.bfloat16)
        ops.append(((M, N, K), x, w))
    base = {}
    for shp, x, w in ops:
        base[shp] = timeit(lambda: F.linear(x, w))
        print(f"default {shp}: {base[shp]:.1f} us", flush=True)
    tun.enable(True)
    tun.tuning_enable(True)
    tun.set_filename(out)
    for shp, x, w in ops:
        t0 = time.time()
        F.linear(x, w)
        torch.cuda.synchronize()
        print(f"tuned {shp} in {time.time() - t0:.1f} s", flush=True)
    tun.tuning_enable(False)  # the results file is written at exit
    for shp, x, w in ops:
        t = timeit(lambda: F.linear(x, w))
        M, N, K = shp
        print(f"tunableop {shp}: {t:.1f} us ({2 * M * N * K / t / 1e6:.0f} TF/s) vs default {base[shp]:.1f} us "
              f"({base[shp] / t:.3f}x)", flush=True)


if __name__ == "__main__":
    main()
