#!/usr/bin/env python3
"""The decode sampler at the bench's batch (4096 rows x 128256 vocabulary, temperature 0.8, top-p 0.95, no
logprobs), `iters` launches — a short single-kernel program for rocprofv3 passes and quick timing.
Usage: sample_probe.py [B] [iters]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from llm_weighted_consensus_amd import ops  # noqa: E402


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    dev = torch.device("cuda")
    V = 128256
    logits = (torch.randn(B, V, device=dev) * 3).to(torch.bfloat16)
    f = lambda v: torch.full((B,), v, dtype=torch.float32, device=dev)  # noqa: E731
    args = dict(temperature=f(0.8), top_p=f(0.95), top_k=torch.zeros(B, dtype=torch.int32, device=dev), min_p=f(0.0),
                top_a=f(0.0), seeds=torch.arange(B, dtype=torch.int64, device=dev),
                offsets=torch.zeros(B, dtype=torch.int64, device=dev), need_logprob=False)
    ops.sample(logits, **args)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        ops.sample(logits, **args)
    e.record()
    torch.cuda.synchronize()
    us = s.elapsed_time(e) / iters * 1e3
    print(f"sample B={B} V={V}: {us:.1f} us ({B * V * 2 / us / 1e6:.2f} TB/s of bf16 logits)", flush=True)


if __name__ == "__main__":
    main()
