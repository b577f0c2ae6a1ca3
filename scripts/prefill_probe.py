#!/usr/bin/env python3
"""Prefill cost vs token count (Llama-3-8B, random init): fixed per-call cost vs per-token cost, with and
without the cached-prefix key-range path (ctx), through the engine's _run_chunk."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from llm_weighted_consensus_amd.engine.engine import LLMEngine
    from llm_weighted_consensus_amd.engine.tokenizer import ByteTokenizer
    from llm_weighted_consensus_amd.models.config import decoder_config
    from llm_weighted_consensus_amd.models.llama import LlamaModel
    from llm_weighted_consensus_amd.utils.tracing import STATS  # noqa: F401

    dev = torch.device("cuda", 0)
    m = LlamaModel(decoder_config(os.environ.get("ARCH", "llama-3-8b")), device=dev, seed=0, max_position=4096)
    tok = ByteTokenizer(m.cfg.vocab_size)
    eng = LLMEngine(m, tok, max_batch=64, max_model_len=4096, kv_memory_fraction=0.3)
    g = torch.Generator().manual_seed(0)

    class G:  # a stand-in group: the probe drives _run_chunk directly
        _n = 0

        def __init__(self, L):
            G._n += 1
            self.id = 10_000 + G._n
            self.prompt_ids = torch.randint(0, 100000, (L,), generator=g).tolist()

    for total, per, start in [(256, 256, 0), (512, 512, 0), (1024, 1024, 0), (2048, 2048, 0), (4096, 512, 0),
                              (384, 48, 0), (384, 48, 300), (2048, 256, 300)]:
        n = total // per
        groups = [G(start + per) for _ in range(n)]
        for gr in groups:
            eng.bm.add_sequence(-gr.id, len(gr.prompt_ids))
        items = [(gr, start, start + per) for gr in groups]
        if start:
            eng._run_chunk([(gr, 0, start) for gr in groups])
        eng._run_chunk(items)
        torch.cuda.synchronize()
        ts = []
        for _ in range(5):
            t = time.perf_counter()
            eng._run_chunk(items)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t)
        ts.sort()
        print(f"prefill {n} x {per} tokens (cached head {start}): {ts[2] * 1e3:7.2f} ms  "
              f"{total / ts[2] / 1e3:7.1f} k tok/s", flush=True)
        for gr in groups:
            eng.bm.free_sequence(-gr.id)


if __name__ == "__main__":
    main()
