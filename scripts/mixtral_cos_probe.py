#!/usr/bin/env python3
"""Prefill logits of mixtral-tiny (bf16 and fp8 experts) vs the fp32 reference: the cosine the model test
bounds (tests/test_model_gpu.py::test_mixtral_moe_matches_reference_and_engine), for several seeds."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from llm_weighted_consensus_amd.models.config import decoder_config
    from llm_weighted_consensus_amd.models.llama import KVCache
    from llm_weighted_consensus_amd.models.mixtral import MixtralModel
    from tests import torch_ref as ref

    gpu = torch.device("cuda", 0)
    for fp8 in (False, True):
        for seed in (2, 3, 4):
            m = MixtralModel(decoder_config("mixtral-tiny"), device=gpu, seed=seed, max_position=1024, fp8=fp8)
            g = torch.Generator(device="cpu").manual_seed(1)
            P = 37
            toks = torch.randint(0, m.cfg.vocab_size, (P,), generator=g).to(gpu)
            r = ref.llama_forward(m, toks)
            cache = KVCache(m.cfg, 16, 16, gpu)
            ar = torch.arange(P, dtype=torch.int32, device=gpu)
            lg = m.prefill(toks.int(), ar, ar, torch.tensor([0, P], dtype=torch.int32, device=gpu), P,
                           torch.tensor([P - 1], device=gpu), cache)
            c = torch.nn.functional.cosine_similarity(lg[0].float(), r[P - 1].float(), dim=0).item()
            print(f"fp8={fp8} seed={seed}: cos {c:.5f}", flush=True)


if __name__ == "__main__":
    main()
