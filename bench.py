#!/usr/bin/env python3
"""Headline benchmark: consensus answers/sec (whole node), N=64 candidates, Llama-3-8B sampler +
bge-large-en-v1.5 scorer (BASELINE.json "metric"; configs 3-4), synthetic prompts, random-init weights.

One consensus answer = one request fully served: prefill its prompt, sample N candidate completions
(top-p, fixed length), embed every candidate with the BGE encoder, cosine-consensus (MFMA GEMM +
row-reduce) and pick the answer.  A bench *step* serves R requests per GPU end-to-end.

Multi-GPU (torchrun, one rank per GPU, RCCL): candidate-parallel — the global batch is R*W requests and
rank r samples candidates [r*N/W, (r+1)*N/W) of EVERY request (per-GPU decode batch stays R*N: weak
scaling).  Each rank prefills only its own R prompts; their KV blocks and last-token logits are
all-gathered (C4) so no prompt is computed twice; one all-gather of the candidate embeddings (C1)
gives every rank all N candidates of every request, then the consensus kernel runs.  Timed region: K steps bracketed by barrier + synchronize on
both sides; the reported time is the max over ranks.

    python bench.py --gpus N --steps K --warmup W
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--requests", type=int, default=48, help="requests per GPU per step (R)")
    ap.add_argument("--candidates", type=int, default=64, help="candidates per request (N)")
    ap.add_argument("--prompt-len", type=int, default=256)
    ap.add_argument("--gen-len", type=int, default=128)
    ap.add_argument("--decoder", default="llama-3-8b")
    ap.add_argument("--encoder", default="bge-large-en-v1.5")
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--no-prefix-sharing", action="store_true", help="disable the cascade prefix attention pass")
    ap.add_argument("--profile-steps", action="store_true", help="print a per-phase breakdown")
    return ap.parse_args()


def main():
    a = parse()
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from llm_weighted_consensus_amd.embeddings.consensus import EmbeddingConsensus
    from llm_weighted_consensus_amd.engine.engine import LLMEngine
    from llm_weighted_consensus_amd.engine.sampling import SamplingParams
    from llm_weighted_consensus_amd.engine.tokenizer import ByteTokenizer
    from llm_weighted_consensus_amd.models.bert import BertEncoder
    from llm_weighted_consensus_amd.models.config import decoder_config, encoder_config
    from llm_weighted_consensus_amd.models.llama import LlamaModel
    from llm_weighted_consensus_amd.parallel import dist as pdist
    from llm_weighted_consensus_amd.parallel.prefill_share import all_gather_prefills

    info = pdist.init_from_env("cuda")
    W, rank = info.world, info.rank
    if W != a.gpus:
        print(f"warning: --gpus {a.gpus} but WORLD_SIZE {W}", file=sys.stderr)
    dev = torch.device("cuda", info.local_rank)
    N, R = a.candidates, a.requests
    assert N % W == 0, "candidates must divide across ranks"
    n_local = N // W
    G = R * W  # global requests per step

    dcfg = decoder_config(a.decoder)
    ecfg = encoder_config(a.encoder)
    model = LlamaModel(dcfg, device=dev, seed=1234, max_position=a.prompt_len + a.gen_len + 64)
    encoder = BertEncoder(ecfg, device=dev, seed=4321)
    tok = ByteTokenizer(dcfg.vocab_size, dcfg.bos_token_id, dcfg.eos_token_id)
    max_len = a.prompt_len + a.gen_len + 16
    engine = LLMEngine(model, tok, max_batch=G * n_local, max_model_len=max_len, use_graphs=not a.no_graphs,
                       kv_memory_fraction=0.5, prefix_sharing=not a.no_prefix_sharing)
    scorer = EmbeddingConsensus(encoder, tau=0.05, max_tokens=512)
    gen = torch.Generator().manual_seed(99)

    def one_step(step_idx: int):
        # identical synthetic prompts on every rank (same generator)
        prompts = [torch.randint(0, dcfg.vocab_size, (a.prompt_len,), generator=gen).tolist() for _ in range(G)]
        t0 = time.perf_counter()
        groups = []
        shared = None
        if W > 1:
            # C4: prefill only this rank's R prompts, all-gather their KV blocks + last logits (RCCL)
            kv, lg, nbl = engine.export_prefill(prompts[rank * R:(rank + 1) * R])
            shared = all_gather_prefills(kv, lg, nbl)
        for gi, p in enumerate(prompts):
            sp = SamplingParams(temperature=0.8, top_p=0.95, max_tokens=a.gen_len, ignore_eos=True,
                                seed=(step_idx * 1000003 + gi) * 131 + rank)
            groups.append(engine.add_request(p, sp, n=n_local, prefilled=shared[gi] if shared else None))
        while engine.has_work():
            engine.step()
        t1 = time.perf_counter()
        cands = [[s.tokens for s in g.seqs] for g in groups]
        res = scorer.score(cands, gather=W > 1)
        torch.cuda.synchronize(dev)
        t2 = time.perf_counter()
        return res, t1 - t0, t2 - t1

    for i in range(a.warmup):
        one_step(i)
    torch.cuda.synchronize(dev)
    pdist.barrier()
    torch.cuda.synchronize(dev)
    t_start = time.perf_counter()
    gen_t = score_t = 0.0
    for i in range(a.steps):
        res, tg, ts = one_step(a.warmup + i)
        gen_t += tg
        score_t += ts
    torch.cuda.synchronize(dev)
    pdist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t_start
    elapsed = pdist.max_over_ranks(elapsed, dev)
    answers = G * a.steps
    value = answers / elapsed
    emb_per_s = G * N * a.steps / elapsed
    if a.profile_steps and rank == 0:
        print(f"# generate {gen_t / a.steps * 1e3:.1f} ms/step, score {score_t / a.steps * 1e3:.1f} ms/step, "
              f"decode steps {engine.stats['steps']}", file=sys.stderr)
    if rank == 0:
        out = {
            "metric": "consensus answers/sec (whole node) + embeddings/sec, N=64 Llama-3-8B@bge-large",
            "value": round(value, 4),
            "unit": "answers/s",
            "n_gpus": W,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(elapsed / a.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic prompts (random token ids), random-init weights",
            "embeddings_per_s": round(emb_per_s, 2),
            "generated_tokens_per_s": round(G * N * a.gen_len * a.steps / elapsed, 1),
            "config": {
                "model": f"{a.decoder} sampler + {a.encoder} scorer",
                "global_batch": G,
                "candidates_per_request": N,
                "seq_len": a.prompt_len + a.gen_len,
                "prompt_len": a.prompt_len,
                "gen_len": a.gen_len,
                "sampling": "temperature 0.8, top_p 0.95",
                "parallelism": (f"candidate-parallel cp{W} (RCCL all-gather of prompt KV + embeddings)" if W > 1
                                else "single GPU"),
            },
        }
        print(json.dumps(out), flush=True)
    pdist.shutdown()


if __name__ == "__main__":
    main()
