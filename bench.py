#!/usr/bin/env python3
"""Headline benchmark: consensus answers/sec (whole node), N=64 candidates, Llama-3-8B sampler +
bge-large-en-v1.5 scorer (BASELINE.json "metric"; configs 3-4), synthetic prompts, random-init weights.

One consensus answer = one request fully served: prefill its prompt, sample N candidate completions
(top-p, fixed length), embed every candidate with the BGE encoder, cosine-consensus (MFMA GEMM +
row-reduce) and pick the answer.  A bench *step* serves R requests per GPU end-to-end.

Multi-GPU (torchrun, one rank per GPU, RCCL): candidate-parallel — the global batch is R*W requests and
the ranks form W/cp candidate-parallel groups of cp GPUs (cp = min(W, N/32) by default, so each GPU
keeps >= 32 candidates of a request and the cascade attention still shares each prompt across >= 32
sequences).  Group d serves R*cp requests; each of its ranks samples N/cp candidates of every one of
them (per-GPU decode batch stays R*N: weak scaling).  Each rank prefills only R of the group's prompts;
their KV blocks and last-token logits are all-gathered inside the group (C4) so no prompt is computed
twice; one all-gather of the candidate embeddings (C1) gives the group all N candidates of its
requests, then the consensus kernel runs.  Timed region: K steps bracketed by barrier + synchronize on
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
    ap.add_argument("--requests", type=int, default=None,
                    help="requests per GPU per step (R); default 4096 // N: a 4096-sequence decode batch per GPU "
                         "(R=64 at the headline's N=64, R=16 for config 4's N=256)")
    ap.add_argument("--candidates", type=int, default=64, help="candidates per request (N)")
    ap.add_argument("--prompt-len", type=int, default=256)
    ap.add_argument("--gen-len", type=int, default=128)
    ap.add_argument("--decoder", default="llama-3-8b")
    ap.add_argument("--encoder", default="bge-large-en-v1.5")
    ap.add_argument("--no-graphs", action="store_true")
    ap.add_argument("--no-prefix-sharing", action="store_true", help="disable the cascade prefix attention pass")
    ap.add_argument("--cp", type=int, default=0,
                    help="candidate-parallel degree (ranks sharing one request's candidates); 0 = auto: "
                         "min(world, candidates // 32) so every GPU keeps >= 32 candidates per request")
    ap.add_argument("--kv-fraction", type=float, default=0.5,
                    help="share of the free device memory the engine's paged KV cache takes")
    ap.add_argument("--profile-steps", action="store_true", help="print a per-phase breakdown")
    return ap.parse_args()


def main():
    a = parse()
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    from llm_weighted_consensus_amd.parallel import launch

    # `python bench.py --gpus N` without torchrun: this process only launches N ranks (never touches the GPU)
    rc = launch.maybe_self_launch(a.gpus, __file__)
    if rc is not None:
        sys.exit(rc)
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
    launch.check_world(a.gpus, W)
    dev = torch.device("cuda", info.local_rank)
    # multi-rank pre-flight (peer access matrix + a checked, timed RCCL all-gather): its result goes into the
    # JSON so a first multi-GPU number explains itself
    from llm_weighted_consensus_amd.parallel import preflight
    pre = preflight.maybe_run(dev)
    N = a.candidates
    R = a.requests or max(1, 4096 // N)
    cp = a.cp or max(1, min(W, N // 32))
    while W % cp or N % cp:
        cp -= 1
    n_local = N // cp
    G = R * W  # global requests per step (weak scaling: R per GPU)
    # ranks form W/cp candidate groups; group d serves requests [d*R*cp, (d+1)*R*cp), each of its cp ranks
    # samples n_local candidates of every one of them (per-GPU decode batch = R*N at any W)
    cgroup, gidx, crank = pdist.candidate_groups(cp)
    Rg = R * cp

    dcfg = decoder_config(a.decoder)
    ecfg = encoder_config(a.encoder)
    model = LlamaModel(dcfg, device=dev, seed=1234, max_position=a.prompt_len + a.gen_len + 64)
    encoder = BertEncoder(ecfg, device=dev, seed=4321)
    tok = ByteTokenizer(dcfg.vocab_size, dcfg.bos_token_id, dcfg.eos_token_id)
    max_len = a.prompt_len + a.gen_len + 16
    # LWC_SHARE_ONE_GPU=1 (multi-rank rehearsal on one GPU): the ranks size their caches from the same free
    # memory at the same time, so each takes its share of the fraction
    shared = os.environ.get("LWC_SHARE_ONE_GPU") == "1" and W > 1
    engine = LLMEngine(model, tok, max_batch=Rg * n_local, max_model_len=max_len, use_graphs=not a.no_graphs,
                       kv_memory_fraction=a.kv_fraction / W if shared else a.kv_fraction,
                       prefix_sharing=not a.no_prefix_sharing)
    scorer = EmbeddingConsensus(encoder, tau=0.05, max_tokens=512)
    gen = torch.Generator().manual_seed(99)

    defer = not a.profile_steps  # the per-phase breakdown needs the score phase synchronised
    last_cands = [None]

    def one_step(step_idx: int, prev=None):
        """Serve one step's requests.  The consensus of the step is returned DEFERRED (its answer indices
        still on the device): the host goes straight on to the next step's admission while the GPU runs
        the encoder, and ``prev`` (the previous step's result) is read back once that admission is queued."""
        # identical synthetic prompts on every rank (same generator)
        all_prompts = [torch.randint(0, dcfg.vocab_size, (a.prompt_len,), generator=gen).tolist() for _ in range(G)]
        prompts = all_prompts[gidx * Rg:(gidx + 1) * Rg]  # this candidate group's requests
        t0 = time.perf_counter()
        groups = []
        shared = None
        if cp > 1:
            # C4: prefill only this rank's R of the group's prompts, all-gather their KV blocks + last
            # logits inside the candidate group (RCCL)
            kv, lg, nbl = engine.export_prefill(prompts[crank * R:(crank + 1) * R])
            with pdist.comm_tag("C4"):
                shared = all_gather_prefills(kv, lg, nbl, group=cgroup)
        for gi, p in enumerate(prompts):
            sp = SamplingParams(temperature=0.8, top_p=0.95, max_tokens=a.gen_len, ignore_eos=True,
                                seed=(step_idx * 1000003 + gidx * Rg + gi) * 131 + crank)
            groups.append(engine.add_request(p, sp, n=n_local, prefilled=shared[gi] if shared else None))
        if prev is not None:
            prev.resolve()
        while engine.has_work():
            engine.step()
        t1 = time.perf_counter()
        cands = [[s.tokens for s in g.seqs] for g in groups]
        with pdist.comm_tag("C1"):
            res = scorer.score(cands, gather=cp > 1, group=cgroup, defer=defer)
        if not defer:
            torch.cuda.synchronize(dev)
        t2 = time.perf_counter()
        last_cands[0] = cands
        return res, t1 - t0, t2 - t1

    res = None
    for i in range(a.warmup):
        res = one_step(i, res)[0]
        if rank == 0:  # progress on stderr (stdout carries only the JSON result line)
            print(f"# warmup step {i + 1}/{a.warmup} done", file=sys.stderr, flush=True)
    if res is not None:
        res.resolve()
    torch.cuda.synchronize(dev)
    pdist.comm_report(reset=True)  # count the timed steps' collectives only
    pdist.barrier()
    torch.cuda.synchronize(dev)
    t_start = time.perf_counter()
    gen_t = score_t = 0.0
    res = None
    for i in range(a.steps):
        res, tg, ts = one_step(a.warmup + i, res)
        gen_t += tg
        score_t += ts
        if rank == 0:
            print(f"# timed step {i + 1}/{a.steps} done", file=sys.stderr, flush=True)
    if res is not None:
        res.resolve()  # every timed step's answers are on the host before the clock stops
    torch.cuda.synchronize(dev)
    pdist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t_start
    elapsed = pdist.max_over_ranks(elapsed, dev)
    comm_stats = pdist.comm_report(a.steps) if W > 1 else {}  # C1 / C4 bytes received + ms per step
    # self-check (untimed, after the clock stopped): the last step's first request re-scored from all of its
    # candidates on one device must match what the candidate-parallel path produced (C1 all-gather +
    # consensus); the verdict is a MIN over every rank, and a mismatch fails the run
    from llm_weighted_consensus_amd.embeddings.consensus import LAST_VERIFY, verify_sharded
    verified = True
    if res is not None and last_cands[0]:
        verified = verify_sharded(scorer, last_cands[0][0], res, group=cgroup if cp > 1 else None)
    answers = G * a.steps
    value = answers / elapsed
    emb_per_s = G * N * a.steps / elapsed
    seen = pdist.world_size_seen()  # collective: ranks that actually took part in an all-reduce
    # which kernels the decode step ran (the largest decode bucket: the step every request goes through) and
    # the engine's in-step A/B of whole captured steps behind that choice — on stderr in every run, and in
    # the JSON record
    Bdec = max(engine.buckets) if engine.buckets else 0
    plan = model.plan_summary(Bdec) if Bdec else {}
    step_ab = {k: (round(v, 3) if isinstance(v, float) else v) for k, v in engine.step_ab.get(Bdec, {}).items()}
    if rank == 0:
        print(f"# decode plan at batch {Bdec}: {plan}; step A/B (ms per decode step): {step_ab}", file=sys.stderr,
              flush=True)
    if a.profile_steps and rank == 0:
        print(f"# generate {gen_t / a.steps * 1e3:.1f} ms/step, score {score_t / a.steps * 1e3:.1f} ms/step, "
              f"decode steps {engine.stats['steps']}", file=sys.stderr)
        from llm_weighted_consensus_amd.ops import gemm_plan
        for k, v in gemm_plan.table().items():
            print(f"# gemm {k}: " + " ".join(f"{b}={t:.1f}us" if isinstance(t, float) else f"{b}={t}"
                                             for b, t in v.items()), file=sys.stderr)
    if rank == 0:
        out = {
            "metric": "consensus answers/sec (whole node) + embeddings/sec, N=64 Llama-3-8B@bge-large",
            "value": round(value, 4),
            "unit": "answers/s",
            "n_gpus": 1 if shared else W,
            "backend": info.backend or "none (single process)",
            "world_size": seen,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(elapsed / a.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16",
            "data": "synthetic prompts (random token ids), random-init weights",
            "embeddings_per_s": round(emb_per_s, 2),
            "verified": verified,
            "verify_detail": dict(LAST_VERIFY),
            "generated_tokens_per_s": round(G * N * a.gen_len * a.steps / elapsed, 1),
            "decode_plan": plan,
            "preflight": pre,
            "comm_per_step": comm_stats,
            "step_ab_ms": step_ab,
            "config": {
                "model": f"{a.decoder} sampler + {a.encoder} scorer",
                "global_batch": G,
                "candidates_per_request": N,
                "seq_len": a.prompt_len + a.gen_len,
                "prompt_len": a.prompt_len,
                "gen_len": a.gen_len,
                "sampling": "temperature 0.8, top_p 0.95",
                "parallelism": (f"cp{cp} x dp{W // cp}: candidate-parallel groups of {cp} GPUs (all-gather of prompt KV "
                                f"+ embeddings inside a group over {info.backend}), request-parallel across groups"
                                if W > 1 else "single GPU") + (" (ranks SHARE one GPU: a rehearsal of the "
                                                                "multi-rank path, not a multi-GPU number)"
                                                                if shared else ""),
            },
        }
        print(json.dumps(out), flush=True)
    pdist.shutdown()
    if not verified:
        print("# VERIFICATION FAILED: the sharded consensus differs from the single-device recomputation",
              file=sys.stderr, flush=True)
        sys.exit(3)


if __name__ == "__main__":
    main()
