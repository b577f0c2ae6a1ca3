#!/usr/bin/env python3
"""Benchmarks for the other BASELINE.json configs (the headline config is bench.py):

  encoder  config 2: bge-base-en-v1.5 bf16 on 1 MI355X, 64-candidate batches -> embeddings/s (+ the
           cosine-consensus GEMM per batch)
  moe      config 5: Mixtral-8x7B sampler (fp8 experts by default) + e5-mistral-7b embedder, N candidates
           per request, embedding consensus -> answers/s.  `--tp 2` self-launches 2 ranks (or run it under
           torchrun) for the TP=2 layout (heads and expert FFN split, RCCL all-reduce per row-parallel projection)

(config 1 is the CPU plumbing test tests/test_server.py::test_config1_cpu_...; config 3 is
`bench.py --candidates 32`; config 4 is `bench.py` under torchrun.)  Synthetic token ids and
random-init weights; timing brackets the steps with synchronize (+ barrier under torchrun); one JSON
line per run on rank 0.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import torch


def _sync(dev, dist_on):
    torch.cuda.synchronize(dev)
    if dist_on:
        from llm_weighted_consensus_amd.parallel import dist as pdist

        pdist.barrier()
        torch.cuda.synchronize(dev)


def bench_encoder(a):
    from llm_weighted_consensus_amd.embeddings.consensus import EmbeddingConsensus
    from llm_weighted_consensus_amd.models.bert import BertEncoder
    from llm_weighted_consensus_amd.models.config import encoder_config

    dev = torch.device("cuda", 0)
    enc = BertEncoder(encoder_config(a.encoder), device=dev, seed=1)
    scorer = EmbeddingConsensus(enc, tau=0.05, max_tokens=512)
    g = torch.Generator().manual_seed(0)
    R, N, L = a.requests, a.candidates, a.seq_len
    reqs = [[torch.randint(1000, 30000, (L,), generator=g).tolist() for _ in range(N)] for _ in range(R)]
    for _ in range(a.warmup):
        scorer.score(reqs)
    _sync(dev, False)
    t0 = time.perf_counter()
    for _ in range(a.steps):
        res = scorer.score(reqs)
    _sync(dev, False)
    dt = (time.perf_counter() - t0) / a.steps
    return {"metric": "embeddings/sec (config 2: bge-base bf16, 64-candidate cosine consensus)",
            "value": round(R * N / dt, 1), "unit": "embeddings/s", "n_gpus": 1, "steps": a.steps,
            "warmup": a.warmup, "ms_per_step": round(dt * 1e3, 3), "higher_is_better": True, "dtype": "bf16",
            "data": "synthetic token ids, random-init weights", "best_of_first_request": int(res.best[0]),
            "config": {"model": a.encoder, "global_batch": R, "candidates_per_request": N, "seq_len": L}}


def bench_moe(a):
    from llm_weighted_consensus_amd.embeddings.consensus import EmbeddingConsensus
    from llm_weighted_consensus_amd.engine.engine import LLMEngine
    from llm_weighted_consensus_amd.engine.sampling import SamplingParams
    from llm_weighted_consensus_amd.engine.tokenizer import ByteTokenizer
    from llm_weighted_consensus_amd.models.config import decoder_config
    from llm_weighted_consensus_amd.models.embedder import DecoderEmbedder
    from llm_weighted_consensus_amd.models.llama import LlamaModel
    from llm_weighted_consensus_amd.models.mixtral import MixtralModel
    from llm_weighted_consensus_amd.models.tp import TPLlamaModel
    from llm_weighted_consensus_amd.parallel import dist as pdist

    info = pdist.init_from_env("cuda")
    # config 5 layout: TP groups of `tp` consecutive ranks (IPC all-reduce inside each), DP across groups
    # (each group serves its own requests): `--tp 2` on 8 GPUs = 4 x TP2
    tp = a.tp if info.world > 1 else 1
    if info.world % tp:
        raise SystemExit(f"--tp {a.tp} must divide the world size {info.world}")
    dp = info.world // tp
    tp_group, dp_idx, tp_rank = pdist.candidate_groups(tp) if info.world > 1 else (None, 0, 0)
    dev = torch.device("cuda", info.local_rank)
    dcfg = decoder_config(a.decoder)
    # multi-rank pre-flight (peer access matrix, a checked RCCL all-gather, the IPC self-test when the TP
    # all-reduce is to run over IPC): a failed peer check runs the TP all-reduce on the process group instead,
    # with the reason in the JSON
    from llm_weighted_consensus_amd.parallel import preflight
    pre = preflight.maybe_run(dev, want_ipc=tp > 1 and a.tp_comm == "ipc")
    tp_comm = a.tp_comm
    if pre is not None and pre["ipc_fallback"]:
        tp_comm = "pg"
        if info.rank == 0:
            print(f"# pre-flight: {pre['ipc']} -> TP all-reduce on the process group", file=sys.stderr, flush=True)
    comm = None
    if tp > 1 and tp_comm == "ipc":
        from llm_weighted_consensus_amd.parallel.allreduce import CustomAllReduce

        # C3 over IPC peer buffers: [decode batch, hidden] bf16 per call, inside the captured decode graph
        comm = CustomAllReduce(group=tp_group, device=dev, max_bytes=a.requests * a.candidates * dcfg.hidden * 2)
    model = MixtralModel(dcfg, device=dev, seed=11, max_position=a.prompt_len + a.gen_len + 64, fp8=not a.bf16,
                         tp_rank=tp_rank, tp_size=tp, tp_group=tp_group, tp_comm=comm)
    # config 5 is fp8 throughout: the embedder's projections too (e4m3 + per-channel scales, fp8 library GEMM).
    # --embedder-par tp (config 5's "TP=2 each"): the embedder's heads / FFN columns split over the TP group
    # like the sampler's, every rank embeds all N candidates, its two all-reduces per layer go through the
    # process group (RCCL; [tokens, d] is GBs per call, beyond the IPC buffer).  dp: each rank holds the whole
    # embedder and embeds 1/tp of the candidates, one all-gather assembles them — same FLOPs, no per-layer
    # collective.
    emb_tp = tp if a.embedder_par == "tp" else 1
    emb_model = TPLlamaModel(decoder_config(a.embedder), device=dev, seed=12, max_position=a.gen_len + 64,
                             fp8_dense=not a.bf16, tp_rank=tp_rank if emb_tp > 1 else 0, tp_size=emb_tp,
                             tp_group=tp_group)
    scorer = EmbeddingConsensus(DecoderEmbedder(emb_model, max_tokens=a.gen_len + 16), tau=0.05)
    tok = ByteTokenizer(dcfg.vocab_size, dcfg.bos_token_id, dcfg.eos_token_id)
    R, N = a.requests, a.candidates
    if N % tp:
        raise SystemExit(f"--candidates {N} must be a multiple of --tp {tp}")
    shared = os.environ.get("LWC_SHARE_ONE_GPU") == "1" and info.world > 1
    # ranks sharing one GPU size their caches concurrently from the same free memory: split the fraction
    engine = LLMEngine(model, tok, max_batch=R * N, max_model_len=a.prompt_len + a.gen_len + 16,
                       kv_memory_fraction=0.4 / info.world if shared else 0.4, use_graphs=model.graph_safe)
    g = torch.Generator().manual_seed(5 + dp_idx)  # each DP group its own prompts

    def step(i):
        groups = []
        for r in range(R):
            p = torch.randint(0, dcfg.vocab_size, (a.prompt_len,), generator=g).tolist()
            sp = SamplingParams(temperature=0.8, top_p=0.95, max_tokens=a.gen_len, ignore_eos=True,
                                seed=(i * 977 + r) * 131 + dp_idx)
            groups.append(engine.add_request(p, sp, n=N))
        while engine.has_work():
            engine.step()
        # the TP ranks hold the same candidates.  dp embedder: each embeds its 1/tp share, one all-gather (C1)
        # inside the TP group assembles all N per request; tp embedder: each embeds all N with its weight
        # shard.  Both ranks then run the (tiny) consensus
        if emb_tp > 1 or tp == 1:
            last[0] = [[s.tokens for s in gr.seqs] for gr in groups]
            return scorer.score(last[0])
        n_loc = N // tp
        last[0] = [[s.tokens for s in gr.seqs[tp_rank * n_loc:(tp_rank + 1) * n_loc]] for gr in groups]
        with pdist.comm_tag("C1"):
            return scorer.score(last[0], gather=True, group=tp_group)

    last = [None]

    for i in range(a.warmup):
        step(i)
    _sync(dev, info.enabled)
    pdist.comm_report(reset=True)  # count the timed steps' collectives only
    t0 = time.perf_counter()
    res = None
    for i in range(a.steps):
        res = step(a.warmup + i)
    _sync(dev, info.enabled)
    dt = pdist.max_over_ranks((time.perf_counter() - t0) / a.steps, dev)
    comm_stats = pdist.comm_report(a.steps) if info.world > 1 else {}
    if comm is not None:
        comm.check()
    # untimed self-check: the last step's first request re-scored from all of its candidates on one device
    # (a MIN over every rank; a mismatch fails the run, see bench.py)
    from llm_weighted_consensus_amd.embeddings.consensus import LAST_VERIFY, verify_sharded
    gathered = not (emb_tp > 1 or tp == 1)
    # the TP embedder's per-layer all-reduces: 2 per layer of [tokens, d] bf16 over the process group
    ecfg = decoder_config(a.embedder)
    emb_tokens = R * N * (a.gen_len + 1)
    # (the re-embedding takes the fp8 dense-MLP path the batch took: MX from DENSE_MX_MIN_ROWS rows on)
    from llm_weighted_consensus_amd import ops as _ops
    batch_rows = emb_tokens // (tp if gathered else 1)
    with _ops.dense_mx_min_rows(0 if batch_rows >= _ops.DENSE_MX_MIN_ROWS else _ops.DENSE_MX_MIN_ROWS):
        verified = verify_sharded(scorer, last[0][0], res, group=tp_group if gathered else None)
    ar_bytes = 2 * ecfg.layers * emb_tokens * ecfg.hidden * 2 if emb_tp > 1 else 0
    return {"metric": "consensus answers/sec (config 5: Mixtral-8x7B sampler + e5-mistral-7b embedder)",
            "value": round(dp * R / dt, 4), "unit": "answers/s", "n_gpus": 1 if shared else info.world,
            "steps": a.steps, "warmup": a.warmup, "ms_per_step": round(dt * 1e3, 3), "higher_is_better": True,
            "scaling": "weak",
            "dtype": ("fp8 e4m3 weights (experts, attention projections, embedder projections; per-channel scales) "
                      "x row-quantised e4m3 activations, bf16 elsewhere") if not a.bf16 else "bf16",
            "data": "synthetic prompts (random token ids), random-init weights",
            "generated_tokens_per_s": round(dp * R * N * a.gen_len / dt, 1),
            "verified": verified,
            "verify_detail": dict(LAST_VERIFY),
            "embedder_allreduce_bytes_per_step": ar_bytes,
            "world_size": pdist.world_size_seen(),
            "preflight": pre,
            "comm_per_step": comm_stats,
            "config": {"model": f"{a.decoder} + {a.embedder}", "global_batch": dp * R, "candidates_per_request": N,
                       "seq_len": a.prompt_len + a.gen_len,
                       "parallelism": f"tp{tp} x dp{dp}" + (" (ranks SHARE one GPU: a rehearsal of the protocol, "
                                                            "not a multi-GPU number)" if shared else ""),
                       "embedder": f"tp{emb_tp}" if emb_tp > 1 else (f"dp{tp} inside the TP group" if tp > 1 else
                                                                      "one GPU"),
                       "tp_allreduce": ("ipc one-shot kernel (hipGraph)" if comm is not None else
                                        "process group (eager)" + (" (pre-flight fallback)" if tp_comm != a.tp_comm
                                                                   else "") if tp > 1 else "none")}}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("which", choices=["encoder", "moe"])
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--requests", type=int, default=None)
    ap.add_argument("--candidates", type=int, default=64)
    ap.add_argument("--seq-len", type=int, default=128)
    ap.add_argument("--prompt-len", type=int, default=256)
    ap.add_argument("--gen-len", type=int, default=128)
    ap.add_argument("--encoder", default="bge-base-en-v1.5")
    ap.add_argument("--decoder", default="mixtral-8x7b")
    ap.add_argument("--embedder", default="e5-mistral-7b")
    ap.add_argument("--bf16", action="store_true", help="bf16 experts instead of fp8")
    ap.add_argument("--tp", type=int, default=1)
    ap.add_argument("--embedder-par", choices=["tp", "dp"], default="dp",
                    help="moe: the embedder across the TP group — data-parallel (default: whole model per rank, "
                         "1/tp of the candidates each, ONE all-gather of the unit rows per step; the layout "
                         "profiles/ep_vs_tp_round4.md measured best) or tensor-parallel like the sampler (config "
                         "5's literal 'TP=2 each': two [tokens, d] bf16 all-reduces per layer through the process "
                         "group, their bytes per step are reported)")
    ap.add_argument("--gpus", type=int, default=0, help="moe: world size (TP groups x DP); default = --tp")
    ap.add_argument("--tp-comm", choices=["ipc", "pg"], default="ipc",
                    help="moe TP all-reduce: IPC one-shot kernel (graph-captured) or the process group (RCCL / gloo, "
                         "eager); spin-waiting IPC kernels of more than one TP pair cannot share one GPU")
    a = ap.parse_args()
    sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
    if a.which == "moe" and max(a.tp, a.gpus) > 1:
        from llm_weighted_consensus_amd.parallel import launch

        # `bench_configs.py moe --tp 2 [--gpus 8]` without torchrun: launch the ranks (this process never
        # touches the GPU); default world = the TP degree
        rc = launch.maybe_self_launch(max(a.tp, a.gpus), __file__)
        if rc is not None:
            sys.exit(rc)
    if a.which == "encoder":
        a.requests = a.requests or 64
        out = bench_encoder(a)
    else:
        a.requests = a.requests or 64  # 4096-sequence decode batch (the headline's): amortises the expert-weight stream
        # (32 requests: 4.68 answers/s, 64: 5.12 on one MI355X, profiles/moe_round4.md)
        out = bench_moe(a)
    if int(os.environ.get("RANK", "0")) == 0:
        from llm_weighted_consensus_amd import ops
        from llm_weighted_consensus_amd.ops import gemm_plan

        for k, v in gemm_plan.table().items():  # bf16 backend choice per shape (encoder / decoder)
            print(f"# gemm {k}: " + " ".join(f"{b}={t:.1f}us" if b != "choice" else f"choice={t}"
                                             for b, t in v.items()), file=sys.stderr, flush=True)
        for k, v in sorted(ops.FP8_TIMINGS.items(), key=str):  # dense fp8 backend choice per (rows bucket, N, K)
            print(f"# fp8 gemm {k}: " + " ".join(f"{b}={t:.1f}us" for b, t in v.items())
                  + f" choice={ops.FP8_CHOICE.get(k)}", file=sys.stderr, flush=True)
        print(json.dumps(out), flush=True)
    if out.get("verified") is False:
        sys.exit(3)


if __name__ == "__main__":
    main()
