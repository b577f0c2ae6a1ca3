#!/usr/bin/env python3
"""Serving-path load test: the real ASGI app (in-process transport, no sockets) with a local Llama-3-8B
voter model (random init) on one MI355X, hit by C concurrent `POST /score/completions` requests, each a
score model of V local voters choosing among K choices (json_schema output mode: constrained decoding,
votes from top-logprobs).  Reports scored requests/s, voter completions/s and latency percentiles, plus
the engine's prefix-cache savings (every voter of a request shares the messages head).

    python scripts/serve_load.py [--concurrency 64] [--requests 256] [--voters 8] [--arch llama-3-8b]

The reference measures nothing of the kind (its voters are upstream HTTP calls); this is the serving
number of the whole stack: HTTP contract, orchestrator, engine service thread, engine, kernels.
"""
import argparse
import asyncio
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--arch", default="llama-3-8b")
    ap.add_argument("--concurrency", type=int, default=64)
    ap.add_argument("--requests", type=int, default=256)
    ap.add_argument("--voters", type=int, default=8)
    ap.add_argument("--choices", type=int, default=4)
    ap.add_argument("--max-batch", type=int, default=1024)
    ap.add_argument("--profile", action="store_true", help="cProfile the engine thread and the event loop")
    ap.add_argument("--gpus", default=os.environ.get("LWC_GPUS", ""),
                    help="comma list: serve through an EngineGroup of worker processes (e.g. '0' = one worker)")
    a = ap.parse_args()
    profs = {}
    import gc

    gc_time = {0: 0.0, 1: 0.0, 2: 0.0}
    gc_n = {0: 0, 1: 0, 2: 0}
    _gc_t0 = [0.0]

    def _gc_cb(phase, info):  # time spent in each generation's collections (stalls every thread)
        if phase == "start":
            _gc_t0[0] = time.perf_counter()
        else:
            gc_time[info["generation"]] += time.perf_counter() - _gc_t0[0]
            gc_n[info["generation"]] += 1

    gc.callbacks.append(_gc_cb)
    if a.profile:
        import cProfile

        from llm_weighted_consensus_amd.engine import service as S

        orig = S.EngineService._run

        def prof_run(self):
            pr = profs.setdefault("engine", cProfile.Profile())
            pr.enable()
            try:
                orig(self)
            finally:
                pr.disable()

        S.EngineService._run = prof_run

        from llm_weighted_consensus_amd.engine import group as G

        orig_read = G.EngineGroup._read

        def prof_read(self):
            pr = profs.setdefault("group-reader", cProfile.Profile())
            pr.enable()
            try:
                orig_read(self)
            finally:
                pr.disable()

        G.EngineGroup._read = prof_read

    import httpx

    from llm_weighted_consensus_amd.server.app import create_app
    from llm_weighted_consensus_amd.server.config import Config
    from llm_weighted_consensus_amd.server.main import build_state

    models = {"local": {"arch": a.arch, "weights": "random:1", "max_model_len": 2048, "max_batch": a.max_batch}}
    t0 = time.time()
    gpus = [int(x) for x in a.gpus.split(",") if x.strip()]
    state = build_state(Config(models=models, kv_fraction=0.6, gpus=gpus,
                               chunked_prefill=int(os.environ.get("LWC_CHUNKED_PREFILL", "2048")),
                               gpu_tally=os.environ.get("LWC_GPU_TALLY")))
    print(f"# model ready in {time.time() - t0:.1f} s", file=sys.stderr, flush=True)
    app = create_app(state)
    client = httpx.AsyncClient(transport=httpx.ASGITransport(app=app), base_url="http://t", timeout=600)
    question = ("You are grading answers to a geography quiz. Consider each candidate carefully, compare them "
                "with what you know, and pick the single best answer. ") * 4
    llms = [{"model": "local", "output_mode": "json_schema", "top_logprobs": 5, "temperature": 0.7 + 0.01 * i}
            for i in range(a.voters)]

    def body(i):
        return {"messages": [{"role": "user", "content": f"{question} Question {i}: which city is the capital?"}],
                "model": {"llms": llms},
                "choices": [f"City number {j} of request {i}" for j in range(a.choices)]}

    lat, errs = [], 0

    async def one(i, sem):
        nonlocal errs
        async with sem:
            t = time.perf_counter()
            r = await client.post("/score/completions", json=body(i))
            lat.append(time.perf_counter() - t)
            if r.status_code != 200:
                errs += 1

    async def run(n):
        sem = asyncio.Semaphore(a.concurrency)
        await asyncio.gather(*(one(i, sem) for i in range(n)))

    asyncio.run(run(min(a.concurrency, a.requests)))  # warmup: graphs, GEMM plans
    lat.clear()
    eng = state.services["local"].engine
    stats = getattr(eng, "stats", None) or {"prefill_tokens": 0, "prefix_cache_tokens": 0, "steps": 0}
    p0, c0 = stats["prefill_tokens"], stats["prefix_cache_tokens"]
    if a.profile:
        import cProfile

        profs["loop"] = cProfile.Profile()
        profs["loop"].enable()
    t = time.perf_counter()
    asyncio.run(run(a.requests))
    el = time.perf_counter() - t
    if a.profile:
        profs["loop"].disable()
    lat.sort()
    pct = lambda q: lat[min(len(lat) - 1, int(q * len(lat)))]  # noqa: E731
    out = {"metric": "score requests/s through the HTTP app (local voters)", "value": round(a.requests / el, 3),
           "voter_completions_per_s": round(a.requests * a.voters / el, 2), "errors": errs,
           "latency_s": {"p50": round(pct(0.5), 3), "p90": round(pct(0.9), 3), "p99": round(pct(0.99), 3)},
           "prefill_tokens": stats["prefill_tokens"] - p0,
           "prefix_cache_tokens": stats["prefix_cache_tokens"] - c0,
           "serving": f"EngineGroup workers on GPUs {gpus}" if gpus else "in-process engine",
           "chunked_prefill": int(os.environ.get("LWC_CHUNKED_PREFILL", "2048")),
           "config": {"arch": a.arch, "concurrency": a.concurrency, "requests": a.requests, "voters": a.voters,
                      "choices": a.choices, "output_mode": "json_schema", "data": "synthetic prompts, random-init"}}
    from llm_weighted_consensus_amd.utils.tracing import STATS

    out["phases"] = {k: [v[0], round(v[1], 3)] for k, v in STATS.snapshot()["phases"].items()}
    from llm_weighted_consensus_amd.ops import gemm_plan

    # the planner's per-shape choices (decode buckets and mixed-step row buckets) with their timings
    out["gemm_plan"] = {k: {b: (round(t, 1) if isinstance(t, float) else t) for b, t in v.items()}
                        for k, v in gemm_plan.table().items()}
    out["engine_steps"] = stats["steps"]
    tb = getattr(state.score, "tally_batcher", None)
    if tb is not None:  # K10b: tallies batched into GPU launches (LWC_GPU_TALLY)
        out["gpu_tally"] = {"min_batch": tb.min_batch, "launches": tb.gpu_batches, "tallies": tb.gpu_tallies}
    out["gc"] = {f"gen{k}": [gc_n[k], round(gc_time[k], 3)] for k in gc_time}
    print(json.dumps(out), flush=True)
    for svc in state.services.values():
        svc.close()
    if a.profile:
        import io
        import pstats

        for name, pr in profs.items():
            for order, k in (("tottime", 25), ("cumulative", 45)):
                buf = io.StringIO()
                pstats.Stats(pr, stream=buf).sort_stats(order).print_stats(k)
                print(f"==== {name} ({order})\n" + buf.getvalue()[:9000], file=sys.stderr)


if __name__ == "__main__":
    main()
