#!/usr/bin/env python3
"""CPU-only cost of the serving front end: /score/completions through the ASGI app with scripted voters
(FakeChatClient) shaped like serve_load.py's local voters — 8 voters, ~16 streamed tokens each with
top-5 logprobs — so the orchestrator, chunk merging, archive and JSON costs are measured without a GPU.
Usage: frontend_bench.py [requests] [--profile]"""
import asyncio
import math
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import httpx  # noqa: E402

from llm_weighted_consensus_amd.chat.fake import FakeChatClient, Scripted, select_keys  # noqa: E402
from llm_weighted_consensus_amd.server.app import create_app  # noqa: E402
from llm_weighted_consensus_amd.server.config import Config  # noqa: E402
from llm_weighted_consensus_amd.server.main import build_state  # noqa: E402


def policy(req):
    keys = select_keys(req)
    good = keys[0][0]
    alts = lambda t: [(t, -0.05)] + [(f"x{j}", -3.0 - j) for j in range(4)]  # noqa: E731
    toks = [(w, alts(w)) for w in ('{"', "response", "_key", '":"')] + [("`", alts("`"))]
    toks += [(good[1], [(good[1], math.log(0.6))] + [(k[0][1], math.log(0.1)) for k in keys[1:4]] +
              [("zz", math.log(0.05))])]
    toks += [("`", alts("`")), ('"}', alts('"}'))] + [(f" pad{j}", alts(f" pad{j}")) for j in range(8)]
    return [Scripted("".join(t for t, _ in toks), logprobs=toks)]


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 and sys.argv[1].isdigit() else 256
    import gc

    gc.set_threshold(200_000, 50, 100)  # as a serving process has it (LLMEngine tune_gc)
    prof = "--profile" in sys.argv
    state = build_state(Config(), chat_client=FakeChatClient(policy, chunk_chars=1000))
    app = create_app(state)
    client = httpx.AsyncClient(transport=httpx.ASGITransport(app=app), base_url="http://t", timeout=600)
    llms = [{"model": f"voter{i}", "top_logprobs": 5, "temperature": 0.7 + 0.01 * i} for i in range(8)]

    def body(i):
        return {"messages": [{"role": "user", "content": f"Question {i}: which city is the capital?"}],
                "model": {"llms": llms}, "choices": [f"City number {j} of request {i}" for j in range(4)]}

    async def run(k):
        sem = asyncio.Semaphore(64)

        async def one(i):
            async with sem:
                r = await client.post("/score/completions", json=body(i))
                assert r.status_code == 200, r.text[:300]

        await asyncio.gather(*(one(i) for i in range(k)))

    asyncio.run(run(32))
    pr = None
    if prof:
        import cProfile

        pr = cProfile.Profile()
        pr.enable()
    rounds = int(os.environ.get("FRONTEND_ROUNDS", "1" if prof else "5"))
    per = []
    for _ in range(rounds):  # the container's CPU time per request is noisy: min and median over rounds
        t, c = time.perf_counter(), time.process_time()
        asyncio.run(run(n))
        el, cpu = time.perf_counter() - t, time.process_time() - c
        per.append((cpu / n * 1e3, el))
    cpus = sorted(p for p, _ in per)
    el = min(e for _, e in per)
    cpu = cpus[0] * n / 1e3
    if pr is not None:
        pr.disable()
        import pstats

        st = pstats.Stats(pr)
        st.sort_stats(os.environ.get("PROF_SORT", "tottime")).print_stats(int(os.environ.get("PROF_N", "30")))
        if "--callers" in sys.argv:
            st.print_callers("main.py:253")
    print(f"front end: {n / el:.1f} score requests/s ({el / n * 1e3:.2f} ms wall, {cpu / n * 1e3:.2f} ms process CPU "
          f"per request, 8 voters x 16 tokens; best of {rounds} rounds, median "
          f"{cpus[len(cpus) // 2]:.2f} ms CPU)")


if __name__ == "__main__":
    main()
