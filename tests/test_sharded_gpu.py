"""Voter-sharded scoring on the GPU (C2): two ranks sharing one MI355X (LWC_SHARE_ONE_GPU=1), each with its
own local engine of a random-init Llama voter model, serve concurrent /score/completions through the ASGI
app on rank 0 (the follower's voters stream back over the shard link).  Every response carries every voter
of its request, each with a parseable vote (json_schema constrained decoding) and confidences that sum to
one; /consensus/completions splits its candidates over both engines."""
import os
import socket

import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

MODELS = {"tiny": {"arch": "llama-tiny", "weights": "random:1", "max_model_len": 2048, "max_batch": 64}}


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE="2", LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), LWC_SHARE_ONE_GPU="1", HSA_ENABLE_IPC_MODE_LEGACY="0")
    import asyncio

    import httpx

    from llm_weighted_consensus_amd.parallel import dist as pdist
    from llm_weighted_consensus_amd.server.app import create_app
    from llm_weighted_consensus_amd.server.config import Config
    from llm_weighted_consensus_amd.server.main import build_state, shard_voters

    try:
        info = pdist.init_from_env("cuda")
        state = build_state(Config(models=MODELS, embed_models={"e": {"arch": "bert-tiny", "weights": "random:1"}},
                                   kv_fraction=0.04, gpu=info.local_rank))
        lead = shard_voters(state)
        if rank != 0:
            q.put((rank, lead.serve()))
        else:
            client = httpx.AsyncClient(transport=httpx.ASGITransport(app=create_app(state)), base_url="http://t",
                                       timeout=300)
            llms = [{"model": "tiny", "output_mode": "json_schema", "top_logprobs": 5, "temperature": 0.6 + 0.1 * i}
                    for i in range(4)]

            async def one(i):
                r = await client.post("/score/completions", json={
                    "messages": [{"role": "user", "content": f"Question {i}: which city is the capital of France?"}],
                    "model": {"llms": llms}, "choices": ["Paris", "Madrid", "Rome"]})
                assert r.status_code == 200, r.text[:500]
                return r.json()

            async def go():
                return await asyncio.gather(*(one(i) for i in range(5)))

            bodies = asyncio.run(go())

            async def consensus():  # candidates split over the ranks, unit rows back over the shard link
                r = await client.post("/consensus/completions", json={
                    "model": "tiny", "messages": [{"role": "user", "content": "Name a colour."}], "n": 6,
                    "max_tokens": 12, "temperature": 0.9, "seed": 3, "embedding_model": "e"})
                assert r.status_code == 200, r.text[:500]
                return r.json()

            cons = asyncio.run(consensus())
            lead.close()
            out = []
            for b in bodies:
                provided = [c for c in b["choices"] if c["index"] < 3]
                voters = [c for c in b["choices"] if c["index"] >= 3]
                out.append((len(provided), sorted(v["model_index"] for v in voters),
                            sum(1 for v in voters if v["message"].get("vote")),
                            round(sum(c["confidence"] for c in provided), 6),
                            sorted(c["index"] for c in b["choices"])))
            out.append((sorted(c["index"] for c in cons["choices"]),
                        round(sum(c["confidence"] for c in cons["choices"]), 5),
                        len(cons["weight_data"]["embeddings_response"]["data"])))
            q.put((rank, out))
        for svc in state.services.values():
            svc.close()
        pdist.shutdown()
    except BaseException as e:  # noqa: BLE001 — report, then fail the rank
        q.put((rank, repr(e)))
        raise


def test_voter_sharded_serving_two_ranks_one_gpu(gpu):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert got[1] == 6, got  # the follower ran its share of every request (5 score shares + 1 consensus slice)
    cons_indices, cons_conf, n_rows = got[0].pop()
    assert cons_indices == list(range(6)) and cons_conf == pytest.approx(1.0) and n_rows == 6
    for n_provided, model_indices, n_votes, conf, indices in got[0]:
        assert n_provided == 3 and model_indices == [0, 1, 2, 3] and n_votes == 4, got[0]
        assert conf == pytest.approx(1.0) and indices == list(range(7))
    assert all(p.exitcode == 0 for p in procs)
