"""Multi-process (gloo, world_size 2, CPU): process-group bring-up from torchrun-style env, the
candidate-parallel embedding all-gather (C1) and the consensus on gathered candidates equals the
single-process result on the full candidate set."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    from llm_weighted_consensus_amd.embeddings.consensus import consensus_reference, gather_candidates
    from llm_weighted_consensus_amd.parallel import dist as pdist

    info = pdist.init_from_env("cpu")
    assert info.world == world and info.backend == "gloo"
    g = torch.Generator().manual_seed(0)
    R, N, d = 3, 8, 16
    full = torch.nn.functional.normalize(torch.randn(R, N, d, generator=g), dim=-1)
    n_local = N // world
    shard = full[:, rank * n_local:(rank + 1) * n_local]
    gathered = gather_candidates(shard)
    res = consensus_reference(gathered, 0.1)
    ref = consensus_reference(full, 0.1)
    ok = torch.allclose(gathered, full) and res.best == ref.best and torch.allclose(res.weights, ref.weights)
    m = pdist.max_over_ranks(float(rank))
    pdist.barrier()
    out_q.put((rank, ok, m))
    pdist.shutdown()


def test_candidate_parallel_gather_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(ok for _, ok, _ in res)
    assert all(m == 1.0 for _, _, m in res)
