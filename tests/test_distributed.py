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


def _prefill_share_worker(rank, world, port, out_q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    from llm_weighted_consensus_amd.parallel import dist as pdist
    from llm_weighted_consensus_amd.parallel.prefill_share import all_gather_prefills

    pdist.init_from_env("cpu")
    L, E, V = 3, 5, 7
    # rank r owns r+1 prompts with r+2 ... blocks each: uneven counts exercise the padding path
    nblocks = [rank + 2 + i for i in range(rank + 1)]
    kv = torch.stack([torch.full((L, 2, E), 100.0 * rank + b) for b in range(sum(nblocks))], dim=2)
    logits = torch.stack([torch.full((V,), 10.0 * rank + i) for i in range(len(nblocks))])
    got = all_gather_prefills(kv, logits, nblocks)
    ok = True
    idx = 0
    for r in range(world):
        nbs = [r + 2 + i for i in range(r + 1)]
        off = 0
        for i, nb in enumerate(nbs):
            k, lg = got[idx]
            ok &= k.shape == (L, 2, nb, E)
            ok &= bool((k[0, 0, :, 0] == torch.arange(off, off + nb) + 100.0 * r).all())
            ok &= bool((lg == 10.0 * r + i).all())
            off += nb
            idx += 1
    ok &= idx == len(got)
    out_q.put((rank, ok))
    pdist.shutdown()


def test_prefill_share_all_gather_gloo():
    """C4: uneven per-rank prompt/block counts are padded, gathered once and split back per prompt."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_prefill_share_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(ok for _, ok in res)


def _groups_worker(rank, world, port, out_q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    from llm_weighted_consensus_amd.embeddings.consensus import gather_candidates
    from llm_weighted_consensus_amd.parallel import dist as pdist

    pdist.init_from_env("cpu")
    g, gidx, crank = pdist.candidate_groups(2)
    E = torch.full((3, 2, 4), float(rank))
    got = gather_candidates(E, g)          # only the 2 ranks of this candidate group
    ok = got.shape == (3, 4, 4) and got[0, :2].eq(gidx * 2).all() and got[0, 2:].eq(gidx * 2 + 1).all()
    out_q.put((rank, bool(ok), gidx, crank))
    pdist.shutdown()


def test_candidate_groups_gloo():
    """cp=2 x dp=2 over 4 ranks: gathers stay inside each candidate group."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_groups_worker, args=(r, 4, port, q)) for r in range(4)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [r[1:] for r in res] == [(True, 0, 0), (True, 0, 1), (True, 1, 0), (True, 1, 1)]


def _dead_peer_worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), LWC_COLLECTIVE_TIMEOUT_S="5")
    import time

    from llm_weighted_consensus_amd.embeddings.consensus import gather_candidates
    from llm_weighted_consensus_amd.parallel import dist as pdist

    pdist.init_from_env("cpu")
    pdist.barrier()
    if rank == 1:
        os._exit(0)  # the peer dies without a word
    E = torch.nn.functional.normalize(torch.randn(2, 3, 8), dim=-1)
    t0 = time.time()
    got = pdist.guarded(gather_candidates, E, None, fallback=lambda: E)
    ok = torch.equal(got, E) and not pdist.info().enabled
    # further collectives are single-rank no-ops now
    ok = ok and pdist.all_gather(E).shape == (1, 2, 3, 8) and pdist.max_over_ranks(3.0) == 3.0
    q.put((ok, time.time() - t0))


def test_collective_failure_aborts_and_falls_back():
    """Failure detection for collectives: a peer dies, the surviving rank's guarded all-gather fails
    within the process-group timeout, the group is aborted and the rank continues single-rank with
    its local shard."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dead_peer_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    ok, dt = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
    assert ok and dt < 60, dt


def test_guarded_without_fallback_raises():
    from llm_weighted_consensus_amd.parallel import dist as pdist

    def boom():
        raise RuntimeError("transport closed")

    with pytest.raises(pdist.CollectiveFailure):
        pdist.guarded(boom)
    assert pdist.guarded(lambda: 7) == 7
