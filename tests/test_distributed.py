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


def _world8_worker(rank, world, port, out_q):
    """The bench's exact multi-GPU layout at world 8: cp=2 candidate groups x dp=4 request groups."""
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    from llm_weighted_consensus_amd.embeddings.consensus import consensus_reference, gather_candidates
    from llm_weighted_consensus_amd.parallel import dist as pdist
    from llm_weighted_consensus_amd.parallel.prefill_share import all_gather_prefills

    from llm_weighted_consensus_amd.parallel import preflight

    pdist.init_from_env("cpu")
    # the benches' start-up pre-flight: a checked all-gather at world 8 (CPU: no devices, no peer pairs);
    # with a forced peer failure the IPC path falls back with the reason
    pre = preflight.run(torch.device("cpu"))
    pre_ok = (pre["world_size_rccl"] == world and pre["rccl_allgather"]["ok"] and pre["peer_access"] == "all"
              and pre["ipc"] == "not requested" and not pre["ipc_fallback"])
    forced = preflight.run(torch.device("cpu"), want_ipc=True, force_peer_fail=True)
    pre_ok &= forced["ipc_fallback"] and forced["ipc"].startswith("fallback: no peer access on forced")
    cp = 2
    cgroup, gidx, crank = pdist.candidate_groups(cp)
    ok = (gidx, crank) == (rank // cp, rank % cp)
    # C4 inside the candidate group: each rank prefilled R=2 prompts of its group's 4 (3 blocks each)
    R, L, E, V, nb = 2, 2, 4, 5, 3
    kv = torch.stack([torch.full((L, 2, E), 1000.0 * rank + b) for b in range(R * nb)], dim=2)
    lg = torch.stack([torch.full((V,), 10.0 * rank + i) for i in range(R)])
    pdist.comm_report(reset=True)
    with pdist.comm_tag("C4"):
        shared = all_gather_prefills(kv, lg, [nb] * R, group=cgroup)
    ok &= len(shared) == R * cp
    for j, (k, l) in enumerate(shared):
        src = gidx * cp + j // R          # global rank that prefilled group prompt j
        ok &= bool((l == 10.0 * src + j % R).all()) and bool((k[0, 0, :, 0] == 1000.0 * src + (j % R) * nb
                                                            + torch.arange(nb)).all())
    # C1 inside the candidate group: rank shard = candidates [crank*n_local, (crank+1)*n_local)
    N, d = 8, 16
    g = torch.Generator().manual_seed(7 + gidx)   # one candidate set per request group
    full = torch.nn.functional.normalize(torch.randn(R * cp, N, d, generator=g), dim=-1)
    n_local = N // cp
    with pdist.comm_tag("C1"):
        got = gather_candidates(full[:, crank * n_local:(crank + 1) * n_local].contiguous(), cgroup)
    ok &= torch.equal(got, full)
    # the per-step accounting the bench JSON reports: bytes received per tag (kv + logits + 2 count gathers
    # for C4, the embeddings for C1), calls, and a time for each
    comm = pdist.comm_report(1)
    c4_bytes = cp * (kv.numel() + lg.numel()) * 4 + cp * 2 * 8 + cp * R * 8
    ok &= comm["C4"]["calls"] == 4 and comm["C4"]["bytes"] == c4_bytes and comm["C4"]["ms"] >= 0
    ok &= comm["C1"]["calls"] == 1 and comm["C1"]["bytes"] == R * cp * N * d * 4
    ok &= pre_ok
    ok &= consensus_reference(got, 0.1).best == consensus_reference(full, 0.1).best
    seen = pdist.world_size_seen()
    ok &= pdist.max_over_ranks(float(rank)) == world - 1
    # bench.py's end-of-run self-check (verify_sharded) through the real scorer: a CPU encoder embeds this
    # rank's shard of every request, C1 gathers them, and the verdict (a MIN over the 8 ranks) is True; the
    # same run with a corrupted all-gather (the group's shards swapped) is caught on every rank
    from llm_weighted_consensus_amd.embeddings import consensus as cons
    from llm_weighted_consensus_amd.models.bert import BertEncoder
    from llm_weighted_consensus_amd.models.config import encoder_config

    scorer = cons.EmbeddingConsensus(BertEncoder(encoder_config("bert-tiny"), device="cpu", seed=3), tau=0.05)
    gt = torch.Generator().manual_seed(100 + gidx)  # the candidate group's requests (same on both its ranks)
    toks = [[torch.randint(0, 1000, (10,), generator=gt).tolist() for _ in range(N)] for _ in range(R)]
    mine = [req[crank * n_local:(crank + 1) * n_local] for req in toks]
    res = scorer.score(mine, gather=True, group=cgroup)
    verified = cons.verify_sharded(scorer, mine[0], res, group=cgroup)
    real = cons.gather_candidates

    def corrupt(E_local, group=None):
        G = real(E_local, group)
        return torch.cat([G[:, n_local:], G[:, :n_local]], dim=1)  # shards in the wrong order

    cons.gather_candidates = corrupt
    try:
        res_bad = scorer.score(mine, gather=True, group=cgroup)
    finally:
        cons.gather_candidates = real
    caught = not cons.verify_sharded(scorer, mine[0], res_bad, group=cgroup)
    out_q.put((rank, bool(ok), seen, verified, caught))
    pdist.shutdown()


def test_bench_layout_cp2_dp4_world8_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_world8_worker, args=(r, 8, port, q)) for r in range(8)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=240) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert [r[0] for r in res] == list(range(8))
    assert all(r[1] for r in res), res
    assert all(r[2] == 8 for r in res)
    assert all(r[3] for r in res), res   # the sharded consensus verified against one-device recomputation
    assert all(r[4] for r in res), res   # and a corrupted all-gather fails the verification everywhere


def test_guarded_reraises_local_errors_without_abort():
    """Only transport failures abort the group; OOM / shape bugs propagate unchanged."""
    from llm_weighted_consensus_amd.parallel import dist as pdist

    def shape_bug():
        raise RuntimeError("shape '[3, 4]' is invalid for input of size 7")

    def oom():
        raise torch.OutOfMemoryError("HIP out of memory")

    with pytest.raises(RuntimeError, match="invalid for input"):
        pdist.guarded(shape_bug, fallback=lambda: 0)
    with pytest.raises(torch.OutOfMemoryError):
        pdist.guarded(oom, fallback=lambda: 0)
    with pytest.raises(ValueError):
        pdist.guarded(lambda: (_ for _ in ()).throw(ValueError("bad")), fallback=lambda: 0)
    assert pdist.is_transport_error(RuntimeError("[gloo/transport/tcp/pair.cc:547] Connection closed by peer"))
    assert pdist.is_transport_error(torch.distributed.DistBackendError("NCCL error: unhandled system error"))


_LAUNCH_CHILD = r'''
import os, sys, torch
sys.path.insert(0, sys.argv[1])
from llm_weighted_consensus_amd.parallel import dist as pdist
info = pdist.init_from_env("cpu")
seen = pdist.world_size_seen()
if info.rank == 0:
    print("WORLD", info.world, seen, info.backend, flush=True)
if len(sys.argv) > 2 and int(sys.argv[2]) == info.rank:
    sys.exit(3)
pdist.barrier()
pdist.shutdown()
'''


def test_self_launch_spawns_ranks(tmp_path):
    """`bench.py --gpus N` self-launch: the launcher starts N ranks with torchrun-style env over 127.0.0.1
    and returns the worst exit status."""
    import subprocess
    import sys

    from llm_weighted_consensus_amd.parallel import launch

    ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    script = tmp_path / "child.py"
    script.write_text(_LAUNCH_CHILD)
    out = tmp_path / "out.txt"
    code = ("import sys; sys.path.insert(0, %r); from llm_weighted_consensus_amd.parallel import launch; "
            "sys.exit(launch.launch(3, [sys.executable, %r, %r]))" % (ROOT, str(script), ROOT))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "WORLD 3 3 gloo" in r.stdout
    # a failing rank makes the launcher fail (the others are stopped, not left hanging in a collective)
    code_fail = code.replace("%r]))" % ROOT, "%r, '1']))" % ROOT)
    r = subprocess.run([sys.executable, "-c", code_fail], env=env, capture_output=True, text=True, timeout=120)
    assert r.returncode == 3, (r.returncode, r.stderr[-2000:])
    with pytest.raises(SystemExit):
        launch.check_world(8, 1)
    launch.check_world(2, 2)


def test_allreduce_selftest_gathers_device_tensors_on_rccl(monkeypatch):
    """CustomAllReduce's start-up self-test builds its input on the host; on an RCCL process group (backend
    "nccl") the all-gather must be handed a tensor on the communicator's device, on gloo a host tensor
    (the NCCL branch passed the host tensor and raised on every multi-GPU bring-up).  No GPU: the
    collective is replaced by a recorder and the device by "meta"."""
    import torch
    import torch.distributed as dist

    from llm_weighted_consensus_amd.parallel.allreduce import CustomAllReduce

    seen = []

    def fake_all_gather(parts, src, group=None):
        seen.append(src.device.type)
        parts[:] = [torch.zeros(src.shape, dtype=src.dtype) for _ in parts]

    ar = CustomAllReduce.__new__(CustomAllReduce)
    ar.group, ar.W, ar.device = None, 2, torch.device("meta")
    monkeypatch.setattr(dist, "all_gather", fake_all_gather)
    x = torch.ones(16, dtype=torch.bfloat16)
    for backend, want in (("nccl", "meta"), ("gloo", "cpu")):
        monkeypatch.setattr(dist, "get_backend", lambda group=None, b=backend: b)
        seen.clear()
        out = ar._gather_ref(x)
        assert seen == [want] and len(out) == 2 and all(p.device.type == "cpu" for p in out)
