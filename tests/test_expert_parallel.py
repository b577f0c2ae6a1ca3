"""Expert parallelism (C4) on CPU: gloo, world_size 2 and 4.  Every rank routes its own tokens, dispatches
the (token, slot) rows to the expert owners over all-to-all, the owners run their experts, and the
combine brings the outputs back.  The result must equal a single-process MoE over all experts, in both
exchange modes (padded: device-only indices; exact: variable splits), including ranks with zero tokens
and experts that receive no rows.  The routing here is a pure-torch stand-in for the K11a kernel with the
same contract (expert-sorted rows, segment offsets, src/inv permutations)."""
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


def route_ref(logits, k):
    """Pure-torch equivalent of ops.moe_route: (w [T,k], row_off [E+1], src [T*k], inv [T*k])."""
    T, E = logits.shape
    top, ids = torch.topk(logits.float(), k, dim=-1)
    w = torch.softmax(top, dim=-1)
    flat = ids.reshape(-1)
    order = torch.sort(flat * (T * k) + torch.arange(T * k), stable=True).indices
    src = order // k
    inv = torch.empty_like(order)
    inv[order] = torch.arange(T * k)
    counts = torch.bincount(flat, minlength=E)
    row_off = torch.zeros(E + 1, dtype=torch.int32)
    row_off[1:] = torch.cumsum(counts, 0).to(torch.int32)
    return w, row_off, src, inv


def experts_ref(x, row_off, w1, w2, e0=0):
    """Grouped two-layer expert FFN over expert-major rows (the grouped GEMM's contract)."""
    out = torch.zeros(x.shape[0], w2.shape[1])
    for e in range(w1.shape[0]):
        a, b = int(row_off[e]), int(row_off[e + 1])
        if b > a:
            out[a:b] = torch.relu(x[a:b] @ w1[e].t()) @ w2[e].t()
    return out


def _moe_full(x, router, w1, w2, k):
    w, row_off, src, inv = route_ref(x @ router.t(), k)
    y = experts_ref(x[src], row_off, w1, w2)
    T = x.shape[0]
    return (y[inv].view(T, k, y.shape[-1]) * w[..., None]).sum(1)


class _ByteAllToAll:
    """Stand-in with CustomAllToAll's contract (equal chunks moved as raw bytes, parallel/allreduce.py) over
    the gloo group, to check the EP layer's routing of its exchanges through a ``comm``."""

    def __init__(self, W):
        self.W, self.calls = W, 0

    def all_to_all(self, out, inp):
        import torch.distributed as dist

        self.calls += 1
        src = inp.contiguous().view(-1).view(torch.uint8)
        recv = torch.empty_like(src)
        dist.all_to_all_single(recv, src)
        out.view(-1).view(torch.uint8).copy_(recv)
        return out


def _worker(rank, world, port, mode, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))
    try:
        from llm_weighted_consensus_amd.parallel import dist as pdist
        from llm_weighted_consensus_amd.parallel.expert import ExpertParallel

        pdist.init_from_env("cpu")
        E, k, d, f = 8, 2, 16, 24
        g = torch.Generator().manual_seed(0)
        router = torch.randn(E, d, generator=g)
        router[E - 1] -= 100.0  # the last expert never wins a top-k slot: an empty segment everywhere
        w1 = torch.randn(E, f, d, generator=g) / 4
        w2 = torch.randn(E, d, f, generator=g) / 4
        sizes = [5, 0, 9, 3][:world]  # rank 1 has no tokens this step
        xs = [torch.randn(n, d, generator=g) for n in sizes]
        x = xs[rank]
        comm = _ByteAllToAll(world) if mode == "padded-comm" else None
        ep = ExpertParallel(E, mode="padded" if mode == "padded-comm" else mode, comm=comm)
        El = ep.El
        lw1, lw2 = w1[rank * El:(rank + 1) * El], w2[rank * El:(rank + 1) * El]
        w, row_off, src, inv = route_ref(x @ router.t(), k)
        y_sorted = ep.run(x[src], row_off, lambda xl, ro, _s: experts_ref(xl, ro, lw1, lw2))
        T = x.shape[0]
        out = (y_sorted[inv].view(T, k, y_sorted.shape[-1]) * w[..., None]).sum(1)
        ref = _moe_full(x, router, w1, w2, k)
        ok = bool(torch.allclose(out, ref, atol=1e-5, rtol=1e-5))
        if comm is not None:  # counts, rows and returned outputs: every exchange went through the comm
            ok = ok and comm.calls == 3
        q.put((rank, ok, float((out - ref).abs().max()) if T else 0.0))
        pdist.shutdown()
    except Exception as e:  # noqa: BLE001
        q.put((rank, False, repr(e)))


@pytest.mark.parametrize("world,mode", [(2, "padded"), (2, "exact"), (4, "padded"), (4, "exact"), (2, "padded-comm"),
                                        (4, "padded-comm")])
def test_expert_parallel_matches_full_moe(world, mode):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, mode, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(ok for _, ok, _ in res), res


def test_route_ref_contract():
    g = torch.Generator().manual_seed(1)
    logits = torch.randn(7, 4, generator=g)
    w, row_off, src, inv = route_ref(logits, 2)
    ids = torch.topk(logits, 2, dim=-1).indices.reshape(-1)
    # sorted row inv[t*k+j] belongs to token t and lies inside expert ids[t*k+j]'s segment
    for tj in range(14):
        p = int(inv[tj])
        assert int(src[p]) == tj // 2
        e = int(ids[tj])
        assert int(row_off[e]) <= p < int(row_off[e + 1])
    assert torch.allclose(w.sum(-1), torch.ones(7))


def test_sane_counts_drop_poisoned_chunks():
    """counts received from a peer that never arrived are all-ones bytes (-1 as int64); a chunk with
    a negative count or more rows than the capacity is zeroed before it can become an index."""
    from llm_weighted_consensus_amd.parallel.expert import ExpertParallel

    rc = torch.tensor([[2, 1], [-1, -1], [5, 4], [0, 3]], dtype=torch.int64)
    out = ExpertParallel._sane_counts(rc, 8)
    assert out.tolist() == [[2, 1], [0, 0], [0, 0], [0, 3]]
