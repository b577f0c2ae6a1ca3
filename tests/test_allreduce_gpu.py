"""C3 one-shot all-reduce over IPC-mapped peer buffers (csrc/kernels/allreduce.hip), two ranks sharing
the test box's GPU (handles exchanged over gloo; the data path is the kernel only): results equal the
fp32 rank-order sum rounded to bf16 on both ranks, across many calls (parity reuse), ragged sizes,
payloads larger than a slot, and inside a replayed hipGraph; and TP=2 Mixtral logits through it match
TP=1."""
import os
import socket

import pytest
import numpy as np
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu



def _collect(q, procs, timeout):
    """Gather (rank, result) pairs. Workers send numpy arrays (pickled by value): a CPU tensor put on a
    queue is shared through a file descriptor that dies with the worker, so a worker that exits before the
    parent reads the queue would reset the connection."""
    out = {}
    for _ in procs:
        r, v = q.get(timeout=timeout)
        out[r] = torch.from_numpy(v) if isinstance(v, np.ndarray) else v
    return out

def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _ref(world, n, seed):
    g = torch.Generator().manual_seed(seed)
    xs = [torch.randn(n, generator=g).to(torch.bfloat16) for _ in range(world)]
    acc = torch.zeros(n)
    for x in xs:
        acc += x.float()
    return xs, acc.to(torch.bfloat16)


def _ar_worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), LWC_SHARE_ONE_GPU="1")
    try:
        from llm_weighted_consensus_amd.parallel import dist as pdist
        from llm_weighted_consensus_amd.parallel.allreduce import CustomAllReduce

        pdist.init_from_env("cuda")
        dev = torch.device("cuda", 0)
        comm = CustomAllReduce(device=dev, max_bytes=1 << 20, blocks=16)
        bad = []
        sizes = [8, 4096, 12344, 1 << 19, (1 << 19) + 4096 * 3, 3 << 20]  # last two exceed one 1 MiB slot
        for it in range(24):
            n = sizes[it % len(sizes)]
            xs, want = _ref(world, n, 1000 + it)
            x = xs[rank].to(dev)
            comm.all_reduce_(x)
            if not torch.equal(x.cpu(), want):
                bad.append(("eager", it, n))
        # captured in a hipGraph, replayed with fresh inputs copied into the static buffer
        n = 65536
        static = torch.zeros(n, dtype=torch.bfloat16, device=dev)
        s = torch.cuda.Stream(dev)
        s.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(s):
            comm.all_reduce_(static)  # warm-up outside capture
        torch.cuda.current_stream(dev).wait_stream(s)
        pdist.barrier()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            comm.all_reduce_(static)
        for it in range(10):
            xs, want = _ref(world, n, 5000 + it)
            static.copy_(xs[rank].to(dev))
            graph.replay()
            torch.cuda.synchronize(dev)
            if not torch.equal(static.cpu(), want):
                bad.append(("graph", it))
        comm.check()
        pdist.barrier()
        comm.close()
        q.put((rank, bad))
        pdist.shutdown()
    except Exception as e:  # noqa: BLE001
        q.put((rank, repr(e)))


def test_ipc_allreduce_two_ranks_one_gpu(gpu):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ar_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = _collect(q, procs, 300)
    for p in procs:
        p.join(timeout=60)
    assert res == {0: [], 1: []}, res


def _tp_worker(rank, world, port, fp8, q, arch="mixtral-tiny"):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), LWC_SHARE_ONE_GPU="1")
    try:
        from llm_weighted_consensus_amd.models.config import decoder_config
        from llm_weighted_consensus_amd.models.llama import KVCache
        from llm_weighted_consensus_amd.models.mixtral import MixtralModel
        from llm_weighted_consensus_amd.models.tp import TPLlamaModel
        from llm_weighted_consensus_amd.parallel import dist as pdist
        from llm_weighted_consensus_amd.parallel.allreduce import CustomAllReduce

        pdist.init_from_env("cuda")
        dev = torch.device("cuda", 0)
        comm = CustomAllReduce(device=dev, max_bytes=1 << 20, blocks=16)
        if arch.startswith("mixtral"):
            m = MixtralModel(decoder_config(arch), device=dev, seed=4, max_position=512, fp8=fp8,
                             tp_rank=rank, tp_size=world, tp_comm=comm)
        else:
            m = TPLlamaModel(decoder_config(arch), device=dev, seed=4, max_position=512, fp8_dense=fp8,
                             tp_rank=rank, tp_size=world, tp_comm=comm)
        assert m.graph_safe
        g = torch.Generator().manual_seed(9)
        P = 29
        toks = torch.randint(0, m.cfg.vocab_size, (P,), generator=g).to(dev)
        cache = KVCache(m.cfg, 8, 16, dev)
        ar = torch.arange(P, dtype=torch.int32, device=dev)
        lg = m.prefill(toks.int(), ar, ar, torch.tensor([0, P], dtype=torch.int32, device=dev), P,
                       torch.tensor([P - 1], device=dev), cache)
        torch.cuda.synchronize(dev)
        comm.check()
        q.put((rank, lg[0].float().cpu().numpy()))
        pdist.barrier()
        comm.close()
        pdist.shutdown()
    except Exception as e:  # noqa: BLE001
        q.put((rank, repr(e)))


@pytest.mark.parametrize("arch", ["mixtral-tiny", "llama-tiny"])
def test_tp2_through_ipc_allreduce(gpu, arch):
    """TP=2 prefill logits (two ranks on one GPU, IPC one-shot all-reduce after o and after down) match TP=1:
    the MoE decoder (experts column-split) and the dense one (TPLlamaModel: heads and FFN columns split)."""
    from llm_weighted_consensus_amd.models.config import decoder_config
    from llm_weighted_consensus_amd.models.llama import KVCache, LlamaModel
    from llm_weighted_consensus_amd.models.mixtral import MixtralModel

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_tp_worker, args=(r, 2, port, False, q, arch)) for r in range(2)]
    for p in procs:
        p.start()
    res = _collect(q, procs, 600)
    for p in procs:
        p.join(timeout=120)
    assert all(isinstance(v, torch.Tensor) for v in res.values()), res
    cls = MixtralModel if arch.startswith("mixtral") else LlamaModel
    m = cls(decoder_config(arch), device=gpu, seed=4, max_position=512)
    g = torch.Generator().manual_seed(9)
    P = 29
    toks = torch.randint(0, m.cfg.vocab_size, (P,), generator=g).to(gpu)
    cache = KVCache(m.cfg, 8, 16, gpu)
    ar = torch.arange(P, dtype=torch.int32, device=gpu)
    lg = m.prefill(toks.int(), ar, ar, torch.tensor([0, P], dtype=torch.int32, device=gpu), P,
                   torch.tensor([P - 1], device=gpu), cache)[0].float().cpu()
    for r in range(2):
        c = torch.nn.functional.cosine_similarity(res[r], lg, dim=0).item()
        assert c > 0.99, (r, c)
    assert torch.equal(res[0], res[1])


def _back_to_back_worker(rank, world, port, q):
    """flags only grow, so a fast peer may publish call e+1's flag before a slow poller read
    e.  Back-to-back calls with no host sync must neither stall nor set the error word."""
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), LWC_SHARE_ONE_GPU="1")
    try:
        from llm_weighted_consensus_amd.parallel import dist as pdist
        from llm_weighted_consensus_amd.parallel.allreduce import CustomAllReduce

        pdist.init_from_env("cuda")
        dev = torch.device("cuda", 0)
        comm = CustomAllReduce(device=dev, max_bytes=1 << 20, blocks=8, spin_ms=2000)
        xs, want = _ref(world, 4096, 77)
        outs = []
        for it in range(300):  # every call waits on the previous one's result: a data dependency chain
            x = xs[rank].to(dev) if it == 0 else outs[-1] * 0 + xs[rank].to(dev)
            comm.all_reduce_(x)
            outs.append(x)
        torch.cuda.synchronize(dev)
        bad = [] if torch.equal(outs[-1].cpu(), want) else ["value"]
        if int(comm.err.item()):
            bad.append("err")
        pdist.barrier()
        comm.close()
        q.put((rank, bad))
        pdist.shutdown()
    except Exception as e:  # noqa: BLE001
        q.put((rank, repr(e)))


def test_ipc_allreduce_back_to_back_no_false_timeout(gpu):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_back_to_back_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = _collect(q, procs, 300)
    for p in procs:
        p.join(timeout=60)
    assert res == {0: [], 1: []}, res


def _skip_worker(rank, world, port, q):
    """Rank 1 skips one call: rank 0 must return within its spin bound with NaN output, the error word
    set, and poll() raising CommFailure — no hang, no silently wrong sum."""
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), LWC_SHARE_ONE_GPU="1")
    try:
        import time

        from llm_weighted_consensus_amd.parallel import dist as pdist
        from llm_weighted_consensus_amd.parallel.allreduce import CommFailure, CustomAllReduce

        pdist.init_from_env("cuda")
        dev = torch.device("cuda", 0)
        comm = CustomAllReduce(device=dev, max_bytes=1 << 20, blocks=4, spin_ms=300)
        xs, want = _ref(world, 8192, 5)
        x = xs[rank].to(dev)
        comm.all_reduce_(x)  # one healthy call
        torch.cuda.synchronize(dev)
        ok_first = torch.equal(x.cpu(), want)
        pdist.barrier()
        out = {"first": ok_first}
        if rank == 0:
            y = xs[0].to(dev)
            t0 = time.perf_counter()
            comm.all_reduce_(y)
            comm.arm()
            torch.cuda.synchronize(dev)
            out["elapsed"] = time.perf_counter() - t0
            out["all_nan"] = bool(torch.isnan(y.float()).all())
            try:
                comm.poll()
                out["raised"] = False
            except CommFailure:
                out["raised"] = True
        pdist.barrier()
        q.put((rank, out))
        comm.close()
        pdist.shutdown()
    except Exception as e:  # noqa: BLE001
        q.put((rank, repr(e)))


def test_ipc_allreduce_missing_peer_fails_loudly(gpu):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_skip_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = _collect(q, procs, 300)
    for p in procs:
        p.join(timeout=60)
    assert isinstance(res[0], dict) and isinstance(res[1], dict), res
    assert res[0]["first"] and res[1]["first"]
    assert res[0]["all_nan"] and res[0]["raised"], res[0]
    assert res[0]["elapsed"] < 5.0, res[0]  # the 300 ms bound, plus launch / sync overhead


def _selftest_worker(rank, world, port, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), LWC_SHARE_ONE_GPU="1")
    try:
        from llm_weighted_consensus_amd.parallel import dist as pdist
        from llm_weighted_consensus_amd.parallel.allreduce import CommFailure, CustomAllReduce, CustomAllToAll

        pdist.init_from_env("cuda")
        dev = torch.device("cuda", 0)
        out = []
        for cls in (CustomAllReduce, CustomAllToAll):
            comm = cls(device=dev, max_bytes=1 << 20, blocks=8, spin_ms=300)  # start-up self-test passes
            good = comm.bases
            comm.bases = [comm._own] * world  # a broken peer mapping: every "peer" is this rank's own region
            try:
                comm.self_test()
                out.append((cls.__name__, "not caught"))
            except CommFailure:
                out.append((cls.__name__, "caught"))
            comm.bases = good
            pdist.barrier()
            comm.close()
        q.put((rank, out))
        pdist.shutdown()
    except Exception as e:  # noqa: BLE001
        q.put((rank, repr(e)))


def test_ipc_collectives_self_test_catches_broken_mapping(gpu):
    """the IPC collectives check themselves against the process group at start-up, and a
    broken peer mapping is caught (CommFailure on every rank) instead of decoding garbage."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_selftest_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = _collect(q, procs, 300)
    for p in procs:
        p.join(timeout=60)
    want = [("CustomAllReduce", "caught"), ("CustomAllToAll", "caught")]
    assert res == {0: want, 1: want}, res
