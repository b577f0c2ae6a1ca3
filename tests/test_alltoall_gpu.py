"""C4 equal-split all-to-all over IPC-mapped peer buffers (csrc/kernels/allreduce.hip ``alltoall_kernel``),
two ranks sharing the test box's GPU (handles exchanged over gloo; the data path is the kernel only):
chunks arrive byte-exact for several dtypes and ragged chunk sizes, across many calls (parity reuse) and
inside a replayed hipGraph; a rank that skips a call makes its peer poison the received chunks and raise
CommFailure within the spin bound; and an expert-parallel Mixtral (EP=2) whose dispatch / combine run
through it gives the single-rank logits, with its decode step hipGraph-safe."""
import os
import socket

import pytest
import numpy as np
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _env(rank, world, port):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), LWC_SHARE_ONE_GPU="1")


def _payload(src, dst, it, shape, dtype):
    """Rank src's chunk for rank dst at call it (deterministic, both ranks can rebuild it)."""
    g = torch.Generator().manual_seed(src * 1000 + dst * 100 + it)
    if dtype in (torch.int64, torch.int32):
        return torch.randint(-1000, 1000, shape, generator=g, dtype=dtype)
    if dtype == torch.float8_e4m3fn:  # built as bytes (no NaN pattern 0x7f / 0xff), viewed as e4m3 on the device
        return torch.randint(0, 127, shape, generator=g, dtype=torch.uint8)
    return torch.randn(shape, generator=g).to(dtype)


def _run(world, target, *args, timeout=300):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, q) + args) for r in range(world)]
    for p in procs:
        p.start()
    res = {}
    for _ in procs:
        r, v = q.get(timeout=timeout)
        res[r] = torch.from_numpy(v) if isinstance(v, np.ndarray) else v
    for p in procs:
        p.join(timeout=60)
    return res


def _a2a_worker(rank, world, port, q):
    _env(rank, world, port)
    try:
        from llm_weighted_consensus_amd.parallel import dist as pdist
        from llm_weighted_consensus_amd.parallel.allreduce import CustomAllToAll

        pdist.init_from_env("cuda")
        dev = torch.device("cuda", 0)
        comm = CustomAllToAll(device=dev, max_bytes=1 << 20, blocks=16)
        bad = []
        cases = [((3, 64), torch.bfloat16), ((2, 4), torch.int64), ((5,), torch.float32), ((128, 96), torch.bfloat16),
                 ((7, 33), torch.float8_e4m3fn), ((1000, 256), torch.bfloat16), ((1,), torch.int32)]
        for it in range(28):
            shape, dt = cases[it % len(cases)]
            inp = torch.stack([_payload(rank, d, it, shape, dt) for d in range(world)]).to(dev)
            if dt == torch.float8_e4m3fn:
                inp = inp.view(dt)
            out = torch.empty_like(inp)
            comm.all_to_all(out.view(world * shape[0], *shape[1:]), inp.view(world * shape[0], *shape[1:]))
            want = torch.stack([_payload(s, rank, it, shape, dt) for s in range(world)])
            got = out.cpu()
            if dt == torch.float8_e4m3fn:
                got = got.view(torch.uint8)
            if not torch.equal(got, want):
                bad.append(("eager", it, shape, str(dt)))
        # captured in a hipGraph, replayed with fresh inputs in the static buffer
        shape = (64, 128)
        s_in = torch.zeros(world * shape[0], shape[1], dtype=torch.bfloat16, device=dev)
        s_out = torch.zeros_like(s_in)
        st = torch.cuda.Stream(dev)
        st.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(st):
            comm.all_to_all(s_out, s_in)
        torch.cuda.current_stream(dev).wait_stream(st)
        pdist.barrier()
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            comm.all_to_all(s_out, s_in)
        for it in range(8):
            s_in.copy_(torch.cat([_payload(rank, d, 500 + it, shape, torch.bfloat16) for d in range(world)]).to(dev))
            graph.replay()
            torch.cuda.synchronize(dev)
            want = torch.cat([_payload(s, rank, 500 + it, shape, torch.bfloat16) for s in range(world)])
            if not torch.equal(s_out.cpu(), want):
                bad.append(("graph", it))
        comm.check()
        pdist.barrier()
        comm.close()
        q.put((rank, bad))
        pdist.shutdown()
    except Exception as e:  # noqa: BLE001
        q.put((rank, repr(e)))


def test_ipc_alltoall_two_ranks_one_gpu(gpu):
    assert _run(2, _a2a_worker) == {0: [], 1: []}


def _skip_worker(rank, world, port, q):
    _env(rank, world, port)
    try:
        from llm_weighted_consensus_amd.parallel import dist as pdist
        from llm_weighted_consensus_amd.parallel.allreduce import CommFailure, CustomAllToAll

        pdist.init_from_env("cuda")
        dev = torch.device("cuda", 0)
        comm = CustomAllToAll(device=dev, max_bytes=1 << 16, blocks=4, spin_ms=300)
        x = torch.ones(world * 16, 8, dtype=torch.bfloat16, device=dev)
        out = torch.zeros_like(x)
        comm.all_to_all(out, x)
        torch.cuda.synchronize(dev)
        ok_first = bool(torch.equal(out.cpu(), x.cpu())) and not int(comm.err.item())
        pdist.barrier()
        res = {"first": ok_first}
        if rank == 0:  # rank 1 never joins this call
            comm.all_to_all(out, x)
            comm.arm()
            torch.cuda.synchronize(dev)
            peer = out.view(world, 16, 8)[1]
            res["nan"] = bool(torch.isnan(peer.float()).all())
            res["own"] = bool(torch.equal(out.view(world, 16, 8)[0].cpu(), x.view(world, 16, 8)[0].cpu()))
            try:
                comm.poll()
                res["raised"] = False
            except CommFailure:
                res["raised"] = True
            # the EP layer over the same exchange — the poisoned per-expert counts (all-ones bytes
            # = -1) must not become out-of-range scatter / gather indices: the layer completes (NaN rows
            # from the missing peer), and the error word raises CommFailure instead of a device fault
            from llm_weighted_consensus_amd.parallel.expert import ExpertParallel

            ep = ExpertParallel(4, mode="padded", comm=comm)
            xs = torch.randn(8, 8, device=dev).to(torch.bfloat16)
            ro = torch.tensor([0, 2, 4, 6, 8], dtype=torch.int32, device=dev)
            y = ep.run(xs, ro, lambda xl, rol, sl: xl, capacity=8)
            comm.arm()
            torch.cuda.synchronize(dev)
            res["ep_shape"] = tuple(y.shape)
            try:
                comm.poll()
                res["ep_raised"] = False
            except CommFailure:
                res["ep_raised"] = True
        pdist.barrier()
        comm.close()
        q.put((rank, res))
        pdist.shutdown()
    except Exception as e:  # noqa: BLE001
        q.put((rank, repr(e)))


def test_ipc_alltoall_missing_peer_fails_loudly(gpu):
    res = _run(2, _skip_worker)
    assert res[1] == {"first": True}, res
    assert res[0] == {"first": True, "nan": True, "own": True, "raised": True, "ep_shape": (8, 8),
                      "ep_raised": True}, res


def _ep_worker(rank, world, port, q, fp8):
    _env(rank, world, port)
    try:
        from llm_weighted_consensus_amd.models.config import decoder_config
        from llm_weighted_consensus_amd.models.mixtral import MixtralModel
        from llm_weighted_consensus_amd.parallel import dist as pdist
        from llm_weighted_consensus_amd.parallel.allreduce import CustomAllToAll
        from tests.test_tp_gpu import _prefill_logits

        pdist.init_from_env("cuda")
        dev = torch.device("cuda", 0)
        comm = CustomAllToAll(device=dev, max_bytes=1 << 20, blocks=16)
        m = MixtralModel(decoder_config("mixtral-tiny"), device=dev, seed=4, max_position=512, fp8=fp8,
                         ep_rank=rank, ep_size=world, ep_mode="padded", ep_capacity=64, ep_comm=comm)
        assert m.graph_safe
        lg = _prefill_logits(m, dev, P=23 + 9 * rank, seed=rank)
        torch.cuda.synchronize(dev)
        comm.check()
        pdist.barrier()
        comm.close()
        q.put((rank, lg.float().cpu().numpy()))  # by value: a shared CPU tensor dies with its sender
        pdist.shutdown()
    except Exception as e:  # noqa: BLE001
        q.put((rank, repr(e)))


@pytest.mark.parametrize("fp8", [False, True])
def test_mixtral_ep2_through_ipc_alltoall(gpu, fp8):
    from llm_weighted_consensus_amd.models.config import decoder_config
    from llm_weighted_consensus_amd.models.mixtral import MixtralModel
    from tests.test_tp_gpu import _prefill_logits

    res = _run(2, _ep_worker, fp8, timeout=600)
    assert all(isinstance(v, torch.Tensor) for v in res.values()), res
    m = MixtralModel(decoder_config("mixtral-tiny"), device=gpu, seed=4, max_position=512, fp8=fp8)
    for r in range(2):
        ref = _prefill_logits(m, gpu, P=23 + 9 * r, seed=r)
        c = torch.nn.functional.cosine_similarity(res[r], ref, dim=0).item()
        assert c > 0.999, (r, c)


def _ep_prompts(rank):
    g = torch.Generator().manual_seed(300 + rank)
    return [torch.randint(0, 4000, (19,), generator=g).tolist() for _ in range(3)]  # same shapes on every rank


def _run_engine(model, prompts, dev):
    from llm_weighted_consensus_amd.engine.engine import LLMEngine
    from llm_weighted_consensus_amd.engine.sampling import SamplingParams
    from llm_weighted_consensus_amd.engine.tokenizer import ByteTokenizer

    cfg = model.cfg
    eng = LLMEngine(model, ByteTokenizer(cfg.vocab_size, cfg.bos_token_id, cfg.eos_token_id), max_batch=8,
                    max_model_len=256, kv_memory_fraction=0.04, use_graphs=model.graph_safe, cascade_min_batch=1 << 30)
    eng.collect_events = True
    sp = SamplingParams(temperature=0.0, max_tokens=10, ignore_eos=True, logprobs=True, top_logprobs=3)
    groups = [eng.add_request(p, sp, n=1) for p in prompts]
    trace = {}
    while eng.has_work():
        for ev in eng.step():
            trace.setdefault(ev.seq.group.id, []).append((ev.token_id, ev.logprob, dict(ev.top_logprobs)))
    return [trace[g.id] for g in groups]


def _ep_engine_worker(rank, world, port, q):
    _env(rank, world, port)
    try:
        from llm_weighted_consensus_amd.models.config import decoder_config
        from llm_weighted_consensus_amd.models.mixtral import MixtralModel
        from llm_weighted_consensus_amd.parallel import dist as pdist
        from llm_weighted_consensus_amd.parallel.allreduce import CustomAllToAll

        pdist.init_from_env("cuda")
        dev = torch.device("cuda", 0)
        comm = CustomAllToAll(device=dev, max_bytes=4 << 20, blocks=16, spin_ms=5000)
        m = MixtralModel(decoder_config("mixtral-tiny"), device=dev, seed=4, max_position=512, ep_rank=rank,
                         ep_size=world, ep_mode="padded", ep_capacity=128, ep_comm=comm)
        assert m.graph_safe
        toks = _run_engine(m, _ep_prompts(rank), dev)
        torch.cuda.synchronize(dev)
        comm.check()
        pdist.barrier()
        comm.close()
        q.put((rank, toks))
        pdist.shutdown()
    except Exception as e:  # noqa: BLE001
        q.put((rank, repr(e)))


def _ep1_engine_worker(rank, world, port, q):
    """The single-rank reference, in its own process too: the engine's graphs and KV pool stay out of the
    test runner's allocator (later kernel tests keep the memory layout they always had)."""
    _env(rank, world, port)
    try:
        from llm_weighted_consensus_amd.models.config import decoder_config
        from llm_weighted_consensus_amd.models.mixtral import MixtralModel

        dev = torch.device("cuda", 0)
        m = MixtralModel(decoder_config("mixtral-tiny"), device=dev, seed=4, max_position=512)
        q.put((rank, [_run_engine(m, _ep_prompts(r), dev) for r in range(2)]))
    except Exception as e:  # noqa: BLE001
        q.put((rank, repr(e)))


def test_ep2_engine_decode_graphs_match_ep1(gpu):
    """Two expert-parallel engines (mixtral-tiny, 2 of 4 experts each, different prompts of the same shapes)
    step in lockstep with their decode steps captured in hipGraphs — the device exchange (ep.hip kernels + IPC
    all-to-alls) inside the graphs — finish without a peer timeout, and generate greedily what a single-rank
    engine with every expert generates for the same prompts: every step's log-probability within 3e-2 of the
    reference up to the first differing token, and a differing token only at a near tie (both tokens in the
    other's top-3 within 3e-2: the grouped expert GEMM splits K by batch size, so the ranks' rounding can
    differ in the last bit).  A broken exchange moves logprobs far more than that at its first step."""
    res = _run(2, _ep_engine_worker, timeout=600)
    assert all(isinstance(v, list) for v in res.values()), res
    refs = _run(1, _ep1_engine_worker, timeout=600)[0]
    assert isinstance(refs, list), refs
    tol = 3e-2
    for r in range(2):
        ref = refs[r]
        assert [len(t) for t in res[r]] == [len(t) for t in ref] == [10] * 3
        for got, want in zip(res[r], ref):
            for step, ((tg, lg, topg), (tw, lw, topw)) in enumerate(zip(got, want)):
                assert abs(lg - lw) < tol, (r, step, lg, lw)
                if tg != tw:
                    assert tw in topg and abs(topg[tw] - lg) < tol, (r, step, tg, tw, topg)
                    assert tg in topw and abs(topw[tg] - lw) < tol, (r, step, tg, tw, topw)
                    break


def _ep_kernels_worker(rank, world, port, q, fp8):
    """ExpertParallel.run_combined (ep.hip: pack / unpack / back / combine around the IPC all-to-all) ==
    the torch-glue padded exchange + moe_combine, bitwise: both regroup the received rows in the same
    expert-major order, so the expert function sees identical inputs."""
    _env(rank, world, port)
    try:
        from llm_weighted_consensus_amd import ops
        from llm_weighted_consensus_amd.parallel import dist as pdist
        from llm_weighted_consensus_amd.parallel.allreduce import CustomAllToAll
        from llm_weighted_consensus_amd.parallel.expert import ExpertParallel

        pdist.init_from_env("cuda")
        dev = torch.device("cuda", 0)
        comm = CustomAllToAll(device=dev, max_bytes=4 << 20, blocks=16, spin_ms=5000)
        E, k, d = 8, 2, 256
        ep = ExpertParallel(E, mode="padded", comm=comm)
        g = torch.Generator(device=dev).manual_seed(40 + rank)
        T = 37 + 11 * rank
        h = torch.randn(T, d, device=dev, generator=g).to(torch.bfloat16)
        logits = torch.randn(T, E, device=dev, generator=g).to(torch.bfloat16)
        _ids, w, row_off, src, inv = ops.moe_route(logits, k)
        if fp8:
            x, xs = ops.quant_fp8_rows(h)
        else:
            x, xs = h, None

        def fn(xl, ro, sl):  # expert e scales its rows by (e + 1): checks the local segments too
            e = torch.searchsorted(ro[1:].long(), torch.arange(xl.shape[0], device=dev), right=True)
            v = xl.float() * (sl[:, None] if sl is not None else 1.0)
            return (v * (1 + rank * 8 + e)[:, None].float()).to(torch.bfloat16)

        out_k = ep.run_combined(x, row_off, src, inv, w, k, fn, x_scale=xs, capacity=128)
        idx = src.long()
        xsort = x.view(torch.uint8)[idx].view(torch.float8_e4m3fn) if fp8 else x[idx]
        y = ep.run(xsort, row_off, fn, x_scale=xs[idx] if fp8 else None, capacity=128)
        out_t = ops.moe_combine(y.contiguous(), inv, w, k)
        torch.cuda.synchronize(dev)
        comm.check()
        res = {"equal": bool(torch.equal(out_k, out_t)), "finite": bool(torch.isfinite(out_k.float()).all()),
               "nonzero": bool(out_k.float().abs().sum() > 0)}
        pdist.barrier()
        comm.close()
        q.put((rank, res))
        pdist.shutdown()
    except Exception as e:  # noqa: BLE001
        import traceback

        q.put((rank, repr(e) + traceback.format_exc()))


@pytest.mark.parametrize("fp8", [False, True])
def test_ep_device_exchange_matches_torch_glue(gpu, fp8):
    res = _run(2, _ep_kernels_worker, fp8, timeout=300)
    assert res == {r: {"equal": True, "finite": True, "nonzero": True} for r in range(2)}, res
