"""Tensor parallelism (C3) on the GPU: a TP=2 Mixtral (heads and expert FFN columns split, row-parallel
outputs all-reduced) computes the same logits as TP=1.  Two ranks share the one GPU of the test box
(LWC_SHARE_ONE_GPU=1: gloo collectives staged through host memory); on an 8-GPU node the same code
runs over RCCL."""
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


def _tp_worker(rank, world, port, fp8, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), LWC_SHARE_ONE_GPU="1")
    try:
        from llm_weighted_consensus_amd.models.config import decoder_config
        from llm_weighted_consensus_amd.models.llama import KVCache
        from llm_weighted_consensus_amd.models.mixtral import MixtralModel
        from llm_weighted_consensus_amd.parallel import dist as pdist

        pdist.init_from_env("cuda")
        dev = torch.device("cuda", 0)
        m = MixtralModel(decoder_config("mixtral-tiny"), device=dev, seed=4, max_position=512, fp8=fp8,
                         tp_rank=rank, tp_size=world)
        g = torch.Generator().manual_seed(9)
        P = 29
        toks = torch.randint(0, m.cfg.vocab_size, (P,), generator=g).to(dev)
        cache = KVCache(m.cfg, 8, 16, dev)
        ar = torch.arange(P, dtype=torch.int32, device=dev)
        lg = m.prefill(toks.int(), ar, ar, torch.tensor([0, P], dtype=torch.int32, device=dev), P,
                       torch.tensor([P - 1], device=dev), cache)
        q.put((rank, lg[0].float().cpu().numpy()))
        pdist.shutdown()
    except Exception as e:  # noqa: BLE001
        q.put((rank, repr(e)))


@pytest.mark.parametrize("fp8", [False, True])
def test_mixtral_tp2_matches_tp1(gpu, fp8):
    from llm_weighted_consensus_amd.models.config import decoder_config
    from llm_weighted_consensus_amd.models.llama import KVCache
    from llm_weighted_consensus_amd.models.mixtral import MixtralModel

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_tp_worker, args=(r, 2, port, fp8, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = _collect(q, procs, 600)
    for p in procs:
        p.join(timeout=120)
    assert all(isinstance(v, torch.Tensor) for v in res.values()), res
    # TP=1 reference in this process
    m = MixtralModel(decoder_config("mixtral-tiny"), device=gpu, seed=4, max_position=512, fp8=fp8)
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
    assert torch.equal(res[0], res[1])  # ranks agree exactly (replicated after the all-reduce)


def _ep_worker(rank, world, port, fp8, mode, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), LWC_SHARE_ONE_GPU="1")
    try:
        from llm_weighted_consensus_amd.models.config import decoder_config
        from llm_weighted_consensus_amd.models.llama import KVCache
        from llm_weighted_consensus_amd.models.mixtral import MixtralModel
        from llm_weighted_consensus_amd.parallel import dist as pdist

        pdist.init_from_env("cuda")
        dev = torch.device("cuda", 0)
        m = MixtralModel(decoder_config("mixtral-tiny"), device=dev, seed=4, max_position=512, fp8=fp8,
                         ep_rank=rank, ep_size=world, ep_mode=mode, ep_capacity=64 if mode == "padded" else None)
        q.put((rank, _prefill_logits(m, dev, P=23 + 9 * rank, seed=rank).float().cpu().numpy()))  # each rank its own prompt
        pdist.shutdown()
    except Exception as e:  # noqa: BLE001
        q.put((rank, repr(e)))


def _prefill_logits(m, dev, P, seed):
    from llm_weighted_consensus_amd.models.llama import KVCache

    g = torch.Generator().manual_seed(100 + seed)
    toks = torch.randint(0, m.cfg.vocab_size, (P,), generator=g).to(dev)
    cache = KVCache(m.cfg, 8, 16, dev)
    ar = torch.arange(P, dtype=torch.int32, device=dev)
    return m.prefill(toks.int(), ar, ar, torch.tensor([0, P], dtype=torch.int32, device=dev), P,
                     torch.tensor([P - 1], device=dev), cache)[0].float().cpu()


@pytest.mark.parametrize("fp8,mode", [(False, "padded"), (True, "padded"), (False, "exact")])
def test_mixtral_ep2_matches_ep1(gpu, fp8, mode):
    """Expert parallelism (C4): two EP ranks (2 of mixtral-tiny's 4 experts each, full FFN width), each
    prefilling a DIFFERENT prompt, give the logits a single-rank model computes for that prompt."""
    from llm_weighted_consensus_amd.models.config import decoder_config
    from llm_weighted_consensus_amd.models.mixtral import MixtralModel

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ep_worker, args=(r, 2, port, fp8, mode, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = _collect(q, procs, 600)
    for p in procs:
        p.join(timeout=120)
    assert all(isinstance(v, torch.Tensor) for v in res.values()), res
    m = MixtralModel(decoder_config("mixtral-tiny"), device=gpu, seed=4, max_position=512, fp8=fp8)
    for r in range(2):
        ref = _prefill_logits(m, gpu, P=23 + 9 * r, seed=r)
        c = torch.nn.functional.cosine_similarity(res[r], ref, dim=0).item()
        assert c > 0.999, (r, c)


def _enc_worker(rank, world, port, fp8, q):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(rank), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port), LWC_SHARE_ONE_GPU="1")
    try:
        from llm_weighted_consensus_amd.models.config import decoder_config
        from llm_weighted_consensus_amd.models.tp import TPLlamaModel
        from llm_weighted_consensus_amd.parallel import dist as pdist

        pdist.init_from_env("cuda")
        dev = torch.device("cuda", 0)
        m = TPLlamaModel(decoder_config("llama-tiny"), device=dev, seed=6, max_position=512, fp8_dense=fp8,
                         tp_rank=rank, tp_size=world)  # no tp_comm: the process group's all-reduce (eager)
        q.put((rank, _encode(m, dev).numpy()))
        pdist.shutdown()
    except Exception as e:  # noqa: BLE001
        q.put((rank, repr(e)))


def _encode(m, dev):
    g = torch.Generator().manual_seed(21)
    lens = [17, 40, 9]
    toks = torch.randint(0, m.cfg.vocab_size, (sum(lens),), generator=g).to(dev)
    pos = torch.cat([torch.arange(n, dtype=torch.int32) for n in lens]).to(dev)
    cu = torch.tensor([0, 17, 57, 66], dtype=torch.int32, device=dev)
    return m.encode(toks.int(), pos, cu, max(lens)).float().cpu()


@pytest.mark.parametrize("fp8", [False, True])
def test_dense_tp2_encode_matches_tp1(gpu, fp8):
    """The config-5 embedder layout (bench_configs.py moe --embedder-par tp): a dense decoder used as an
    embedder at TP=2 (TPLlamaModel, process-group all-reduce) gives the TP=1 hidden states."""
    from llm_weighted_consensus_amd.models.config import decoder_config
    from llm_weighted_consensus_amd.models.llama import LlamaModel

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_enc_worker, args=(r, 2, port, fp8, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = _collect(q, procs, 600)
    for p in procs:
        p.join(timeout=120)
    assert all(isinstance(v, torch.Tensor) for v in res.values()), res
    ref = _encode(LlamaModel(decoder_config("llama-tiny"), device=gpu, seed=6, max_position=512, fp8_dense=fp8), gpu)
    for r in range(2):
        c = torch.nn.functional.cosine_similarity(res[r], ref, dim=1)
        assert c.min().item() > 0.99, (r, c.min().item())
    assert torch.equal(res[0], res[1])
