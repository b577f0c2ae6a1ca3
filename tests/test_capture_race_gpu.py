"""the K10b tally batcher (score/tally_batch.py) launches, allocates and reads back on a worker
thread while the engine thread may be capturing a decode graph for a bucket it meets for the first time.
The capture runs with capture_error_mode="thread_local" (engine/engine.py, _ensure_graph), so neither side
fails: every capture completes and every tally matches the host tally."""
import threading

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_tallies_concurrent_with_first_time_captures(gpu):
    import torch

    from llm_weighted_consensus_amd import _runtime as RT
    from llm_weighted_consensus_amd.engine.engine import LLMEngine
    from llm_weighted_consensus_amd.engine.sampling import SamplingParams
    from llm_weighted_consensus_amd.engine.tokenizer import ByteTokenizer
    from llm_weighted_consensus_amd.models.config import decoder_config
    from llm_weighted_consensus_amd.models.llama import LlamaModel
    from llm_weighted_consensus_amd.score.tally_batch import tally_many_gpu

    cfg = decoder_config("llama-tiny")
    model = LlamaModel(cfg, device=gpu, seed=0, max_position=512)
    tok = ByteTokenizer(cfg.vocab_size)
    eng = LLMEngine(model, tok, num_blocks=512, max_batch=64, max_model_len=256)
    rng = np.random.default_rng(0)
    items = []
    for _ in range(16):
        L, C = int(rng.integers(1, 9)), int(rng.integers(2, 6))
        votes = [list(rng.dirichlet(np.ones(C))) for _ in range(L)]
        items.append((votes, list(rng.uniform(0.1, 2.0, L)), C))
    want = [RT.tally(v, w, C) for v, w, C in items]
    stop, errors, rounds = threading.Event(), [], [0]
    side = torch.cuda.Stream(device=gpu)

    def tallies():
        try:
            with torch.cuda.device(gpu):
                while not stop.is_set():
                    got = tally_many_gpu(items, gpu, side)
                    for g, w in zip(got, want):
                        assert np.allclose(g.confidence, w.confidence, atol=1e-6)
                    rounds[0] += 1
        except BaseException as e:  # noqa: BLE001
            errors.append(e)

    t = threading.Thread(target=tallies)
    t.start()
    try:
        # batch sizes 1..48 walk through several decode buckets: each first visit captures a graph
        for n in (1, 3, 9, 17, 33, 48):
            out = eng.generate([tok.encode("race")], SamplingParams(temperature=0.7, max_tokens=4, ignore_eos=True,
                                                                   seed=n), n=n)
            assert len(out[0]) == n
    finally:
        stop.set()
        t.join(60)
    assert not errors, errors
    assert rounds[0] > 0 and len(eng.buckets) >= 3
