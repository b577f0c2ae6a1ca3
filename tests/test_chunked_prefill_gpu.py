"""Mixed chunked prefill (engine ``chunked_prefill``): each step is ONE forward over the running
sequences' decode rows and a token-budget chunk of the admitted prompts (earlier chunks read from the
paged cache by the paged-KV prefill kernel).  Chunked prompts give the same first-token logprobs and
greedy continuations as whole-prompt prefill; running sequences advance a token in every step while a
long (4k) prompt prefills; prompts sharing a head inside one admission still compute it once (prefix
cache); aborting a half-prefilled request releases everything."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def tiny(gpu):
    from llm_weighted_consensus_amd.models.config import decoder_config
    from llm_weighted_consensus_amd.models.llama import LlamaModel

    return LlamaModel(decoder_config("llama-tiny"), device=gpu, seed=0, max_position=1024)


def _run(tiny, prompts, chunk, prefix_caching=False, n=2):
    from llm_weighted_consensus_amd.engine.engine import LLMEngine
    from llm_weighted_consensus_amd.engine.sampling import SamplingParams
    from llm_weighted_consensus_amd.engine.tokenizer import ByteTokenizer

    tok = ByteTokenizer(tiny.cfg.vocab_size)
    eng = LLMEngine(tiny, tok, num_blocks=512, max_batch=32, max_model_len=768, chunked_prefill=chunk,
                    prefix_caching=prefix_caching)
    eng.collect_events = True
    sp = SamplingParams(temperature=0.0, max_tokens=10, ignore_eos=True, logprobs=True, top_logprobs=3)
    groups = [eng.add_request(p, sp, n=n) for p in prompts]
    trace = {}
    while eng.has_work():
        for ev in eng.step():  # events arrive in token order
            trace.setdefault((ev.seq.group.id, ev.seq.index), []).append((ev.token_id, ev.logprob, dict(ev.top_logprobs)))
    traces = [[trace[(g.id, s.index)] for s in g.seqs] for g in groups]
    assert eng.bm.num_free == 512 or prefix_caching  # prefix-cached blocks may stay resident (evictable)
    return traces, eng


def _assert_same_greedy(got, want, tol=2e-2):
    """Greedy continuations of two runs agree token for token, or up to a NEAR TIE: at the first
    differing step both runs' tokens are in the other's top-3 with log-probabilities within ``tol`` (decode
    rows that share a forward with prompt-chunk rows run other GEMM shapes: last-bit differences can flip
    an exact tie of the random-init model, never a clear winner — the prompt logits too: a mixed step's
    gate|up runs on the row-bucket planner's backend, so a first token can flip between two exactly tied
    logits).  The log-probabilities up to the divergence must match within ``tol``."""
    for tg, tw in zip(got, want):
        for a, b in zip(tg, tw):
            assert len(a) == len(b)
            for step, ((ta, la, topa), (tb, lb, topb)) in enumerate(zip(a, b)):
                assert abs(la - lb) < tol, (step, la, lb)
                if ta != tb:
                    assert tb in topa and abs(topa[tb] - la) < tol, (step, ta, tb, topa)
                    assert ta in topb and abs(topb[ta] - lb) < tol, (step, ta, tb, topb)
                    break


def test_chunked_matches_whole_prompt_prefill(tiny):
    g = torch.Generator().manual_seed(3)
    prompts = [torch.randint(0, 4000, (L,), generator=g).tolist() for L in (300, 17, 130, 64)]
    want, _ = _run(tiny, prompts, 0)
    for chunk in (48, 100):
        got, eng = _run(tiny, prompts, chunk)
        assert eng.stats["prefill_chunks"] >= sum(len(p) for p in prompts) // chunk
        assert eng.stats["mixed_steps"] == eng.stats["prefill_chunks"]
        _assert_same_greedy(got, want)


def test_decode_continues_while_a_long_prompt_prefills(tiny):
    from llm_weighted_consensus_amd.engine.engine import LLMEngine
    from llm_weighted_consensus_amd.engine.sampling import SamplingParams
    from llm_weighted_consensus_amd.engine.tokenizer import ByteTokenizer

    tok = ByteTokenizer(tiny.cfg.vocab_size)
    eng = LLMEngine(tiny, tok, num_blocks=512, max_batch=32, max_model_len=768, chunked_prefill=32)
    eng.collect_events = True
    sp = SamplingParams(temperature=0.0, max_tokens=40, ignore_eos=True)
    short = eng.add_request(tok.encode("hello"), sp, n=1)
    while not eng.running:
        eng.step()
    long_ = eng.add_request(list(range(256, 256 + 600)), SamplingParams(temperature=0.0, max_tokens=4, ignore_eos=True))
    overlapped = 0
    while eng.has_work():
        before = len(short.seqs[0].tokens)
        eng.step()
        if any(g is long_ for g in eng.prefilling) and len(short.seqs[0].tokens) > before:
            overlapped += 1
    assert overlapped >= 10  # 600 tokens / 32 per chunk: the short sequence decoded alongside the chunks
    assert len(long_.seqs[0].tokens) == 4 and len(short.seqs[0].tokens) == 40


def test_chunked_with_prefix_cache_and_shared_heads(tiny):
    g = torch.Generator().manual_seed(5)
    head = torch.randint(0, 4000, (200,), generator=g).tolist()
    prompts = [head + torch.randint(0, 4000, (k,), generator=g).tolist() for k in (9, 30, 3)]
    want, _ = _run(tiny, prompts, 0)
    got, eng = _run(tiny, prompts, 64, prefix_caching=True)
    assert eng.stats["prefix_cache_tokens"] >= 2 * 192  # the later prompts took the head from the cache
    _assert_same_greedy(got, want)


def test_abort_half_prefilled_request_releases_blocks(tiny):
    from llm_weighted_consensus_amd.engine.engine import LLMEngine
    from llm_weighted_consensus_amd.engine.sampling import SamplingParams
    from llm_weighted_consensus_amd.engine.tokenizer import ByteTokenizer

    tok = ByteTokenizer(tiny.cfg.vocab_size)
    eng = LLMEngine(tiny, tok, num_blocks=512, max_batch=32, max_model_len=768, chunked_prefill=32)
    grp = eng.add_request(list(range(300, 700)), SamplingParams(temperature=0.0, max_tokens=4, ignore_eos=True), n=3)
    eng.step()
    eng.step()
    assert eng.prefilling and 0 < grp.pf_pos < 400
    eng.abort(grp)
    assert not eng.has_work() and eng.bm.num_free == 512 and eng.free_blocks_unreserved == 512
    assert all(s.finished and s.finish_reason == "abort" for s in grp.seqs)


def test_decode_advances_every_step_during_4k_prompt(gpu):
    """A 4096-token prompt admitted next to running sequences: every one of its 16 chunks shares a forward
    with the decode rows (each running sequence gains a token per step), and its first tokens match a
    whole-prompt prefill of the same prompt."""
    from llm_weighted_consensus_amd.engine.engine import LLMEngine
    from llm_weighted_consensus_amd.engine.sampling import SamplingParams
    from llm_weighted_consensus_amd.engine.tokenizer import ByteTokenizer
    from llm_weighted_consensus_amd.models.config import decoder_config
    from llm_weighted_consensus_amd.models.llama import LlamaModel

    m = LlamaModel(decoder_config("llama-tiny"), device=gpu, seed=0, max_position=4608)
    tok = ByteTokenizer(m.cfg.vocab_size)
    g = torch.Generator().manual_seed(9)
    long_prompt = torch.randint(0, 4000, (4096,), generator=g).tolist()

    sp_long = SamplingParams(temperature=0.0, max_tokens=4, ignore_eos=True, logprobs=True, top_logprobs=3)
    whole = LLMEngine(m, tok, num_blocks=1024, max_batch=32, max_model_len=4352)
    whole.collect_events = True
    want = []
    gw = whole.add_request(long_prompt, sp_long)
    while whole.has_work():
        want += [(ev.token_id, ev.logprob, dict(ev.top_logprobs)) for ev in whole.step() if ev.seq.group is gw]

    eng = LLMEngine(m, tok, num_blocks=1024, max_batch=32, max_model_len=4352, chunked_prefill=256)
    sp = SamplingParams(temperature=0.0, max_tokens=64, ignore_eos=True)
    shorts = [eng.add_request(tok.encode(f"hello {i}"), sp, n=2) for i in range(3)]
    while len(eng.running) < 6:
        eng.step()
    eng.collect_events = True
    long_ = eng.add_request(long_prompt, sp_long)
    chunk_steps = advanced = 0
    got = []
    while eng.has_work():
        before = [len(s.tokens) for gr in shorts for s in gr.seqs]
        was_prefilling = bool(eng.prefilling) or bool(eng.waiting)
        got += [(ev.token_id, ev.logprob, dict(ev.top_logprobs)) for ev in eng.step() if ev.seq.group is long_]
        after = [len(s.tokens) for gr in shorts for s in gr.seqs]
        if was_prefilling and long_.pf_pos > 0:
            chunk_steps += 1
            advanced += all(b > a or len(s.tokens) >= 64 for a, b, s in
                            zip(before, after, [s for gr in shorts for s in gr.seqs]))
    assert eng.stats["mixed_steps"] >= 16
    assert chunk_steps >= 16 and advanced >= chunk_steps - 1, (chunk_steps, advanced)
    _assert_same_greedy([[got]], [[want]])
    assert all(len(s.tokens) == 64 for gr in shorts for s in gr.seqs)


@pytest.mark.parametrize("where", ["mixed", "prefill"])
def test_poisoned_collective_delivers_no_tokens(tiny, monkeypatch, where):
    """a tensor-parallel peer that never arrives poisons the forward (NaN activations) and sets
    the collective's error word.  The engine must read that word back for EVERY step whose tokens reach the
    host — the mixed chunked-prefill step and the whole-batch prefill as well as the graph decode step — and
    raise CommFailure before delivering any token sampled from the poisoned forward.  Here a fake comm
    stands in for the IPC all-reduce: the poisoned forward's logits put all mass on a sentinel token."""
    from llm_weighted_consensus_amd.engine.engine import LLMEngine
    from llm_weighted_consensus_amd.engine.sampling import SamplingParams
    from llm_weighted_consensus_amd.engine.tokenizer import ByteTokenizer
    from llm_weighted_consensus_amd.parallel.allreduce import CommFailure

    dev = tiny.device
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    host = torch.zeros(2, dtype=torch.int32).pin_memory()
    evs = [None, None]
    n_arm = [0]
    sentinel = tiny.cfg.vocab_size - 7

    def arm():
        i = n_arm[0] & 1
        n_arm[0] += 1
        host[i:i + 1].copy_(err, non_blocking=True)
        e = torch.cuda.Event()
        e.record()
        evs[i] = e

    def poll():
        for i in (0, 1):
            if evs[i] is not None and evs[i].query():
                evs[i] = None
                if int(host[i]):
                    raise CommFailure("fake peer never arrived")

    def poison(out):
        err.fill_(1)
        out = torch.full_like(out, -1e4)
        out[:, sentinel] = 1e4
        return out

    monkeypatch.setattr(tiny, "comm_arm", arm, raising=False)
    monkeypatch.setattr(tiny, "comm_poll", poll, raising=False)
    armed = {"on": False}
    if where == "mixed":
        orig = tiny.forward_mixed
        monkeypatch.setattr(tiny, "forward_mixed",
                            lambda *a, **k: poison(orig(*a, **k)) if armed["on"] else orig(*a, **k))
    else:
        orig = tiny.prefill
        monkeypatch.setattr(tiny, "prefill", lambda *a, **k: poison(orig(*a, **k)) if armed["on"] else orig(*a, **k))
    tok = ByteTokenizer(tiny.cfg.vocab_size)
    eng = LLMEngine(tiny, tok, num_blocks=512, max_batch=32, max_model_len=768,
                    chunked_prefill=64 if where == "mixed" else 0)
    eng.collect_events = True
    sp = SamplingParams(temperature=0.0, max_tokens=40, ignore_eos=True)
    g = torch.Generator().manual_seed(5)
    eng.add_request(torch.randint(0, 4096, (50,), generator=g).tolist(), sp, n=2)
    delivered = []
    for _ in range(6):  # the first request decodes in steady state
        delivered += eng.step()
    assert delivered
    armed["on"] = True
    eng.add_request(torch.randint(0, 4096, (90,), generator=g).tolist(), sp, n=2)
    with pytest.raises(CommFailure):
        for _ in range(8):
            delivered += eng.step()
    assert all(ev.token_id != sentinel for ev in delivered), "a token sampled from the poisoned forward was delivered"
