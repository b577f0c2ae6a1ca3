"""Chunked prefill mixed with decode (engine ``chunked_prefill``): prompts prefilled in token-budget chunks
(earlier chunks read back from the paged cache through the key-range prefill path) give the same
first-token logprobs and greedy continuations as whole-prompt prefill; running sequences keep decoding
while a long prompt is being prefilled; prompts sharing a head inside one admission still compute it
once (prefix cache); aborting a half-prefilled request releases everything."""
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
    first_lp = {}
    while eng.has_work():
        for ev in eng.step():
            first_lp.setdefault((ev.seq.group.id, ev.seq.index), ev.logprob)  # events arrive in token order
    toks = [[list(s.tokens) for s in g.seqs] for g in groups]
    lps = [[first_lp[(g.id, s.index)] for s in g.seqs] for g in groups]
    assert eng.bm.num_free == 512 or prefix_caching  # prefix-cached blocks may stay resident (evictable)
    return toks, lps, eng


def test_chunked_matches_whole_prompt_prefill(tiny):
    g = torch.Generator().manual_seed(3)
    prompts = [torch.randint(0, 4000, (L,), generator=g).tolist() for L in (300, 17, 130, 64)]
    want, lp_w, _ = _run(tiny, prompts, 0)
    for chunk in (48, 100):
        got, lp_g, eng = _run(tiny, prompts, chunk)
        assert eng.stats["prefill_chunks"] >= sum(len(p) for p in prompts) // chunk
        assert got == want, chunk
        for a, b in zip(lp_g, lp_w):
            assert max(abs(x - y) for x, y in zip(a, b)) < 2e-2, (a, b)


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
    want, lp_w, _ = _run(tiny, prompts, 0)
    got, lp_g, eng = _run(tiny, prompts, 64, prefix_caching=True)
    assert eng.stats["prefix_cache_tokens"] >= 2 * 192  # the later prompts took the head from the cache
    assert got == want
    for a, b in zip(lp_g, lp_w):
        assert max(abs(x - y) for x, y in zip(a, b)) < 2e-2


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
