"""KV over-subscription with preemption by swapping (engine/engine.py): a pool three times too small for the
requests' max_tokens still completes every request, with exactly the tokens of an uninterrupted run."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def tiny(gpu):
    from llm_weighted_consensus_amd.models.config import decoder_config
    from llm_weighted_consensus_amd.models.llama import LlamaModel

    return LlamaModel(decoder_config("llama-tiny"), device=gpu, seed=0, max_position=1024)


def test_kv_oversubscription_swaps_and_matches_uninterrupted(tiny, gpu):
    from llm_weighted_consensus_amd import ops
    from llm_weighted_consensus_amd.engine.engine import LLMEngine
    from llm_weighted_consensus_amd.engine.sampling import SamplingParams
    from llm_weighted_consensus_amd.engine.tokenizer import ByteTokenizer
    from llm_weighted_consensus_amd.ops import gemm_plan

    # a batch-composition-invariant forward, so the two runs can be compared token for token: every GEMM
    # on gemm4w (a row's result does not depend on the other rows), split-K 1 and the wave-per-item
    # decode kernel for every batch, no cascade tiles
    old_mode, old_min = gemm_plan.MODE, ops.set_decode_wave_min_items(0)
    gemm_plan.MODE = "g4"
    try:
        tok = ByteTokenizer(tiny.cfg.vocab_size)
        prompts = [tok.encode(f"request {i}: " + "abcdefgh"[i] * (20 + 3 * i)) for i in range(6)]
        assert sum(len(p) for p in prompts) < 256
        sp = SamplingParams(temperature=0.9, top_p=0.95, max_tokens=160, ignore_eos=True, seed=11, top_logprobs=3,
                            logprobs=True)
        kw = dict(max_batch=64, max_model_len=512, prefix_sharing=False, decode_splits=1)
        ref = LLMEngine(tiny, tok, num_blocks=1024, kv_reserve_tokens=None, **kw)
        want = ref.generate(prompts, sp, n=4)
        assert ref.stats["preemptions"] == 0
        need = sum(-(-len(p) // 16) + 4 * -(-(len(p) + 160) // 16) for p in prompts)
        small_blocks = need // 3
        eng = LLMEngine(tiny, tok, num_blocks=small_blocks, kv_reserve_tokens=16, **kw)
        got = eng.generate(prompts, sp, n=4)
        assert eng.stats["preemptions"] > 0, eng.stats
        assert got == want
        assert eng.bm.num_free == small_blocks and not eng.swapped  # every block released, nothing parked
    finally:
        gemm_plan.MODE = old_mode
        ops.set_decode_wave_min_items(old_min)
