#!/usr/bin/env python3
"""Chunked-prefill cost (Llama-3-8B, random init): a prompt chunk after a cached head, through
 (a) the old path: model.prefill with the key range gathered from the paged cache per layer (kv_gather),
 (b) forward_mixed with no decode rows: the paged-KV prefill kernel reads the head through block tables,
 (c) forward_mixed with B decode rows riding along (one GEMM per projection over both),
 (d) the plain decode step of the same B rows alone (eager),
so (c) - (d) is what a chunk costs the running batch."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    from llm_weighted_consensus_amd.engine.engine import LLMEngine
    from llm_weighted_consensus_amd.engine.tokenizer import ByteTokenizer
    from llm_weighted_consensus_amd.models.config import decoder_config
    from llm_weighted_consensus_amd.models.llama import LlamaModel

    dev = torch.device("cuda", 0)
    m = LlamaModel(decoder_config(os.environ.get("ARCH", "llama-3-8b")), device=dev, seed=0, max_position=8192)
    tok = ByteTokenizer(m.cfg.vocab_size)
    eng = LLMEngine(m, tok, max_batch=256, max_model_len=8192, kv_memory_fraction=0.3)
    bm, BS = eng.bm, eng.block_size
    g = torch.Generator().manual_seed(0)
    i32 = lambda x: torch.tensor(np.asarray(x), dtype=torch.int32, device=dev)  # noqa: E731
    i64 = lambda x: torch.tensor(np.asarray(x), dtype=torch.int64, device=dev)  # noqa: E731
    from llm_weighted_consensus_amd._runtime import slots_range

    def timeit(fn, n=5):
        fn()
        torch.cuda.synchronize()
        ts = []
        for _ in range(n):
            t = time.perf_counter()
            fn()
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t)
        return sorted(ts)[n // 2] * 1e3

    # B running decode rows with 384-token contexts
    B = int(os.environ.get("DEC_B", "64"))
    for i in range(B):
        bm.add_sequence(1_000_000 + i, 384)
    dec_ids = [1_000_000 + i for i in range(B)]
    W = eng.width
    bt_d = np.zeros((B, W), np.int32)
    for i, sid in enumerate(dec_ids):
        t = list(bm.block_table(sid))
        bt_d[i, :len(t)] = t
    dec = {"block_tables": i32(bt_d), "ctx_lens": i32([384] * B), "splits": 4}
    dec_tok = i32(torch.randint(0, 100000, (B,), generator=g).numpy())
    dec_pos = i32([383] * B)
    dec_slot = i32([int(slots_range(bm, sid, 383, 1)[0]) for sid in dec_ids])

    def decode_only():
        return m.decode(dec_tok, dec_pos, dec_slot, dec["block_tables"], dec["ctx_lens"], eng.cache, num_splits=4)

    print(f"decode step alone, B={B}: {timeit(decode_only):7.2f} ms", flush=True)
    for n, per, start in [(1, 256, 0), (1, 512, 0), (1, 512, 1024), (1, 512, 3584), (4, 256, 256), (8, 64, 300)]:
        pids = [-(2_000_000 + k) for k in range(n)]
        prompts = [torch.randint(0, 100000, (start + per,), generator=g).tolist() for _ in range(n)]
        for pid, p in zip(pids, prompts):
            bm.add_sequence(pid, len(p))
        toks = i32(np.concatenate([p[start:] for p in prompts]))
        pos = i32(np.concatenate([np.arange(start, start + per)] * n))
        slots = i32(np.concatenate([slots_range(bm, pid, start, per) for pid in pids]))
        cu = i32(np.arange(n + 1) * per)
        last = i64(np.arange(1, n + 1) * per - 1)
        ks = np.concatenate([slots_range(bm, pid, 0, start + per) for pid in pids]).astype(np.int64)
        ctx = {"k_slots": i64(ks), "cu_k": i32(np.arange(n + 1) * (start + per)), "q_lens": [per] * n,
               "k_lens": [start + per] * n}
        wc = 2 * -(-(start + per) // 32)
        btc = np.zeros((n, wc), np.int32)
        for i, pid in enumerate(pids):
            t = list(bm.block_table(pid))
            btc[i, :len(t)] = t
        chunk = {"cu_q": cu, "block_tables": i32(btc), "k_lens": i32([start + per] * n), "max_q": per,
                 "lens": ([per] * n, [start + per] * n)}

        def gather():
            return m.prefill(toks, pos, slots, cu, per, last, eng.cache, ctx=ctx)

        def paged():
            return m.forward_mixed(toks, pos, slots, eng.cache, 0, None, chunk, last)

        mtok = torch.cat([dec_tok, toks])
        mpos = torch.cat([dec_pos, pos])
        mslot = torch.cat([dec_slot, slots])
        rows = i64(list(range(B)) + [B + x for x in (np.arange(1, n + 1) * per - 1)])

        def mixed():
            return m.forward_mixed(mtok, mpos, mslot, eng.cache, B, dec, chunk, rows)

        a, b, c = timeit(gather), timeit(paged), timeit(mixed)
        diff = (gather().float() - paged().float()).abs().max().item()
        print(f"chunk {n} x {per} after head {start}: gather {a:7.2f} ms  paged {b:7.2f} ms  "
              f"mixed(+{B} decode rows) {c:7.2f} ms  |logits gather - paged| {diff:.3g}", flush=True)
        for pid in pids:
            bm.free_sequence(pid)


if __name__ == "__main__":
    main()
