#!/usr/bin/env python3
"""Config-5 MoE layer, expert-parallel vs tensor-parallel, per rank, on ONE GPU (for rocprofv3 --kernel-trace
--stats): what each layout costs a rank of a 2-GPU split of Mixtral-8x7B (fp8 experts) at the config-5
decode batch, exchange kernels and expert GEMMs timed as they would run on the node.

* EP=2 rank: T tokens of its own, route, the ep.hip exchange (pack -> all-to-all -> unpack -> experts ->
  back -> all-to-all -> combine) for 4 local experts at full FFN width; the exchange is a local copy here (a
  fake 2-rank transport: both "sources" are this rank's own chunks), so the kernels run on exactly the
  buffer shapes of the node and the xGMI transfer is priced separately from its bytes;
* TP=2 rank: the same 2T tokens of the replica (TP splits the columns, not the tokens), route, the grouped
  fp8 GEMMs over all 8 experts at half FFN width, combine; its all-reduce of [2T, d] bf16 per MoE layer (and
  one per attention block) is priced from its bytes.

    python scripts/ep_probe.py [T] [iters]
"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


class _LocalSwap:
    """A 2-rank all-to-all transport stand-in: out = inp (every chunk 'received' from itself)."""

    W = 2

    def all_to_all(self, out, inp):
        return out.copy_(inp)


def main():
    from llm_weighted_consensus_amd import ops
    from llm_weighted_consensus_amd.parallel.expert import ExpertParallel

    T = int(sys.argv[1]) if len(sys.argv) > 1 else 2048
    iters = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    dev = torch.device("cuda", 0)
    d, F, E, k = 4096, 14336, 8, 2
    g = torch.Generator(device=dev).manual_seed(0)

    def fp8_w(*shape):
        w = (torch.randn(*shape, device=dev, generator=g) * 0.02).to(torch.bfloat16)
        return ops.quant_fp8_weight(w)

    def experts(w13, s13, w2, s2):
        def fn(x, ro, sc, a_rows=None, rows=None):
            gu = ops.grouped_gemm(x, w13, ro, a_rows=a_rows, rows=rows, a_scale=sc, w_scale=s13)
            aq, as_ = ops.silu_mul_quant_fp8(gu)
            return ops.grouped_gemm(aq, w2, ro, a_scale=as_, w_scale=s2)
        return fn

    # ---- EP=2 rank: 4 experts, full width
    w13e, s13e = fp8_w(E // 2, 2 * F, d)
    w2e, s2e = fp8_w(E // 2, d, F)
    ep = ExpertParallel.__new__(ExpertParallel)
    ep.W, ep.E, ep.El, ep.group, ep.mode, ep.comm = 2, E, E // 2, None, "padded", _LocalSwap()
    h = torch.randn(T, d, device=dev, generator=g).to(torch.bfloat16)
    router = (torch.randn(E, d, device=dev, generator=g) * 0.1).to(torch.bfloat16)
    fn_ep = experts(w13e, s13e, w2e, s2e)

    def ep_layer():
        _ids, w, row_off, src, inv = ops.moe_route(torch.nn.functional.linear(h, router), k)
        hq, hs = ops.quant_fp8_rows(h)
        return ep.run_combined(hq, row_off, src, inv, w, k, fn_ep, x_scale=hs, capacity=T * k)

    # ---- TP=2 rank: all 8 experts, half width, the replica's 2T tokens
    w13t, s13t = fp8_w(E, F, d)   # gate|up halves of this rank: 2 * F/2 rows
    w2t, s2t = fp8_w(E, d, F // 2)
    h2 = torch.randn(2 * T, d, device=dev, generator=g).to(torch.bfloat16)
    fn_tp = experts(w13t, s13t, w2t, s2t)

    def tp_layer():
        _ids, w, row_off, src, inv = ops.moe_route(torch.nn.functional.linear(h2, router), k)
        hq, hs = ops.quant_fp8_rows(h2)
        y = fn_tp(hq, row_off, hs, a_rows=src, rows=2 * T * k)  # as MixtralModel._mlp: A rows gathered
        return ops.moe_combine(y, inv, w, k)

    out = {}
    for name, fn in (("ep2", ep_layer), ("tp2", tp_layer)):
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(iters):
            fn()
        torch.cuda.synchronize()
        out[name] = (time.perf_counter() - t0) / iters * 1e6
    ep_bytes = T * k // 2 * (d + 4) + T * k // 2 * d * 2  # dispatched e4m3 rows + scales, returned bf16 rows
    tp_bytes = 2 * T * d * 2  # one-shot all-reduce of [2T, d] bf16: the whole tensor crosses once per direction
    print(f"T={T}: MoE layer per rank  EP=2 {out['ep2']:8.1f} us (exchange over xGMI not included: "
          f"{ep_bytes / 1e6:.1f} MB per direction)  TP=2 {out['tp2']:8.1f} us (+ all-reduce "
          f"{tp_bytes / 1e6:.1f} MB per direction; attention adds one more all-reduce under TP, none under EP)",
          flush=True)


if __name__ == "__main__":
    main()
