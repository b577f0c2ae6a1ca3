"""Numerics of every hand-written gfx950 kernel against a plain PyTorch fp32 reference."""
import math

import pytest
import numpy as np
import torch

from tests import torch_ref as ref

pytestmark = pytest.mark.gpu


def _bf(*shape, dev, scale=1.0, g=None):
    return (torch.randn(*shape, device=dev, generator=g) * scale).to(torch.bfloat16)


def _close(a, b, atol, rtol=0.0):
    a, b = a.float(), b.float()
    err = (a - b).abs()
    lim = atol + rtol * b.abs()
    assert torch.isfinite(a).all(), "non-finite output"
    assert (err <= lim).all(), f"max err {err.max().item():.4g} (atol {atol}, rtol {rtol})"


@pytest.mark.parametrize("d,rows", [(384, 37), (1024, 37), (4096, 37), (2048, 301), (4096, 258), (8192, 256)])
@pytest.mark.parametrize("with_res", [False, True])
def test_rmsnorm(gpu, d, rows, with_res):
    """rows >= 256 at d in {2048, 4096, 8192} take the wave-per-row kernel (ragged last workgroup)."""
    from llm_weighted_consensus_amd import ops

    x = _bf(rows, d, dev=gpu)
    w = _bf(d, dev=gpu, scale=0.5) + 1
    if with_res:
        r = _bf(rows, d, dev=gpu)
        r0 = r.clone()
        y = ops.rmsnorm(x, w, 1e-5, residual=r)
        h = (x.float() + r0.float()).to(torch.bfloat16)
        _close(r, h, 1e-2, 1e-2)
        _close(y, ref.rmsnorm(h, w, 1e-5), 3e-2, 2e-2)
    else:
        y = ops.rmsnorm(x, w, 1e-5)
        _close(y, ref.rmsnorm(x, w, 1e-5), 3e-2, 2e-2)


@pytest.mark.parametrize("d", [256, 768, 1024])
def test_layernorm(gpu, d):
    from llm_weighted_consensus_amd import ops

    x, r = _bf(53, d, dev=gpu), _bf(53, d, dev=gpu)
    g, b = _bf(d, dev=gpu, scale=0.2) + 1, _bf(d, dev=gpu, scale=0.2)
    y = ops.layernorm(x, g, b, 1e-12, residual=r)
    _close(y, ref.layernorm(x.float() + r.float(), g, b, 1e-12), 4e-2, 2e-2)
    y2 = ops.layernorm(x, g, b, 1e-12)
    _close(y2, ref.layernorm(x, g, b, 1e-12), 4e-2, 2e-2)
    # pre-norm bias (the encoder's residual-fused projections), in place
    pb = _bf(d, dev=gpu)
    x3 = x.clone()
    ops.layernorm(x3, g, b, 1e-12, out=x3, pre_bias=pb)
    _close(x3, ref.layernorm(x.float() + pb.float(), g, b, 1e-12), 4e-2, 2e-2)


def test_silu_mul_embedding(gpu):
    from llm_weighted_consensus_amd import ops

    gu = _bf(19, 2 * 1024, dev=gpu)
    y = ops.silu_mul(gu)
    g, u = gu.float().chunk(2, -1)
    _close(y, torch.nn.functional.silu(g) * u, 2e-2, 2e-2)
    table = _bf(1000, 384, dev=gpu)
    ids = torch.randint(0, 1000, (77,), device=gpu, dtype=torch.int32)
    _close(ops.embedding(table, ids), table[ids.long()], 0)


def test_rope_kv_write(gpu):
    from llm_weighted_consensus_amd import ops
    from llm_weighted_consensus_amd.models.config import decoder_config
    from llm_weighted_consensus_amd.models.llama import rope_tables

    cfg = decoder_config("llama-tiny")
    Hq, Hkv, D, BS, NB = cfg.heads, cfg.kv_heads, cfg.head_dim, 16, 12
    cos, sin = rope_tables(cfg, gpu, 256)
    T = 21
    qkv = _bf(T, (Hq + 2 * Hkv) * D, dev=gpu)
    q0 = qkv.clone()
    pos = torch.randint(0, 200, (T,), device=gpu, dtype=torch.int32)
    slots = torch.randperm(NB * BS, device=gpu)[:T].to(torch.int32)
    kc = torch.zeros(NB, Hkv, BS, D, dtype=torch.bfloat16, device=gpu)
    vc = torch.zeros(NB, Hkv, BS // 4, D, 4, dtype=torch.bfloat16, device=gpu)
    q2 = qkv.clone()
    kc2, vc2 = kc.clone(), vc.clone()
    ops.rope_kv_write(qkv, pos, cos, sin, kc, vc, Hq, Hkv, D, slots=slots)
    # rope_q=False (pure decode steps): q untouched, k rotated and cached exactly as above; qkv's own k / v
    # columns are not written back (the decode kernels read k and v from the cache only)
    ops.rope_kv_write(q2, pos, cos, sin, kc2, vc2, Hq, Hkv, D, slots=slots, rope_q=False)
    assert torch.equal(q2, q0)
    assert torch.equal(kc2, kc) and torch.equal(vc2, vc)
    q_ref = ref.rope(q0[:, : Hq * D].view(T, Hq, D), pos, cos, sin)
    k_ref = ref.rope(q0[:, Hq * D:(Hq + Hkv) * D].view(T, Hkv, D), pos, cos, sin)
    v_ref = q0[:, (Hq + Hkv) * D:].view(T, Hkv, D)
    _close(qkv[:, : Hq * D].view(T, Hq, D), q_ref, 2e-2, 1e-2)
    _close(qkv[:, Hq * D:(Hq + Hkv) * D].view(T, Hkv, D), k_ref, 2e-2, 1e-2)
    blk, off = (slots // BS).long(), (slots % BS).long()
    _close(kc[blk, :, off, :], k_ref, 2e-2, 1e-2)
    _close(ops.v_token(vc, blk, off), v_ref, 0)
    # padding rows of a decode bucket (slot -1) on the k-only path: no cache write, k rotated in place, q as is
    sl3 = slots.clone()
    sl3[::3] = -1
    q3 = q0.clone()
    kc3, vc3 = torch.zeros_like(kc), torch.zeros_like(vc)
    ops.rope_kv_write(q3, pos, cos, sin, kc3, vc3, Hq, Hkv, D, slots=sl3, rope_q=False)
    pad, real = sl3 < 0, sl3 >= 0
    assert torch.equal(q3[:, : Hq * D], q0[:, : Hq * D]) and torch.equal(q3[real], q0[real])
    assert torch.equal(q3[pad, Hq * D:(Hq + Hkv) * D], qkv[pad, Hq * D:(Hq + Hkv) * D])
    b3, o3 = blk[real], off[real]
    assert torch.equal(kc3[b3, :, o3, :], kc[b3, :, o3, :])
    assert torch.equal(ops.v_token(vc3, b3, o3), ops.v_token(vc, b3, o3))
    assert int((kc3 != 0).sum()) == int((kc3[b3, :, o3, :] != 0).sum())


@pytest.fixture(params=["wg4", "wave"])
def decode_path(request, gpu):
    """Run a decode test through the 4-waves-per-sequence kernel and the wave-per-item kernel."""
    from llm_weighted_consensus_amd import ops

    old = ops.set_decode_wave_min_items(1 << 30 if request.param == "wg4" else 0)
    yield request.param
    ops.set_decode_wave_min_items(old)


def _q_rope(gpu, B):
    """(cos, sin, positions) for the decode kernels' load-time RoPE: q arrives un-rotated."""
    from llm_weighted_consensus_amd.models.config import decoder_config
    from llm_weighted_consensus_amd.models.llama import rope_tables

    cos, sin = rope_tables(decoder_config("llama-tiny"), gpu, 512)
    pos = torch.randint(0, 500, (B,), device=gpu, dtype=torch.int32)
    return cos, sin, pos


def _q_ref(q_full, b, Hq, D, rope):
    q = q_full[b, : Hq * D].view(1, Hq, D)
    if rope is None:
        return q
    cos, sin, pos = rope
    return ref.rope(q, pos[b:b + 1], cos, sin).to(torch.bfloat16)


@pytest.mark.parametrize("rope", [False, True])
@pytest.mark.parametrize("G,splits", [(4, 1), (4, 3), (1, 1), (8, 2)])
def test_paged_decode(gpu, G, splits, decode_path, rope):
    """rope=True: q un-rotated, rotated at load (pure decode steps; rope_kv_write rope_q=False)."""
    from llm_weighted_consensus_amd import ops

    torch.manual_seed(0)
    Hkv, D, BS, NB = 2, 128, 16, 64
    Hq = Hkv * G
    B = 5
    ctx = torch.tensor([1, 15, 16, 77, 200], dtype=torch.int32, device=gpu)
    width = 16
    kc = _bf(NB, Hkv, BS, D, dev=gpu)
    vc = _bf(NB, Hkv, BS // 4, D, 4, dev=gpu)
    # poison the cache beyond context with NaNs to check masking
    perm = torch.randperm(NB, device=gpu)
    bt = torch.zeros(B, width, dtype=torch.int32, device=gpu)
    k = 0
    for b in range(B):
        nb = (int(ctx[b]) + BS - 1) // BS
        bt[b, :nb] = perm[k:k + nb].to(torch.int32)
        k += nb
    for b in range(B):
        L = int(ctx[b])
        last = int(bt[b, (L - 1) // BS])
        o = L % BS
        if o:
            kc[last, :, o:, :] = float("nan")
            for tt in range(o, BS):
                ops.v_token(vc, last, tt).fill_(float("nan"))
    q_full = _bf(B, (Hq + 2 * Hkv) * D, dev=gpu)
    rp = _q_rope(gpu, B) if rope else None
    out = ops.paged_decode(q_full, kc, vc, bt, ctx, Hq, 1 / math.sqrt(D), num_splits=splits, rope=rp)
    for b in range(B):
        L = int(ctx[b])
        toks = torch.arange(L, device=gpu)
        blk = bt[b, toks // BS].long()
        kk = kc[blk, :, toks % BS, :]  # [L, Hkv, D]
        vv = ops.v_gather(vc, blk, toks % BS)  # [L, Hkv, D]
        q = _q_ref(q_full, b, Hq, D, rp)
        o = ref.attention(q, kk, vv, False, 1 / math.sqrt(D))[0]
        _close(out[b], o, 2e-2, 2e-2)


@pytest.mark.parametrize("rope", [False, True])
@pytest.mark.parametrize("G", [4, 2, 1, 8])
def test_paged_decode_cascade(gpu, G, rope):
    """One-launch cascade kernel (LDS-staged shared prompt + per-sequence suffix) == reference, over
    groups spanning several super-tiles, odd prefix block counts, plain rows and NaN-poisoned slots; a
    prompt of one LDS chunk takes the interleaved pass (its DMA overlapping the suffix loads, its pairs
    attended between suffix pairs), a longer one (19 blocks > 16) the chunked pass."""
    from llm_weighted_consensus_amd import ops
    from llm_weighted_consensus_amd.engine.engine import cascade_tiles

    torch.manual_seed(11)
    Hkv, D, BS = 2, 128, 16
    Hq = Hkv * G
    per = ops.cascade_rows_per_tile(G)
    # (count, prefix blocks): a group larger than one super-tile, an odd prefix, a singleton, a
    # group with an empty prefix (plain), a short group, and a prompt longer than one LDS chunk
    groups = [(per + 9, 2), (7, 5), (1, 4), (3, 0), (3, 3), (5, 19)]
    B = sum(c for c, _ in groups)
    width = 24
    NB = 4 + sum(p + c * (width - p) for c, p in groups)
    kc = _bf(NB, Hkv, BS, D, dev=gpu)
    vc = _bf(NB, Hkv, BS // 4, D, 4, dev=gpu)
    bt = torch.zeros(B, width, dtype=torch.int32)
    ctx = torch.zeros(B, dtype=torch.int32)
    nxt, row, runs = 0, 0, []
    g = torch.Generator().manual_seed(3)
    for c, pblk in groups:
        shared = torch.arange(nxt, nxt + pblk, dtype=torch.int32)
        nxt += pblk
        for _ in range(c):
            L = pblk * BS + int(torch.randint(1, (width - pblk) * BS, (1,), generator=g))
            nb = -(-L // BS)
            bt[row, :pblk] = shared
            bt[row, pblk:nb] = torch.arange(nxt, nxt + nb - pblk, dtype=torch.int32)
            nxt += nb - pblk
            ctx[row] = L
            row += 1
        runs.append((row - c, c, pblk))
    for b in range(B):  # poison slots past the context
        L = int(ctx[b])
        if L % BS:
            last = int(bt[b, (L - 1) // BS])
            kc[last, :, L % BS:, :] = float("nan")
            for tt in range(L % BS, BS):
                ops.v_token(vc, last, tt).fill_(float("nan"))
    tiles_np = np.zeros((-(-B // per) + len(groups) + 2, 3), dtype=np.int32)
    nt = cascade_tiles(runs, per, tiles_np)
    assert nt >= len(groups)
    bt, ctx = bt.to(gpu), ctx.to(gpu)
    tiles = torch.from_numpy(tiles_np).to(gpu)
    q_full = _bf(B, (Hq + 2 * Hkv) * D, dev=gpu)
    rp = _q_rope(gpu, B) if rope else None
    out = ops.paged_decode_cascade(q_full, kc, vc, bt, ctx, tiles, Hq, 1 / math.sqrt(D), rope=rp)
    assert torch.isfinite(out.float()).all()
    for b in range(B):
        L = int(ctx[b])
        toks = torch.arange(L, device=gpu)
        blk = bt[b, toks // BS].long()
        o = ref.attention(_q_ref(q_full, b, Hq, D, rp), kc[blk, :, toks % BS, :], ops.v_gather(vc, blk, toks % BS),
                          False, 1 / math.sqrt(D))[0]
        _close(out[b], o, 2e-2, 2e-2)
    # MX output (the fp8 o projection's operand): e4m3 rows + one e8m0 scale per 32 dims of a head, from the
    # same softmax state — dequantised, within e4m3 rounding of the bf16 output; every block's scale tight
    a = ops.paged_decode_cascade(q_full, kc, vc, bt, ctx, tiles, Hq, 1 / math.sqrt(D), rope=rp, mx=True)
    assert a.q.shape == (B, Hq * D) and a.mx.shape == (Hq * D // 128, B, 4)
    dims = torch.arange(Hq * D, device=gpu)
    deq = a.q.float() * torch.exp2(a.mx.float() - 127.0)[dims // 128, :, (dims % 128) // 32].t()
    want = out.float().reshape(B, -1)
    assert ((deq - want).norm() / want.norm()).item() < 4e-2
    bmax = a.q.float().abs().view(B, -1, 32).amax(-1)
    assert (bmax[bmax > 0] >= 224).all()


def test_paged_decode_cascade_short_tile_q_at_allocation_end(gpu):
    """Round-3 fault regression: a super-tile with fewer sequences than waves leaves waves that own no
    sequence; they must not read Q rows past the batch.  q is a view ending exactly at the end of its own
    2 MiB-multiple allocation (a caching-allocator segment of its own), B = 33 gives a last super-tile of one
    sequence, and the result must equal the reference (an out-of-bounds read past q faulted here)."""
    from llm_weighted_consensus_amd import ops
    from llm_weighted_consensus_amd.engine.engine import cascade_tiles

    G, Hkv, D, BS = 4, 8, 128, 16
    Hq = Hkv * G
    per = ops.cascade_rows_per_tile(G)
    B, pblk, width = per + 1, 3, 6
    NB = pblk + B * (width - pblk) + 2
    kc = _bf(NB, Hkv, BS, D, dev=gpu)
    vc = _bf(NB, Hkv, BS // 4, D, 4, dev=gpu)
    bt = torch.zeros(B, width, dtype=torch.int32)
    ctx = torch.zeros(B, dtype=torch.int32)
    nxt = pblk
    for b in range(B):
        L = pblk * BS + 5 + b % 30
        nb = -(-L // BS)
        bt[b, :pblk] = torch.arange(pblk, dtype=torch.int32)
        bt[b, pblk:nb] = torch.arange(nxt, nxt + nb - pblk, dtype=torch.int32)
        nxt += nb - pblk
        ctx[b] = L
    tiles_np = np.zeros((-(-B // per) + 3, 3), dtype=np.int32)
    cascade_tiles([(0, B, pblk)], per, tiles_np)
    assert tiles_np[1, 1] == 1  # the short last super-tile: one sequence, seven idle waves
    stride = (Hq + 2 * Hkv) * D
    seg = 2 << 20
    total = -(-(B * stride * 2) // seg) * seg  # bytes: a whole number of 2 MiB pages
    buf = torch.empty(total // 2, dtype=torch.bfloat16, device=gpu)
    q_full = buf[buf.numel() - B * stride:].view(B, stride)
    q_full.copy_(_bf(B, stride, dev=gpu))
    bt, ctx, tiles = bt.to(gpu), ctx.to(gpu), torch.from_numpy(tiles_np).to(gpu)
    out = ops.paged_decode_cascade(q_full, kc, vc, bt, ctx, tiles, Hq, 1 / math.sqrt(D))
    torch.cuda.synchronize()
    for b in (0, per - 1, per):
        L = int(ctx[b])
        toks = torch.arange(L, device=gpu)
        blk = bt[b, toks // BS].long()
        o = ref.attention(q_full[b, : Hq * D].view(1, Hq, D), kc[blk, :, toks % BS, :], ops.v_gather(vc, blk, toks % BS),
                          False, 1 / math.sqrt(D))[0]
        _close(out[b], o, 2e-2, 2e-2)


@pytest.mark.parametrize("D,Hq,Hkv,causal", [(128, 8, 2, True), (64, 4, 4, False), (128, 4, 4, False),
                                             (64, 8, 2, True), (32, 12, 12, False), (32, 4, 2, True)])
def test_prefill_attention(gpu, D, Hq, Hkv, causal):
    from llm_weighted_consensus_amd import ops

    torch.manual_seed(1)
    lens = [1, 17, 64, 100, 130]
    T = sum(lens)
    cu = torch.tensor([0] + list(torch.tensor(lens).cumsum(0)), dtype=torch.int32, device=gpu)
    row = (Hq + 2 * Hkv) * D
    qkv = _bf(T, row, dev=gpu)
    q, k, v = qkv[:, : Hq * D], qkv[:, Hq * D:(Hq + Hkv) * D], qkv[:, (Hq + Hkv) * D:]
    out = ops.prefill_attention(q, k, v, cu, max(lens), Hq, Hkv, D, 1 / math.sqrt(D), causal)
    for i, L in enumerate(lens):
        s0 = int(cu[i])
        o = ref.attention(q[s0:s0 + L].reshape(L, Hq, D), k[s0:s0 + L].reshape(L, Hkv, D),
                          v[s0:s0 + L].reshape(L, Hkv, D), causal, 1 / math.sqrt(D))
        _close(out[s0:s0 + L].view(L, Hq, D), o, 2e-2, 2e-2)


@pytest.mark.parametrize("Hq,Hkv,causal", [(8, 2, True), (4, 4, False)])
def test_prefill_attention_mx_matches_fp32(gpu, Hq, Hkv, causal):
    """MX epilogue of the prefill kernel (the fp8 o projection's operand, config 5's embedder / prefill):
    e4m3 rows + one e8m0 scale per 32 dims of a head.  Dequantised it is within e4m3 rounding of the fp32
    attention oracle (per-sequence relative Frobenius norm), every block's scale is tight (block amax lands
    in the top binade of e4m3), and the kept-row selection picks whole rows + their scales."""
    from llm_weighted_consensus_amd import ops

    torch.manual_seed(3)
    D = 128
    lens = [1, 17, 64, 100, 130]
    T = sum(lens)
    cu = torch.tensor([0] + list(torch.tensor(lens).cumsum(0)), dtype=torch.int32, device=gpu)
    qkv = _bf(T, (Hq + 2 * Hkv) * D, dev=gpu)
    q, k, v = qkv[:, : Hq * D], qkv[:, Hq * D:(Hq + Hkv) * D], qkv[:, (Hq + Hkv) * D:]
    a = ops.prefill_attention_mx(q, k, v, cu, max(lens), Hq, Hkv, 1 / math.sqrt(D), causal)
    assert a.q.shape == (T, Hq * D) and a.mx.shape == (Hq, T, 4)
    dims = torch.arange(Hq * D, device=gpu)
    deq = a.q.float() * torch.exp2(a.mx.float() - 127.0)[dims // 128, :, (dims % 128) // 32].t()
    for i, L in enumerate(lens):
        s0 = int(cu[i])
        o = ref.attention(q[s0:s0 + L].reshape(L, Hq, D).float(), k[s0:s0 + L].reshape(L, Hkv, D).float(),
                          v[s0:s0 + L].reshape(L, Hkv, D).float(), causal, 1 / math.sqrt(D)).reshape(L, -1)
        got = deq[s0:s0 + L]
        assert ((got - o).norm() / o.norm()).item() < 4e-2, i
    bmax = a.q.float().abs().view(T, -1, 32).amax(-1)
    assert (bmax[bmax > 0] >= 224).all()
    keep = torch.tensor([0, 17, 80, T - 1], device=gpu)
    sub = a.index_select(keep)
    assert torch.equal(sub.q.view(torch.uint8), a.q.view(torch.uint8)[keep])
    assert torch.equal(sub.mx, a.mx[:, keep])


@pytest.mark.parametrize("D,Hq,Hkv", [(128, 8, 2), (64, 4, 4)])
def test_prefill_attention_key_ranges(gpu, D, Hq, Hkv):
    """Cached-prefix prefill: each sequence's queries are the LAST rows of a longer key range (causal
    with that offset); k/v come from their own packed buffer."""
    from llm_weighted_consensus_amd import ops

    torch.manual_seed(2)
    ql, kl = [1, 17, 64, 70], [33, 17, 200, 118]
    cu_q = torch.tensor([0] + list(torch.tensor(ql).cumsum(0)), dtype=torch.int32, device=gpu)
    cu_k = torch.tensor([0] + list(torch.tensor(kl).cumsum(0)), dtype=torch.int32, device=gpu)
    q = _bf(sum(ql), Hq * D, dev=gpu)
    k, v = _bf(sum(kl), Hkv * D, dev=gpu), _bf(sum(kl), Hkv * D, dev=gpu)
    sc = 1 / math.sqrt(D)
    out = ops.prefill_attention(q, k, v, cu_q, max(ql), Hq, Hkv, D, sc, True, cu_seqlens_k=cu_k, lens=(ql, kl))
    for i, (a, b) in enumerate(zip(ql, kl)):
        q0, k0 = int(cu_q[i]), int(cu_k[i])
        o = ref.attention(q[q0:q0 + a].reshape(a, Hq, D), k[k0:k0 + b].reshape(b, Hkv, D),
                          v[k0:k0 + b].reshape(b, Hkv, D), True, sc)
        _close(out[q0:q0 + a].view(a, Hq, D), o, 2e-2, 2e-2)
    with pytest.raises(ValueError):  # a key range shorter than its queries is refused on the host
        ops.prefill_attention(q, k, v, cu_q, max(ql), Hq, Hkv, D, sc, True, cu_seqlens_k=cu_k, lens=(ql, [1, 1, 1, 1]))


@pytest.mark.parametrize("Hq,Hkv", [(8, 2), (4, 4), (32, 8)])
def test_prefill_attention_paged(gpu, Hq, Hkv):
    """Mixed chunked prefill: query chunks at the END of each key range, keys/values read from the paged
    cache through block tables (scattered blocks, ragged last block poisoned with NaN past k_len), q a
    strided view of a qkv row block."""
    from llm_weighted_consensus_amd import ops

    torch.manual_seed(5)
    D, BS = 128, 16
    ql, kl = [1, 17, 64, 70, 32, 5], [33, 17, 200, 118, 32, 300]
    n = len(ql)
    W = 2 * -(-max(kl) // 32)
    NB = 4 + sum(-(-k // BS) for k in kl)
    kc, vc = _bf(NB, Hkv, BS, D, dev=gpu), _bf(NB, Hkv, BS // 4, D, 4, dev=gpu)
    perm = torch.randperm(NB).to(torch.int32)
    bt = torch.zeros(n, W, dtype=torch.int32)
    used = 0
    for i, k in enumerate(kl):
        nb = -(-k // BS)
        bt[i, :nb] = perm[used:used + nb]
        used += nb
        if k % BS:  # slots past the key range hold garbage: the kernel must mask them
            last = int(bt[i, nb - 1])
            kc[last, :, k % BS:, :] = float("nan")
            for t in range(k % BS, BS):
                ops.v_token(vc, last, t).fill_(float("nan"))
    bt_d = bt.to(gpu)
    cu_q = torch.tensor([0] + list(np.cumsum(ql)), dtype=torch.int32, device=gpu)
    k_lens = torch.tensor(kl, dtype=torch.int32, device=gpu)
    qkv = _bf(sum(ql), (Hq + 2 * Hkv) * D, dev=gpu)
    sc = 1 / math.sqrt(D)
    out = ops.prefill_attention_paged(qkv, kc, vc, cu_q, bt_d, k_lens, max(ql), Hq, sc, lens=(ql, kl))
    for i, (a, b) in enumerate(zip(ql, kl)):
        toks = torch.arange(b, device=gpu)
        blk = bt_d[i, toks // BS].long()
        kk, vv = kc[blk, :, toks % BS, :], ops.v_gather(vc, blk, toks % BS)
        q0 = int(cu_q[i])
        o = ref.attention(qkv[q0:q0 + a, : Hq * D].reshape(a, Hq, D), kk, vv, True, sc)
        _close(out[q0:q0 + a].view(a, Hq, D), o, 2e-2, 2e-2)
    with pytest.raises(ValueError):  # block tables too narrow for a key range: refused on the host
        ops.prefill_attention_paged(qkv, kc, vc, cu_q, bt_d[:, :2], k_lens, max(ql), Hq, sc, lens=(ql, kl))


def _sample(logits, dev, n=None, **kw):
    from llm_weighted_consensus_amd import ops

    B = logits.shape[0]
    f = lambda v: torch.full((B,), float(v), device=dev)
    args = dict(temperature=f(kw.pop("temperature", 1.0)), top_p=f(kw.pop("top_p", 1.0)),
                top_k=torch.full((B,), int(kw.pop("top_k", 0)), dtype=torch.int32, device=dev),
                min_p=f(kw.pop("min_p", 0.0)), top_a=f(kw.pop("top_a", 0.0)),
                seeds=kw.pop("seeds", torch.arange(B, device=dev, dtype=torch.int64) * 7919 + 1),
                offsets=kw.pop("offsets", torch.zeros(B, device=dev, dtype=torch.int64)))
    args.update(kw)
    return ops.sample(logits, **args)


def test_sample_greedy_and_logprobs(gpu):
    torch.manual_seed(2)
    V = 128256
    logits = _bf(6, V, dev=gpu, scale=3.0)
    tok, lp, ids, tlp = _sample(logits, gpu, temperature=0.0, num_logprobs=20)
    lsm = torch.log_softmax(logits.float(), -1)
    assert torch.equal(tok.long(), logits.float().argmax(-1))
    _close(lp, lsm.gather(1, tok.long()[:, None])[:, 0], 2e-3, 1e-3)
    ref_lp, ref_ids = lsm.topk(20, dim=-1)
    _close(tlp, ref_lp, 2e-3, 1e-3)
    # ids equal up to ties
    _close(lsm.gather(1, ids.long()), ref_lp, 2e-3, 1e-3)


def test_sample_distribution_top_p_top_k(gpu):
    V = 4096
    B = 4096  # many rows of the same logits, different seeds -> empirical distribution
    base = torch.full((V,), -20.0, device=gpu)
    base[:6] = torch.tensor([2.0, 1.5, 1.0, 0.5, 0.0, -0.5], device=gpu)
    logits = base.to(torch.bfloat16).expand(B, V)
    p = torch.softmax(base.to(torch.bfloat16).float(), -1)
    for kw, keep in [({}, 6), ({"top_p": 0.8}, None), ({"top_k": 3}, 3), ({"min_p": 0.3}, None)]:
        tok, *_ = _sample(logits, gpu, **kw)
        cnt = torch.bincount(tok.long(), minlength=V).float() / B
        if "top_p" in kw:
            cum = p[:6].cumsum(0)
            keep = int((cum < kw["top_p"]).sum().item()) + 1
        if "min_p" in kw:
            keep = int((p[:6] >= kw["min_p"] * p[0]).sum().item())
        q = p[:keep] / p[:keep].sum()
        assert cnt[keep:].sum().item() == 0.0, kw
        assert (cnt[:keep] - q).abs().max().item() < 0.04, (kw, cnt[:keep], q)


@pytest.mark.parametrize("kw", [{}, {"top_p": 0.9}, {"top_k": 10}, {"top_p": 0.7, "top_k": 20}])
def test_sample_distribution_full_vocab(gpu, kw):
    """The Llama-3 vocabulary (V = 128256: the 16-slot instance the decode batch runs): 40 live tokens
    spread over different threads, slots and lanes of the row, the rest at -20; 4096 draws (one row per
    seed) against the fp32 torch distribution after temperature / top-p / top-k.  Exercises the packed
    u16 threshold masses, the top-k count search and the one-wave walk over the owner's registers."""
    V, B = 128256, 4096
    g = torch.Generator().manual_seed(8)
    idx = torch.randperm(V, generator=g)[:40].sort().values
    base = torch.full((V,), -20.0)
    base[idx] = torch.linspace(2.0, -1.0, 40)[torch.randperm(40, generator=g)]
    lg1 = base.to(torch.bfloat16).to(gpu)
    T = 0.8
    p = torch.softmax(lg1.float() / T, -1)
    order = p.argsort(descending=True)
    keep = torch.zeros(V, dtype=torch.bool, device=gpu)
    n = int(kw.get("top_k", 0)) or V
    keep[order[:n]] = True
    if "top_p" in kw:
        ps = p[order[:n]] / p[order[:n]].sum()
        m = int((ps.cumsum(0) < kw["top_p"]).sum().item()) + 1
        keep = torch.zeros_like(keep)
        keep[order[:m]] = True
    q = torch.where(keep, p, torch.zeros_like(p))
    q = q / q.sum()
    tok, *_ = _sample(lg1.expand(B, V), gpu, temperature=T, **kw)
    cnt = torch.bincount(tok.long(), minlength=V).float() / B
    assert cnt[~keep].sum().item() == 0.0, (kw, cnt.nonzero()[:8])
    assert (cnt - q).abs().max().item() < 0.03, (kw, (cnt - q).abs().max().item())


def test_sample_denormal_tail_mass(gpu):
    """The probability form of the row is fp16 (u = exp((y - ymax) / T) in [0, 1]): a flat tail of 128k tokens
    whose u lie in the fp16 SUBNORMAL range (here ~3.7e-6 each, ~4-5 % of the mass together) must keep its
    mass through the packed sums (v_dot2) and the walk, or no draw ever lands in it."""
    V, B = 128256, 4096
    g = torch.Generator().manual_seed(9)
    idx = torch.randperm(V, generator=g)[:40]
    base = torch.full((V,), -8.0)
    base[idx] = torch.linspace(2.0, -1.0, 40)
    lg1 = base.to(torch.bfloat16).to(gpu)
    T = 0.8
    p = torch.softmax(lg1.float() / T, -1)
    live = torch.zeros(V, dtype=torch.bool, device=gpu)
    live[idx.to(gpu)] = True
    u_tail = torch.exp(torch.tensor((-8.0 - 2.0) / T)).item()
    assert u_tail < 6.1e-5  # fp16 subnormal
    tok, *_ = _sample(lg1.expand(B, V), gpu, temperature=T)
    cnt = torch.bincount(tok.long(), minlength=V).float() / B
    tail_ref = p[~live].sum().item()
    assert 0.02 < tail_ref < 0.1
    assert abs(cnt[~live].sum().item() - tail_ref) < 0.015, (cnt[~live].sum().item(), tail_ref)
    assert (cnt[live] - p[live]).abs().max().item() < 0.03


def _penalised_ref(logits_bf16, counts, fpen, ppen, rpen):
    """fp32 torch reference of the sampler's logit processing (reference src/score/llm/mod.rs:39-72):
    for tokens already generated (count c > 0): y = y / rep if y > 0 else y * rep; y -= freq * c + pres;
    the kernel stores the processed row back as bf16 before sampling."""
    y = logits_bf16.float().clone()
    c = counts.float()
    seen = c > 0
    y = torch.where(seen & (y > 0), y / rpen, torch.where(seen, y * rpen, y))
    y = torch.where(seen, y - fpen * c - ppen, y)
    return y.to(torch.bfloat16).float()


@pytest.mark.parametrize("fpen,ppen,rpen", [(0.5, 0.0, 1.0), (0.0, 0.7, 1.0), (0.0, 0.0, 1.5), (0.3, 0.2, 1.3),
                                            (0.0, 0.0, 0.7)])
def test_sample_penalties_match_torch_distribution(gpu, fpen, ppen, rpen):
    """frequency / presence / repetition penalties: the empirical distribution of 4096 draws of one row
    (separate count rows, same content) matches softmax of the fp32 torch reference, and greedy picks its
    argmax on random rows."""
    V, B = 4096, 4096
    base = torch.full((V,), -20.0, device=gpu)
    base[:6] = torch.tensor([2.0, 1.5, 1.0, 0.5, 0.0, -0.5], device=gpu)
    lg1 = base.to(torch.bfloat16)
    c1 = torch.zeros(V, dtype=torch.int16, device=gpu)
    c1[0], c1[2], c1[4], c1[5] = 2, 1, 3, 1
    counts = c1.expand(B, V).contiguous()
    rows = torch.arange(B, dtype=torch.int32, device=gpu)
    f = lambda v: torch.full((B,), float(v), device=gpu)
    tok, *_ = _sample(lg1.expand(B, V), gpu, counts=counts, count_rows=rows, freq_pen=f(fpen), pres_pen=f(ppen),
                      rep_pen=f(rpen))
    q = torch.softmax(_penalised_ref(lg1, c1, fpen, ppen, rpen), -1)
    cnt = torch.bincount(tok.long(), minlength=V).float() / B
    assert (cnt - q).abs().max().item() < 0.04, (cnt[:6], q[:6])
    # every row counted exactly its own draw
    assert torch.equal(counts.long().sum(1) - c1.long().sum(), torch.ones(B, dtype=torch.long, device=gpu))
    # greedy on random rows with random counts = argmax of the reference
    torch.manual_seed(11)
    Bg = 64
    lg = _bf(Bg, V, dev=gpu, scale=2.0)
    cg = (torch.rand(Bg, V, device=gpu) < 0.05).to(torch.int16) * torch.randint(1, 4, (Bg, V), device=gpu).to(torch.int16)
    ref = _penalised_ref(lg, cg, fpen, ppen, rpen)
    fg = lambda v: torch.full((Bg,), float(v), device=gpu)
    tok, *_ = _sample(lg, gpu, temperature=0.0, counts=cg.clone(), count_rows=torch.arange(Bg, dtype=torch.int32, device=gpu),
                      freq_pen=fg(fpen), pres_pen=fg(ppen), rep_pen=fg(rpen))
    got = ref.gather(1, tok.long()[:, None])[:, 0]
    assert torch.equal(got, ref.max(-1).values)  # the chosen token is a maximiser (ties allowed)


@pytest.mark.parametrize("top_a", [0.5, 1.0, 2.0])
def test_sample_top_a_matches_torch(gpu, top_a):
    """top_a keeps tokens with p_i >= top_a * p_max^2 (renormalised): empirical vs the torch reference."""
    V, B = 4096, 4096
    base = torch.full((V,), -20.0, device=gpu)
    base[:6] = torch.tensor([2.0, 1.5, 1.0, 0.5, 0.0, -0.5], device=gpu)
    lg1 = base.to(torch.bfloat16)
    p = torch.softmax(lg1.float(), -1)
    keep = p >= top_a * p.max() ** 2
    keep[p.argmax()] = True
    q = torch.where(keep, p, torch.zeros_like(p))
    q = q / q.sum()
    tok, *_ = _sample(lg1.expand(B, V), gpu, top_a=top_a)
    cnt = torch.bincount(tok.long(), minlength=V).float() / B
    assert cnt[~keep].sum().item() == 0.0, (top_a, cnt[:6], q[:6])
    assert (cnt - q).abs().max().item() < 0.04, (top_a, cnt[:6], q[:6])


def test_sample_bias_mask_penalty(gpu):
    V = 4096
    B = 3
    logits = torch.zeros(B, V, device=gpu, dtype=torch.bfloat16)
    bias = torch.zeros(2, V, device=gpu)
    bias[0, 123] = 100.0
    bias[1, 7] = 100.0
    tok, *_ = _sample(logits, gpu, bias=bias, bias_rows=torch.tensor([0, 1, -1], dtype=torch.int32, device=gpu))
    assert tok[0].item() == 123 and tok[1].item() == 7
    mask = torch.zeros(1, V // 32, dtype=torch.int32, device=gpu)
    mask[0, 3] = 1 << 5  # only token 3*32+5 = 101 allowed
    tok, *_ = _sample(logits, gpu, mask=mask, mask_rows=torch.tensor([0, 0, -1], dtype=torch.int32, device=gpu))
    assert tok[0].item() == 101 and tok[1].item() == 101
    # repetition penalty pushes a dominant, already-generated token down
    lg = torch.zeros(1, V, device=gpu, dtype=torch.bfloat16)
    lg[0, 42] = 5.0
    counts = torch.zeros(1, V, dtype=torch.int16, device=gpu)
    counts[0, 42] = 3
    one = lambda v: torch.tensor([v], device=gpu, dtype=torch.float32)
    tok, *_ = _sample(lg, gpu, temperature=0.0, counts=counts, count_rows=torch.zeros(1, dtype=torch.int32, device=gpu),
                      freq_pen=one(2.0), pres_pen=one(0.0), rep_pen=one(1.0))
    assert tok[0].item() != 42
    assert counts[0, tok[0].long()].item() == 1  # the sampled token was counted


def test_sample_reproducible(gpu):
    logits = _bf(8, 32000, dev=gpu, scale=2.0)
    a, *_ = _sample(logits, gpu, top_p=0.9)
    b, *_ = _sample(logits, gpu, top_p=0.9)
    assert torch.equal(a, b)
    c, *_ = _sample(logits, gpu, top_p=0.9, offsets=torch.ones(8, dtype=torch.int64, device=gpu))
    assert not torch.equal(a, c)


def test_sample_skip_logprob(gpu):
    """need_logprob=False skips the raw log-sum-exp: same tokens as the full path for every sampling mode,
    NaN token logprob; the full path's logprob matches the fp32 log-softmax (fused into the sampling
    pass for unprocessed rows, into the bias pass for processed ones)."""
    torch.manual_seed(5)
    B, V = 16, 128256
    logits = _bf(B, V, dev=gpu, scale=2.0)
    lsm = torch.log_softmax(logits.float(), -1)
    bias = torch.zeros(1, V, device=gpu)
    bias[0, :64] = 3.0
    rows = torch.tensor([0, -1] * (B // 2), dtype=torch.int32, device=gpu)
    for kw in ({"temperature": 0.0}, {"top_p": 0.9, "temperature": 0.8}, {"top_k": 50}, {"bias": bias, "bias_rows": rows},
               {"temperature": 0.0, "bias": bias, "bias_rows": rows}):
        t1, lp1, *_ = _sample(logits, gpu, **kw)
        t0, lp0, *_ = _sample(logits, gpu, need_logprob=False, **kw)
        assert torch.equal(t0, t1), kw
        assert torch.isnan(lp0).all(), kw
        _close(lp1, lsm.gather(1, t1.long()[:, None])[:, 0], 2e-3, 1e-3)


def test_pool_cosine(gpu):
    from llm_weighted_consensus_amd import ops

    torch.manual_seed(3)
    lens = [3, 9, 1, 30]
    T, d = sum(lens), 1024
    h = _bf(T, d, dev=gpu)
    cu = torch.tensor([0, 3, 12, 13, 43], dtype=torch.int32, device=gpu)
    for mode in (ops.POOL_CLS, ops.POOL_MEAN, ops.POOL_LAST):
        of, ob = ops.pool_l2norm(h, cu, mode)
        for i in range(4):
            seg = h[int(cu[i]):int(cu[i + 1])].float()
            v = seg[0] if mode == 0 else (seg.mean(0) if mode == 1 else seg[-1])
            _close(of[i], v / v.norm(), 2e-3, 1e-2)
    R, n = 3, 37
    E = torch.nn.functional.normalize(torch.randn(R, n, d, device=gpu), dim=-1).to(torch.bfloat16)
    S, cen, w, best = ops.cosine_consensus(E, tau=0.1)
    Sr = E.float() @ E.float().transpose(1, 2)
    _close(S, Sr, 2e-3, 1e-2)
    cr = (Sr.sum(-1) - Sr.diagonal(dim1=1, dim2=2)) / (n - 1)
    _close(cen, cr, 2e-3, 1e-2)
    _close(w, torch.softmax(cr / 0.1, -1), 2e-3, 2e-2)
    assert torch.equal(best.long(), cr.argmax(-1))
    # the bench's deferred form: answer indices stay on the device until resolve()
    from llm_weighted_consensus_amd.embeddings.consensus import EmbeddingConsensus
    sc = EmbeddingConsensus(encoder=None, tau=0.1)
    lazy = sc.score_local(E, defer=True)
    assert isinstance(lazy.best, torch.Tensor) and lazy.resolve().best == sc.score_local(E).best == cr.argmax(-1).tolist()


def test_kv_block_copy(gpu):
    from llm_weighted_consensus_amd import ops

    cache = _bf(6, 10, 2 * 16 * 128, dev=gpu)
    ref_c = cache.clone()
    pairs = torch.tensor([[1, 4], [7, 2]], dtype=torch.int32, device=gpu)
    ops.kv_block_copy(cache, pairs)
    ref_c[:, 4] = ref_c[:, 1]
    ref_c[:, 2] = ref_c[:, 7]
    assert torch.equal(cache, ref_c)


@pytest.mark.parametrize("fp8", [False, True])
@pytest.mark.parametrize("splits", [None, 3])
def test_grouped_gemm(gpu, fp8, splits):
    """Grouped MFMA GEMM (MoE expert segments on the device, incl. an empty and a ragged group) vs
    per-group fp32 matmuls; fp8 e4m3fn operands with per-row / per-channel scales."""
    from llm_weighted_consensus_amd import ops

    torch.manual_seed(3)
    G, N, K = 4, 384, 256
    sizes = [130, 0, 7, 300]
    rows = sum(sizes)
    off = torch.tensor([0] + list(np.cumsum(sizes)), dtype=torch.int32, device=gpu)
    A = torch.randn(rows, K, device=gpu)
    W = torch.randn(G, N, K, device=gpu) * 0.05
    bias = (torch.randn(G, N, device=gpu) * 0.1).to(torch.bfloat16)
    if fp8:
        a_s = A.abs().amax(1).clamp(min=1e-6) / 448.0
        w_s = W.abs().amax(2).clamp(min=1e-6) / 448.0
        Aq = (A / a_s[:, None]).to(torch.float8_e4m3fn)
        Wq = (W / w_s[:, :, None]).to(torch.float8_e4m3fn)
        out = ops.grouped_gemm(Aq, Wq, off, a_scale=a_s.float().contiguous(), w_scale=w_s.float().contiguous(),
                               bias=bias, splits=splits)
        Ar = Aq.float() * a_s[:, None]
        Wr = Wq.float() * w_s[:, :, None]
    else:
        Ab, Wb = A.to(torch.bfloat16), W.to(torch.bfloat16)
        out = ops.grouped_gemm(Ab, Wb, off, bias=bias, splits=splits)
        Ar, Wr = Ab.float(), Wb.float()
    o = off.tolist()
    for g in range(G):
        if o[g + 1] == o[g]:
            continue
        ref_g = Ar[o[g]:o[g + 1]] @ Wr[g].t() + bias[g].float()
        _close(out[o[g]:o[g + 1]], ref_g, 2e-2, 2e-2)


@pytest.mark.parametrize("M,N,K,epi", [
    (512, 768, 256, "plain"), (300, 1024, 512, "res"), (4096, 4096, 4096, "plain"),  # data-parallel only
    (200, 8, 64, "plain"),                      # one partial tile, one K tile
    (3072, 6144, 4096, "plain"),                # 288 tiles: all stream-K, 1-2 workgroups per tile
    (1000, 4096, 14336, "res"),                 # 64 tiles: 4 workgroups per tile, 3 partials each
    (777, 2048, 1024, "swiglu"),                # shrunken grid, half-tile ranges
    (5000, 1280, 128, "plain"),                 # 2-iteration ranges, stream-K + 3 data-parallel rounds
    (3072, 28672, 4096, "swiglu")])             # gate_up: 320 stream-K tiles + 4 data-parallel rounds
def test_gemm8p(gpu, M, N, K, epi):
    """8-phase 256x256 MFMA GEMM with the stream-K tail (plain / residual / SwiGLU epilogue) vs an fp32
    matmul: ragged M and N tails, single-K-tile problems, tiles split over 1-4 workgroups.  Each case runs
    twice (the second launch depends on the first leaving the partial flags zero)."""
    from llm_weighted_consensus_amd import ops

    torch.manual_seed(M + N + K)
    A = torch.randn(M, K, device=gpu).to(torch.bfloat16)
    W = (torch.randn(N, K, device=gpu) / K ** 0.5).to(torch.bfloat16)
    ref = A.float() @ W.float().t()
    for _ in range(2):
        if epi == "swiglu":
            F = N // 2
            out = ops.gemm8p(A, ops.swiglu_interleave(W), swiglu=True)
            _close(out, torch.nn.functional.silu(ref[:, :F]) * ref[:, F:], 3e-2, 1e-2)
            continue
        R = torch.randn(M, N, device=gpu).to(torch.bfloat16) if epi == "res" else None
        out = ops.gemm8p(A, W, residual=R)
        _close(out, ref + (R.float() if R is not None else 0), 3e-2, 1e-2)
    torch.cuda.synchronize()
    assert int(ops.gemm8p_workspace(A.device)[1].abs().sum()) == 0, "stream-K flags left set"


@pytest.mark.parametrize("backend", ["g8", "g4", "g4n192", "blas"])
@pytest.mark.parametrize("M,N,K", [(520, 1024, 2048), (3072, 4096, 4096)])
def test_linear_add_inplace(gpu, backend, M, N, K):
    """gemm_plan.linear_add_: acc += A W^T in place (gemm8p's residual epilogue writing over its residual
    operand / hipBLASLt beta = 1) vs an fp32 matmul + add, repeated so the second call accumulates onto
    the first call's result."""
    from llm_weighted_consensus_amd.ops import gemm_plan

    torch.manual_seed(M + K)
    A = torch.randn(M, K, device=gpu).to(torch.bfloat16)
    W = (torch.randn(N, K, device=gpu) / K ** 0.5).to(torch.bfloat16)
    acc = torch.randn(M, N, device=gpu).to(torch.bfloat16)
    ref = acc.float()
    key = (M, N, K, "residual")
    old = gemm_plan._CHOICE.get(key)
    gemm_plan._CHOICE[key] = backend
    try:
        for _ in range(2):
            ref = ref + A.float() @ W.float().t()
            out = gemm_plan.linear_add_(A, W, acc)
            assert out.data_ptr() == acc.data_ptr()
            _close(acc, ref, 5e-2, 2e-2)
            ref = acc.float()  # the next call accumulates onto the rounded stream, as the model does
    finally:
        if old is None:
            gemm_plan._CHOICE.pop(key, None)
        else:
            gemm_plan._CHOICE[key] = old


def test_sample_constrained_logprobs(gpu):
    """mask_logprobs: a masked row's top-k logprobs are the restricted log-softmax over the allowed
    tokens (sum of their probabilities = 1), in the raw order of the allowed logits; unmasked rows and
    the default keep raw-distribution logprobs."""
    from llm_weighted_consensus_amd import ops

    V = 4096
    torch.manual_seed(2)
    logits = (torch.randn(2, V, device=gpu) * 3).to(torch.bfloat16)
    allowed = [65, 66, 67, 70, 84]  # 'A' 'B' 'C' 'F' 'T'
    mask = torch.zeros(1, V // 32, dtype=torch.int32, device=gpu)
    for a in allowed:
        mask[0, a // 32] |= 1 << (a % 32)
    rows = torch.tensor([0, -1], dtype=torch.int32, device=gpu)
    f = lambda v: torch.full((2,), float(v), device=gpu)
    args = (logits, f(1.0), f(1.0), torch.zeros(2, dtype=torch.int32, device=gpu), f(0), f(0),
            torch.arange(2, device=gpu, dtype=torch.int64), torch.zeros(2, device=gpu, dtype=torch.int64))
    tok, lp, ids, lps = ops.sample(*args, num_logprobs=8, mask=mask, mask_rows=rows, mask_logprobs=True)
    got = {int(i): float(v) for i, v in zip(ids[0].tolist(), lps[0].tolist()) if v > -1e30}
    assert set(got) == set(allowed)
    ref_lp = torch.log_softmax(logits[0, allowed].float(), 0)
    for a, r in zip(allowed, ref_lp.tolist()):
        assert abs(got[a] - r) < 2e-2
    raw = torch.log_softmax(logits[1].float(), 0)
    assert abs(lps[1, 0].item() - raw.max().item()) < 2e-2  # unmasked row: raw distribution
    _, _, ids2, lps2 = ops.sample(*args, num_logprobs=8, mask=mask, mask_rows=rows)
    assert abs(lps2[0, 0].item() - torch.log_softmax(logits[0].float(), 0).max().item()) < 2e-2


@pytest.mark.parametrize("fp8", [False, True])
def test_grouped_gemm_xcd_grouped_mapping(gpu, fp8):
    """Groups with several m-tiles each (rows >= 2*128*G) take the XCD-grouped 1-D grid; n-tile count
    not a multiple of 8, ragged groups, a gathered A (MoE dispatch) — vs fp32 matmuls."""
    from llm_weighted_consensus_amd import ops

    torch.manual_seed(5)
    G, N, K = 2, 3 * 128 + 16, 256
    sizes = [300, 433]
    rows = sum(sizes)
    off = torch.tensor([0] + list(np.cumsum(sizes)), dtype=torch.int32, device=gpu)
    A = torch.randn(rows + 11, K, device=gpu)
    src = torch.randperm(rows + 11, device=gpu)[:rows].to(torch.int32)
    W = torch.randn(G, N, K, device=gpu) * 0.05
    if fp8:
        a_s = A.abs().amax(1).clamp(min=1e-6) / 448.0
        w_s = W.abs().amax(2).clamp(min=1e-6) / 448.0
        Aq = (A / a_s[:, None]).to(torch.float8_e4m3fn)
        Wq = (W / w_s[:, :, None]).to(torch.float8_e4m3fn)
        out = ops.grouped_gemm(Aq, Wq, off, a_scale=a_s.float().contiguous(), w_scale=w_s.float().contiguous(),
                               a_rows=src, rows=rows)
        Ar, Wr = Aq.float() * a_s[:, None], Wq.float() * w_s[:, :, None]
    else:
        Ab, Wb = A.to(torch.bfloat16), W.to(torch.bfloat16)
        out = ops.grouped_gemm(Ab, Wb, off, a_rows=src, rows=rows)
        Ar, Wr = Ab.float(), Wb.float()
    o = off.tolist()
    Ag = Ar[src.long()]
    for g in range(G):
        _close(out[o[g]:o[g + 1]], Ag[o[g]:o[g + 1]] @ Wr[g].t(), 2e-2, 2e-2)


@pytest.mark.parametrize("F,block", [(14336, 0), (512, 32), (40000, 0)])
def test_silu_mul_quant_fp8_matches_unfused(gpu, F, block):
    """Fused SwiGLU + e4m3 row quantisation == quant_fp8_rows(silu_mul(x)) (register-held rows and the
    recompute path for rows wider than 16384)."""
    from llm_weighted_consensus_amd import ops

    torch.manual_seed(9)
    gu = (torch.randn(37, 2 * F, device=gpu) * 3).to(torch.bfloat16)
    q, s = ops.silu_mul_quant_fp8(gu, block=block)
    q_ref, s_ref = ops.quant_fp8_rows(ops.silu_mul(gu, block=block))
    torch.testing.assert_close(s, s_ref, rtol=0, atol=0)
    assert torch.equal(q.view(torch.uint8), q_ref.view(torch.uint8))


def test_kv_gather_matches_cache_layout(gpu):
    """Paged K / 4-token-interleaved V rows -> contiguous [n, Hkv*D] (cached-prefix prefill) vs torch
    indexing of the same cache."""
    from llm_weighted_consensus_amd import ops

    torch.manual_seed(4)
    NB, Hkv, BS, D = 9, 2, 16, 128
    kc = torch.randn(NB, Hkv, BS, D, device=gpu).to(torch.bfloat16)
    vc = torch.randn(NB, Hkv, BS // 4, D, 4, device=gpu).to(torch.bfloat16)
    slots = torch.tensor([0, 1, 2, 3, 5, 17, 31, 32, 70, 143, 100, 99], dtype=torch.int64, device=gpu)
    k, v = ops.kv_gather(kc, vc, slots)
    blk, off = slots // BS, slots % BS
    k_ref = kc.permute(0, 2, 1, 3)[blk, off].reshape(len(slots), -1)
    v_ref = vc.permute(0, 2, 4, 1, 3)[blk, off // 4, off % 4].reshape(len(slots), -1)
    assert torch.equal(k, k_ref) and torch.equal(v, v_ref)


@pytest.mark.parametrize("gather", [False, True])
def test_gemm8g_grouped_fp8_matches_reference(gpu, gather, monkeypatch):
    """8-phase grouped fp8 GEMM (csrc/kernels/gemm8g.hip): ragged expert groups (empty, < one tile, several
    tiles, a partial last tile), optional A-row gather, per-row / per-channel scales, vs an fp32 reference
    and vs the 128x128 grouped kernel; rows outside every group are never written."""
    from llm_weighted_consensus_amd import ops

    torch.manual_seed(11)
    G, N, K = 5, 640, 512
    sizes = [300, 0, 17, 700, 256]
    rows = sum(sizes)
    off = torch.tensor([0] + list(np.cumsum(sizes)), dtype=torch.int32, device=gpu)
    A = torch.randn(rows + 37, K, device=gpu)
    W = torch.randn(G, N, K, device=gpu) * 0.05
    a_s = A.abs().amax(1).clamp(min=1e-6) / 448.0
    w_s = W.abs().amax(2).clamp(min=1e-6) / 448.0
    Aq = (A / a_s[:, None]).to(torch.float8_e4m3fn)
    Wq = (W / w_s[:, :, None]).to(torch.float8_e4m3fn)
    a_rows = torch.randperm(rows + 37, device=gpu)[:rows].to(torch.int32) if gather else None
    out = torch.full((rows, N), float("nan"), dtype=torch.bfloat16, device=gpu)
    ops.kernels().gemm8g_fp8(Aq, Wq, out, off, -(-rows // 256) + G, a_rows, a_s.float().contiguous(),
                             w_s.float().contiguous(), 0, None, None)
    Ar = Aq.float() * a_s[:, None]
    if gather:
        Ar = Ar[a_rows.long()]
    Wr = Wq.float() * w_s[:, :, None]
    o = off.tolist()
    for g in range(G):
        if o[g + 1] > o[g]:
            _close(out[o[g]:o[g + 1]], Ar[o[g]:o[g + 1]] @ Wr[g].t(), 2e-2, 2e-2)
    assert not torch.isnan(out).any()
    # the routed path agrees with the 128x128 kernel on the same operands
    monkeypatch.setattr(ops, "MOE_GEMM", "classic")
    Ac, sc = (Aq, a_s) if gather else (Aq[:rows], a_s[:rows])
    classic = ops.grouped_gemm(Ac, Wq, off, a_scale=sc.float().contiguous(), w_scale=w_s.float().contiguous(),
                               a_rows=a_rows, rows=rows, splits=1, max_slots=-(-rows // 128) + G)
    _close(out, classic, 2e-2, 2e-2)


@pytest.mark.parametrize("sizes", [[300, 0, 77, 520], [100, 200, 129, 128]])
@pytest.mark.parametrize("gather", [False, True])
@pytest.mark.parametrize("moe_gemm", ["g8", "classic"])
def test_grouped_fp8_swiglu_matches_reference(gpu, gather, moe_gemm, sizes, monkeypatch):
    """MoE gate|up with the SwiGLU fused (gemm8g's epilogue; the 128x128 kernel + the SwiGLU pass when it
    takes the batch): gate / up rows interleaved in blocks of 32 per expert, ragged groups, A-row gather,
    per-row / per-channel scales -> silu(A Wg^T) * (A Wu^T) [rows, F] vs an fp32 reference."""
    from llm_weighted_consensus_amd import ops

    monkeypatch.setattr(ops, "MOE_GEMM", moe_gemm)
    torch.manual_seed(13)
    G, F, K = 4, 320, 512
    rows = sum(sizes)
    off = torch.tensor([0] + list(np.cumsum(sizes)), dtype=torch.int32, device=gpu)
    A = torch.randn(rows + 11, K, device=gpu)
    W = torch.randn(G, 2 * F, K, device=gpu) * 0.05       # [gate (F); up (F)] per expert
    Wi = torch.stack([ops.swiglu_interleave(W[g]) for g in range(G)])
    a_s = A.abs().amax(1).clamp(min=1e-6) / 448.0
    w_s = Wi.abs().amax(2).clamp(min=1e-6) / 448.0
    Aq = (A / a_s[:, None]).to(torch.float8_e4m3fn)
    Wq = (Wi / w_s[:, :, None]).to(torch.float8_e4m3fn)
    a_rows = torch.randperm(rows + 11, device=gpu)[:rows].to(torch.int32) if gather else None
    Ac, sc = (Aq, a_s) if gather else (Aq[:rows], a_s[:rows])
    out = ops.grouped_gemm(Ac, Wq, off, a_scale=sc.float().contiguous(), w_scale=w_s.float().contiguous(),
                           a_rows=a_rows, rows=rows, swiglu=True)
    assert out.shape == (rows, F)
    Ar = Aq.float() * a_s[:, None]
    if gather:
        Ar = Ar[a_rows.long()]
    Wr = Wq.float() * w_s[:, :, None]
    o = off.tolist()
    for g in range(G):
        if o[g + 1] > o[g]:
            y = Ar[o[g]:o[g + 1]] @ Wr[g].t()                        # interleaved gate / up columns
            yb = y.view(-1, F // 32, 2, 32)
            want = (torch.nn.functional.silu(yb[:, :, 0]) * yb[:, :, 1]).reshape(-1, F)
            _close(out[o[g]:o[g + 1]], want, 3e-2, 2e-2)


@pytest.mark.parametrize("T,E,k", [(1, 8, 2), (77, 8, 2), (4096, 8, 2), (300, 16, 4)])
def test_moe_route_matches_torch(gpu, T, E, k):
    """MoE routing (K11a, one workgroup, per-wave aggregated LDS counters / cursors): top-k ids and softmax
    weights as torch computes them; row_off the per-expert counts' prefix sum; src_row groups every routed
    (token, slot) under its expert; inv points each (token, slot) at its row."""
    from llm_weighted_consensus_amd import ops

    torch.manual_seed(29)
    logits = torch.randn(T, E, device=gpu).to(torch.bfloat16)
    ids, w, row_off, src, inv = ops.moe_route(logits, k)
    top, _ = logits.float().topk(k, dim=-1)
    tid = ids.long()  # (bf16 ties: the kernel takes the lower expert id, torch's order is unspecified)
    assert torch.equal(logits.float().gather(1, tid), top)
    assert all(len(set(r)) == k for r in tid.tolist())
    torch.testing.assert_close(w, top.softmax(-1), rtol=1e-5, atol=1e-6)
    cnt = torch.bincount(tid.flatten(), minlength=E)
    assert torch.equal(row_off.long().cpu(), torch.cat([torch.zeros(1, dtype=torch.long), cnt.cumsum(0).cpu()]))
    inv_l, src_l = inv.long(), src.long()
    tok = torch.arange(T, device=gpu).repeat_interleave(k)
    assert torch.equal(src_l[inv_l], tok)                      # row of (t, j) holds token t
    assert torch.equal(torch.sort(inv_l).values, torch.arange(T * k, device=gpu))  # a permutation
    ro = row_off.long().tolist()
    for e in range(E):                                         # expert e's rows are exactly its tokens
        got = torch.sort(src_l[ro[e]:ro[e + 1]]).values
        want = torch.sort(tok[tid.flatten() == e]).values
        assert torch.equal(got, want), e


def _check_permutation(gpu, ids, row_off, src, inv, T, E, k):
    tid = ids.long()
    cnt = torch.bincount(tid.flatten(), minlength=E)
    assert torch.equal(row_off.long().cpu(), torch.cat([torch.zeros(1, dtype=torch.long), cnt.cumsum(0).cpu()]))
    inv_l, src_l = inv.long(), src.long()
    tok = torch.arange(T, device=gpu).repeat_interleave(k)
    assert torch.equal(src_l[inv_l], tok)
    assert torch.equal(torch.sort(inv_l).values, torch.arange(T * k, device=gpu))
    ro = row_off.long().tolist()
    for e in range(E):
        got = torch.sort(src_l[ro[e]:ro[e + 1]]).values
        want = torch.sort(tok[tid.flatten() == e]).values
        assert torch.equal(got, want), e


@pytest.mark.parametrize("T,E,k,d,ld", [(1, 8, 2, 4096, 4096), (77, 8, 2, 4096, 4096), (4096, 8, 2, 4096, 4096),
                                        (300, 6, 2, 512, 520), (129, 16, 4, 1024, 1024), (50, 8, 3, 256, 256),
                                        # > 8192 routed rows: the permutation's re-reading path (prefill batches)
                                        (16500, 8, 2, 512, 512)])
def test_moe_router_matches_fp32(gpu, T, E, k, d, ld):
    """The router GEMV fused with the top-k (K11a moe_router: TPW tokens per wave, wave reduce-scatter of
    the E x TPW partial sums): logits within a bf16 rounding of the fp32 product (the kernel rounds them to
    bf16 as F.linear would); the experts are the top-k of the kernel's own logits and match the fp32 top-k
    wherever the fp32 logits are not within a rounding of a tie; weights = softmax of the selected logits;
    the permutation as in moe_route.  E = 6 / row stride 520 cover a padded expert set and strided rows."""
    from llm_weighted_consensus_amd import ops

    torch.manual_seed(31)
    hb = (torch.randn(T, ld, device=gpu) * 0.5).to(torch.bfloat16)
    h = hb[:, :d]
    router = (torch.randn(E, d, device=gpu) * 0.05).to(torch.bfloat16)
    ids, w, row_off, src, inv, lg = ops.moe_router(h, router, k, want_logits=True)
    ref = h.float() @ router.float().t()
    torch.testing.assert_close(lg.float(), ref, rtol=1.6e-2, atol=1e-3)
    tid = ids.long()
    lgf = lg.float()
    top, _ = lgf.topk(k, dim=-1)
    assert torch.equal(lgf.gather(1, tid), top)
    assert all(len(set(r)) == k for r in tid.tolist())
    torch.testing.assert_close(w, top.softmax(-1), rtol=1e-5, atol=1e-6)
    # vs the fp32 oracle: the chosen set equals fp32's top-k unless the k-th / (k+1)-th logits nearly tie
    rs, _ = ref.sort(-1, descending=True)
    clear = (rs[:, k - 1] - rs[:, k]) > 0.02 * rs.abs().max(-1).values.clamp_min(1e-3) if k < E else \
        torch.ones(T, dtype=torch.bool, device=gpu)
    ref_set = ref.topk(k, -1).indices.sort(-1).values
    assert torch.equal(tid.sort(-1).values[clear], ref_set[clear])
    assert clear.float().mean() > 0.8
    _check_permutation(gpu, ids, row_off, src, inv, T, E, k)
    # the unfused pair on the same bf16 logits routes identically
    ids2, w2, row_off2, _, _ = ops.moe_route(lg, k)
    assert torch.equal(ids2, ids) and torch.equal(row_off2, row_off)
    torch.testing.assert_close(w2, w, rtol=0, atol=0)


def _mx_scale_map(mx: torch.Tensor, K: int) -> torch.Tensor:
    """[K/128, rows, 4] e8m0 bytes -> per-element scales [rows, K]: element k of 128-slice t is in block
    (k % 128) // 32."""
    blk = (torch.arange(K, device=mx.device) % 128) // 32
    kt = torch.arange(K, device=mx.device) // 128
    return torch.exp2(mx.float() - 127.0)[kt, :, blk].t()


@pytest.mark.parametrize("sizes", [[300, 0, 77, 520], [1024, 1003, 990, 1079],
                                   # ragged tails of 65..128 rows (the wave rows' 128-row boundary)
                                   [100, 200, 129, 128]])
def test_grouped_fp8_mx_a_matches_reference(gpu, sizes):
    """The down-projection side of the MX expert FFN: gemm8g with A's e8m0 block scales applied by the
    block-scaled MFMA (the scale tile DMA'd beside A, one scale byte per lane and row fragment via op_sel)
    vs fp32 of the dequantised operands; ragged groups, an empty group, block scales spread over 2^-3..2^3
    (the MFMA sums a 128-term slice in its own internal format: terms many binades below the slice's largest
    lose low bits there, so the bound is relative to the output's scale, not per element)."""
    from llm_weighted_consensus_amd import ops

    torch.manual_seed(17)
    G, N, K = len(sizes), 512, 1024
    rows = sum(sizes)
    off = torch.tensor([0] + list(np.cumsum(sizes)), dtype=torch.int32, device=gpu)
    Aq = (torch.randn(rows, K, device=gpu) * 100).clamp(-448, 448).to(torch.float8_e4m3fn)
    mx = torch.randint(124, 131, (K // 128, rows, 4), dtype=torch.uint8, device=gpu)
    W = torch.randn(G, N, K, device=gpu) * 0.05
    w_s = W.abs().amax(2).clamp(min=1e-6) / 448.0
    Wq = (W / w_s[:, :, None]).to(torch.float8_e4m3fn)
    out = ops.grouped_gemm(Aq, Wq, off, w_scale=w_s.float().contiguous(), a_mx=mx)
    Ar = Aq.float() * _mx_scale_map(mx, K)
    Wr = Wq.float() * w_s[:, :, None]
    o = off.tolist()
    for g in range(G):
        if o[g + 1] > o[g]:
            ref_ = Ar[o[g]:o[g + 1]] @ Wr[g].t()
            _close(out[o[g]:o[g + 1]], ref_, 1e-2 * ref_.abs().max().item(), 2e-2)
            assert ((out[o[g]:o[g + 1]].float() - ref_).norm() / ref_.norm()).item() < 1e-2


@pytest.mark.parametrize("sizes", [[300, 0, 77, 520], [100, 200, 129, 128]])
@pytest.mark.parametrize("gather", [False, True])
def test_grouped_fp8_swiglu_mx_matches_reference(gpu, gather, sizes):
    """The gate|up side of the MX expert FFN: SwiGLU in gemm8g's epilogue, the activation written as e4m3
    with one e8m0 scale per (row, block of 32; one quad of lanes per block) vs fp32; then the
    whole middle (MX gate|up -> MX down) vs fp32 silu(gate) * up through the down projection."""
    from llm_weighted_consensus_amd import ops

    torch.manual_seed(19)
    G, F, K, D = 4, 512, 512, 256
    rows = sum(sizes)
    off = torch.tensor([0] + list(np.cumsum(sizes)), dtype=torch.int32, device=gpu)
    A = torch.randn(rows + 11, K, device=gpu)
    W = torch.randn(G, 2 * F, K, device=gpu) * 0.05
    Wi = torch.stack([ops.swiglu_interleave(W[g]) for g in range(G)])
    a_s = A.abs().amax(1).clamp(min=1e-6) / 448.0
    w_s = Wi.abs().amax(2).clamp(min=1e-6) / 448.0
    Aq = (A / a_s[:, None]).to(torch.float8_e4m3fn)
    Wq = (Wi / w_s[:, :, None]).to(torch.float8_e4m3fn)
    a_rows = torch.randperm(rows + 11, device=gpu)[:rows].to(torch.int32) if gather else None
    Ac, sc = (Aq, a_s) if gather else (Aq[:rows], a_s[:rows])
    q, mx = ops.grouped_gemm_swiglu_mx(Ac, Wq, off, sc.float().contiguous(), w_s.float().contiguous(),
                                       a_rows=a_rows, rows=rows)
    assert q.shape == (rows, F) and mx.shape == (2 * F // 256, rows, 4)
    Ar = Aq.float() * a_s[:, None]
    if gather:
        Ar = Ar[a_rows.long()]
    Wr = Wq.float() * w_s[:, :, None]
    want = torch.zeros(rows, F, device=gpu)
    o = off.tolist()
    for g in range(G):
        if o[g + 1] > o[g]:
            yb = (Ar[o[g]:o[g + 1]] @ Wr[g].t()).view(-1, F // 32, 2, 32)
            want[o[g]:o[g + 1]] = (torch.nn.functional.silu(yb[:, :, 0]) * yb[:, :, 1]).reshape(-1, F)
    got = q.float() * _mx_scale_map(mx, F)
    rel = (got - want).norm() / want.norm()
    assert rel < 4e-2, rel  # e4m3's 3 mantissa bits
    # every block's scale is tight: its largest |q| lands in e4m3's top binade [256, 448]
    bmax = q.float().abs().view(rows, F // 128, 4, 32).amax(-1)  # [rows, F/128, 4]
    live = bmax > 0
    assert (bmax[live] >= 224).all()
    # down projection from the MX activation vs fp32
    W2 = torch.randn(G, D, F, device=gpu) * 0.05
    s2 = W2.abs().amax(2).clamp(min=1e-6) / 448.0
    W2q = (W2 / s2[:, :, None]).to(torch.float8_e4m3fn)
    y = ops.grouped_gemm(q, W2q, off, w_scale=s2.float().contiguous(), a_mx=mx)
    W2r = W2q.float() * s2[:, :, None]
    for g in range(G):
        if o[g + 1] > o[g]:
            ref_ = want[o[g]:o[g + 1]] @ W2r[g].t()
            rel = (y[o[g]:o[g + 1]].float() - ref_).norm() / ref_.norm()
            assert rel < 5e-2, (g, rel)


@pytest.mark.parametrize("d,rows", [(4096, 1), (4096, 301), (2048, 64), (8192, 257), (1024, 33)])
@pytest.mark.parametrize("with_res", [False, True])
def test_rmsnorm_quant_fp8_fused(gpu, d, rows, with_res):
    """RMSNorm with the per-row e4m3 quantisation fused (K1 + K11e): the e4m3 rows and scales are bitwise
    quant_fp8_rows of the kernel's own bf16 output (same rounding before the row max); that output and the
    residual update equal the plain RMSNorm (bitwise where both take the wave-per-row kernel, rows >= 256;
    the workgroup-per-row kernel of smaller batches reduces in another order); d = 1024 takes the
    two-kernel fallback."""
    from llm_weighted_consensus_amd import ops

    x = _bf(rows, d, dev=gpu)
    w = _bf(d, dev=gpu, scale=0.5) + 1
    r = _bf(rows, d, dev=gpu) if with_res else None
    r2 = r.clone() if with_res else None
    y = ops.rmsnorm(x, w, 1e-5, residual=r)
    a = ops.rmsnorm_quant_fp8(x, w, 1e-5, residual=r2, keep_bf16=True)
    q_ref, s_ref = ops.quant_fp8_rows(a.bf16)
    assert torch.equal(a.q.view(torch.uint8), q_ref.view(torch.uint8))
    assert torch.equal(a.s, s_ref)
    if rows >= 256 or d == 1024:
        assert torch.equal(a.bf16, y)
    else:
        _close(a.bf16, y, 2e-2, 1e-2)
    if with_res:
        assert torch.equal(r2, r)
    # dequantised rows track the fp32 reference within e4m3 precision
    deq = a.q.float() * a.s[:, None]
    _close(deq, y.float(), 0.07 * a.s.max().item() * 448 / 16 + 1e-3, 0.07)


@pytest.mark.parametrize("M,N,K", [(1, 512, 256), (255, 640, 512), (2048, 6144, 4096), (4097, 1024, 1024)])
def test_dense_fp8_gemm8g(gpu, M, N, K, monkeypatch):
    """Dense fp8 projections on the hand-written 8-phase core (gemm8g, no row table): per-row activation and
    per-channel weight scales vs an fp32 reference of the dequantised operands, and vs hipBLASLt's
    row-scaled fp8 GEMM; the planner path (linear_fp8) forced to each backend agrees."""
    from llm_weighted_consensus_amd import ops

    torch.manual_seed(5)
    x = torch.randn(M, K, device=gpu).to(torch.bfloat16)
    w = ops.Fp8Weight(torch.randn(N, K, device=gpu).to(torch.bfloat16) * 0.05)
    xq, xs = ops.quant_fp8_rows(x)
    out = ops.gemm8g_dense(xq, xs, w)
    ref_ = (xq.float() * xs[:, None]) @ (w.q.float() * w.s.view(-1, 1)).t()
    _close(out, ref_, 2e-2, 2e-2)
    blas = ops._fp8_blas(xq, xs, w)
    _close(out, blas, 2e-2, 2e-2)
    monkeypatch.setattr(ops, "FP8_GEMM", "g8g")
    _close(ops.linear_fp8(x, w), out, 1e-6)
    monkeypatch.setattr(ops, "FP8_GEMM", "auto")
    monkeypatch.setattr(ops, "FP8_CHOICE", {})
    _close(ops.linear_fp8(x, w), out, 2e-2, 2e-2)
    assert len(ops.FP8_CHOICE) == 1


def test_dense_fp8_gemm8g_row_blocks(gpu, monkeypatch):
    """A beyond gemm8g's 32-bit buffer range goes as row blocks, one launch each (the embedder's ~0.5 M-row
    prefill): with the span shrunk to force five blocks (the last one ragged) the result is unchanged."""
    from llm_weighted_consensus_amd import ops

    torch.manual_seed(6)
    M, N, K = 1200, 512, 256
    x = torch.randn(M, K, device=gpu).to(torch.bfloat16)
    w = ops.Fp8Weight(torch.randn(N, K, device=gpu).to(torch.bfloat16) * 0.05)
    xq, xs = ops.quant_fp8_rows(x)
    whole = ops.gemm8g_dense(xq, xs, w)
    monkeypatch.setattr(ops, "G8G_SPAN", 256 * K + 1)
    blocks = ops.gemm8g_dense(xq, xs, w)
    assert torch.equal(whole, blocks)
    ref_ = (xq.float() * xs[:, None]) @ (w.q.float() * w.s.view(-1, 1)).t()
    _close(blocks, ref_, 2e-2, 2e-2)


def test_dense_fp8_mlp_mx(gpu, monkeypatch):
    """The dense fp8 MLP middle in MX form (config 5's embedder prefill): gemm8g dense SwiGLU epilogue writing
    e4m3 + e8m0 block scales, the down projection applying them — with the row-block split forced (span shrunk)
    so the scale planes are passed as row-range views — vs fp32 silu(gate) * up through the down projection."""
    from llm_weighted_consensus_amd import ops

    torch.manual_seed(23)
    M, F, K, D = 1200, 512, 256, 384
    x = torch.randn(M, K, device=gpu).to(torch.bfloat16)
    wgu = ops.Fp8Weight(ops.swiglu_interleave(torch.randn(2 * F, K, device=gpu).to(torch.bfloat16) * 0.05))
    wd = ops.Fp8Weight(torch.randn(D, F, device=gpu).to(torch.bfloat16) * 0.05)
    monkeypatch.setattr(ops, "DENSE_MX_MIN_ROWS", 1)
    assert ops.dense_mx_ok(x, wgu, wd, 32)
    q1, mx1 = ops.linear_fp8_swiglu_mx(x, wgu)
    y1 = ops.linear_fp8_mx(q1, mx1, wd)
    monkeypatch.setattr(ops, "G8G_SPAN", 256 * F + 1)  # row blocks of 256: five launches per projection
    q2, mx2 = ops.linear_fp8_swiglu_mx(x, wgu)
    y2 = ops.linear_fp8_mx(q2, mx2, wd)
    assert torch.equal(q1.view(torch.uint8), q2.view(torch.uint8)) and torch.equal(mx1, mx2) and torch.equal(y1, y2)
    xq, xs = ops.quant_fp8_rows(x)
    gu = ((xq.float() * xs[:, None]) @ (wgu.q.float() * wgu.s.view(-1, 1)).t()).view(M, -1, 2, 32)
    act = torch.nn.functional.silu(gu[:, :, 0].reshape(M, -1)) * gu[:, :, 1].reshape(M, -1)
    got = q1.float() * _mx_scale_map(mx1, F)
    assert ((got - act).norm() / act.norm()).item() < 4e-2
    ref_ = act @ (wd.q.float() * wd.s.view(-1, 1)).t()
    assert ((y1.float() - ref_).norm() / ref_.norm()).item() < 5e-2


@pytest.mark.parametrize("M,N,K", [(1000, 1024, 512), (4096, 2048, 1024)])
@pytest.mark.parametrize("backend", ["g8g", "blas", "auto"])
def test_dense_fp8_swiglu(gpu, M, N, K, backend, monkeypatch):
    """The dense fp8 MLP middle (ops.linear_fp8_swiglu): gate|up rows interleaved in blocks of 32, fp8 GEMM,
    SwiGLU (gemm8g's epilogue, or hipBLASLt + the fused silu_mul_quant pass), per-row e4m3 quantisation —
    the dequantised activation vs fp32 silu(gate) * up of the dequantised operands."""
    from llm_weighted_consensus_amd import ops

    torch.manual_seed(7)
    x = torch.randn(M, K, device=gpu).to(torch.bfloat16)
    wgu = torch.randn(N, K, device=gpu).to(torch.bfloat16) * 0.05
    w = ops.Fp8Weight(ops.swiglu_interleave(wgu))
    monkeypatch.setattr(ops, "FP8_GEMM", backend)
    monkeypatch.setattr(ops, "FP8_CHOICE", {})
    aq, as_ = ops.linear_fp8_swiglu(x, w, 32)
    assert aq.shape == (M, N // 2) and aq.dtype == torch.float8_e4m3fn and as_.shape == (M,)
    xq, xs = ops.quant_fp8_rows(x)
    gu = ((xq.float() * xs[:, None]) @ (w.q.float() * w.s.view(-1, 1)).t()).view(M, -1, 2, 32)
    g, u = gu[:, :, 0].reshape(M, -1), gu[:, :, 1].reshape(M, -1)
    ref_ = torch.nn.functional.silu(g) * u
    got = aq.float() * as_[:, None]
    rel = (got - ref_).norm() / ref_.norm()
    assert rel < 4e-2, rel  # e4m3 rounding of the activation (~2^-4 relative per element)
    if backend == "auto":
        assert len(ops.FP8_CHOICE) == 1


@pytest.mark.parametrize("M,N,K", [(1000, 1024, 512), (4096, 3072, 1024), (300, 4096, 1024)])
@pytest.mark.parametrize("gelu", [False, True])
def test_gemm8p_bias_gelu_epilogue(gpu, M, N, K, gelu):
    """gemm8p bias / bias + exact-erf GELU epilogue on the fp32 accumulators vs an fp32 torch reference
    (the encoder's FFN1 / projections); the planner's library path gives the same function."""
    from llm_weighted_consensus_amd import ops
    from llm_weighted_consensus_amd.ops import gemm_plan

    torch.manual_seed(M + N + gelu)
    A = torch.randn(M, K, device=gpu).to(torch.bfloat16)
    W = (torch.randn(N, K, device=gpu) * 0.05).to(torch.bfloat16)
    b = (torch.randn(N, device=gpu) * 0.5).to(torch.bfloat16)
    ref = A.float() @ W.float().t() + b.float()
    if gelu:
        ref = torch.nn.functional.gelu(ref)
    _close(ops.gemm8p(A, W, bias=b, gelu=gelu), ref, 3e-2, 1e-2)
    _close(gemm_plan.linear_bias(A, W, b, gelu=gelu), ref, 3e-2, 1e-2)


@pytest.mark.parametrize("var", [32, 64])
@pytest.mark.parametrize("bn", [256, 192])
@pytest.mark.parametrize("M,N,K,epi", [(300, 520, 64, "plain"), (4096, 6144, 4096, "plain"), (513, 1000, 128, "res"),
                                       (1024, 1024, 14336, "res"), (700, 2048, 1024, "swiglu"),
                                       (257, 776, 320, "bias"), (520, 4096, 1024, "gelu"),
                                       (64, 384, 192, "plain"), (2048, 128256 // 8, 4096, "plain"),
                                       # > 256 tiles: every epilogue across persistent rounds (VAR 64's
                                       # cross-tile prefetch under the epilogue)
                                       (4096, 4352, 256, "res"), (4352, 4096, 128, "swiglu"),
                                       (4352, 4096, 192, "gelu"),
                                       # the encoders' small-K projections (config 2 bge-base K = 768, bge-large
                                       # K = 1024): qkv / o / FFN1+GELU / FFN2 over several persistent rounds
                                       (4352, 2304, 768, "bias"), (4352, 768, 768, "bias"),
                                       (4352, 3072, 768, "gelu"), (4352, 768, 3072, "bias"),
                                       (2100, 1024, 1024, "bias")])
def test_gemm4w(gpu, M, N, K, epi, bn, var):
    """4-wave interleaved MFMA GEMM (AGPR accumulators, in-place inline-asm MFMA) vs an fp32 matmul for every
    epilogue: ragged M / N tails, one / two / many K tiles (the peeled last iterations), both tile widths,
    several rounds of tiles per workgroup, both schedules (32: the block-staged epilogue; 64: the wave-local
    transposed-layout epilogue with the next tile's first K tiles DMA'd inside the last two iterations — odd K
    tile counts run 32).  Launched twice (persistent rounds must leave LDS reusable)."""
    from llm_weighted_consensus_amd import ops

    if epi == "swiglu" and bn != 256:
        pytest.skip("SwiGLU epilogue needs bn 256")
    torch.manual_seed(M + N + K + bn)
    A = torch.randn(M, K, device=gpu).to(torch.bfloat16)
    W = (torch.randn(N, K, device=gpu) / K ** 0.5).to(torch.bfloat16)
    ref = A.float() @ W.float().t()
    for _ in range(2):
        if epi == "swiglu":
            F = N // 2
            out = ops.gemm4w(A, ops.swiglu_interleave(W), swiglu=True, bn=bn, var=var)
            _close(out, torch.nn.functional.silu(ref[:, :F]) * ref[:, F:], 3e-2, 1e-2)
        elif epi in ("bias", "gelu"):
            b = (torch.randn(N, device=gpu) * 0.5).to(torch.bfloat16)
            want = ref + b.float()
            if epi == "gelu":
                want = torch.nn.functional.gelu(want)
            _close(ops.gemm4w(A, W, bias=b, gelu=epi == "gelu", bn=bn, var=var), want, 3e-2, 1e-2)
        else:
            R = torch.randn(M, N, device=gpu).to(torch.bfloat16) if epi == "res" else None
            want = ref + (R.float() if R is not None else 0)
            out = ops.gemm4w(A, W, residual=R, out=R if R is not None else None, bn=bn, var=var)
            _close(out, want, 3e-2, 1e-2)


@pytest.mark.parametrize("var", [32, 64])
@pytest.mark.parametrize("M,N,K,epi,bn,P", [(300, 4096, 256, "plain", 256, 1), (4096 + 37, 6144, 512, "plain", 192, 16),
                                           (1000, 1536, 320, "swiglu", 256, 3), (257, 128256 // 16, 128, "plain", 256, 2),
                                           (1000, 1536, 384, "swiglu", 256, 3), (4352, 16384, 256, "swiglu", 256, 16),
                                           (2100, 128256 // 4, 256, "plain", 256, 16)])
def test_gemm4w_rowscale(gpu, M, N, K, epi, bn, P, var):
    """Folded RMSNorm, consumer side (RS 1): P partial row sums of squares [P, M] arrive by LDS-DMA, the
    prologue reduces them to r = rsqrt(sum / K + eps) and the epilogue scales the accumulator rows (plain,
    SwiGLU), ragged M (partials past the last row read zeros), multi-round tiles; vs the fp32 product of the
    scaled rows.  Twice (the LDS regions across rounds and launches).  VAR 64 (even K tile counts; odd ones run
    VAR 32): the transposed-layout epilogue, and each persistent tile DMAs the next tile's partials under its
    main loop."""
    from llm_weighted_consensus_amd import ops

    torch.manual_seed(M + N + K)
    A = torch.randn(M, K, device=gpu).to(torch.bfloat16)
    W = (torch.randn(N, K, device=gpu) / K ** 0.5).to(torch.bfloat16)
    chain = ops.NormChain(M + 64, 256 * P, 1e-5, gpu)
    chain.ss[:P, :M] = torch.rand(P, M, device=gpu) * K / P + 0.01
    chain.P = P
    rs = torch.rsqrt(chain.ss[:P, :M].sum(0) / K + 1e-5)
    ref = rs[:, None] * (A.float() @ W.float().t())
    for _ in range(2):
        if epi == "swiglu":
            F = N // 2
            out = ops.gemm4w(A, ops.swiglu_interleave(W), swiglu=True, bn=bn, chain=chain, var=var)
            _close(out, torch.nn.functional.silu(ref[:, :F]) * ref[:, F:], 3e-2, 1e-2)
        else:
            _close(ops.gemm4w(A, W, bn=bn, chain=chain, var=var), ref, 3e-2, 1e-2)


@pytest.mark.parametrize("var", [32, 64])
@pytest.mark.parametrize("M,N,K", [(4096, 4096, 256), (300, 4096, 512), (1000, 1024, 128), (4096 + 37, 4096, 64)])
def test_gemm4w_residual_rowsum(gpu, M, N, K, var):
    """Folded RMSNorm, producer side (RS 2): the residual epilogue writes C = R + A.W^T and the N/256 partial
    row sums of squares of the bf16 output (fp32 reference on the returned C), with the block-staged (32) and the
    wave-local (64) epilogue; three launches in a row; then
    the chain end to end: an RS 1 projection of C with those partials == the projection of rmsnorm(C), and a
    chain started by rms_rowsumsq gives the same scales."""
    from llm_weighted_consensus_amd import ops

    torch.manual_seed(M + N + K)
    eps = 1e-5
    chain = ops.NormChain(M + 64, N, eps, gpu)
    chain.ss.fill_(-7.0)
    A = torch.randn(M, K, device=gpu).to(torch.bfloat16)
    W = (torch.randn(N, K, device=gpu) / K ** 0.5).to(torch.bfloat16)
    for it in range(3):
        R = torch.randn(M, N, device=gpu).to(torch.bfloat16)
        want = R.float() + A.float() @ W.float().t()
        C = ops.gemm4w(A, W, residual=R, out=R, chain=chain, var=var)
        torch.cuda.synchronize()
        _close(C, want, 3e-2, 1e-2)
        P = N // 256
        assert chain.P == P
        parts = C.float().pow(2).view(M, P, 256).sum(-1).t()
        assert torch.allclose(chain.ss[:P, :M], parts, rtol=1e-5, atol=1e-4), (it, (chain.ss[:P, :M] - parts).abs().max())
        assert bool((chain.ss[:P, M:] == -7.0).all())  # rows past M untouched
    Wn = (torch.randn(512, N, device=gpu) / N ** 0.5).to(torch.bfloat16)
    h = ops.rmsnorm(C, torch.ones(N, device=gpu, dtype=torch.bfloat16), eps)
    want = h.float() @ Wn.float().t()
    _close(ops.gemm4w(C, Wn, chain=chain), want, 3e-2, 1e-2)
    ops.rms_rowsumsq(C, chain)
    assert chain.P == 1 and torch.allclose(chain.ss[0, :M], C.float().pow(2).sum(-1), rtol=1e-5)
    _close(ops.gemm4w(C, Wn, chain=chain), want, 3e-2, 1e-2)


@pytest.mark.parametrize("n,d,k", [(37, 1024, 5), (1000, 1024, 16), (70000, 384, 64), (300, 4096, 1)])
def test_knn_topk(gpu, n, d, k):
    """K10c training-table neighbour search == torch.topk of the fp32 dot products (rows with tied scores:
    duplicates of a row, the lower row first)."""
    from llm_weighted_consensus_amd import ops

    g = torch.Generator(device=gpu).manual_seed(n)
    E = torch.nn.functional.normalize(torch.randn(n, d, device=gpu, generator=g), dim=1)
    q = torch.nn.functional.normalize(torch.randn(d, device=gpu, generator=g), dim=0)
    if n > 10:
        best = int((E @ q).argmax())
        E[n - 3] = E[best]  # a tie with the best row
    vals, rows = ops.knn_topk(E, q, k)
    ref_v, _ = (E.double() @ q.double()).topk(k)
    assert torch.allclose(vals.double(), ref_v, atol=1e-5)
    got = (E.double() @ q.double())[rows]
    assert torch.allclose(got, ref_v, atol=1e-5)  # the rows hold those values
    assert len(set(rows.tolist())) == k
    if n > 10 and k > 1:
        r = rows.tolist()
        assert r.index(best) < r.index(n - 3)  # ties: lower row first


@pytest.mark.parametrize("M", [1, 7, 16, 33, 64])
@pytest.mark.parametrize("N,K", [(4096, 4096), (6144, 4096), (4096, 14336), (1040, 2048)])
@pytest.mark.parametrize("res", [False, True])
def test_skinny_gemm_matches_fp32(gpu, M, N, K, res):
    """Decode-sized weight-stream GEMM (skinny.hip): every m-tile count (1 / 2 / 4 with ragged rows), the
    headline projections' N and K, a 65-workgroup N, plain and in-place residual epilogues vs fp32."""
    from llm_weighted_consensus_amd import ops

    torch.manual_seed(M * 7 + N + K + res)
    A = torch.randn(M, K, device=gpu).to(torch.bfloat16)
    W = (torch.randn(N, K, device=gpu) / K ** 0.5).to(torch.bfloat16)
    ref = A.float() @ W.float().t()
    if res:
        R = torch.randn(M, N, device=gpu).to(torch.bfloat16)
        want = ref + R.float()
        out = ops.skinny_gemm(A, W, residual=R, out=R)
        assert out.data_ptr() == R.data_ptr()
    else:
        want = ref
        out = ops.skinny_gemm(A, W)
    _close(out, want, 3e-2, 1e-2)
    # a view of rows (lda > K) takes the same path
    if not res and M > 1:
        big = torch.randn(M, K + 64, device=gpu).to(torch.bfloat16)
        _close(ops.skinny_gemm(big[:, :K], W), big[:, :K].float() @ W.float().t(), 3e-2, 1e-2)



@pytest.mark.parametrize("M", [1, 16, 33, 64])
@pytest.mark.parametrize("N,K", [(28672, 4096), (1024, 2048)])
def test_skinny_gemm_swiglu_matches_fp32(gpu, M, N, K):
    """The skinny GEMM's SwiGLU epilogue over a 32-row gate/up interleaved W (each workgroup's gate and up
    tiles on the same activation fragments) vs fp32 silu(x Wg^T) * (x Wu^T)."""
    from llm_weighted_consensus_amd import ops

    torch.manual_seed(M + N + K)
    A = torch.randn(M, K, device=gpu).to(torch.bfloat16)
    W = (torch.randn(N, K, device=gpu) / K ** 0.5).to(torch.bfloat16)
    ref = A.float() @ W.float().t()
    F = N // 2
    out = ops.skinny_gemm(A, ops.swiglu_interleave(W), swiglu=True)
    assert out.shape == (M, F)
    _close(out, torch.nn.functional.silu(ref[:, :F]) * ref[:, F:], 3e-2, 1e-2)

def test_gemm4w_row_blocks_past_2gib(gpu):
    """gemm4w addresses A through one 32-bit buffer range; ops.gemm4w runs an A of 2 GiB or more (the encoders'
    FFN2 input at config 2's 0.5 M tokens is 3 GiB) as row blocks: rows on both sides of the block boundary and
    the ragged last rows match fp32, for the bias epilogue and the in-place residual one."""
    from llm_weighted_consensus_amd import ops

    torch.manual_seed(43)
    K, N = 8192, 256
    step = ((1 << 31) - 1) // (K * 2) // 256 * 256
    M = step + 300
    A = (torch.rand(M, K, device=gpu) - 0.5).to(torch.bfloat16)
    W = ((torch.rand(N, K, device=gpu) - 0.5) / K ** 0.5).to(torch.bfloat16)
    b = (torch.rand(N, device=gpu) - 0.5).to(torch.bfloat16)
    out = ops.gemm4w(A, W, bias=b, var=64)
    R = torch.randn(M, N, device=gpu).to(torch.bfloat16)
    R0 = R.clone()
    ops.gemm4w(A, W, residual=R, out=R)
    for r0, r1 in ((0, 256), (step - 128, step + 128), (M - 300, M)):
        ref = A[r0:r1].float() @ W.float().t()
        _close(out[r0:r1], ref + b.float(), 3e-2, 1e-2)
        _close(R[r0:r1], ref + R0[r0:r1].float(), 3e-2, 1e-2)


@pytest.mark.parametrize("splits", [2, 3, 4])
@pytest.mark.parametrize("M,N,K,epi,split_from", [(2048, 4096, 4096, "res", 0), (700, 2048, 1024, "swiglu", 0),
                                                  (1000, 128256 // 16, 512, "plain", 64), (300, 6144, 512, "plain", 0),
                                                  (4352, 4096, 512, "res", 200)])
def test_gemm4w_split_k(gpu, M, N, K, epi, split_from, splits):
    """gemm4w split-K (VAR 64): the tiles from split_from on run as `splits` units over K / splits; the first
    arrivers publish fp32 partials, the last adds them in its epilogue.  Plain / residual / SwiGLU, all tiles
    or only a tail (whole tiles and split tiles in one launch, several persistent rounds), ragged M / N; three
    launches in a row (the ticket counters reset by each tile's last arriver); vs fp32."""
    from llm_weighted_consensus_amd import ops

    torch.manual_seed(M + N + K + splits)
    A = torch.randn(M, K, device=gpu).to(torch.bfloat16)
    W = (torch.randn(N, K, device=gpu) / K ** 0.5).to(torch.bfloat16)
    ref = A.float() @ W.float().t()
    for _ in range(3):
        if epi == "swiglu":
            F = N // 2
            out = ops.gemm4w(A, ops.swiglu_interleave(W), swiglu=True, var=64, splits=splits, split_from=split_from)
            _close(out, torch.nn.functional.silu(ref[:, :F]) * ref[:, F:], 3e-2, 1e-2)
        elif epi == "res":
            R = torch.randn(M, N, device=gpu).to(torch.bfloat16)
            want = ref + R.float()
            _close(ops.gemm4w(A, W, residual=R, out=R, var=64, splits=splits, split_from=split_from), want, 3e-2, 1e-2)
        else:
            _close(ops.gemm4w(A, W, var=64, splits=splits, split_from=split_from), ref, 3e-2, 1e-2)
    torch.cuda.synchronize()
    _, cnt = ops.split_workspace(M, N, 256, splits, split_from, A.device)
    assert int(cnt.abs().sum()) == 0  # every tile's counters were reset by its last arriver


@pytest.mark.parametrize("M,N,K,splits", [(2560, 4096, 1024, 7), (2304, 4096, 1792, 3), (2560, 4096, 3584, 6)])
def test_gemm4w_split_k_uneven(gpu, M, N, K, splits):
    """Split-K with S not dividing the K tile count (units of K tile pairs [s H / S, (s + 1) H / S), H = K / 128)
    and more units than one round of CUs (144-160 tiles x 3-7 units): residual epilogue, twice in a row, vs
    fp32; the counters end reset."""
    from llm_weighted_consensus_amd import ops

    torch.manual_seed(M + K + splits)
    A = torch.randn(M, K, device=gpu).to(torch.bfloat16)
    W = (torch.randn(N, K, device=gpu) / K ** 0.5).to(torch.bfloat16)
    ref = A.float() @ W.float().t()
    for _ in range(2):
        R = torch.randn(M, N, device=gpu).to(torch.bfloat16)
        want = ref + R.float()
        _close(ops.gemm4w(A, W, residual=R, out=R, var=64, splits=splits), want, 3e-2, 1e-2)
    torch.cuda.synchronize()
    _, cnt = ops.split_workspace(M, N, 256, splits, 0, A.device)
    assert int(cnt.abs().sum()) == 0


@pytest.mark.parametrize("splits", [2, 3, 4])
def test_gemm4w_split_k_norm_chain(gpu, splits):
    """Split-K with the folded-RMSNorm epilogues: a row-scaled consumer (RS 1) and a residual producer that
    writes the row sums of squares (RS 2) — only the last arriver of a tile runs them."""
    from llm_weighted_consensus_amd import ops

    M, N, K, P = 1000, 4096, 1024, 4
    torch.manual_seed(7 + splits)
    A = torch.randn(M, K, device=gpu).to(torch.bfloat16)
    W = (torch.randn(N, K, device=gpu) / K ** 0.5).to(torch.bfloat16)
    chain = ops.NormChain(M + 64, 256 * 16, 1e-5, gpu)
    chain.ss[:P, :M] = torch.rand(P, M, device=gpu) * K / P + 0.01
    chain.P = P
    rs = torch.rsqrt(chain.ss[:P, :M].sum(0) / K + 1e-5)
    _close(ops.gemm4w(A, W, chain=chain, var=64, splits=splits), rs[:, None] * (A.float() @ W.float().t()), 3e-2, 1e-2)
    R = torch.randn(M, N, device=gpu).to(torch.bfloat16)
    want = R.float() + A.float() @ W.float().t()
    C = ops.gemm4w(A, W, residual=R, out=R, chain=chain, var=64, splits=splits)
    torch.cuda.synchronize()
    _close(C, want, 3e-2, 1e-2)
    parts = C.float().pow(2).view(M, N // 256, 256).sum(-1).t()
    assert torch.allclose(chain.ss[:N // 256, :M], parts, rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("var", [32, 64])
def test_gemm4w_gelu_epilogue_values(gpu, var):
    """The GELU epilogue's math alone: W = identity, so the output is gelu(A + b) of the operand's own bf16
    values over [-10, 10] (the VAR 64 tanh form and the VAR 32 erf form) against the fp32
    erf GELU: within 1e-3 plus the bf16 output's rounding."""
    from llm_weighted_consensus_amd import ops

    M, K = 512, 128
    x = torch.linspace(-10, 10, M * K, device=gpu).view(M, K).to(torch.bfloat16)
    W = torch.eye(K, device=gpu).to(torch.bfloat16)
    b = torch.zeros(K, device=gpu).to(torch.bfloat16)
    y = ops.gemm4w(x, W, bias=b, gelu=True, var=var)
    _close(y, torch.nn.functional.gelu(x.float()), 1e-3, 8e-3)


@pytest.mark.parametrize("var", [32, 64])
def test_gemm4w_operand_past_2gib_one_launch(gpu, var):
    """A of more than 2 GiB in one launch (the kernel's A buffer resource spans one tile's rows): the first
    and the last rows of a [1049088, 1024] bf16 operand (2.0 GiB + 1 MiB) against fp32, residual epilogue."""
    from llm_weighted_consensus_amd import ops

    M, K, N = (1 << 20) + 512, 1024, 256
    A = torch.empty(M, K, device=gpu, dtype=torch.bfloat16)
    A[:1024] = torch.randn(1024, K, device=gpu).to(torch.bfloat16)
    A[-1024:] = torch.randn(1024, K, device=gpu).to(torch.bfloat16)
    W = (torch.randn(N, K, device=gpu) / K ** 0.5).to(torch.bfloat16)
    R = torch.zeros(M, N, device=gpu, dtype=torch.bfloat16)
    R[-1024:] = torch.randn(1024, N, device=gpu).to(torch.bfloat16)
    out = ops.gemm4w(A, W, residual=R, var=var)
    for sl in (slice(0, 1024), slice(M - 1024, M)):
        want = R[sl].float() + A[sl].float() @ W.float().t()
        _close(out[sl], want, 3e-2, 1e-2)
    del A, R, out
