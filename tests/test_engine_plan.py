"""Host-side decode planning (CPU): cascade super-tile tables cover every batch row exactly once,
keep shared tiles inside one group, and degrade gracefully when the table is small."""
import numpy as np
import pytest
import torch
from hypothesis import given, settings, strategies as st

from llm_weighted_consensus_amd.engine.engine import cascade_tiles


def _runs(spec):
    runs, r = [], 0
    for n, p in spec:
        runs.append((r, n, p))
        r += n
    return runs, r


def _check(runs, B, per, tiles, nt):
    cover = np.zeros(B, dtype=int)
    group_of = np.zeros(B, dtype=int)
    for gi, (s, n, _p) in enumerate(runs):
        group_of[s:s + n] = gi
    for r0, n, p in tiles[:nt]:
        assert 1 <= n <= per
        cover[r0:r0 + n] += 1
        if p > 0:  # a shared tile stays inside one group and uses that group's prefix
            gi = group_of[r0]
            assert (group_of[r0:r0 + n] == gi).all()
            assert p == runs[gi][2] and runs[gi][1] >= 2
    assert (cover == 1).all()
    assert (tiles[nt:] == 0).all()


def test_cascade_tiles_basic():
    runs, B = _runs([(64, 16), (64, 16), (1, 16), (3, 0), (2, 4)])
    tiles = np.zeros((B // 32 + 16, 3), dtype=np.int32)
    nt = cascade_tiles(runs, 32, tiles)
    _check(runs, B, 32, tiles, nt)
    assert [tuple(t) for t in tiles[:nt]] == [(0, 32, 16), (32, 32, 16), (64, 32, 16), (96, 32, 16),
                                             (128, 4, 0), (132, 2, 4)]


@settings(max_examples=200, deadline=None)
@given(spec=st.lists(st.tuples(st.integers(1, 70), st.integers(0, 5)), min_size=1, max_size=30),
       per=st.sampled_from([2, 4, 16, 32]), extra=st.integers(0, 8))
def test_cascade_tiles_cover_and_degrade(spec, per, extra):
    runs, B = _runs(spec)
    T = -(-B // per) + extra  # engine sizing: ceil(B/per) + slack
    tiles = np.zeros((T, 3), dtype=np.int32)
    nt = cascade_tiles(runs, per, tiles)
    assert nt <= T
    _check(runs, B, per, tiles, nt)


def test_cascade_tiles_overflow_raises_only_without_room():
    tiles = np.zeros((1, 3), dtype=np.int32)
    with pytest.raises(RuntimeError):
        cascade_tiles([(0, 40, 0)], 32, tiles)


def test_step_plans_candidates_and_apply(monkeypatch):
    """LlamaModel.step_plans (the engine's in-step A/B candidates) from recorded planner state, on CPU: the
    planner's own choice, all-library (norm chain off) and all-hand-written (fastest own backend per shape, the
    chain fully folded with the fastest consumer / producer variants); apply_step_plan installs one and
    plan_summary reports it."""
    from llm_weighted_consensus_amd.models.config import decoder_config
    from llm_weighted_consensus_amd.models.llama import LlamaModel
    from llm_weighted_consensus_amd.ops import gemm_plan

    m = LlamaModel.__new__(LlamaModel)
    m.cfg = decoder_config("llama-3-8b")
    m.g8_ws = object()
    m.fp8_dense = False
    m.chain = type("Ch", (), {"max_rows": 8192})()
    M = 4096
    keys = m._plan_keys(M)
    choices, timings = dict(gemm_plan._CHOICE), dict(gemm_plan.TIMINGS)
    try:
        for n, k in keys.items():
            gemm_plan._CHOICE[k] = "blas"
            gemm_plan.TIMINGS[k] = {"blas": 100.0, "g4": 101.0, "g4p": 99.0, "g8": 120.0}
        t = {f"qkv_rs{bn}v{v}": 150.0 + bn / 100 + v / 100 for bn in (192, 256) for v in (32, 64)}
        t.update({"gu_rsv32": 660.0, "gu_rsv64": 650.0, "lm_rsv32": 3000.0, "lm_rsv64": 2990.0,
                  "o_own32": 110.0, "o_own64": 101.0, "down_own32": 330.0, "down_own64": 320.0})
        gemm_plan.TIMINGS[(M, m.cfg.hidden, 0, "norm_chain")] = t
        m.chain_m = {M: {"attn": True, "mlp": False, "final": False, "qkv_bn": 192, "qkv_var": 32, "o": "own64",
                         "down": "sumsq"}}
        plans = m.step_plans(M)
        assert set(plans) == {"planner", "library", "own"}
        assert plans["library"]["choices"] == {n: "blas" for n in keys}
        assert not plans["library"]["chain"]["attn"]
        assert plans["own"]["choices"] == {n: "g4p" for n in keys}
        assert plans["own"]["chain"] == {"attn": True, "mlp": True, "final": True, "qkv_bn": 192, "qkv_var": 32,
                                         "gu_var": 64, "lm_var": 64, "lm_split": False, "o": "own64",
                                         "down": "own64"}
        m.apply_step_plan(M, plans["own"])
        assert all(gemm_plan._CHOICE[k] == "g4p" for k in keys.values()) and m.chain_m[M]["mlp"]
        s = m.plan_summary(M)
        assert s["gu"] == "g4 rs v64" and s["o"] == "g4 rs2 v64" and s["qkv"] == "g4 rs192 v32"
        # coordinate-descent moves: from the all-own plan (chain owns every projection) only chain decisions
        labels = [lb for lb, _ in m.step_moves(M, plans["own"])]
        assert "attn_fold=False" in labels and "gu_var=32" in labels and "o_producer=sumsq" in labels
        assert "lm_split=True" in labels
        assert not any(lb.startswith(("qkv=", "gu=", "lm=")) for lb in labels)
        # from the planner's plan: the projections the chain does not own can switch backend
        mv = dict(m.step_moves(M, plans["planner"]))
        assert "gu=g4p" in mv and "qkv=g4p" not in mv
        p1 = m.with_move(plans["planner"], mv["gu=g4p"])
        assert p1["choices"]["gu"] == "g4p" and p1["chain"] == plans["planner"]["chain"]
        # no move that leaves the step unchanged: a schedule / tile width / producer mode only where its norm
        # point is folded
        pc = plans["planner"]["chain"]
        assert ("gu_var=32" in mv or "gu_var=64" in mv) == bool(pc["mlp"])
        assert any(k.startswith("lm_") and k != "lm=g4p" for k in mv) == bool(pc["final"])
        assert any(k.startswith("o_producer=") for k in mv) == bool(pc["mlp"])
        p2 = m.with_move(p1, mv["mlp_fold=True"])  # moves compose
        assert p2["chain"]["mlp"] and p2["choices"]["gu"] == "g4p" and not plans["planner"]["chain"]["mlp"]
        m.apply_step_plan(M, plans["library"])
        assert m.plan_summary(M) == {n: "blas" for n in keys}
    finally:
        gemm_plan._CHOICE.clear()
        gemm_plan._CHOICE.update(choices)
        gemm_plan.TIMINGS.clear()
        gemm_plan.TIMINGS.update(timings)


def test_split_plan():
    """gemm4w split-K planning: whole-call splits only while the units fit one round; ragged last rounds of at
    most half the CUs split their tiles; every unit an even K tile count."""
    from llm_weighted_consensus_amd.ops import split_plan

    assert split_plan(2048, 4096, 4096) == (2, 0)  # 128 tiles -> 256 units
    assert split_plan(512, 4096, 4096) == (4, 0)  # 32 tiles -> 128 units
    assert split_plan(2304, 4096, 4096) == (1, 0)  # 144 tiles: a split would need a second round
    assert split_plan(4096, 128256, 4096) == (2, 7936)  # lm_head: 31 rounds + 80 tiles
    assert split_plan(3072, 6144, 4096) == (4, 256)  # 288 tiles: 32-tile tail
    assert split_plan(4096, 28672, 4096) == (1, 0)  # 7 whole rounds
    assert split_plan(2048, 4096, 192) == (1, 0)  # 3 K tiles: no even split


def test_split_workspace_grows_and_keeps_old_buffers():
    """gemm4w split-K workspace: per (device, thread); growing it keeps the old buffers alive (graphs captured
    before the growth still address them); a smaller request reuses the current one."""
    import threading

    from llm_weighted_consensus_amd import ops

    dev = torch.device("cpu")
    p1, c1 = ops.split_workspace(2048, 4096, 256, 2, 0, dev)
    assert p1.numel() >= 128 * 256 * 256 and c1.numel() >= 2 * 128 and int(c1.abs().sum()) == 0
    assert ops.split_workspace(512, 4096, 256, 2, 0, dev)[0] is p1  # fits: same buffer
    p2, _ = ops.split_workspace(2048, 4096, 256, 4, 0, dev)  # 3 slabs per tile: grows
    assert p2 is not p1 and p2.numel() >= 3 * 128 * 256 * 256
    assert any(ws[0] is p1 for ws in ops._SPLIT_WS_RETIRED)
    other = {}
    t = threading.Thread(target=lambda: other.setdefault("ws", ops.split_workspace(2048, 4096, 256, 2, 0, dev)))
    t.start()
    t.join()
    assert other["ws"][0] is not p2  # another host thread gets its own counters


def test_dense_mx_min_rows_context():
    """The benches' self-check re-embeds on the batch's fp8 MLP path: the MX threshold is overridden inside the
    context only, and restored on the way out (also after an exception)."""
    from llm_weighted_consensus_amd import ops

    base = ops.DENSE_MX_MIN_ROWS
    with ops.dense_mx_min_rows(0):
        assert ops.DENSE_MX_MIN_ROWS == 0
    assert ops.DENSE_MX_MIN_ROWS == base
    try:
        with ops.dense_mx_min_rows(7):
            raise ValueError
    except ValueError:
        pass
    assert ops.DENSE_MX_MIN_ROWS == base
