"""Host-side decode planning (CPU): cascade super-tile tables cover every batch row exactly once,
keep shared tiles inside one group, and degrade gracefully when the table is small."""
import numpy as np
import pytest
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
