"""Pins the BSI oracle (tests/_bsi.py) to the reference's own known answers.

bsi/src/test/java/org/roaringbitmap/bsi/RBBsiTest.java (RBT_BSI/ below): values
1..99 at columns 1..99, then compare / sum results checked at set level.
"""
import numpy as np
import pytest

import _bsi
import _oracle as O


def vals(b):
    return list(O.to_values(b))


@pytest.fixture(scope="module")
def bsi():
    return _bsi.BSI.from_columns(np.arange(1, 100), np.arange(1, 100))


@pytest.mark.parametrize("run_opt", [False, True])
def test_rbbsitest_compare_known_answers(run_opt):
    b = _bsi.BSI.from_columns(np.arange(1, 100), np.arange(1, 100), run_opt)
    r = range
    cases = [  # RBT_BSI/:228-299
        ("GT", 50, 0, list(r(51, 100))), ("GT", 0, 0, list(r(1, 100))), ("GT", 99, 0, []),
        ("GE", 50, 0, list(r(50, 100))), ("GE", 1, 0, list(r(1, 100))), ("GE", 100, 0, []),
        ("LT", 50, 0, list(r(1, 50))), ("LT", 2**31 - 1, 0, list(r(1, 100))), ("LT", 1, 0, []),
        ("LE", 50, 0, list(r(1, 51))), ("LE", 2**31 - 1, 0, list(r(1, 100))), ("LE", 0, 0, []),
        ("RANGE", 10, 20, list(r(10, 21))), ("RANGE", 1, 200, list(r(1, 100))), ("RANGE", 1000, 2000, []),
    ]
    for op, a, e, exp in cases:
        assert vals(b.compare(op, a, e)) == exp, (op, a, e)


def test_rbbsitest_neq_and_zero():
    b = _bsi.BSI.from_columns([1, 2, 3], [99, 1, 50])  # RBT_BSI/:200-221
    assert vals(b.compare("NEQ", 99)) == [2, 3]
    assert vals(b.compare("NEQ", 100)) == [1, 2, 3]
    b = _bsi.BSI.from_columns([1, 2, 3], [99, 99, 99])
    assert vals(b.compare("NEQ", 99)) == []
    assert vals(b.compare("NEQ", 1)) == [1, 2, 3]
    b = _bsi.BSI.from_columns([0, 1, 2], [0, 0, 1])  # RBT_BSI/:321-331
    assert vals(b.compare("EQ", 0)) == [0, 1]
    assert vals(b.compare("EQ", 1)) == [2]


def test_rbbsitest_sum(bsi):
    found = O.from_values(np.arange(1, 51))  # RBT_BSI/:301-318
    s, c = bsi.sum(found)
    assert s == sum(range(1, 51)) and c == 50


def test_rbbsitest_eq_half():
    """RBT_BSI/:184-194: values 1 for even columns, x otherwise; EQ 1 -> 50 columns"""
    cols = np.arange(1, 100)
    v = np.where(cols % 2 == 0, 1, cols)
    assert O.stats(_bsi.BSI.from_columns(cols, v).compare("EQ", 1))["card"] == 50


@pytest.mark.parametrize("seed", range(4))
def test_oracle_matches_brute_force(seed):
    rng = np.random.default_rng(seed)
    cols = np.sort(rng.choice(1 << 18, 3000, replace=False))
    v = rng.integers(0, 1 << int(rng.integers(3, 20)), cols.size)
    b = _bsi.BSI.from_columns(cols, v, run_optimize=bool(seed % 2))
    for op in _bsi.OPS:
        a, e = sorted(rng.integers(0, int(v.max()) + 2, 2))
        got = set(vals(b.compare(op, int(a), int(e))))
        m = {"EQ": v == a, "NEQ": v != a, "LE": v <= a, "LT": v < a, "GE": v >= a, "GT": v > a,
             "RANGE": (v >= a) & (v <= e)}[op]
        assert got == set(cols[m].tolist()), op
    found = O.from_values(cols[::3])
    assert b.sum(found) == (int(v[::3].sum()), len(cols[::3]))


def test_parallel_range_sum_leg_matches_single_thread():
    """The bench's key-parallel CPU leg (rbo_time_bsi_range_sum_parallel) gives the single-thread
    compare(RANGE) + sum (BSI/:482-513, 581-592) for any worker count."""
    rng = np.random.default_rng(8)
    cols = np.unique(rng.integers(0, 40 << 16, 60000))
    vals = rng.integers(0, 1 << 20, cols.size)
    ebm = O.from_values(cols, True)
    slices = [O.from_values(cols[(vals >> i) & 1 == 1], True) for i in range(20)]
    lo, hi = 1 << 17, 3 << 18
    _, one = O.time_bsi_range_sum(ebm, slices, lo, hi, 1)
    m = (vals >= lo) & (vals <= hi)
    assert one == (int(vals[m].sum()), int(m.sum()))
    for t in (1, 2, 3, 7, 64):
        assert O.time_bsi_range_sum_parallel(ebm, slices, lo, hi, t, 1)[1] == one
