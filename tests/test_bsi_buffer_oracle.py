"""Pins the buffer-package BSI oracle (tests/_bsi.BufferBSI) to the reference's own known answers.

bsi/src/test/java/org/roaringbitmap/bsi/BufferBSITest.java (BBT/ below): ImmutableBitSliceIndex /
MutableBitSliceIndex compare and sum, checked at set level, plus a brute force over random
columns.  The container types of every step follow BitSliceIndexBase
(bsi/src/main/java/org/roaringbitmap/bsi/buffer/BitSliceIndexBase.java, BBSI/), whose circuit differs
from the heap BSI's; test_buffer_types_differ_from_heap shows it on bytes.
"""
import numpy as np
import pytest

import _bsi
import _oracle as O


def vals(b):
    return list(O.to_values(b))


@pytest.mark.parametrize("run_opt", [False, True])
def test_bufferbsitest_compare_known_answers(run_opt):
    b = _bsi.BufferBSI.from_columns(np.arange(1, 100), np.arange(1, 100), run_opt)  # BBT/:37-45
    r = range
    cases = [  # BBT/:272-342
        ("GT", 50, 0, list(r(51, 100))), ("GT", 0, 0, list(r(1, 100))), ("GT", 99, 0, []),
        ("GE", 50, 0, list(r(50, 100))), ("GE", 1, 0, list(r(1, 100))), ("GE", 100, 0, []),
        ("LT", 50, 0, list(r(1, 50))), ("LT", 2**31 - 1, 0, list(r(1, 100))), ("LT", 1, 0, []),
        ("LE", 50, 0, list(r(1, 51))), ("LE", 2**31 - 1, 0, list(r(1, 100))), ("LE", 0, 0, []),
        ("RANGE", 10, 20, list(r(10, 21))), ("RANGE", 1, 200, list(r(1, 100))), ("RANGE", 1000, 2000, []),
    ]
    for op, a, e, exp in cases:
        assert vals(b.compare(op, a, e)) == exp, (op, a, e)


def test_bufferbsitest_eq():
    """BBT/:219-239: values 1 for columns <= 50, x otherwise; rangeEQ directly"""
    cols = np.arange(1, 100)
    b = _bsi.BufferBSI.from_columns(cols, np.where(cols <= 50, 1, cols))
    assert O.stats(b.range_eq(None, 1))["card"] == 50
    assert O.stats(b.range_eq(None, 129))["card"] == 0
    assert vals(b.range_eq(None, 99)) == [99]


def test_bufferbsitest_neq_and_zero():
    b = _bsi.BufferBSI.from_columns([1, 2, 3], [99, 1, 50])  # BBT/:241-267
    assert vals(b.compare("NEQ", 99)) == [2, 3]
    assert vals(b.compare("NEQ", 100)) == [1, 2, 3]
    b = _bsi.BufferBSI.from_columns([1, 2, 3], [99, 99, 99])
    assert vals(b.compare("NEQ", 99)) == []
    assert vals(b.compare("NEQ", 1)) == [1, 2, 3]
    b = _bsi.BufferBSI.from_columns([0, 1, 2], [0, 0, 1])  # BBT/:344-358
    assert vals(b.compare("EQ", 0)) == [0, 1]
    assert vals(b.compare("EQ", 1)) == [2]


def test_bufferbsitest_sum():
    b = _bsi.BufferBSI.from_columns(np.arange(1, 100), np.arange(1, 100))  # BBT/:198-217
    s, c = b.sum(O.from_values(np.arange(1, 51)))
    assert s == sum(range(1, 51)) and c == 50


def test_bufferbsitest_add_and_evaluate():
    """BBT/:119-135: after bsiA.add(bsiB) columns 1..99 hold 120 and columns 100..119 hold 120 - col;
    the index is built here straight from those values (add's own slice types are construction)."""
    cols = np.arange(1, 120)
    v = np.where(cols < 100, 120, 120 - cols)
    b = _bsi.BufferBSI.from_columns(cols, v)
    b.min, b.max = 1, 120  # MutableBitSliceIndex.add recomputes minValue() / maxValue() (BBSI mutable :216-218)
    assert vals(b.compare("EQ", 120)) == list(range(1, 100))
    assert vals(b.compare("RANGE", 1, 20)) == list(range(100, 120))


def test_range_start_at_most_zero_is_empty():
    """owenGreatEqual with predicate <= 0 (BBSI/:246-250): beGtrThan = -1, ~beGtrThan = 0, so
    Long.numberOfTrailingZeros gives 64, no orInput is made and horizontal_or() of nothing is
    the empty bitmap.  compare(RANGE, 0, end) reaches it whenever compareUsingMinMax does not decide."""
    b = _bsi.BufferBSI.from_columns(np.arange(1, 100), np.arange(1, 100))
    assert vals(b.compare("RANGE", 0, 50)) == []
    assert vals(_bsi.BSI.from_columns(np.arange(1, 100), np.arange(1, 100)).compare("RANGE", 0, 50)) == \
        list(range(1, 51))


def test_neq_with_found_set_uses_ebm():
    """rangeNEQ (BBSI/:384-387) subtracts from ebM, not from the found set."""
    cols = np.arange(0, 200)
    b = _bsi.BufferBSI.from_columns(cols, cols % 7)
    found = O.from_values(np.arange(0, 100))
    got = set(vals(b.compare("NEQ", 3, 0, found)))
    assert got == set(cols.tolist()) - set(c for c in range(100) if c % 7 == 3)


def test_buffer_types_differ_from_heap():
    """Run AND run keeps the merged run container in the buffer package: an EQ chain over
    run-compressed slices gives different bytes (same set) than the heap BSI."""
    cols = np.arange(0, 1 << 16)
    m = cols % 200  # bit 1: 100-column runs, bit 0: 101-column runs overlapping them at one column
    v = (m < 100) * 2 + (m >= 99)
    hb = _bsi.BSI.from_columns(cols, v, run_optimize=True)
    bb = _bsi.BufferBSI.from_columns(cols, v, run_optimize=True)
    h, b = hb.compare("EQ", 3), bb.compare("EQ", 3)  # the single columns 200k + 99
    assert vals(h) == vals(b)
    assert O.stats(b)["run"] == 1 and O.stats(h)["array"] == 1


@pytest.mark.parametrize("seed", range(6))
def test_buffer_oracle_matches_brute_force(seed):
    rng = np.random.default_rng(100 + seed)
    cols = np.sort(rng.choice(1 << 18, 3000, replace=False))
    v = rng.integers(0, 1 << int(rng.integers(3, 20)), cols.size)
    b = _bsi.BufferBSI.from_columns(cols, v, run_optimize=bool(seed % 2))
    fmask = rng.random(cols.size) < 0.5
    for found in (None, O.from_values(cols[fmask])):
        fm = np.ones(cols.size, bool) if found is None else fmask
        for op in _bsi.OPS:
            a, e = sorted(rng.integers(1, int(v.max()) + 2, 2))
            got = set(vals(b.compare(op, int(a), int(e), found)))
            m = {"EQ": v == a, "NEQ": v != a, "LE": v <= a, "LT": v < a, "GE": v >= a, "GT": v > a,
                 "RANGE": (v >= a) & (v <= e)}[op]
            want = m & fm
            if op == "NEQ":  # ebM minus the found EQ columns (BBSI/:384-387)
                want = ~((v == a) & fm)
            if op == "LE":  # or(LT, and(fixedFoundSet, EQ)): LT is not restricted (BBSI/:217-228)
                want = (v < a) | ((v == a) & fm)
            assert got == set(cols[want].tolist()), (op, found is None)
    assert b.sum(O.from_values(cols[::3])) == (int(v[::3].sum()), len(cols[::3]))
