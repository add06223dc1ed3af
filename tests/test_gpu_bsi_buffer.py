"""The buffer package's bit-sliced index on the MI355X vs its oracle (tests/_bsi.BufferBSI).

bsi/src/main/java/org/roaringbitmap/bsi/buffer/BitSliceIndexBase.java (BBSI/): compare :422-453
(rangeEQ :351-375, rangeNEQ :384-387, oNeilCompare :190-234, owenGreatEqual over
BufferFastAggregation.horizontal_or :243-275, RANGE :444-449, compareUsingMinMax :455-519), sum
:521-532.  Byte-identical results (container types included): every op x foundSet {null, set} x
runOptimize, predicates with up to 30 owenGreatEqual inputs (the horizontal_or queue's tie order
replayed on the host) and run containers above 2047 runs (C5 at 10^9 rows: test_gpu_fullsize.py).  The
reference's own known answers (BufferBSITest.java) are replayed through the engine as well.
"""
import numpy as np
import pytest

import _bsi
import _fmt
import _oracle as O

pytestmark = pytest.mark.gpu


def _pair(cols, vals, run_opt=False):
    from roaringbitmap_amd import MutableBitSliceIndex
    g = MutableBitSliceIndex.from_columns(cols, vals, run_opt)
    o = _bsi.BufferBSI.from_columns(cols, vals, run_opt)
    assert g.ebM.serialize() == o.ebm and [b.serialize() for b in g.bA] == o.ba
    assert (g.minValue, g.maxValue) == (o.min, o.max)
    return g, o


def _from_bytes(ebm, slices, mn, mx):
    from roaringbitmap_amd import ImmutableBitSliceIndex, RoaringBitmap
    g = ImmutableBitSliceIndex(RoaringBitmap(ebm), [RoaringBitmap(s) for s in slices], mn, mx)
    return g, _bsi.BufferBSI(ebm, slices, mn, mx)


def _check(g, o, op, a, e, found=None):
    from roaringbitmap_amd import RoaringBitmap
    fg = RoaringBitmap(found) if found is not None else None
    got = g.compare(op, a, e, fg).serialize()
    exp = o.compare(op, a, e, found)
    assert got == exp, (op, a, e, found is None, O.stats(got), O.stats(exp))
    return exp


def test_bufferbsitest_known_answers(gpu):
    """BufferBSITest.java:272-342 (GT / GE / LT / LE / RANGE), :198-217 (sum)"""
    g, o = _pair(np.arange(1, 100), np.arange(1, 100))
    r = range
    for op, a, e, exp in [
            ("GT", 50, 0, r(51, 100)), ("GT", 0, 0, r(1, 100)), ("GT", 99, 0, []),
            ("GE", 50, 0, r(50, 100)), ("GE", 1, 0, r(1, 100)), ("GE", 100, 0, []),
            ("LT", 50, 0, r(1, 50)), ("LT", 2**31 - 1, 0, r(1, 100)), ("LT", 1, 0, []),
            ("LE", 50, 0, r(1, 51)), ("LE", 2**31 - 1, 0, r(1, 100)), ("LE", 0, 0, []),
            ("RANGE", 10, 20, r(10, 21)), ("RANGE", 1, 200, r(1, 100)), ("RANGE", 1000, 2000, []),
            ("EQ", 7, 0, [7]), ("NEQ", 7, 0, [x for x in r(1, 100) if x != 7])]:
        got = _check(g, o, op, a, e)
        assert list(O.to_values(got)) == list(exp), (op, a, e)
    from roaringbitmap_amd import RoaringBitmap
    assert g.sum(RoaringBitmap.from_values(np.arange(1, 51))) == (sum(range(1, 51)), 50)
    assert g.sum(None) == (0, 0) and g.sum(RoaringBitmap()) == (0, 0)


def test_bufferbsitest_eq_neq_zero(gpu):
    """BufferBSITest.java:219-267, :344-358: rangeEQ direct, NEQ, zero values"""
    cols = np.arange(1, 100)
    g, o = _pair(cols, np.where(cols <= 50, 1, cols))
    for v, card in ((1, 50), (129, 0), (99, 1)):
        got = g.rangeEQ(None, v).serialize()
        assert got == o.range_eq(None, v) and O.stats(got)["card"] == card
    for cols, vals, tests in (([1, 2, 3], [99, 1, 50], [(99, [2, 3]), (100, [1, 2, 3])]),
                              ([1, 2, 3], [99, 99, 99], [(99, []), (1, [1, 2, 3])])):
        g, o = _pair(cols, vals)
        for v, exp in tests:
            assert list(O.to_values(_check(g, o, "NEQ", v, 0))) == exp
    g, o = _pair([0, 1, 2], [0, 0, 1])
    assert list(O.to_values(_check(g, o, "EQ", 0, 0))) == [0, 1]
    assert list(O.to_values(_check(g, o, "EQ", 1, 0))) == [2]


def test_range_neq_direct(gpu):
    """rangeNEQ called directly (BBSI/:384-387) skips compare's NEQ shortcut (:500-503)."""
    from roaringbitmap_amd import RoaringBitmap
    cols = np.arange(0, 300)
    g, o = _pair(cols, np.full(cols.size, 9))  # min == max
    f = O.from_values(np.arange(0, 300, 4))
    for v in (9, 10):
        for found in (None, f):
            exp = o._andnot(o.ebm, o.range_eq(found, v))
            got = g.rangeNEQ(RoaringBitmap(found) if found is not None else None, v).serialize()
            assert got == exp, (v, found is None)
    g, o = _pair(cols, cols % 5)
    for found in (None, f):
        exp = o._andnot(o.ebm, o.range_eq(found, 3))
        assert g.rangeNEQ(RoaringBitmap(found) if found is not None else None, 3).serialize() == exp


@pytest.mark.parametrize("seed", range(8))
def test_random_buffer_bsi(gpu, seed):
    """every op x foundSet {null, set}, runOptimize on odd seeds"""
    rng = np.random.default_rng(5000 + seed)
    n = int(rng.integers(100, 60000))
    span = int(rng.choice([1 << 16, 1 << 18, 1 << 20]))
    cols = np.sort(rng.choice(span, n, replace=False))
    bits = int(rng.integers(1, 31))
    vals = rng.integers(0, 1 << bits, n)
    if seed % 4 == 2:  # clustered values: long runs in the slices
        vals = (cols // 3000) % (1 << bits)
    if seed % 4 == 3:  # periodic values: equal slice cardinalities (horizontal_or queue ties)
        vals = cols % (1 << min(bits, 12))
    g, o = _pair(cols, vals, run_opt=bool(seed % 2))
    found = O.from_values(rng.choice(cols, n // 3, replace=False), bool(seed % 2))
    vmax = int(vals.max())
    for op in _bsi.OPS:
        for f in (None, found):
            for _ in range(2):
                a, e = sorted(int(x) for x in rng.integers(0, vmax + 2, 2))
                _check(g, o, op, a, e, f)
    # many owenGreatEqual inputs: start - 1 with many zero bits
    for a in (1 << (bits - 1), (1 << (bits - 1)) + 1, 3, 5, vmax // 3 + 1):
        for f in (None, found):
            _check(g, o, "GE", int(a), 0, f)
            _check(g, o, "RANGE", int(a), vmax - 1, f)
    _check(g, o, "RANGE", 0, vmax // 2)  # start <= 0: owenGreatEqual has no input (the empty bitmap)
    from roaringbitmap_amd import RoaringBitmap
    res = o.compare("RANGE", int(vals.min()) + 1, vmax - 1)
    assert g.sum(RoaringBitmap(res)) == o.sum(res)


def test_owen_queue_ties(gpu):
    """orInputs of equal cardinality on many keys: the chain follows the queue's heap order"""
    rng = np.random.default_rng(77)
    cols = np.arange(0, 40 << 16)  # 40 keys, every column
    vals = (cols * 2654435761) % (1 << 10)  # each residue class equally often per key
    g, o = _pair(cols, vals, run_opt=False)
    for a in (1, 2, 3, 5, 9, 17, 129, 513):
        for f in (None, O.from_values(rng.choice(cols, 1 << 18, replace=False))):
            _check(g, o, "GE", a, 0, f)
    g, o = _pair(cols, cols % (1 << 10), run_opt=True)  # run slices, periodic: ties everywhere
    for a in (1, 2, 3, 5, 9, 17, 129, 513):
        _check(g, o, "GE", a, 0)
        _check(g, o, "RANGE", a, 700)


def _big_run_slices(nkeys):
    """bit 0: runs [32k, 32k + 20], bit 1: runs [32k + 15, 32k + 35] (k < 2000), both run containers;
    their AND has two runs per k (~4000 runs: more than a slot holds)"""
    a = np.concatenate([np.arange(32 * k, 32 * k + 21) for k in range(2000)])
    b = np.concatenate([np.arange(32 * k + 15, 32 * k + 36) for k in range(2000)])
    full = np.arange(0, 1 << 16)
    s0 = _fmt.encode([(k, _fmt.R, a) for k in range(nkeys)])
    s1 = _fmt.encode([(k, _fmt.R, b) for k in range(nkeys)])
    ebm = _fmt.encode([(k, _fmt.R, full) for k in range(nkeys)])
    return ebm, [s0, s1]


@pytest.mark.parametrize("nkeys", [1, 1300])
def test_run_containers_above_2047_runs(gpu, nkeys):
    """EQ 3 = ebM & bA[1] & bA[0]: run AND run keeps the merged run container (~4000 runs, 16 KB):
    written to the big-run arena (1300 keys overflow its first 16 MiB: the op is rerun)"""
    ebm, sl = _big_run_slices(nkeys)
    g, o = _from_bytes(ebm, sl, 0, 3)
    got = _check(g, o, "EQ", 3, 0)
    assert O.stats(got)["run"] == nkeys and len(got) > 15000 * nkeys
    _check(g, o, "GT", 2, 0)
    _check(g, o, "RANGE", 3, 3)
