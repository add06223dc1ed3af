"""Bit-sliced index compare / sum on the MI355X vs the BSI oracle (tests/_bsi.py).

bsi/src/main/java/org/roaringbitmap/bsi/RoaringBitmapSliceIndex.java: compare
:482-513 (compareUsingMinMax :515-579, oNeilCompare :432-468), sum :581-592.
Byte-identical results (container types included); the reference's own known
answers (RBBsiTest.java) are replayed through the engine as well.
"""
import numpy as np
import pytest

import _bsi
import _oracle as O

pytestmark = pytest.mark.gpu


def _pair(cols, vals, run_opt=False):
    from roaringbitmap_amd import RoaringBitmapSliceIndex
    g = RoaringBitmapSliceIndex.from_columns(cols, vals, run_opt)
    o = _bsi.BSI.from_columns(cols, vals, run_opt)
    assert g.ebM.serialize() == o.ebm and [b.serialize() for b in g.bA] == o.ba
    assert (g.minValue, g.maxValue) == (o.min, o.max)
    return g, o


def _check(g, o, op, a, e, found=None):
    from roaringbitmap_amd import RoaringBitmap
    fg = RoaringBitmap(found) if found is not None else None
    got = g.compare(op, a, e, fg).serialize()
    exp = o.compare(op, a, e, found)
    assert got == exp, (op, a, e, O.stats(got), O.stats(exp))
    return exp


def test_rbbsitest_known_answers(gpu):
    g, o = _pair(np.arange(1, 100), np.arange(1, 100))
    for op, a, e in [("GT", 50, 0), ("GT", 0, 0), ("GT", 99, 0), ("GE", 50, 0), ("GE", 1, 0), ("GE", 100, 0),
                     ("LT", 50, 0), ("LT", 2**31 - 1, 0), ("LT", 1, 0), ("LE", 50, 0), ("LE", 2**31 - 1, 0),
                     ("LE", 0, 0), ("RANGE", 10, 20), ("RANGE", 1, 200), ("RANGE", 1000, 2000), ("EQ", 7, 0),
                     ("NEQ", 7, 0)]:
        _check(g, o, op, a, e)
    from roaringbitmap_amd import RoaringBitmap
    assert g.sum(RoaringBitmap.from_values(np.arange(1, 51))) == (sum(range(1, 51)), 50)
    assert g.sum(None) == (0, 0)


@pytest.mark.parametrize("seed", range(6))
def test_random_bsi(gpu, seed):
    rng = np.random.default_rng(4000 + seed)
    n = int(rng.integers(100, 60000))
    span = int(rng.choice([1 << 16, 1 << 18, 1 << 20]))
    cols = np.sort(rng.choice(span, n, replace=False))
    bits = int(rng.integers(1, 31))
    vals = rng.integers(0, 1 << bits, n)
    if seed % 3 == 2:  # clustered values: long runs in the slices
        vals = (cols // 3000) % (1 << bits)
    g, o = _pair(cols, vals, run_opt=bool(seed % 2))
    for op in _bsi.OPS:
        for _ in range(3):
            a, e = sorted(int(x) for x in rng.integers(0, int(vals.max()) + 2, 2))
            _check(g, o, op, a, e)
    found = O.from_values(rng.choice(cols, n // 3, replace=False), bool(seed % 2))
    for op in ("EQ", "NEQ", "GT", "LE", "RANGE"):
        a, e = sorted(int(x) for x in rng.integers(0, int(vals.max()) + 2, 2))
        _check(g, o, op, a, e, found)
    from roaringbitmap_amd import RoaringBitmap
    res = o.compare("RANGE", int(vals.min()) + 1, int(vals.max()) - 1)
    assert g.sum(RoaringBitmap(res)) == o.sum(res)
    assert g.sum(RoaringBitmap(found)) == o.sum(found)


def test_single_value_and_empty(gpu):
    g, o = _pair([5, 70000, 131071], [3, 3, 3])  # min == max: compareUsingMinMax shortcuts
    for op in _bsi.OPS:
        for a in (2, 3, 4):
            _check(g, o, op, a, a + 1)
    g, o = _pair([0, 1, 2], [0, 0, 1])
    _check(g, o, "EQ", 0, 0)
    _check(g, o, "EQ", 1, 0)


def _splitmix(x):
    x = (x + np.uint64(0x9E3779B97F4A7C15))
    x = (x ^ (x >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
    x = (x ^ (x >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
    return x ^ (x >> np.uint64(31))


def test_c5_synthetic_bsi(gpu):
    """C5 generator (csrc/synth.hip) + fused compare(RANGE) + sum, against the oracle on the same bitmaps."""
    from roaringbitmap_amd import Engine
    rows, seed = 200_000, 0xC5
    e = Engine(0)
    b = e.synth(4, seed, rows)
    mn, mx = e.batch_minmax(b)
    with np.errstate(over="ignore"):
        r = np.arange(rows, dtype=np.uint64)
        v = (_splitmix(np.uint64(seed) ^ (r * np.uint64(0x9E3779B97F4A7C15))) & np.uint64(0x7FFFFFFF)).astype(np.int64)
    assert (mn, mx) == (int(v.min()), int(v.max()))
    bms = [e.batch_fetch(b, i).serialize() for i in range(32)]
    assert list(O.to_values(bms[0])) == list(range(rows))
    assert list(O.to_values(bms[5])) == np.nonzero((v >> 4) & 1)[0].tolist()  # slice 4
    assert O.run_optimize(bms[7]) == bms[7]  # runOptimize'd types
    o = _bsi.BSI(bms[0], bms[1:], mn, mx)
    lo, hi = 1 << 29, 1 << 30
    e.bsi(b, "RANGE", 31, lo, hi, mn, mx, want_sum=True)
    exp = o.compare("RANGE", lo, hi)
    assert e.fetch().serialize() == exp
    assert e.bsi_sums() == o.sum(exp)
    assert o.sum(exp)[0] == int(v[(v >= lo) & (v <= hi)].sum())
    # the same (sum, count) copied to device memory on the engine stream (the bench's all-reduce input)
    import torch
    d = torch.empty(2, dtype=torch.int64, device="cuda:0")  # no fill on torch's stream to race the engine's write
    e.bsi_sums_device(d)
    e.sync()
    assert (int(d[0]), int(d[1])) == o.sum(exp)
    # a compare without want_sum leaves (0, 0)
    e.bsi(b, "RANGE", 31, lo, hi, mn, mx, want_sum=False)
    assert e.bsi_sums() == (0, 0)
    assert e.fetch().serialize() == exp
    # without sum shares the low slices are read only where EQ survives the high ones: every op,
    # with predicates whose EQ dies early, survives into the low slices, or matches exactly
    for op in _bsi.OPS:
        for a, z in ((lo, hi), (int(v[7]), int(v[7]) + 3), (int(v[11]) - 1, int(v[11]))):
            e.bsi(b, op, 31, a, z, mn, mx)
            assert e.fetch().serialize() == o.compare(op, a, z), (op, a, z)
    # the sums target (the bench's C5 step): every sum also lands in d, written by the summing kernel
    d2 = torch.empty(2, dtype=torch.int64, device="cuda:0")
    e.bsi_sums_target(d2)
    e.bsi(b, "RANGE", 31, lo, hi, mn, mx, want_sum=True)
    e.sync()
    assert (int(d2[0]), int(d2[1])) == o.sum(exp)
    assert e._bsi_target is d2  # the engine holds the target while kernels may write it
    e.bsi_sums_target(None)
    assert e._bsi_target is None
    for bad in (torch.empty(2, dtype=torch.int32, device="cuda:0"), torch.empty(1, dtype=torch.int64, device="cuda:0"),
                torch.empty(2, dtype=torch.int64), torch.empty(4, dtype=torch.int64, device="cuda:0")[::2]):
        with pytest.raises(ValueError):
            e.bsi_sums_target(bad)
    # a second index on the same engine: each batch keeps its own task list and input table
    b2 = e.synth(4, seed + 1, rows // 3)
    mn2, mx2 = e.batch_minmax(b2)
    o2 = _bsi.BSI(e.batch_fetch(b2, 0).serialize(), [e.batch_fetch(b2, i).serialize() for i in range(1, 32)], mn2, mx2)
    for _ in range(2):
        for bb, oo, m0, m1 in ((b, o, mn, mx), (b2, o2, mn2, mx2)):
            e.bsi(bb, "GE", 31, lo, 0, m0, m1, want_sum=True)
            ex = oo.compare("GE", lo, 0)
            assert e.fetch().serialize() == ex
            assert e.bsi_sums() == oo.sum(ex)
    e.release(b2)
