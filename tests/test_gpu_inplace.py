"""In-place instance ops and RoaringBitmapSliceIndex.merge on the MI355X vs the oracle.

x1.and(x2) / x1.or(x2) / x1.xor(x2) / x1.andNot(x2) in place (RB/RoaringBitmap.java:1272-1296,
2481-2523, 3296-3348, 1346-1382) through rbg_pairwise_inplace: every 18x18 container-mode pair,
the full bitmap | array case of Container.ior (RB/BitmapContainer.java:740-757), x2 being x1
itself, and random bitmaps.  merge (bsi/.../RoaringBitmapSliceIndex.java:379-405 and the buffer
MutableBitSliceIndex.merge) on random disjoint indexes, with and without runOptimize.
"""
import numpy as np
import pytest

import _bsi
import _fmt
import _gen
import _oracle as O

pytestmark = pytest.mark.gpu

EXPECT = {"and": "and", "or": "ior", "xor": "xor", "andNot": "andnot"}


def _inplace(op, a, b):
    import roaringbitmap_amd as rb
    x = rb.RoaringBitmap(a)
    getattr(x, op)(rb.RoaringBitmap(b))  # the Java names: x.and(y), x.or(y), x.xor(y), x.andNot(y)
    return x.serialize()


def test_every_container_mode_pair_in_place(gpu):
    rng = np.random.default_rng(17)
    for m1 in _gen.MODES:
        for m2 in _gen.MODES:
            k1, v1 = _gen.container(rng, m1)
            k2, v2 = _gen.container(rng, m2)
            a, b = _fmt.encode([(3, k1, v1)]), _fmt.encode([(3, k2, v2)])
            for op, oop in EXPECT.items():
                assert _inplace(op, a, b) == O.pairwise(oop, a, b), (m1, m2, op)


def test_full_bitmap_or_array_stays_bitmap(gpu):
    hole = np.sort(np.random.default_rng(3).choice(65536, 100, replace=False)).astype(np.uint16)
    bvals = np.setdiff1d(np.arange(65536), hole).astype(np.uint16)
    rng = np.random.default_rng(4)
    other = [(k, _fmt.A, _gen.container(rng, "a_small")[1]) for k in (1, 5)]
    a = _fmt.encode([(9, _fmt.B, bvals)] + other)
    b = _fmt.encode([(9, _fmt.A, hole), (5, _fmt.B, np.arange(0, 60000, 2))])
    got = _inplace("or", a, b)
    assert got == O.pairwise("ior", a, b)
    assert [c[1] for c in _fmt.decode(got) if c[0] == 9] == [_fmt.B]
    assert _inplace("or", b, a) == O.pairwise("ior", b, a)  # A.ior(B) = B.or(A): R.full


@pytest.mark.parametrize("seed", range(6))
def test_random_in_place(gpu, seed):
    rng = np.random.default_rng(300 + seed)
    keys = np.sort(rng.choice(256, size=int(rng.integers(1, 60)), replace=False))
    a, b = _gen.bitmap(rng, keys), _gen.bitmap(rng, keys, p_present=0.6)
    for op, oop in EXPECT.items():
        assert _inplace(op, a, b) == O.pairwise(oop, a, b), op


def test_self_in_place(gpu):
    """x1.and(x1) / or(x1) return at once; xor(x1) / andNot(x1) clear (RB/RoaringBitmap.java:1271,
    2482, 3297-3300, 1347-1350)"""
    import roaringbitmap_amd as rb
    rng = np.random.default_rng(9)
    buf = _gen.bitmap(rng, np.arange(40))
    for op, exp in (("and_", buf), ("or_", buf), ("xor", O.from_values([])), ("andNot", O.from_values([]))):
        x = rb.RoaringBitmap(buf)
        getattr(x, op)(x)
        assert x.serialize() == exp, op
    # the static forms are untouched by the overloading
    x, y = rb.RoaringBitmap(buf), rb.RoaringBitmap(_gen.bitmap(rng, np.arange(40)))
    assert rb.RoaringBitmap.and_(x, y).serialize() == O.pairwise("and", buf, y.serialize())
    assert getattr(rb.RoaringBitmap, "or")(x, y).serialize() == O.pairwise("or", buf, y.serialize())


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("buffer", [False, True])
def test_merge_random_disjoint(gpu, seed, buffer):
    from roaringbitmap_amd import MutableBitSliceIndex, RoaringBitmapSliceIndex
    cls, ocls = (MutableBitSliceIndex, _bsi.BufferBSI) if buffer else (RoaringBitmapSliceIndex, _bsi.BSI)
    rng = np.random.default_rng(700 + seed)
    cols = rng.permutation(1 << 20)[:int(rng.integers(1000, 80000))]
    split = int(rng.integers(1, cols.size - 1))
    ca, cb = np.sort(cols[:split]), np.sort(cols[split:])
    va = rng.integers(0, 1 << int(rng.integers(1, 20)), ca.size)
    vb = rng.integers(0, 1 << int(rng.integers(1, 20)), cb.size)
    if seed % 3 == 2:  # runs in both
        va, vb = (ca // 500) % 64, (cb // 700) % 1000
    ra, rb_ = bool(seed & 1), bool(seed & 2)
    ga, gb = cls.from_columns(ca, va, ra), cls.from_columns(cb, vb, rb_)
    oa, ob = ocls.from_columns(ca, va, ra), ocls.from_columns(cb, vb, rb_)
    ga.merge(gb)
    oa.merge(ob)
    assert ga.ebM.serialize() == oa.ebm
    assert [x.serialize() for x in ga.bA] == oa.ba
    assert (ga.minValue, ga.maxValue, ga.runOptimized) == (oa.min, oa.max, oa.run_optimized)
    # the merged index answers queries over both column sets
    allc, allv = np.concatenate([ca, cb]), np.concatenate([va, vb])
    lo = int(np.median(allv))
    got = set(ga.compare("GE", lo).toArray().tolist())
    assert got == set(allc[allv >= lo].tolist())


def test_merge_rejects_intersecting(gpu):
    from roaringbitmap_amd import IllegalArgumentException, RoaringBitmapSliceIndex
    a = RoaringBitmapSliceIndex.from_columns([1, 2, 3], [1, 2, 3])
    b = RoaringBitmapSliceIndex.from_columns([3, 4], [5, 6])
    with pytest.raises(IllegalArgumentException):
        a.merge(b)
