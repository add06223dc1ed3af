"""RoaringBitmap.contains(RoaringBitmap subset) (RB/RoaringBitmap.java:2781-2802; ImmutableRoaringBitmap
.contains(ImmutableRoaringBitmap), RB/buffer/ImmutableRoaringBitmap.java:1242) on the MI355X
(rbg_pairwise_card RBG_CONTAINS: |a AND b| == |b| in 64 bits) against set inclusion of the decoded values
(the reference walks both key lists and asks Container.contains(Container), a set test; its advanceUntil
call on the subset's key array only ever advances pos1 by one)."""
import numpy as np
import pytest

import _gen
import _oracle as O
from _fmt import A, B, R, container_table, encode

pytestmark = pytest.mark.gpu


def _sub(buf_a, buf_b):
    a = O.to_values(buf_a)
    b = O.to_values(buf_b)
    return bool(np.isin(b, a).all())


def _check(buf_a, buf_b, tag=""):
    import roaringbitmap_amd as rb
    want = _sub(buf_a, buf_b)
    assert rb.RoaringBitmap(buf_a).contains(rb.RoaringBitmap(buf_b)) == want, tag
    assert rb.ImmutableRoaringBitmap(buf_a).contains(rb.ImmutableRoaringBitmap(buf_b)) == want, tag
    return want


@pytest.mark.parametrize("seed", range(4))
def test_random_subsets(gpu, seed):
    rng = np.random.default_rng(1300 + seed)
    a = _gen.bitmap(rng, np.arange(8), p_present=0.9)
    va = O.to_values(a)
    seen = set()
    for frac in (0.0, 0.01, 0.5, 1.0):
        sub = va[rng.random(va.size) < frac] if frac < 1 else va
        b = O.from_values(sub)
        seen.add(_check(a, b, f"subset {frac}"))
        seen.add(_check(a, O.run_optimize(b), f"subset {frac} runopt"))
        if sub.size:  # one value not in a: a missing value inside a present key, and one in a new key
            miss = np.setdiff1d(np.arange(int(sub[0]), int(sub[0]) + 70000, dtype=np.uint32), va)[:1]
            seen.add(_check(a, O.from_values(np.union1d(sub, miss)), f"subset {frac} + {miss}"))
            seen.add(_check(a, O.from_values(np.union1d(sub, [0xFFFFFFF0])), f"subset {frac} + new key"))
    assert seen == {True, False}


def test_container_kinds_and_edges(gpu):
    full = encode([(k, R, np.arange(65536)) for k in (0, 1, 2)])
    for kind_sub in (A, B, R):
        vals = np.arange(0, 65536, 3) if kind_sub != A else np.arange(0, 9000, 3)
        assert _check(full, encode([(1, kind_sub, vals)]))
        assert not _check(encode([(1, B, np.arange(1, 65536, 3))]), encode([(1, kind_sub, vals)]))
    empty = O.from_values(np.zeros(0, dtype=np.uint32))
    assert _check(full, empty) and _check(empty, empty)
    assert not _check(empty, full)


def test_full_universe(gpu):
    """2^32 values: an int andNot-cardinality would wrap to 0 here; the 64-bit count does not"""
    import roaringbitmap_amd as rb
    univ = rb.RoaringBitmap.add(rb.RoaringBitmap(), 0, 1 << 32)
    empty = rb.RoaringBitmap()
    assert univ.contains(univ) and univ.contains(empty)
    assert not empty.contains(univ)
    holed = rb.RoaringBitmap.remove(univ, 123456, 123457)
    assert univ.contains(holed) and not holed.contains(univ)


def test_is_hamming_similar(gpu):
    """RB/RoaringBitmap.java:1831-1863: true iff the XOR cardinality is within the tolerance"""
    import roaringbitmap_amd as rb
    rng = np.random.default_rng(77)
    a = _gen.bitmap(rng, np.arange(6), p_present=0.9)
    va = O.to_values(a)
    flip = va[rng.random(va.size) < 0.001]
    extra = np.array([0xFFFF0000, 0xFFFF0001, 5], dtype=np.uint32)
    b = O.from_values(np.setxor1d(np.setdiff1d(va, flip), extra))
    d = len(np.setxor1d(va, O.to_values(b)))
    x, y = rb.RoaringBitmap(a), rb.RoaringBitmap(b)
    assert x.isHammingSimilar(y, d) and y.isHammingSimilar(x, d + 5)
    assert not x.isHammingSimilar(y, d - 1)
    assert x.isHammingSimilar(x, 0) and not x.isHammingSimilar(x, -1)
    univ = rb.RoaringBitmap.add(rb.RoaringBitmap(), 0, 1 << 32)
    assert univ.isHammingSimilar(univ, 0)
    assert not univ.isHammingSimilar(rb.RoaringBitmap(), 2 ** 31 - 1)


def test_select_range(gpu):
    """x.selectRange(start, end) (RB/RoaringBitmap.java:3095-3147) and ImmutableRoaringBitmap.selectRange
    (RB/buffer/ImmutableRoaringBitmap.java:701-757) against the oracle's selection (the range
    aggregations' selectRangeWithoutCopy, the same container steps)"""
    import roaringbitmap_amd as rb
    rng = np.random.default_rng(5)
    for m in _gen.MODES:
        ctrs = [(k, *_gen.container(rng, m)) for k in range(3)]
        buf = encode(ctrs)
        for st, en in ((5, 60000), (70000, (2 << 16) + 123), (1 << 16, 3 << 16), (100, 100), (9, 3),
                       (0, 1 << 32), ((1 << 16) + 12288, 2 << 16)):
            got = rb.RoaringBitmap(buf).selectRange(st, en)
            assert type(got) is rb.RoaringBitmap
            assert got.serialize() == O.range_op("select", [buf], st, en), (m, st, en)
            gotb = rb.ImmutableRoaringBitmap(buf).selectRange(st, en)
            assert isinstance(gotb, rb.MutableRoaringBitmap)
            assert gotb.serialize() == O.range_op("select_buf", [buf], st, en), (m, st, en, "buffer")
    x = encode([(1, B, np.arange(0, 65536, 3))])  # 4,096 values kept: heap array, buffer bitmap
    h = rb.RoaringBitmap(x).selectRange(1 << 16, (1 << 16) + 12288).serialize()
    bb = rb.ImmutableRoaringBitmap(x).selectRange(1 << 16, (1 << 16) + 12288).serialize()
    assert h == O.range_op("select", [x], 1 << 16, (1 << 16) + 12288)
    assert bb == O.range_op("select_buf", [x], 1 << 16, (1 << 16) + 12288)
    assert h != bb and len(h) == len(bb)  # 4,096 values: 8,192 payload bytes either way, different bytes
    # no rangeSanityCheck: the bounds are cast like Util.highbits / lowbits (RB/Util.java:436-438,481-483)
    full = encode([(k, R, np.arange(65536)) for k in (0, 1, 65535)])
    for cls in (rb.RoaringBitmap, rb.ImmutableRoaringBitmap):
        sel = "select" if cls is rb.RoaringBitmap else "select_buf"
        # selectRange(x, Long.MAX_VALUE): the last key cut after lowbits(MAX - 1) = 0xFFFE
        assert cls(full).selectRange(5, (1 << 63) - 1).serialize() == O.range_op(sel, [full], 5, (1 << 32) - 1)
        # bounds past 2^32 wrap to their low 32 bits' keys
        assert cls(full).selectRange((1 << 32) + 5, (1 << 32) + 70).serialize() == O.range_op(sel, [full], 5, 70)
        for st, en in ((-1, 10), ((1 << 32) - 70000, (1 << 32) + 10)):  # negative; key casts out of order
            with pytest.raises(ValueError):
                cls(full).selectRange(st, en)


def test_remove_run_compression(gpu):
    import roaringbitmap_amd as rb
    rng = np.random.default_rng(11)
    for m in _gen.MODES:
        buf = encode([(k, *_gen.container(rng, m)) for k in (0, 7, 65535)])
        for cls in (rb.RoaringBitmap, rb.MutableRoaringBitmap):
            x = cls(buf)
            had = x.removeRunCompression()
            assert had == bool((container_table(buf)[1] == R).any())
            assert x.serialize() == O.remove_run_compression(buf), m
            assert x.container_stats()[2] == 0
    y = rb.RoaringBitmap(O.from_values(np.arange(10, dtype=np.uint32), run_optimize=True))
    assert y.removeRunCompression() is True and y.removeRunCompression() is False


def test_limit(gpu):
    """x.limit(n) (RB/RoaringBitmap.java:2457-2476) against the oracle: every mode as the cut container,
    cuts inside containers, at container edges, n <= 0 and n past the cardinality"""
    import roaringbitmap_amd as rb
    rng = np.random.default_rng(21)
    for m in _gen.MODES:
        ctrs = [(k, *_gen.container(rng, m)) for k in (2, 9, 40000)]
        buf = encode(ctrs)
        cards = [len(c[2]) for c in ctrs]
        tot = sum(cards)
        ns = {0, -3, 1, cards[0] - 1, cards[0], cards[0] + 1, cards[0] + cards[1] // 2, tot - 1, tot, tot + 5,
              cards[0] + 4096, cards[0] + 4097, int(rng.integers(1, tot + 1))}
        for n in sorted(ns):
            got = rb.RoaringBitmap(buf).limit(n)
            assert type(got) is rb.RoaringBitmap
            assert got.serialize() == O.limit(buf, n), (m, n)
    got = rb.ImmutableRoaringBitmap(buf).limit(1000)  # RB/buffer/ImmutableRoaringBitmap.java:1658
    assert isinstance(got, rb.MutableRoaringBitmap) and got.serialize() == O.limit(buf, 1000)
    assert rb.ImmutableRoaringBitmap.removeRunCompression is None
    alt = np.arange(0, 65536, 2)  # a run container of 32,768 runs cut after 30,000 of them
    buf = encode([(0, R, alt), (1, A, [3])])
    assert rb.RoaringBitmap(buf).limit(30000).serialize() == O.limit(buf, 30000)


def test_bitmap_of_range(gpu):
    import roaringbitmap_amd as rb
    for lo, hi in ((5, 6), (5, 7), (5, 8), (65535, 65537), (70000, 5 << 16), (12345, (40000 << 16) + 7),
                   (0, 1 << 32), (9, 9), (9, 3)):
        got = rb.RoaringBitmap.bitmapOfRange(lo, hi)
        assert got.serialize() == O.bitmap_of_range(lo, hi), (lo, hi)
    with pytest.raises(rb.IllegalArgumentException):
        rb.RoaringBitmap.bitmapOfRange(0, (1 << 32) + 1)


def test_limit_reference_cases(gpu):
    """RBT/TestRoaringBitmap.java:136-162 through the GPU, byte-exact to the oracle"""
    import roaringbitmap_amd as rb
    i = np.arange(500 * 9943, dtype=np.int64)
    blocks = O.from_values(i[(i // 9943) % 2 == 0].astype(np.uint32))
    got = rb.RoaringBitmap(blocks).limit(1000000)
    assert got.getCardinality() == 1000000 and got.serialize() == O.limit(blocks, 1000000)
    r = rb.RoaringBitmap.add(rb.RoaringBitmap(), 0, 10000000)
    for n in (1, 10, 100, 1000, 10000, 100000, 1000000):
        lim = r.limit(n)
        assert lim.getCardinality() == n and lim.serialize() == O.limit(r.serialize(), n)
