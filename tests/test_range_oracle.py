"""Range-restricted aggregations of the oracle (oracle/rbcpu.cpp: select_range, range_aggregate,
op_andnot_range) against the reference's own tests.  No GPU.

RB/RoaringBitmap.java: and(Iterator, rangeStart, rangeEnd) :1308-1316, or :2536-2543, xor :3359-3365,
andNot(x1, x2, rangeStart, rangeEnd) :1396-1404; each input goes through the private static
selectRangeWithoutCopy (:3160-3214), then FastAggregation.and / or / xor(Iterator) or RoaringBitmap.andNot.
The reference's tests (RBT/TestRoaringBitmap.java:4521-4925, testRanged{Or,And,Xor,AndNot}[BigInts]) check
the sets against a brute force over random bitmaps of 500 values below 1000 (and the same at 2^31 +);
the container types at the cut come from the restatement of Container.remove (A stays A, B becomes A at
<= 4096 values, R stays R with its runs clipped), checked here.
"""
import numpy as np
import pytest

import _oracle as O
from _fmt import A, B, R, decode, encode
from _gen import bitmap


def _set(buf):
    return set(O.to_values(buf).tolist())


@pytest.mark.parametrize("base", [0, 1 << 31])
@pytest.mark.parametrize("op", ["or", "and", "xor", "andnot"])
def test_ranged_ops_brute_force(op, base):
    """RBT/TestRoaringBitmap.java:4521-4925 at their sizes (two bitmaps of 500 draws below 1000, ten ranges
    each, fifty rounds), with runOptimize'd inputs as well."""
    rng = np.random.default_rng(1234 + base % 7)
    for test in range(50):
        v1 = base + rng.integers(0, 1000, 500)
        v2 = base + rng.integers(0, 1000, 500)
        s1, s2 = set(v1.tolist()), set(v2.tolist())
        full = {"or": s1 | s2, "and": s1 & s2, "xor": s1 ^ s2, "andnot": s1 - s2}[op]
        bufs = [O.from_values(v1, test % 2 == 1), O.from_values(v2, test % 3 == 1)]
        for _ in range(10):
            st = int(rng.integers(0, 999))
            en = st + int(rng.integers(0, 1000 - st)) + 1
            got = _set(O.range_op(op, bufs, base + st, base + en))
            assert got == {x for x in full if base + st <= x < base + en}


def test_cut_container_types():
    """Container.remove at the range's first and last keys: an array stays an array, a bitmap left with
    <= 4096 values becomes an array (else stays a bitmap), a run container stays a run container even
    where toEfficientContainer would pick an array; the keys inside the range are untouched and a
    container emptied by the cut is dropped."""
    runs = np.sort(np.concatenate([np.arange(0, 60000, 8), np.arange(1, 60000, 8)]))  # 7,500 runs of 2
    x = encode([(1, B, np.arange(0, 65536, 3)), (2, R, runs), (3, A, np.arange(0, 4000, 2)),
                (4, B, np.arange(0, 65536, 2)), (5, A, np.arange(10, 20))])
    y = encode([(9, A, [1])])
    # [key 1 + 60000, key 4 + 30000): key 1 cut to 1,846 values (A), key 4 to 15,000 (B), key 2 / 3 as is
    got = decode(O.range_op("or", [x, y], (1 << 16) + 60000, (4 << 16) + 30000))
    # (key 2: naive_or of a single run container repairs it to the efficient form, a bitmap of 7,500 runs)
    assert [(c[0], c[1], c[2]) for c in got] == [(1, A, len(range(60000, 65536, 3))), (2, B, 15000),
                                                 (3, A, 2000), (4, B, 15000)]
    # one key: both cuts on key 2, a run container of 2-value runs clipped on both sides stays a run
    # (andNot with a bitmap that lacks the key clones x1's cut container as it is, RB/RoaringBitmap.java:463)
    got = decode(O.range_op("andnot", [x, y], (2 << 16) + 101, (2 << 16) + 20001))
    assert got[0][:2] == (2, R)
    assert list(got[0][3]) == [v for v in runs if 101 <= v <= 20000]
    # a cut that leaves nothing: key 5's array [10, 20) cut to [30, ...) is dropped
    assert decode(O.range_op("or", [x], (5 << 16) + 30, (5 << 16) + 100)) == []


def test_range_sanity_check():
    """rangeSanityCheck (RB/RoaringBitmap.java:204-213): start in [0, 2^32 - 1], end in [0, 2^32]."""
    x = O.from_values([1, 2, 3])
    for st, en in ((-1, 5), (0, (1 << 32) + 1), (1 << 32, (1 << 32)), (0, -3)):
        with pytest.raises(O.OracleError):
            O.range_op("or", [x], st, en)
    assert O.range_op("or", [x], 5, 2) == O.from_values([])  # end <= start: empty
    assert O.range_op("and", [x, x], 0, 1 << 32) == x


@pytest.mark.parametrize("seed", range(4))
def test_ranged_ops_mixed_containers(seed):
    """Every container family at the cut (generator modes incl. full, one-value runs, edge arrays), ranges
    on and off key boundaries: sets equal the brute force, and the unrestricted op of the pre-cut inputs
    restricted afterwards has the same set."""
    rng = np.random.default_rng(70 + seed)
    keys = np.arange(6)
    bufs = [bitmap(rng, keys, p_present=0.8) for _ in range(3)]
    sets = [_set(b) for b in bufs]
    for _ in range(12):
        st = int(rng.integers(0, 6 << 16))
        en = st + int(rng.integers(1, 3 << 16))
        inr = lambda s: {v for v in s if st <= v < en}
        assert _set(O.range_op("or", bufs, st, en)) == inr(sets[0] | sets[1] | sets[2])
        assert _set(O.range_op("and", bufs, st, en)) == inr(sets[0] & sets[1] & sets[2])
        assert _set(O.range_op("xor", bufs, st, en)) == inr(sets[0] ^ sets[1] ^ sets[2])
        assert _set(O.range_op("andnot", bufs[:2], st, en)) == inr(sets[0] - sets[1])


@pytest.mark.parametrize("seed", range(3))
def test_buffer_range_ops_sets(seed):
    """ImmutableRoaringBitmap's range forms (RB/buffer/ImmutableRoaringBitmap.java:261 and -> workShyAnd,
    992 or, 1048 xor, 402 andNot): the same sets as the heap's."""
    rng = np.random.default_rng(90 + seed)
    keys = np.arange(6)
    bufs = [bitmap(rng, keys, p_present=0.8) for _ in range(3)]
    for _ in range(8):
        st = int(rng.integers(0, 6 << 16))
        en = st + int(rng.integers(1, 3 << 16))
        for op in ("and", "or", "xor"):
            assert _set(O.range_op(op + "_buf", bufs, st, en)) == _set(O.range_op(op, bufs, st, en))
        assert _set(O.range_op("andnot_buf", bufs[:2], st, en)) == _set(O.range_op("andnot", bufs[:2], st, en))


def test_buffer_selection_keeps_4096_value_bitmaps():
    """MappeableBitmapContainer.remove makes an array only below 4096 values (RB/buffer/
    MappeableBitmapContainer.java:1597-1612): a bitmap cut to exactly 4096 values stays a bitmap -- its
    payload the 1024 words -- where the heap's BitmapContainer.remove gives an array.  A single input's
    container is cloned by or / xor / andNot, so the result keeps it; workShyAnd repairs it to an array."""
    x = encode([(0, B, np.arange(0, 8192)), (1, A, np.arange(5))])
    words = np.zeros(1024, dtype=np.uint64)
    words[:64] = np.uint64(0xFFFFFFFFFFFFFFFF)
    bits = words.astype("<u8").tobytes()
    vals = np.arange(4096, dtype="<u2").tobytes()
    heap = O.range_op("select", [x], 0, 4096)
    buf = O.range_op("select_buf", [x], 0, 4096)
    assert heap.endswith(vals) and buf.endswith(bits)
    for op in ("or", "xor"):
        assert O.range_op(op, [x], 0, 4096).endswith(vals)
        assert O.range_op(op + "_buf", [x], 0, 4096).endswith(bits)
    empty = O.from_values([])
    assert O.range_op("andnot_buf", [x, empty], 0, 4096).endswith(bits)
    assert O.range_op("and_buf", [x], 0, 4096).endswith(vals)
    assert O.range_op("and_buf", [x, x], 0, 4096) == O.range_op("and", [x, x], 0, 4096)
