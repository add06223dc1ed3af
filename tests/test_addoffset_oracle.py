"""RoaringBitmap.addOffset(x, offset) in the oracle (oracle/rbcpu.cpp op_add_offset), restating
RB/RoaringBitmap.java:230-288 and Util.addOffset (RB/Util.java:32-126); MutableRoaringBitmap.addOffset
(RB/buffer/MutableRoaringBitmap.java:84-142) types its containers alike.  No GPU.

The sets are what the reference's tests check: RBT/TestConcatenation.java:32-109 (its value-list data
files, tests/golden/testdata/addoffset_*.u32.gz, and container-kind layouts at offsets 20 and 65536),
RBT/TestRoaringBitmap.java:5219-5307 (addoffset, issue418, addNegativeOffset).  The container types
follow the per-key steps: the two parts of each container (arrays split, bitmaps shifted then
repairAfterLazy, run containers split unconverted), a low part OR-ed into the previous high part with
Container.ior, and repairAfterLazy over the result (run containers through toEfficientContainer).
"""
import gzip
import zlib
import os

import numpy as np
import pytest

import _oracle as O
from _fmt import A, B, R, container_table, decode, encode
from _gen import MODES, bitmap, container

TD = os.path.join(os.path.dirname(__file__), "golden", "testdata")


def fixture_values(name):
    with gzip.open(os.path.join(TD, f"addoffset_{name}.u32.gz"), "rb") as f:
        return np.frombuffer(f.read(), dtype="<u4")


def shifted(vals, offset):
    v = vals.astype(np.int64) + offset
    return v[(v >= 0) & (v < 1 << 32)].astype(np.uint32)


def _check_set(buf, offset):
    got = O.to_values(O.add_offset(buf, offset))
    np.testing.assert_array_equal(got, shifted(O.to_values(buf), offset))


@pytest.mark.parametrize("name,offset", [("testIssue260", 5950), ("offset_failure_case_1", 20),
                                         ("offset_failure_case_2", 20), ("offset_failure_case_3", 20)])
def test_concatenation_data_files(name, offset):
    vals = fixture_values(name)
    for ro in (False, True):
        buf = O.from_values(vals, run_optimize=ro)
        _check_set(buf, offset)
        assert O.to_values(O.add_offset(buf, offset)).size == vals.size  # testCardinalityPreserved


@pytest.mark.parametrize("layout", ["B0 R1 A2", "R0 B1 B2", "B0 B1 R2", "B0 R2 A4", "R0 B2 B4", "A0 B2 R4", "B0",
                                    "R0", "A0", "B0 R1", "R0 B1", "A0 B1", "B0 R2", "R0 B2", "A0 B2", "A0 B1 R2"])
@pytest.mark.parametrize("offset", [20, 1 << 16])
def test_concatenation_layouts(layout, offset):
    """TestConcatenation's testCase().withBitmapAt(..).withRunAt(..).withArrayAt(..) layouts"""
    rng = np.random.default_rng(zlib.crc32(f"{layout}@{offset}".encode()))
    mode = {"A": "a_mid", "B": "b_mid", "R": "r_many"}
    ctrs = []
    for item in layout.split():
        kind, vals = container(rng, mode[item[0]])
        ctrs.append((int(item[1:]), kind, vals))
    buf = encode(ctrs)
    _check_set(buf, offset)


def test_full_range_at_offset_20():
    buf = O.from_values(np.arange(1 << 16, dtype=np.uint32), run_optimize=True)  # withRange(0, 1 << 16)
    _check_set(buf, 20)
    got = decode(O.add_offset(buf, 20))
    assert [(c[0], c[1], c[2]) for c in got] == [(0, R, 65516), (1, R, 20)]  # both parts one-run containers


def _ref_bitmap():
    """RBT/TestRoaringBitmap.java:5221-5228"""
    v = [10, 0xFFFF, 0x010101] + list(range(100000, 200000, 4)) + list(range(400000, 1400000))
    return O.from_values(np.array(v, dtype=np.uint32), run_optimize=True)


def test_addoffset_and_negative_offset():
    rb = _ref_bitmap()
    offs = []
    o = 3
    while o < 1000000:
        offs.append(o)
        o *= 3
    o = 1024
    while o < 1000000:
        offs.append(o)
        o *= 2
    for off in offs:
        _check_set(rb, off)
        back = O.add_offset(O.add_offset(rb, off), -off)
        np.testing.assert_array_equal(O.to_values(back), O.to_values(rb))


def test_issue418():
    rb = O.from_values(np.array([0], dtype=np.uint32))
    for s in (100, 0xFFFF0000, 0xFFFF0001):
        sh = O.add_offset(rb, s)
        assert O.to_values(sh).tolist() == [s]
        assert O.to_values(O.add_offset(sh, -s)).tolist() == [0]


@pytest.mark.parametrize("seed", range(4))
def test_random_sets_and_limits(seed):
    rng = np.random.default_rng(40 + seed)
    buf = bitmap(rng, np.sort(rng.choice(65536, 12, replace=False)), p_present=0.9)
    offs = [1, 63, 64, 65, 4096, 65535, 65536, 65537, -1, -65535, -65536, -65537, (1 << 32) - 1, -(1 << 32) + 1,
            1 << 32, -(1 << 32), int(rng.integers(-(1 << 32), 1 << 32))]
    for off in offs:
        _check_set(buf, off)
    # a container offset outside [-65536, 65535]: empty
    assert O.to_values(O.add_offset(buf, 1 << 40)).size == 0


def test_part_types():
    """The types of the merged parts: two arrays by cardinality; a bitmap part OR-ed with an array part
    keeps a full bitmap when the low part is the array (BitmapContainer.ior(ArrayContainer), RB/
    BitmapContainer.java:740-757) and becomes a full run container otherwise; run parts end through
    toEfficientContainer; a bitmap part of <= 4096 values is an array (repairAfterLazy)."""
    off = 65536 - 100
    # key 0: the bitmap [100, 65536) moves whole to key 1 as [0, 65436); key 1: the array [0, 100) stays
    # as [65436, 65536); B.ior(A) at key 1 keeps the full bitmap
    x = encode([(0, B, np.arange(100, 65536)), (1, A, np.arange(0, 100))])
    got = decode(O.add_offset(x, off))
    assert [(c[0], c[1], c[2]) for c in got] == [(1, B, 65536)]
    # the same with an array first and a bitmap second: A.ior(B) = B.or(A) -> full run container
    y = encode([(0, A, np.arange(65436, 65536)), (1, B, np.arange(0, 65436))])
    got = decode(O.add_offset(y, 100))
    assert [(c[0], c[1], c[2]) for c in got] == [(1, R, 65536)]
    # run parts: one-value runs end as an array / bitmap (toEfficientContainer)
    z = encode([(0, R, np.arange(0, 65536, 2))])
    got = decode(O.add_offset(z, 1))
    assert [(c[0], c[1]) for c in got] == [(0, B)]
    # a bitmap part of <= 4096 values is an array
    w = encode([(0, B, np.arange(0, 65536, 4))])
    got = decode(O.add_offset(w, 65536 - 4000))
    assert [(c[0], c[1]) for c in got] == [(0, A), (1, B)]


def test_whole_key_offset_clones_and_drops():
    """offset a multiple of 65536: the containers are cloned under the shifted keys, types untouched (a run
    container that toEfficientContainer would convert stays one); keys leaving [0, 65535] are dropped"""
    x = encode([(0, R, np.arange(0, 100, 2)), (5, A, [1, 2, 3]), (65535, B, np.arange(0, 65536, 3))])
    got = decode(O.add_offset(x, 3 << 16))
    assert [(c[0], c[1]) for c in got] == [(3, R), (8, A)]
    got = decode(O.add_offset(x, -(5 << 16)))
    assert [(c[0], c[1]) for c in got] == [(0, A), (65530, B)]
    assert O.add_offset(x, 0) == x


@pytest.mark.parametrize("mode", MODES)
def test_every_mode_neighbours(mode):
    """each generator mode next to each kind, at offsets that split inside words and at word edges"""
    rng = np.random.default_rng(MODES.index(mode) + 7)
    for other in ("a_mid", "b_mid", "r_many"):
        k1, v1 = container(rng, mode)
        k2, v2 = container(rng, other)
        buf = encode([(3, k1, v1), (4, k2, v2)])
        for off in (1, 37, 64, 4099, 65535, 65536 * 2 + 300, -70000):
            _check_set(buf, off)
            keys, kinds, cards, _, _ = container_table(O.add_offset(buf, off))
            assert np.all(np.diff(keys.astype(np.int64)) > 0)


def test_remove_run_compression():
    """x.removeRunCompression() (RB/RoaringBitmap.java:2738-2749): run containers by cardinality
    (RunContainer.toBitmapOrArrayContainer, RB/RunContainer.java:2300-2323), a full one a bitmap"""
    x = encode([(0, R, np.arange(65536)), (1, R, np.arange(100, 4196)), (2, R, np.arange(100, 4197)),
                (3, A, [1, 2]), (4, B, np.arange(0, 65536, 2))])
    got = decode(O.remove_run_compression(x))
    assert [(c[0], c[1], c[2]) for c in got] == [(0, B, 65536), (1, A, 4096), (2, B, 4097), (3, A, 2),
                                                 (4, B, 32768)]
    np.testing.assert_array_equal(O.to_values(O.remove_run_compression(x)), O.to_values(x))


def test_limit():
    """x.limit(n) (RB/RoaringBitmap.java:2457-2476): the first n values; the cut container through
    Container.limit (an array stays one; a bitmap an array at <= 4096 values; a run container keeps its
    runs up to the n-th value)"""
    x = encode([(0, A, np.arange(0, 3000, 3)), (1, B, np.arange(0, 65536, 2)), (2, R, np.arange(10, 60000)),
                (3, A, [5])])
    vals = O.to_values(x)
    for n in (0, -5, 1, 999, 1000, 1001, 1000 + 4096, 1000 + 4097, 1000 + 32768, 1000 + 32768 + 7,
              len(vals) - 1, len(vals), len(vals) + 10, 2 ** 31 - 1):
        got = O.limit(x, n)
        np.testing.assert_array_equal(O.to_values(got), vals[:max(n, 0)])
    kinds = lambda n: [(c[0], c[1]) for c in decode(O.limit(x, n))]
    assert kinds(1000 + 4096) == [(0, A), (1, A)]
    assert kinds(1000 + 4097) == [(0, A), (1, B)]
    assert kinds(1000 + 32768 + 7) == [(0, A), (1, B), (2, R)]
    assert kinds(500) == [(0, A)]


def test_bitmap_of_range():
    """RoaringBitmap.bitmapOfRange(min, max) (RB/RoaringBitmap.java:588-615): run containers only, even for
    one or two values, where the static add over an empty bitmap writes arrays (Container.rangeOfOnes)"""
    empty = O.from_values(np.zeros(0, dtype=np.uint32))
    for lo, hi in ((5, 6), (5, 7), (5, 8), (65535, 65537), (70000, 5 << 16), (0, 1 << 32), (9, 9), (9, 3)):
        got = O.bitmap_of_range(lo, hi)
        keys, kinds, cards, _, _ = container_table(got)
        assert int(cards.sum()) == max(hi - lo, 0)
        assert (kinds == R).all()
        assert (container_table(O.range_mut("add", empty, lo, hi))[2] == cards).all()
    assert O.bitmap_of_range(5, 7) != O.range_mut("add", empty, 5, 7)
    with pytest.raises(O.OracleError):
        O.bitmap_of_range(-1, 5)


def test_limit_reference_cases():
    """RBT/TestRoaringBitmap.java:136-162: limit of alternating 9,943-value blocks, and limitTest's
    [0, 10^7) at 1 .. 10^6"""
    i = np.arange(500 * 9943, dtype=np.int64)
    blocks = O.from_values(i[(i // 9943) % 2 == 0].astype(np.uint32))
    assert O.to_values(O.limit(blocks, 1000000)).size == 1000000
    empty = O.from_values(np.zeros(0, dtype=np.uint32))
    r = O.range_mut("add", empty, 0, 10000000)
    for n in (1, 10, 100, 1000, 10000, 100000, 1000000):
        got = O.to_values(O.limit(r, n))
        assert got.size == n and int(got[-1]) == n - 1
