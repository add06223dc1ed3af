"""Static range mutations of the oracle (oracle/rbcpu.cpp op_range_mut): RoaringBitmap.add(rb, rangeStart,
rangeEnd) (RB/RoaringBitmap.java:298-345), remove(rb, ...) (:995-1040), flip(rb, ...) (:626-668), and
MutableRoaringBitmap's (RB/buffer/MutableRoaringBitmap.java:152-205, 649-700, 455-505).  No GPU.

The sets are what RBT/TestRoaringBitmap.java's ranged add / remove / flip tests check (brute force over
random bitmaps); the container types follow the per-key steps: Container.add (an array above 4096 values
becomes a bitmap, a bitmap stays a bitmap even when full, a run container stays one), the keys between
the first and last replaced by full run containers (add) or dropped (remove), Container.remove, and
Container.not (arrays / bitmaps by cardinality, run containers through toEfficientContainer).
"""
import numpy as np
import pytest

import _oracle as O
from _fmt import A, B, R, container_table, decode, encode
from _gen import bitmap


def _set(buf):
    return set(O.to_values(buf).tolist())


@pytest.mark.parametrize("seed", range(6))
def test_sets_brute_force(seed):
    rng = np.random.default_rng(seed)
    keys = np.arange(5)
    buf = bitmap(rng, keys, p_present=0.7)
    s = _set(buf)
    ranges = [(0, 0), (5, 3), (0, 5 << 16), (1 << 16, 2 << 16), (65535, 65537)]
    ranges += [(int(a), int(a) + int(rng.integers(1, 3 << 16))) for a in rng.integers(0, 5 << 16, 10)]
    for st, en in ranges:
        rng_set = set(range(st, en))
        for buffer in (False, True):
            assert _set(O.range_mut("add", buf, st, en, buffer)) == s | rng_set, (st, en)
            assert _set(O.range_mut("remove", buf, st, en, buffer)) == s - rng_set, (st, en)
            assert _set(O.range_mut("flip", buf, st, en, buffer)) == s ^ rng_set, (st, en)
    # the whole universe: add fills every key, remove empties the bitmap, flip complements it
    keys, kinds, cards, _, _ = container_table(O.range_mut("add", buf, 0, 1 << 32))
    assert len(keys) == 65536 and int(cards.sum()) == 1 << 32
    assert O.range_mut("remove", buf, 0, 1 << 32) == O.from_values(np.zeros(0, dtype=np.uint32))
    keys, kinds, cards, _, _ = container_table(O.range_mut("flip", buf, 0, 1 << 32))
    assert int(cards.sum()) == (1 << 32) - len(s)


def test_container_types():
    x = encode([(0, A, np.arange(0, 4000, 2)), (1, B, np.arange(0, 65536, 3)), (2, R, np.arange(100, 200)),
                (4, R, np.concatenate([np.arange(k, k + 2) for k in range(0, 40000, 16)]))])
    kinds = lambda b: [(c[0], c[1]) for c in decode(b)]
    # add: key 0 array -> 4000 + 2000 values > 4096: bitmap; keys 1..3 between first and last: full
    # run containers (key 3 missing); key 4 run container plus [0, 10): a run container
    got = decode(O.range_mut("add", x, 3000, (4 << 16) + 10))
    assert [(c[0], c[1]) for c in got] == [(0, B), (1, R), (2, R), (3, R), (4, R)]
    assert got[1][2] == 65536 and got[3][2] == 65536
    # a bitmap filled completely stays a bitmap (BitmapContainer.add)
    full_b = decode(O.range_mut("add", x, 1 << 16, 2 << 16))
    assert (1, B) in [(c[0], c[1]) for c in full_b] and [c[2] for c in full_b if c[0] == 1] == [65536]
    # a missing key: rangeOfOnes, an array up to two values
    assert kinds(O.range_mut("add", x, (3 << 16) + 5, (3 << 16) + 7))[3] == (3, A)
    assert kinds(O.range_mut("add", x, (3 << 16) + 5, (3 << 16) + 8))[3] == (3, R)
    # remove: a bitmap cut to <= 4096 values becomes an array (the heap), below 4096 (the buffer package);
    # key 1 holds 21,846 values, so keep [0, 12288): 4,096 values
    heap = decode(O.range_mut("remove", x, (1 << 16) + 12288, 2 << 16))
    buf = decode(O.range_mut("remove", x, (1 << 16) + 12288, 2 << 16, buffer=True))
    assert [c[1] for c in heap if c[0] == 1] == [A]
    assert [c[2] for c in heap if c[0] == 1] == [4096]
    assert O.range_mut("remove", x, (1 << 16) + 12288, 2 << 16, buffer=True) != \
        O.range_mut("remove", x, (1 << 16) + 12288, 2 << 16)
    assert len(buf) == len(heap)
    # remove over whole keys drops them, a run container keeps its clipped runs
    assert [c[0] for c in decode(O.range_mut("remove", x, 1 << 16, 3 << 16))] == [0, 4]
    assert kinds(O.range_mut("remove", x, (4 << 16) + 1, (4 << 16) + 30000))[-1] == (4, R)
    # flip: a run container through toEfficientContainer; emptied containers dropped
    assert kinds(O.range_mut("flip", x, (2 << 16) + 100, (2 << 16) + 200)) == [(0, A), (1, B), (4, R)]
    assert kinds(O.range_mut("flip", x, (2 << 16), (3 << 16)))[2] == (2, R)


def test_range_sanity_and_empty_range():
    x = O.from_values(np.array([1, 2, 3], dtype=np.uint32))
    for op in ("add", "remove", "flip"):
        assert O.range_mut(op, x, 7, 7) == x
        assert O.range_mut(op, x, 9, 2) == x
        for st, en in ((-1, 5), (0, (1 << 32) + 1)):
            with pytest.raises(O.OracleError):
                O.range_mut(op, x, st, en)


def test_in_place_add_keeps_container_kinds_between():
    """x.add(rangeStart, rangeEnd) in place (RB/RoaringBitmap.java:1181-1206) runs Container.iadd on every key
    of the range: an array between the first and last key becomes a full bitmap (toBitmapContainer().iadd),
    a bitmap a full bitmap, a run container a full run; the static add puts full run containers there"""
    x = encode([(0, A, np.arange(5)), (1, A, np.arange(7)), (2, B, np.arange(0, 65536, 2)), (3, R, np.arange(9)),
                (5, A, [1])])
    got = decode(O.range_mut("add_inplace", x, 3, (5 << 16) + 2))
    assert [(c[0], c[1], c[2]) for c in got] == [(0, B, 65536), (1, B, 65536), (2, B, 65536), (3, R, 65536),
                                                 (4, R, 65536), (5, A, 2)]
    stat = [(c[0], c[1]) for c in decode(O.range_mut("add", x, 3, (5 << 16) + 2))]
    assert stat == [(0, B), (1, R), (2, R), (3, R), (4, R), (5, A)]
    assert _set(O.range_mut("add_inplace", x, 3, (5 << 16) + 2)) == _set(O.range_mut("add", x, 3, (5 << 16) + 2))
    for buffer in (False, True):
        assert O.range_mut("add_inplace", x, 9, 7, buffer) == x
