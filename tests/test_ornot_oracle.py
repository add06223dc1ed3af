"""orNot of the oracle (oracle/rbcpu.cpp op_ornot, c_not_prefix) against the reference's own tests.  No GPU.

RB/RoaringBitmap.java: x1.orNot(x2, rangeEnd) in place :1431-1506, RoaringBitmap.orNot(x1, x2, rangeEnd)
:1521-1603.  Per key up to maxKey = (rangeEnd - 1) >>> 16: both present -> Container.orNot / iorNot
(RB/Container.java:191-196, 536-541: or / ior with x2.not(0, end).iremove(end, 0x10000)); x1 only -> full,
or x1.ior(rangeOfOnes(0, lastRun)) at maxKey; x2 only -> x2.not(0, end) (not clipped at rangeEnd); neither
-> full, or rangeOfOnes at maxKey; x1's keys above maxKey appended.  The key loop is bounded by the
reference's maxSize estimate, which can stop it early (pinned below as the reference computes it).

Pinned by RBT/TestRoaringBitmapOrNot.java (orNot1..11, the full-bitmap cases, testBigOrNot[Static] over
the fixture testdata/ornot-fuzz-failure.json -> tests/golden/testdata/ornot_fuzz_{l,r}.bin.gz) and
RBT/OrNotTruncationTest.java; a value-level brute force of the key loop covers random inputs.
"""
import gzip
import os
import struct

import numpy as np
import pytest

import _oracle as O
from _fmt import A, B, R, container_table, decode, encode

HERE = os.path.dirname(os.path.abspath(__file__))


def bm(*vals):
    return O.from_values(np.array(vals, dtype=np.uint32))


def vals(buf):
    return O.to_values(buf).astype(np.int64)


def last_value(buf):
    """max value of a serialized bitmap, from its last container alone"""
    keys, kinds, cards, offs, lens = container_table(buf)
    k, kind, off = int(keys[-1]), int(kinds[-1]), int(offs[-1])
    if kind == R:
        nr = struct.unpack_from("<H", buf, off)[0]
        s, ln = struct.unpack_from("<HH", buf, off + 2 + 4 * (nr - 1))
        lo = s + ln
    elif kind == A:
        lo = struct.unpack_from("<H", buf, off + 2 * (int(cards[-1]) - 1))[0]
    else:
        w = np.frombuffer(buf, dtype="<u8", count=1024, offset=off)
        i = int(np.nonzero(w)[0][-1])
        lo = 64 * i + int(w[i]).bit_length() - 1
    return (k << 16) | lo


def both_forms(a, b, end):
    """static and in-place results (the same values on every reference test)"""
    return O.ornot(a, b, end), O.ornot(a, b, end, inplace=True)


def test_ornot_1_to_7():
    """RBT/TestRoaringBitmapOrNot.java:25-210 (in place; the static form gives the same values)"""
    cases = [
        ((2, 1, 1 << 16, 2 << 16, 3 << 16), (1 << 16, 3 << 16), (4 << 16) - 1, np.arange((4 << 16) - 1)),
        ((0, 1 << 16, 3 << 16), ((4 << 16) - 1,), 4 << 16, np.arange((4 << 16) - 1)),
        ((2 << 16,), (1 << 14, 3 << 16), 5 << 16, np.setdiff1d(np.arange(5 << 16), [1 << 14, 3 << 16])),
        ((1,), (3 << 16,), (2 << 16) + (2 << 14), np.arange((2 << 16) + (2 << 14))),
        ((1, 1 << 16, 2 << 16, 3 << 16), (), 5 << 16, np.arange(5 << 16)),
        ((1, (1 << 16) - 1, 1 << 16, 2 << 16, 3 << 16), (), 1 << 14,
         np.concatenate([np.arange(1 << 14), [(1 << 16) - 1, 1 << 16, 2 << 16, 3 << 16]])),
        ((1 << 16, 2 << 16, 3 << 16), (), 1 << 14, np.concatenate([np.arange(1 << 14), [1 << 16, 2 << 16, 3 << 16]])),
    ]
    for x1, x2, end, want in cases:
        for got in both_forms(bm(*x1), bm(*x2), end):
            assert np.array_equal(vals(got), want), (x1, x2, end)


def test_ornot_9_static():
    """RBT/TestRoaringBitmapOrNot.java:212-307"""
    rb1 = bm(1 << 16, 2 << 16, 3 << 16)
    got = vals(O.ornot(rb1, bm(), 1 << 14))
    assert np.array_equal(got, np.concatenate([np.arange(1 << 14), [1 << 16, 2 << 16, 3 << 16]]))
    got = vals(O.ornot(rb1, bm(), 2 << 16))
    assert np.array_equal(got, np.concatenate([np.arange((2 << 16) + 1), [196608]]))
    rb2 = bm((1 << 16) + (1 << 13), (1 << 16) + (1 << 14), (1 << 16) + (1 << 15))
    got = vals(O.ornot(rb1, rb2, 2 << 16))
    assert len(got) == (2 << 16) - 1
    rb2 = bm(1 << 16, 3 << 16, 4 << 16)
    assert np.array_equal(vals(O.ornot(rb1, rb2, 5 << 16)), np.setdiff1d(np.arange(5 << 16), [4 << 16]))
    assert np.array_equal(vals(O.ornot(rb2, rb1, 5 << 16)), np.setdiff1d(np.arange(5 << 16), [2 << 16]))


def test_ornot_10_11():
    """RBT/TestRoaringBitmapOrNot.java:309-332: the last value stays below / at the range end"""
    for got in both_forms(bm(5), bm(10), 6):
        assert last_value(got) == 5
    a = bm(65535 * 65536 + 65523)
    b = bm(65493 * 65536 + 65520)
    assert last_value(O.ornot(a, b, 65535 * 65536 + 65524)) == 65535 * 65536 + 65523


def test_against_full_bitmap():
    """RBT/TestRoaringBitmapOrNot.java:334-368"""
    full = O.from_values(np.arange(0x40000, dtype=np.uint32))
    for got in both_forms(bm(), full, 0x30000):
        assert len(vals(got)) == 0
    for got in both_forms(bm(1, 0x10001, 0x20001), full, 0x30000):
        assert vals(got).tolist() == [1, 0x10001, 0x20001]


def _range_bitmap(limit):
    """[0, limit) as run containers, serialized directly (65536-value runs per key)"""
    nk = (limit + 65535) >> 16
    keys = np.arange(nk)
    lens = np.full(nk, 65535, dtype=np.int64)
    lens[-1] = (limit - 1) - ((nk - 1) << 16)
    fl = bytearray((nk + 7) // 8)
    for i in range(nk):
        fl[i // 8] |= 1 << (i % 8)
    out = bytearray(struct.pack("<I", 12347 | ((nk - 1) << 16)) + fl)
    out += np.stack([keys, lens], 1).astype("<u2").tobytes()
    header = len(out) + (4 * nk if nk >= 4 else 0)
    if nk >= 4:
        out += (header + 6 * np.arange(nk)).astype("<u4").tobytes()
    pay = np.zeros((nk, 3), dtype="<u2")
    pay[:, 0] = 1
    pay[:, 2] = lens
    return bytes(out + pay.tobytes())


def test_big_ornot_fuzz_fixture():
    """RBT/TestRoaringBitmapOrNot.java:370-424 testBigOrNot / testBigOrNotStatic: with limit = l.last() + 1,
    orNot(l, r, limit) equals or(l, andNot([0, limit), r)) (value equality)."""
    td = os.path.join(HERE, "golden", "testdata")
    l = gzip.open(os.path.join(td, "ornot_fuzz_l.bin.gz")).read()
    r = gzip.open(os.path.join(td, "ornot_fuzz_r.bin.gz")).read()
    last = decode(l)[-1]
    limit = (int(last[0]) << 16) + int(last[3][-1]) + 1
    expected = O.pairwise("or", l, O.pairwise("andnot", _range_bitmap(limit), r))
    for got in both_forms(l, r, limit):
        assert O.pairwise_card("xor", got, expected) == 0


def test_truncation_cases():
    """RBT/OrNotTruncationTest.java: one = {0, 10}; one.orNot(other, 7) keeps 10"""
    others = [bm(), bm(2), bm(2, 3, 4), bm(3, 4), bm(1), bm(*range(7)),
              encode([(0, A, np.arange(0, 3000, 7))]), encode([(0, R, np.arange(100, 5000))]),
              encode([(0, B, np.arange(0, 60000, 3))]),
              encode([(0, A, np.arange(10, 90)), (1, R, np.arange(5, 500))]),
              encode([(1, A, np.arange(10, 90))]), encode([(1, R, np.arange(5, 500)), (2, R, np.arange(9, 99))]),
              encode([(1, B, np.arange(0, 60000, 3)), (2, R, np.arange(9, 99))])]
    for other in others:
        got = vals(O.ornot(bm(0, 10), other, 7, inplace=True))
        assert 10 in got.tolist()


def _brute(x1, x2, end, inplace):
    """Value-level restatement of the key loop of RB/RoaringBitmap.java:1521-1603 (static) / :1431-1506
    (per key a 65536-entry membership mask)."""
    def by_key(v):
        v = np.asarray(v, dtype=np.int64)
        d = {}
        for k in np.unique(v >> 16).tolist():
            m = np.zeros(65536, dtype=bool)
            m[v[(v >> 16) == k] & 0xFFFF] = True
            d[k] = m
        return d
    k1, k2 = by_key(x1), by_key(x2)
    max_key = -1 if end == 0 else (end - 1) >> 16
    last_run = 0x10000 if end & 0xFFFF == 0 else end & 0xFFFF
    keys1, keys2 = sorted(k1), sorted(k2)
    rem = sum(1 for k in keys1 if k > max_key)
    corr = 0
    for i in range(len(keys2) - rem):
        corr += bool(k2[keys2[i]].all())
        if keys2[i] >= max_key:
            break
    max_size = min(max_key + 1 + rem - corr + len(keys1), 0x10000)
    if max_size < 0:
        return None
    out, size = [], 0
    idx = np.arange(65536)
    for key in range(max_key + 1):
        if size >= max_size:
            break
        rng_mask = idx < (last_run if key == max_key else 0x10000)
        if key in k1 and key in k2:
            c = k1[key] | (rng_mask & ~k2[key])
        elif key in k1:
            c = k1[key] | rng_mask
        elif key in k2:
            c = (rng_mask & ~k2[key]) | (~rng_mask & k2[key])
        else:
            c = rng_mask
        if c.any():
            out.append((key << 16) + np.nonzero(c)[0])
            size += 1
    for k in keys1:
        if k > max_key:
            out.append((k << 16) + np.nonzero(k1[k])[0])
    return np.concatenate(out).tolist() if out else []


@pytest.mark.parametrize("seed", range(12))
def test_random_against_brute_force(seed):
    rng = np.random.default_rng(seed)
    for _ in range(3):
        v1 = np.unique(rng.integers(0, 4 << 16, int(rng.integers(0, 300)))).astype(np.uint32)
        v2 = np.unique(rng.integers(0, 4 << 16, int(rng.integers(0, 300)))).astype(np.uint32)
        if seed % 3 == 1:  # a full container in x2 (the maxSize correction)
            v2 = np.union1d(v2, np.arange(1 << 16, 2 << 16)).astype(np.uint32)
        a, b = O.from_values(v1, seed % 2 == 1), O.from_values(v2, seed % 4 >= 2)
        for end in (0, 1, 2, 3, 7, 65535, 65536, 65537, (1 << 16) + 300, 3 << 16, (3 << 16) + 12345, 5 << 16):
            for inplace in (False, True):
                want = _brute(v1.tolist(), v2.tolist(), end, inplace)
                got = vals(O.ornot(a, b, end, inplace))
                assert got.tolist() == want, (seed, end, inplace)


def test_reference_quirks():
    """Edge behaviour of the reference kept: an x2-only container at maxKey keeps its values >= rangeEnd;
    the maxSize estimate stops the key loop early; a negative maxSize throws; rangeSanityCheck."""
    # x2 only at maxKey: not(0, lastRun) is not clipped
    assert vals(O.ornot(bm(), bm(5, 100), 50)).tolist() == [x for x in range(50) if x != 5] + [100]
    # x1 empty, x2 = {key 5: full}, rangeEnd = 2 keys: maxSize = 1 -> only key 0
    full5 = encode([(5, R, np.arange(65536))])
    assert vals(O.ornot(bm(), full5, 2 << 16)).tolist() == list(range(1 << 16))
    # rangeEnd = 0, x1 empty, x2[0] full: maxSize = -1
    full01 = encode([(0, R, np.arange(65536)), (1, R, np.arange(65536))])
    with pytest.raises(O.NegativeArraySize):
        O.ornot(bm(), full01, 0)
    assert O.ornot(bm(3, 1 << 20), full01, 0) == bm(3, 1 << 20)
    for end in (-1, (1 << 32) + 1):
        with pytest.raises(O.OracleError):
            O.ornot(bm(1), bm(2), end)


def test_container_types():
    """Result types follow the container chain: not() types, iremove, then or / ior."""
    # x2-only array of 10 values -> not -> bitmap (card 65526)
    got = decode(O.ornot(bm(), encode([(0, A, np.arange(10))]) + b"", 1 << 17))
    assert [(c[0], c[1]) for c in got] == [(0, B), (1, R)]
    # x2-only run [0, 65534] -> not -> {65535}: run (6 B) vs array (4 B) -> array
    got = decode(O.ornot(bm(), encode([(0, R, np.arange(65535))]), 1 << 16))
    assert [(c[0], c[1], c[2]) for c in got] == [(0, A, 1)]
    # neither at maxKey with lastRun <= 2 -> rangeOfOnes is an array; above 2 a run
    assert [c[1] for c in decode(O.ornot(bm(), bm(), 2))] == [A]
    assert [c[1] for c in decode(O.ornot(bm(), bm(), 3))] == [R]
    # BitmapContainer.ior(ArrayContainer) keeps a full bitmap (in place); or() gives the full run
    c1 = encode([(0, B, np.arange(1, 65536))])
    c2 = encode([(0, A, np.arange(1, 4000))])  # not -> 61537 values, bitmap; or with c1 -> full
    assert [c[1] for c in decode(O.ornot(c1, c2, 1 << 16))] == [R]
    c2 = encode([(0, B, np.arange(1, 65536))])  # not -> {0}: array
    assert [c[1] for c in decode(O.ornot(c1, c2, 1 << 16))] == [R]
    assert [c[1] for c in decode(O.ornot(c1, c2, 1 << 16, inplace=True))] == [B]


def test_buffer_package_types():
    """ImmutableRoaringBitmap.orNot / MutableRoaringBitmap.orNot (RB/buffer/ImmutableRoaringBitmap.java:484-548,
    MutableRoaringBitmap.java:962-1030) run the same loop; their containers type like the heap's except
    MappeableBitmapContainer.iremove, an array only below 4096 values (RB/buffer/MappeableBitmapContainer.java
    :1003-1017).  x2's complement clipped to exactly 4096 values, or'ed with a subset of it: the heap gives an
    array, the buffer package a bitmap -- whose 4096-value payload is its 1024 words (a card-4096 container
    reads back as an array in the portable format, so only the payload bytes tell them apart)."""
    e = 10000
    c2 = encode([(0, B, np.concatenate([np.arange(0, e - 4096), np.arange(20000, 30001)]))])
    c1 = encode([(0, A, np.array([e - 4096, e - 1]))])
    want = np.arange(e - 4096, e)
    words = np.zeros(1024, dtype=np.uint64)
    np.bitwise_or.at(words, want >> 6, np.uint64(1) << (want.astype(np.uint64) & np.uint64(63)))
    for inplace in (False, True):
        heap, buf = O.ornot(c1, c2, e, inplace), O.ornot(c1, c2, e, inplace, buffer=True)
        assert heap[-8192:] == want.astype("<u2").tobytes()
        assert buf[-8192:] == words.astype("<u8").tobytes()
    # elsewhere the bytes agree
    rng = np.random.default_rng(4)
    for _ in range(6):
        v1 = np.unique(rng.integers(0, 3 << 16, 200)).astype(np.uint32)
        v2 = np.unique(rng.integers(0, 3 << 16, 5000)).astype(np.uint32)
        a, b = O.from_values(v1), O.from_values(v2)
        for end in (1 << 16, (2 << 16) + 999, 3 << 16):
            assert O.ornot(a, b, end, buffer=True) == O.ornot(a, b, end)
