"""RoaringBitmap.orNot on the MI355X (rbg_ornot: ornot.hip k_ornot_scan / k_plan_ornot / k_ornot) vs the
oracle (oracle/rbcpu.cpp op_ornot, pinned by tests/test_ornot_oracle.py), byte for byte: the result
container types of Container.not / iremove / or / ior are part of the bytes.

RB/RoaringBitmap.java: static orNot(x1, x2, rangeEnd) :1521-1603, x1.orNot(x2, rangeEnd) in place
:1431-1506 (ends in Container.iorNot and ior).
"""
import gzip
import os

import numpy as np
import pytest

import _gen
import _oracle as O
from _fmt import A, B, R, encode

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))


def _rb():
    import roaringbitmap_amd as rb
    return rb


def _check(a, b, end, tag=""):
    rb = _rb()
    x1, x2 = rb.RoaringBitmap(a), rb.RoaringBitmap(b)
    got = rb.RoaringBitmap.orNot(x1, x2, end).serialize()
    assert got == O.ornot(a, b, end), f"static {tag} end={end}"
    assert x1.serialize() == a  # x1 left unchanged
    y = rb.RoaringBitmap(a)
    y.orNot(x2, end)
    assert y.serialize() == O.ornot(a, b, end, inplace=True), f"inplace {tag} end={end}"
    # the buffer package: ImmutableRoaringBitmap.orNot (static) and MutableRoaringBitmap.orNot (in place)
    got = rb.ImmutableRoaringBitmap.orNot(rb.ImmutableRoaringBitmap(a), rb.ImmutableRoaringBitmap(b), end)
    assert isinstance(got, rb.MutableRoaringBitmap)
    assert got.serialize() == O.ornot(a, b, end, buffer=True), f"buffer static {tag} end={end}"
    m = rb.MutableRoaringBitmap(a)
    m.orNot(rb.ImmutableRoaringBitmap(b), end)
    assert m.serialize() == O.ornot(a, b, end, inplace=True, buffer=True), f"buffer inplace {tag} end={end}"



def test_every_container_mode_pair(gpu):
    """All 18x18 container-mode pairs on key 3, cut at and around maxKey; plus each mode alone in x1 / x2."""
    rng = np.random.default_rng(23)
    for m1 in _gen.MODES:
        for m2 in _gen.MODES:
            k1, v1 = _gen.container(rng, m1)
            k2, v2 = _gen.container(rng, m2)
            a = encode([(1, k1, v1), (3, k1, v1), (6, k2, v2)])
            b = encode([(2, k2, v2), (3, k2, v2), (7, k1, v1)])
            for end in ((3 << 16) + 65536, (3 << 16) + int(rng.integers(1, 65536)), (2 << 16) + 100, 8 << 16):
                _check(a, b, end, f"{m1}x{m2}")


@pytest.mark.parametrize("seed", range(6))
def test_random_bitmaps(gpu, seed):
    rng = np.random.default_rng(300 + seed)
    keys = np.sort(rng.choice(48, size=int(rng.integers(1, 40)), replace=False))
    a, b = _gen.bitmap(rng, keys, p_present=0.7), _gen.bitmap(rng, keys, p_present=0.7)
    for end in [0, 1, 2, 3, 1 << 16, 48 << 16, 1 << 32] + [int(rng.integers(0, 50 << 16)) for _ in range(8)]:
        _check(a, b, end, f"seed{seed}")


def test_reference_cases(gpu):
    """RBT/TestRoaringBitmapOrNot.java orNot1..11 and the full-bitmap cases, and RBT/OrNotTruncationTest.java,
    through the GPU (bytes against the oracle, whose values those tests pin)."""
    bm = lambda *v: O.from_values(np.array(v, dtype=np.uint32))
    cases = [
        (bm(2, 1, 1 << 16, 2 << 16, 3 << 16), bm(1 << 16, 3 << 16), (4 << 16) - 1),
        (bm(0, 1 << 16, 3 << 16), bm((4 << 16) - 1), 4 << 16),
        (bm(2 << 16), bm(1 << 14, 3 << 16), 5 << 16),
        (bm(1), bm(3 << 16), (2 << 16) + (2 << 14)),
        (bm(1, 1 << 16, 2 << 16, 3 << 16), bm(), 5 << 16),
        (bm(1, (1 << 16) - 1, 1 << 16, 2 << 16, 3 << 16), bm(), 1 << 14),
        (bm(1 << 16, 2 << 16, 3 << 16), bm(), 1 << 14),
        (bm(1 << 16, 2 << 16, 3 << 16), bm(1 << 16, 3 << 16, 4 << 16), 5 << 16),
        (bm(5), bm(10), 6),
        (bm(65535 * 65536 + 65523), bm(65493 * 65536 + 65520), 65535 * 65536 + 65524),
    ]
    full = O.from_values(np.arange(0x40000, dtype=np.uint32))
    cases += [(bm(), full, 0x30000), (bm(1, 0x10001, 0x20001), full, 0x30000)]
    for other in (bm(), bm(2), bm(2, 3, 4), bm(1), bm(*range(7)), encode([(0, R, np.arange(100, 5000))]),
                  encode([(1, B, np.arange(0, 60000, 3)), (2, R, np.arange(9, 99))])):
        cases.append((bm(0, 10), other, 7))
    for i, (a, b, end) in enumerate(cases):
        _check(a, b, end, f"case{i}")


def test_fuzz_fixture(gpu):
    """RBT/TestRoaringBitmapOrNot.java:370-424 testBigOrNot[Static] (fixture ornot-fuzz-failure.json):
    65,366 result containers, most of them full."""
    td = os.path.join(HERE, "golden", "testdata")
    l = gzip.open(os.path.join(td, "ornot_fuzz_l.bin.gz")).read()
    r = gzip.open(os.path.join(td, "ornot_fuzz_r.bin.gz")).read()
    from test_ornot_oracle import last_value
    limit = last_value(l) + 1
    _check(l, r, limit, "fuzz")
    _check(r, l, limit, "fuzz-swapped")
    _check(l, r, 1 << 32, "fuzz-full-range")


def test_quirks_and_errors(gpu):
    rb = _rb()
    bm = lambda *v: O.from_values(np.array(v, dtype=np.uint32))
    # the maxSize bound cutting the loop short, x2-only maxKey values above rangeEnd kept
    _check(bm(), encode([(5, R, np.arange(65536))]), 2 << 16, "truncated")
    _check(bm(), bm(5, 100), 50, "unclipped")
    # BitmapContainer.ior(ArrayContainer) keeps a full bitmap in place; or() gives the full run
    _check(encode([(0, B, np.arange(1, 65536))]), encode([(0, B, np.arange(1, 65536))]), 1 << 16, "ior-full")
    _check(encode([(0, B, np.arange(1, 65536))]), bm(), 1, "ior-full-maxkey")
    # the buffer package keeps a 4096-value bitmap through iremove (its payload the 1024 words)
    e = 10000
    c2 = encode([(0, B, np.concatenate([np.arange(0, e - 4096), np.arange(20000, 30001)]))])
    c1 = encode([(0, A, np.array([e - 4096, e - 1]))])
    assert O.ornot(c1, c2, e, buffer=True) != O.ornot(c1, c2, e)
    _check(c1, c2, e, "buffer-4096")
    # rangeEnd == 0: x1 cloned, or NegativeArraySizeException (x1 empty, x2's first container full)
    full01 = encode([(0, R, np.arange(65536)), (1, R, np.arange(65536))])
    _check(bm(3, 1 << 20), full01, 0, "end0")
    _check(bm(), bm(7), 0, "end0-empty")
    with pytest.raises(O.NegativeArraySize):
        O.ornot(bm(), full01, 0)
    with pytest.raises(rb.IllegalArgumentException):
        rb.RoaringBitmap.orNot(rb.RoaringBitmap(bm()), rb.RoaringBitmap(full01), 0)
    for end in (-1, (1 << 32) + 1):
        with pytest.raises(rb.IllegalArgumentException):
            rb.RoaringBitmap.orNot(rb.RoaringBitmap(bm(1)), rb.RoaringBitmap(bm(2)), end)
    x = rb.RoaringBitmap(bm(1, 2))
    with pytest.raises(NotImplementedError):
        x.orNot(x, 10)


def test_dense_full_universe(gpu):
    """rangeEnd = 2^32 over 4096-key operands: 65,536 result containers (the full-run fast path)."""
    rng = np.random.default_rng(77)
    keys = np.sort(rng.choice(65536, size=4096, replace=False))
    a = _gen.bitmap(rng, keys, p_present=0.6)
    b = _gen.bitmap(rng, keys, p_present=0.6)
    _check(a, b, 1 << 32, "dense")
    _check(a, b, (int(keys[2000]) << 16) + 777, "dense-cut")


def test_resident_batches(gpu):
    """rbg_ctx_ornot over device-resident batches (Engine.ornot), fetched through the context"""
    rb = _rb()
    rng = np.random.default_rng(9)
    keys = np.arange(20)
    a, b = _gen.bitmap(rng, keys), _gen.bitmap(rng, keys)
    eng = rb.Engine()
    ia, ib = eng.load_pair(a, b)
    for end, inplace in ((7 << 16, False), ((12 << 16) + 5, True), (1 << 32, False)):
        eng.ornot(ia, ib, end, inplace)
        assert eng.fetch().serialize() == O.ornot(a, b, end, inplace), (end, inplace)


def _realdata(ds):
    z = np.load(os.path.join(HERE, "golden", "realdata", ds + ".npz"))
    v, o = z["values"], z["offsets"]
    return [v[o[i]:o[i + 1]] for i in range(len(o) - 1)]


@pytest.mark.parametrize("ds", ["census1881", "wikileaks-noquotes", "uscensus2000"])
def test_realdata_pairwise_ornot(gpu, ds):
    """jmh/.../realdata/RealDataBenchmarkOrNot.java:20-27 pairwiseOrNot: for k, b[k].clone().orNot(b[k+1],
    b[k].last()) in place and RoaringBitmap.orNot(b[k], b[k+1], toUnsignedLong(b[k].last())), every 9th pair
    (runOptimize'd inputs on odd pairs) against the oracle"""
    rb = _rb()
    sets = _realdata(ds)
    for k in range(0, len(sets) - 1, 9):
        a = O.from_values(sets[k], k % 2 == 1)
        b = O.from_values(sets[k + 1], k % 2 == 1)
        last = int(sets[k].max())
        _check(a, b, last, f"{ds}[{k}]")
