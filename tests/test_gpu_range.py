"""Range-restricted aggregations on the MI355X vs the oracle, byte for byte.

RB/RoaringBitmap.java: and(Iterator, rangeStart, rangeEnd) :1308-1316, or :2536-2543, xor :3359-3365,
andNot(x1, x2, rangeStart, rangeEnd) :1396-1404; every input through selectRangeWithoutCopy (:3160-3214)
on the device (rbg_ctx_select_range: k_rsel_plan / k_rsel_write), then the wide / pairwise kernels.
The sets are what RBT/TestRoaringBitmap.java:4521-4925 check; the bytes are the oracle's
(tests/test_range_oracle.py pins it).
"""
import numpy as np
import pytest

import _gen
import _oracle as O
from _fmt import A, B, R, decode, encode

pytestmark = pytest.mark.gpu


def _rb():
    import roaringbitmap_amd as rb
    return rb


def _gpu(op, bufs, start, end):
    rb = _rb()
    bms = [rb.RoaringBitmap(b) for b in bufs]
    if op == "andnot":
        return getattr(rb.RoaringBitmap, "andNot")(bms[0], bms[1], start, end).serialize()
    return getattr(rb.RoaringBitmap, op)(iter(bms), start, end).serialize()


def _ranges(rng, nkeys):
    out = [(0, 1 << 32), (0, 0), (7, 3), (1 << 16, 2 << 16), (65535, 65537), (12345, 12346)]
    for _ in range(10):
        st = int(rng.integers(0, nkeys << 16))
        out.append((st, st + int(rng.integers(1, 3 << 16))))
    return out


@pytest.mark.parametrize("seed", range(4))
def test_range_ops_mixed(gpu, seed):
    rng = np.random.default_rng(500 + seed)
    keys = np.arange(8)
    bufs = [_gen.bitmap(rng, keys, p_present=0.85) for _ in range(4)]
    for st, en in _ranges(rng, 8):
        for op in ("and", "or", "xor"):
            assert _gpu(op, bufs, st, en) == O.range_op(op, bufs, st, en), (op, st, en)
        assert _gpu("andnot", bufs[:2], st, en) == O.range_op("andnot", bufs[:2], st, en), (st, en)


def test_range_select_types(gpu):
    """The device selection keeps the reference's cut types (A stays A, B -> A at <= 4096, R stays R,
    clipped) and drops emptied containers: the selected batch's bytes equal the oracle's select_range."""
    from roaringbitmap_amd import Engine
    runs = np.sort(np.concatenate([np.arange(0, 60000, 8), np.arange(1, 60000, 8)]))
    x = encode([(1, B, np.arange(0, 65536, 3)), (2, R, runs), (3, A, np.arange(0, 4000, 2)),
                (4, B, np.arange(0, 65536, 2)), (5, A, np.arange(10, 20)), (6, R, np.arange(65536))])
    e = Engine(0)
    b = e.load([x])
    for st, en in (((1 << 16) + 60000, (4 << 16) + 30000), ((2 << 16) + 101, (2 << 16) + 20001),
                   ((5 << 16) + 30, (5 << 16) + 100), ((6 << 16) + 5, (6 << 16) + 65535), (0, 1 << 32),
                   ((4 << 16) + 1, (4 << 16) + 8193), (9, 3)):
        s = e.select_range(b, st, en)
        assert e.batch_fetch(s).serialize() == O.range_op("select", [x], st, en), (st, en)
        e.release(s)
    e.release(b)


def test_range_ops_runs_and_many_inputs(gpu):
    """Inputs with long run containers (up to 32,768 runs) and ten bitmaps: the run clipping of k_rsel_write
    and a multi-bitmap selection (per-bitmap container counts, the key CSR rebuilt on the device)."""
    rng = np.random.default_rng(9)
    bufs = []
    for i in range(10):
        ctrs = [(k, R, np.arange(i % 2, 65536, 2)) if (i + k) % 3 == 0 else
                (k, B, np.sort(rng.choice(65536, 30000, replace=False))) if (i + k) % 3 == 1 else
                (k, A, np.sort(rng.choice(65536, 3000, replace=False))) for k in range(0, 12, 2)]
        bufs.append(encode(ctrs))
    for st, en in ((3 << 16, (9 << 16) + 777), ((2 << 16) + 30001, (2 << 16) + 30002), (1000, (11 << 16)),
                   ((4 << 16) + 65535, (10 << 16) + 1)):
        for op in ("and", "or", "xor"):
            assert _gpu(op, bufs, st, en) == O.range_op(op, bufs, st, en), (op, st, en)
        assert _gpu("andnot", bufs[:2], st, en) == O.range_op("andnot", bufs[:2], st, en)


def test_range_sanity(gpu):
    rb = _rb()
    x = rb.RoaringBitmap.bitmapOf(1, 2, 3)
    for st, en in ((-1, 5), (0, (1 << 32) + 1), (1 << 32, 1 << 32)):
        with pytest.raises(rb.IllegalArgumentException):
            rb.RoaringBitmap.or_(iter([x, x]), st, en)
    assert getattr(rb.RoaringBitmap, "and")(iter([x, x]), 2, 3).toArray().tolist() == [2]


def _gpu_buf(op, bufs, start, end):
    rb = _rb()
    I = rb.ImmutableRoaringBitmap
    bms = [I(b) for b in bufs]
    if op == "andnot":
        got = I.andNot(bms[0], bms[1], start, end)
    else:
        got = getattr(I, op)(iter(bms), start, end)
    assert isinstance(got, rb.MutableRoaringBitmap)
    return got.serialize()


@pytest.mark.parametrize("seed", range(3))
def test_buffer_range_ops(gpu, seed):
    """ImmutableRoaringBitmap's range forms (RB/buffer/ImmutableRoaringBitmap.java:261 and -> workShyAnd,
    992 or, 1048 xor, 402 andNot with the buffer run types) against the oracle's range_aggregate_buf"""
    rng = np.random.default_rng(700 + seed)
    keys = np.arange(8)
    bufs = [_gen.bitmap(rng, keys, p_present=0.85) for _ in range(4)]
    for st, en in _ranges(rng, 8):
        for op in ("and", "or", "xor"):
            assert _gpu_buf(op, bufs, st, en) == O.range_op(op + "_buf", bufs, st, en), (op, st, en)
        assert _gpu_buf("andnot", bufs[:2], st, en) == O.range_op("andnot_buf", bufs[:2], st, en), (st, en)
    # one input, and no input at all
    for op in ("and", "or", "xor"):
        assert _gpu_buf(op, bufs[:1], 1000, 5 << 16) == O.range_op(op + "_buf", bufs[:1], 1000, 5 << 16)
        assert _gpu_buf(op, [], 0, 1 << 32) == O.range_op(op + "_buf", [], 0, 1 << 32)


def test_buffer_range_keeps_4096_value_bitmaps(gpu):
    """MappeableBitmapContainer.remove keeps a bitmap of exactly 4096 values (RB/buffer/
    MappeableBitmapContainer.java:1597-1612); the heap's becomes an array"""
    x = encode([(0, B, np.arange(0, 8192)), (1, A, np.arange(5)), (2, B, np.arange(0, 65536, 2))])
    y = encode([(3, A, [7])])
    for st, en in ((0, 4096), (4096, 8192), (0, (2 << 16) + 8192)):
        for op in ("or", "xor", "and"):
            assert _gpu_buf(op, [x], st, en) == O.range_op(op + "_buf", [x], st, en), (op, st, en)
            assert _gpu(op, [x], st, en) == O.range_op(op, [x], st, en), (op, st, en)
        assert _gpu_buf("andnot", [x, y], st, en) == O.range_op("andnot_buf", [x, y], st, en)
    assert O.range_op("or_buf", [x], 0, 4096) != O.range_op("or", [x], 0, 4096)
