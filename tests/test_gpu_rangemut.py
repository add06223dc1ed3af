"""Static range mutations on the MI355X (rbg_range_mut: rangemut.hip k_plan_rmut / k_rmut) vs the oracle
(oracle/rbcpu.cpp op_range_mut, pinned by tests/test_rangemut_oracle.py), byte for byte.

RB/RoaringBitmap.java: add(rb, rangeStart, rangeEnd) :298-345, remove :995-1040, flip :626-668; the buffer
package's MutableRoaringBitmap.add / remove / flip (RB/buffer/MutableRoaringBitmap.java:152, 649, 455) and
ImmutableRoaringBitmap.flip (:592).
"""
import numpy as np
import pytest

import _gen
import _oracle as O
from _fmt import A, B, R, container_table, encode

pytestmark = pytest.mark.gpu


def _rb():
    import roaringbitmap_amd as rb
    return rb


def _check(buf, st, en, tag=""):
    rb = _rb()
    x = rb.RoaringBitmap(buf)
    m = rb.MutableRoaringBitmap(buf)
    for op in ("add", "remove", "flip"):
        got = getattr(rb.RoaringBitmap, op)(x, st, en).serialize()
        assert got == O.range_mut(op, buf, st, en), f"{tag} {op} [{st}, {en})"
        gotb = getattr(rb.MutableRoaringBitmap, op)(m, st, en)
        assert isinstance(gotb, rb.MutableRoaringBitmap)
        assert gotb.serialize() == O.range_mut(op, buf, st, en, buffer=True), f"{tag} buffer {op} [{st}, {en})"
    assert x.serialize() == buf
    # in place: x.add / remove / flip(rangeStart, rangeEnd) (RB/RoaringBitmap.java:1181, 2656, 1893)
    for cls, buffer in ((rb.RoaringBitmap, False), (rb.MutableRoaringBitmap, True)):
        for op in ("add", "remove", "flip"):
            y = cls(buf)
            assert getattr(y, op)(st, en) is None
            want = O.range_mut("add_inplace" if op == "add" else op, buf, st, en, buffer=buffer)
            assert y.serialize() == want, f"{tag} in-place {cls.__name__}.{op} [{st}, {en})"
            assert y.getLongCardinality() == int(container_table(want)[2].sum())


def _ranges(rng, nkeys):
    out = [(0, 0), (9, 3), (0, 1 << 32), (0, nkeys << 16), (1 << 16, 2 << 16), (65535, 65537), (5, 6), (5, 8)]
    for _ in range(10):
        st = int(rng.integers(0, nkeys << 16))
        out.append((st, st + int(rng.integers(1, 3 << 16))))
    return out


@pytest.mark.parametrize("seed", range(5))
def test_random_bitmaps(gpu, seed):
    rng = np.random.default_rng(900 + seed)
    keys = np.arange(8)
    buf = _gen.bitmap(rng, keys, p_present=0.75)
    for st, en in _ranges(rng, 8):
        _check(buf, st, en, f"seed{seed}")


def test_every_container_mode(gpu):
    """each generator mode (incl. run containers above 2047 runs, which add / remove keep as run containers:
    the big-run arena) at the first, last and a middle key of a range"""
    rng = np.random.default_rng(31)
    for m in _gen.MODES:
        ctrs = []
        for k in range(4):
            kind, vals = _gen.container(rng, m)
            ctrs.append((k, kind, vals))
        buf = encode(ctrs)
        for st, en in ((int(rng.integers(0, 65536)), (3 << 16) + int(rng.integers(0, 65536))),
                       ((1 << 16) + 77, (1 << 16) + 40000), (0, 4 << 16), ((2 << 16) + 1, (2 << 16) + 2)):
            _check(buf, st, en, m)


def test_buffer_remove_keeps_4096_value_bitmap(gpu):
    x = encode([(0, A, np.arange(0, 4000, 2)), (1, B, np.arange(0, 65536, 3))])
    assert O.range_mut("remove", x, (1 << 16) + 12288, 2 << 16, buffer=True) != \
        O.range_mut("remove", x, (1 << 16) + 12288, 2 << 16)
    _check(x, (1 << 16) + 12288, 2 << 16, "b4096")


def test_in_place_add_between_keys(gpu):
    """the in-place add's Container.iadd on the keys between the first and last (an array there becomes a
    full bitmap) against the static add's full run containers"""
    rb = _rb()
    x = encode([(0, A, np.arange(5)), (1, A, np.arange(7)), (2, B, np.arange(0, 65536, 2)), (3, R, np.arange(9)),
                (5, A, [1])])
    y = rb.RoaringBitmap(x)
    y.add(3, (5 << 16) + 2)
    assert y.serialize() == O.range_mut("add_inplace", x, 3, (5 << 16) + 2)
    assert y.serialize() != rb.RoaringBitmap.add(rb.RoaringBitmap(x), 3, (5 << 16) + 2).serialize()
    with pytest.raises(NotImplementedError):
        rb.ImmutableRoaringBitmap(x).flip(3, 9)
    with pytest.raises(rb.IllegalArgumentException):
        y.add(-1, 3)


def test_immutable_flip_and_errors(gpu):
    rb = _rb()
    rng = np.random.default_rng(3)
    buf = _gen.bitmap(rng, np.arange(6))
    got = rb.ImmutableRoaringBitmap.flip(rb.ImmutableRoaringBitmap(buf), 1000, 5 << 16)
    assert isinstance(got, rb.MutableRoaringBitmap)
    assert got.serialize() == O.range_mut("flip", buf, 1000, 5 << 16, buffer=True)
    for st, en in ((-1, 5), (0, (1 << 32) + 1)):
        with pytest.raises(rb.IllegalArgumentException):
            rb.RoaringBitmap.add(rb.RoaringBitmap(buf), st, en)


def test_resident_batch(gpu):
    """rbg_ctx_range_mut over a device-resident batch"""
    rb = _rb()
    import roaringbitmap_amd._lib as L
    rng = np.random.default_rng(8)
    buf = _gen.bitmap(rng, np.arange(10))
    eng = rb.Engine()
    (ia,) = eng.load_pair(buf)
    for op in ("add", "remove", "flip"):
        L.check(L.lib().rbg_ctx_range_mut(eng._ctx, L.RMUT_OP[op], ia, 0, 12345, (7 << 16) + 5))
        assert eng.fetch().serialize() == O.range_mut(op, buf, 12345, (7 << 16) + 5), op


def test_max_run_count_inputs(gpu):
    """run containers of 32,768 one-value runs (the most a container can hold): add / remove keep them as
    run containers of that size (the big-run arena), flip makes them bitmaps; orNot and the buffer
    package's and / andNot take them as operands"""
    rb = _rb()
    alt = np.arange(0, 65536, 2)
    x = encode([(0, R, alt), (1, R, alt + 1), (2, A, np.arange(0, 4000, 3))])
    y = encode([(0, R, alt + 1), (1, B, np.arange(0, 65536, 5)), (3, R, alt)])
    for st, en in ((5, 60000), (0, 3 << 16), (70000, (2 << 16) + 9)):
        _check(x, st, en, "maxruns")
    for end in (1 << 16, (1 << 16) + 1001, 4 << 16):
        got = rb.RoaringBitmap.orNot(rb.RoaringBitmap(x), rb.RoaringBitmap(y), end).serialize()
        assert got == O.ornot(x, y, end), end
    I = rb.ImmutableRoaringBitmap
    assert getattr(I, "and")(I(x), I(y)).serialize() == O.pairwise("and_buf", x, y)
    assert I.andNot(I(x), I(y)).serialize() == O.pairwise("andnot_buf", x, y)
