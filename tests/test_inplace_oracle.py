"""The oracle's in-place instance ops and RoaringBitmapSliceIndex.merge (CPU, test infrastructure).

x1.or(x2) in place (RB/RoaringBitmap.java:2481-2523) runs Container.ior per matched key, whose
types are the static or's except BitmapContainer.ior(ArrayContainer) (RB/BitmapContainer.java:
740-757): a full result stays a bitmap, where BitmapContainer.or(ArrayContainer) (:1064-1085)
returns RunContainer.full().  x1.and / xor / andNot(x2) in place (Container.iand / ixor / iandNot)
type like the static ops.  merge is pinned to RBBsiTest.testMerge /
BufferBSITest.testMerge (bsi/src/test/.../RBBsiTest.java:47-61, BufferBSITest.java:62-76).
"""
import numpy as np
import pytest

import _bsi
import _fmt
import _gen
import _oracle as O


def test_ior_equals_or_but_full_bitmap_or_array():
    rng = np.random.default_rng(31)
    for m1 in _gen.MODES:
        for m2 in _gen.MODES:
            k1, v1 = _gen.container(rng, m1)
            k2, v2 = _gen.container(rng, m2)
            a, b = _fmt.encode([(3, k1, v1)]), _fmt.encode([(3, k2, v2)])
            full_ba = k1 == _fmt.B and k2 == _fmt.A and len(np.union1d(v1, v2)) == 65536
            if not full_ba:
                assert O.pairwise("ior", a, b) == O.pairwise("or", a, b), (m1, m2)
    # a bitmap missing exactly an array's values: the in-place union is a full BITMAP container
    hole = np.sort(np.random.default_rng(3).choice(65536, 100, replace=False)).astype(np.uint16)
    bvals = np.setdiff1d(np.arange(65536), hole).astype(np.uint16)
    a, b = _fmt.encode([(9, _fmt.B, bvals)]), _fmt.encode([(9, _fmt.A, hole)])
    got = _fmt.decode(O.pairwise("ior", a, b))
    assert [(c[0], c[1], c[2]) for c in got] == [(9, _fmt.B, 65536)]
    assert [(c[0], c[1], c[2]) for c in _fmt.decode(O.pairwise("or", a, b))] == [(9, _fmt.R, 65536)]
    assert [(c[1]) for c in _fmt.decode(O.pairwise("ior", b, a))] == [_fmt.R]  # A.ior(B) = B.or(A)


def test_merge_known_answers():
    """RBBsiTest.java:47-61 / BufferBSITest.java:62-76: values x on columns 1..99 merged with
    values x on columns 100..198"""
    for cls in (_bsi.BSI, _bsi.BufferBSI):
        a = cls.from_columns(np.arange(1, 100), np.arange(1, 100))
        b = cls.from_columns(np.arange(100, 199), np.arange(100, 199))
        assert O.stats(a.ebm)["card"] == 99 and O.stats(b.ebm)["card"] == 99
        a.merge(b)
        for x in range(1, 199, 7):
            assert a.get_value(x) == (x, True)
        assert (a.min, a.max) == (1, 198) and a.bit_count() == 8


def test_merge_rejects_intersecting_indexes():
    a = _bsi.BSI.from_columns([1, 2, 3], [1, 2, 3])
    b = _bsi.BSI.from_columns([3, 4], [5, 6])
    with pytest.raises(ValueError):
        a.merge(b)
