"""RoaringBitmap.addOffset on the MI355X (rbg_add_offset: addoffset.hip k_plan_aoff / k_aoff) vs the oracle
(oracle/rbcpu.cpp op_add_offset, pinned by tests/test_addoffset_oracle.py), byte for byte.

RB/RoaringBitmap.java:230-288 (Util.addOffset RB/Util.java:32-126); the buffer package's
MutableRoaringBitmap.addOffset (RB/buffer/MutableRoaringBitmap.java:84-142).  The cases follow
RBT/TestConcatenation.java and RBT/TestRoaringBitmap.java:5219-5307.
"""
import numpy as np
import pytest

import _gen
import _oracle as O
from _fmt import A, B, R, encode
from test_addoffset_oracle import _ref_bitmap, fixture_values

pytestmark = pytest.mark.gpu


def _rb():
    import roaringbitmap_amd as rb
    return rb


def _check(buf, off, tag=""):
    rb = _rb()
    got = rb.RoaringBitmap.addOffset(rb.RoaringBitmap(buf), off)
    assert isinstance(got, rb.RoaringBitmap)
    want = O.add_offset(buf, off)
    assert got.serialize() == want, f"{tag} offset {off}"
    gm = rb.MutableRoaringBitmap.addOffset(rb.ImmutableRoaringBitmap(buf), off)
    assert isinstance(gm, rb.MutableRoaringBitmap)
    assert gm.serialize() == want, f"{tag} buffer offset {off}"


OFFSETS = [1, 20, 37, 63, 64, 65, 4096, 5950, 65535, 65536, 65537, 3 << 16, -1, -65535, -65536, -65537, -70000,
           (1 << 32) - 1, -(1 << 32) + 1, 1 << 32, 1 << 40]


@pytest.mark.parametrize("seed", range(4))
def test_random_bitmaps(gpu, seed):
    rng = np.random.default_rng(700 + seed)
    keys = np.sort(rng.choice(65536, 10, replace=False)) if seed % 2 else np.arange(10)
    buf = _gen.bitmap(rng, keys, p_present=0.8)
    for off in OFFSETS + [int(rng.integers(-(1 << 32), 1 << 32)) for _ in range(4)]:
        _check(buf, off, f"seed{seed}")


def test_every_container_mode_pair(gpu):
    """each generator mode next to each kind (the parts OR-ed at one key), at offsets inside words, at
    word edges and negative ones"""
    rng = np.random.default_rng(17)
    for m in _gen.MODES:
        for other in ("a_tiny", "a_mid", "b_mid", "b_dense", "r_few", "r_many", "full_r"):
            k1, v1 = _gen.container(rng, m)
            k2, v2 = _gen.container(rng, other)
            for buf in (encode([(3, k1, v1), (4, k2, v2)]), encode([(3, k2, v2), (4, k1, v1)])):
                for off in (1, 64, 4099, 65535 - 17, -70000):
                    _check(buf, off, f"{m}/{other}")


def test_reference_cases(gpu):
    for name, off in (("testIssue260", 5950), ("offset_failure_case_1", 20), ("offset_failure_case_2", 20),
                      ("offset_failure_case_3", 20)):
        vals = fixture_values(name)
        for ro in (False, True):
            _check(O.from_values(vals, run_optimize=ro), off, name)
    rb = _ref_bitmap()
    for off in (3, 9, 27, 243, 6561, 1024, 65536, 524288):
        _check(rb, off, "addoffset")
        _check(O.add_offset(rb, off), -off, "addNegativeOffset")
    one = O.from_values(np.array([0], dtype=np.uint32))
    for s in (100, 0xFFFF0000, 0xFFFF0001):
        _check(one, s, "issue418")
        _check(O.add_offset(one, s), -s, "issue418 back")


def test_part_type_edges(gpu):
    """full unions: bitmap part then array part keeps a full bitmap, array then bitmap gives a full run
    container; one-value runs; a bitmap part of <= 4096 values; a run container of 32,768 runs"""
    cases = [(encode([(0, B, np.arange(100, 65536)), (1, A, np.arange(0, 100))]), 65436),
             (encode([(0, A, np.arange(65436, 65536)), (1, B, np.arange(0, 65436))]), 100),
             (encode([(0, R, np.arange(0, 65536, 2))]), 1),
             (encode([(0, R, np.arange(0, 65536, 2)), (1, R, np.arange(1, 65536, 2))]), 3),
             (encode([(0, B, np.arange(0, 65536, 4))]), 65536 - 4000),
             (encode([(0, R, np.arange(65536)), (1, R, np.arange(65536)), (65535, R, np.arange(65536))]), 20),
             (encode([(0, R, np.arange(0, 100, 2)), (5, A, [1, 2, 3]), (65535, B, np.arange(0, 65536, 3))]), 3 << 16)]
    for buf, off in cases:
        _check(buf, off, "edge")
        _check(buf, -off, "edge neg")


def test_resident_batch(gpu):
    """rbg_ctx_add_offset over a device-resident batch"""
    rb = _rb()
    rng = np.random.default_rng(9)
    buf = _gen.bitmap(rng, np.arange(12))
    eng = rb.Engine()
    (ia,) = eng.load_pair(buf)
    for off in (777, -(1 << 16) - 5, 1 << 20, 1 << 41):
        eng.add_offset(ia, off)
        assert eng.fetch().serialize() == O.add_offset(buf, off), off
