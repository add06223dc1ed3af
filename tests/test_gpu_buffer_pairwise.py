"""ImmutableRoaringBitmap / MutableRoaringBitmap pairwise ops on the GPU (rbg_pairwise RBG_AND_BUFFER /
RBG_ANDNOT_BUFFER, csrc/bsi.hip k_pair_buf) against the oracle's and_buf / andnot_buf
(oracle/rbcpu.cpp c_and_buf / c_andnot_buf: RB/buffer/MappeableRunContainer.java:474-536, 600-663 keep
the merged run container; every other pair types like the heap's)."""
import numpy as np
import pytest

import _gen
import _oracle as O
from _fmt import A, R, decode, encode

pytestmark = pytest.mark.gpu


def _rb():
    import roaringbitmap_amd as rb
    return rb


def _check(a, b, tag):
    rb = _rb()
    I = rb.ImmutableRoaringBitmap
    x1, x2 = rb.RoaringBitmap(a), rb.RoaringBitmap(b)
    for op, f in (("and_buf", getattr(I, "and")), ("andnot_buf", I.andNot)):
        got = f(x1, x2)
        assert isinstance(got, rb.MutableRoaringBitmap)
        assert got.serialize() == O.pairwise(op, a, b), f"{tag} {op}"
    # or / xor of the buffer package type like the heap's
    assert getattr(I, "or")(x1, x2).serialize() == O.pairwise("or", a, b), f"{tag} or"
    assert I.xor(x1, x2).serialize() == O.pairwise("xor", a, b), f"{tag} xor"


def test_every_container_mode_pair(gpu):
    """All 18x18 container-mode combinations on one key, plus a key held by one operand only."""
    rng = np.random.default_rng(17)
    for m1 in _gen.MODES:
        for m2 in _gen.MODES:
            k1, v1 = _gen.container(rng, m1)
            k2, v2 = _gen.container(rng, m2)
            k3, v3 = _gen.container(rng, m1)
            _check(encode([(3, k1, v1), (9, k3, v3)]), encode([(3, k2, v2), (11, k3, v3)]), f"{m1}x{m2}")


@pytest.mark.parametrize("seed", range(6))
def test_random_bitmaps(gpu, seed):
    rng = np.random.default_rng(100 + seed)
    keys = np.sort(rng.choice(64, size=int(rng.integers(1, 40)), replace=False))
    _check(_gen.bitmap(rng, keys), _gen.bitmap(rng, keys), f"seed{seed}")


def test_run_results_above_2047_runs(gpu):
    """R AND R into 16,384 one-value runs and R ANDNOT R into 32,768 runs: kept as run containers
    (the big-run arena), where the heap ops convert them."""
    ev = lambda ph: np.sort(np.concatenate([np.arange(ph, 65536, 4), np.arange(1 + ph, 65536, 4)]))
    a = encode([(1, R, ev(0)), (2, R, np.concatenate([np.arange(k, k + 3) for k in range(0, 65530, 4)])),
                (4, A, np.arange(0, 8000, 3))])
    b = encode([(1, R, ev(1)), (2, R, np.arange(1, 65536, 4)), (5, R, np.arange(10, 20))])
    _check(a, b, "bigruns")
    rb = _rb()
    I = rb.ImmutableRoaringBitmap
    got_and = decode(getattr(I, "and")(rb.RoaringBitmap(a), rb.RoaringBitmap(b)).serialize())
    got_andnot = decode(I.andNot(rb.RoaringBitmap(a), rb.RoaringBitmap(b)).serialize())
    assert [c[:2] for c in got_and] == [(1, R), (2, R)]
    assert (2, R) in [c[:2] for c in got_andnot]
    assert O.pairwise("and_buf", a, b) != O.pairwise("and", a, b)
    assert O.pairwise("andnot_buf", a, b) != O.pairwise("andnot", a, b)


def test_mutable_in_place(gpu):
    """MutableRoaringBitmap.and / andNot in place (RB/buffer/MutableRoaringBitmap.java:886-954): the
    static ops' bytes; x1.and(x1) leaves x1, x1.andNot(x1) clears it."""
    rb = _rb()
    rng = np.random.default_rng(5)
    keys = np.arange(12)
    a, b = _gen.bitmap(rng, keys), _gen.bitmap(rng, keys)
    x = rb.MutableRoaringBitmap(a)
    getattr(x, "and")(rb.RoaringBitmap(b))
    assert x.serialize() == O.pairwise("and_buf", a, b)
    y = rb.MutableRoaringBitmap(a)
    y.andNot(rb.RoaringBitmap(b))
    assert y.serialize() == O.pairwise("andnot_buf", a, b)
    z = rb.MutableRoaringBitmap(a)
    getattr(z, "and")(z)
    assert z.serialize() == a
    z.andNot(z)
    assert z.isEmpty()
    # the static forms on the Mutable class are the Immutable ones
    assert getattr(rb.MutableRoaringBitmap, "and")(rb.RoaringBitmap(a), rb.RoaringBitmap(b)).serialize() == \
        O.pairwise("and_buf", a, b)
