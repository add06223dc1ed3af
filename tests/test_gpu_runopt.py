"""runOptimize on the device (RB/RoaringBitmap.java:2764-2774) vs the oracle's runOptimize.

Every container family of tests/_gen.py (arrays, bitmaps, runs, full containers, edge
cardinalities) is run through rbg_run_optimize_many / Engine.run_optimize; the result
bytes must equal the oracle's, and runOptimize's boolean must be "any run container".
"""
import numpy as np
import pytest

import _gen
import _oracle as O

pytestmark = pytest.mark.gpu


def _answer(buf):
    return O.stats(buf)["run"] > 0


@pytest.mark.parametrize("seed", range(4))
def test_run_optimize_many_families(gpu, seed):
    import roaringbitmap_amd as rb
    rng = np.random.default_rng(900 + seed)
    bufs = []
    for i in range(60):
        keys = np.sort(rng.choice(1 << 16, size=int(rng.integers(1, 12)), replace=False))
        bufs.append(_gen.bitmap(rng, keys))
    bufs.append(O.from_values([]))                             # empty bitmap
    bufs.append(O.from_values(np.arange(1 << 16)))              # one full container
    bufs.append(O.from_values(np.arange(0, 1 << 17, 2)))        # alternating bits: stays B
    bufs.append(O.from_values(np.arange(100, 4196)))            # A -> R
    bufs.append(O.from_values([5, 70000, 140000]))               # single values stay A
    bms = [rb.RoaringBitmap(b) for b in bufs]
    ans = rb.run_optimize_many(bms)
    for b, bm, a in zip(bufs, bms, ans):
        exp = O.run_optimize(b)
        assert bm.serialize() == exp
        assert a == _answer(exp)


@pytest.mark.parametrize("seed", range(2))
def test_single_bitmap_run_optimize(gpu, seed):
    """RoaringBitmap.runOptimize() (rbg_run_optimize: the device pass over a one-bitmap batch)."""
    import roaringbitmap_amd as rb
    rng = np.random.default_rng(950 + seed)
    for i in range(12):
        keys = np.sort(rng.choice(1 << 16, size=int(rng.integers(1, 20)), replace=False))
        buf = _gen.bitmap(rng, keys)
        bm = rb.RoaringBitmap(buf)
        answer = bm.runOptimize()
        exp = O.run_optimize(buf)
        assert bm.serialize() == exp
        assert answer == _answer(exp)
    bm = rb.RoaringBitmap(O.from_values([]))
    assert bm.runOptimize() is False and bm.serialize() == O.from_values([])


def test_engine_run_optimize_c2_batch(gpu):
    """A synthetic C2 operand (65,536 keys, mixed A/B/R) optimized on the device and then
    used as an operand: bytes equal to the oracle's runOptimize, and AND results equal to
    the oracle's AND of the optimized inputs."""
    from roaringbitmap_amd import Engine
    e = Engine(0)
    a = e.synth(0, 0xC2A0)
    b = e.synth(0, 0xC2B0)
    oa, ans = e.run_optimize(a)
    ob, _ = e.run_optimize(b)
    src_a, src_b = e.batch_fetch(a).serialize(), e.batch_fetch(b).serialize()
    opt_a, opt_b = e.batch_fetch(oa).serialize(), e.batch_fetch(ob).serialize()
    assert opt_a == O.run_optimize(src_a)
    assert opt_b == O.run_optimize(src_b)
    assert ans == [_answer(opt_a)]
    st = e.batch_stats(oa)
    ost = O.stats(opt_a)
    assert (st["array"], st["bitmap"], st["run"]) == (ost["array"], ost["bitmap"], ost["run"])
    assert st["serialized_bytes"] in (0, len(opt_a))
    e.pairwise("and", oa, ob)
    assert e.fetch().serialize() == O.pairwise("and", opt_a, opt_b)
    for x in (a, b, oa, ob):
        e.release(x)


def test_bsi_run_optimize(gpu):
    import roaringbitmap_amd as rb
    rng = np.random.default_rng(5)
    cols = np.sort(rng.choice(1 << 20, 20000, replace=False))
    v = rng.integers(0, 1 << 12, cols.size)
    bsi = rb.RoaringBitmapSliceIndex.from_columns(cols, v)
    before = [bsi.ebM.serialize()] + [s.serialize() for s in bsi.bA]
    bsi.runOptimize()
    assert bsi.runOptimized
    after = [bsi.ebM.serialize()] + [s.serialize() for s in bsi.bA]
    assert after == [O.run_optimize(b) for b in before]


def test_run_optimize_reuses_released_buffers(gpu):
    """A context keeps the device buffers of released batches for the next batch of a similar
    size (engine.cpp pool_take / pool_put): back-to-back runOptimize + release cycles over
    different inputs reuse them, and every result still equals the oracle's (no stale bytes of
    an earlier batch leak into a later one)."""
    from roaringbitmap_amd import Engine
    rng = np.random.default_rng(990)
    e = Engine(0)
    try:
        for cycle in range(6):
            bufs = []
            for i in range(8):
                keys = np.sort(rng.choice(1 << 16, size=int(rng.integers(1, 30)), replace=False))
                bufs.append(_gen.bitmap(rng, keys))
            a = e.load(bufs)
            o, answers = e.run_optimize(a)
            got = e.batch_fetch_range(o)
            for b, g, ans in zip(bufs, got, answers):
                exp = O.run_optimize(b)
                assert g.serialize() == exp, cycle
                assert bool(ans) == _answer(exp)
            e.release(o)
            e.release(a)
    finally:
        e.close()


def test_engine_run_optimize_without_readback(gpu):
    """runOptimize with no booleans asked for (the bench's timed loop): the new batch's statistics stay
    on the device; the first host-side use reads them (kinds, payload bytes), an op uses the batch
    before that, and releasing it needs no read-back.  Same bytes as the synchronous form."""
    from roaringbitmap_amd import Engine
    e = Engine(0)
    a = e.synth(0, 0xC2A0)
    b = e.synth(0, 0xC2B0)
    src_a, src_b = e.batch_fetch(a).serialize(), e.batch_fetch(b).serialize()
    for _ in range(3):  # released without read-back, buffers back to the pool and reused
        o, none = e.run_optimize(a, answers=False)
        assert none is None
        e.release(o)
    oa, _ = e.run_optimize(a, answers=False)
    ob, _ = e.run_optimize(b, answers=False)
    e.pairwise("and", oa, ob)  # an op on the pending batches (reads their statistics first)
    exp_a, exp_b = O.run_optimize(src_a), O.run_optimize(src_b)
    assert e.fetch().serialize() == O.pairwise("and", exp_a, exp_b)
    st = e.batch_stats(oa)
    ost = O.stats(exp_a)
    assert (st["array"], st["bitmap"], st["run"]) == (ost["array"], ost["bitmap"], ost["run"])
    assert e.batch_fetch(oa).serialize() == exp_a
    oc, ans = e.run_optimize(oa)  # runOptimize of an optimized batch: nothing changes
    assert e.batch_fetch(oc).serialize() == exp_a and ans == [_answer(exp_a)]
    for x in (a, b, oa, ob, oc):
        e.release(x)


def test_all_array_result_with_holes(gpu):
    """runOptimize writes every container at its own slot offset, so an R -> A conversion leaves a hole
    after the new array.  A batch of arrays and such run containers becomes all-array with holes: the
    wide OR must not take the back-to-back value stream over it (Batch::gapped), and its bytes equal the
    oracle's naive_or of the optimized inputs."""
    from _fmt import A, R, encode
    from roaringbitmap_amd import Engine
    rng = np.random.default_rng(31)
    bufs = []
    for i in range(6):
        ctrs = []
        for k in range(8):
            if (i + k) % 2:  # one-value runs: R -> A (2 card < 2 + 4 nruns)
                ctrs.append((k, R, np.arange(3 * i + k, 3 * i + k + 400, 2)))
            else:
                ctrs.append((k, A, np.sort(rng.choice(65536, int(rng.integers(1, 3000)), replace=False))))
        bufs.append(encode(ctrs))
    e = Engine(0)
    try:
        a = e.load(bufs)
        o, _ = e.run_optimize(a, answers=False)
        e.wide("or", o)
        opt = [O.run_optimize(b) for b in bufs]
        assert all(O.stats(b)["run"] == 0 and O.stats(b)["bitmap"] == 0 for b in opt)
        assert e.fetch().serialize() == O.wide("or", opt)
        e.wide("xor", o)
        assert e.fetch().serialize() == O.wide("xor", opt)
        got = e.batch_fetch_range(o)
        assert [g.serialize() for g in got] == opt
    finally:
        e.close()
