"""Batched andCardinality (config C4) vs a loop of the oracle's andCardinality."""
import numpy as np
import pytest

import _gen
import _oracle as O

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("seed", range(3))
def test_batch_and_card(gpu, seed):
    import roaringbitmap_amd as rb
    rng = np.random.default_rng(77 + seed)
    pairs = []
    for i in range(300):
        keys = np.sort(rng.choice(64, size=int(rng.integers(1, 5)), replace=False))
        keys2 = np.sort(rng.choice(64, size=int(rng.integers(1, 5)), replace=False)) if i % 3 else keys
        modes = None if i % 2 else ["a_small", "a_mid", "a_tiny"]
        pairs.append((_gen.bitmap(rng, keys, modes=modes, p_present=1.0),
                      _gen.bitmap(rng, keys2, modes=modes, p_present=1.0)))
    got = rb.batch_and_cardinality([(rb.RoaringBitmap(a), rb.RoaringBitmap(b)) for a, b in pairs])
    exp = np.array([O.pairwise_card("and", a, b) for a, b in pairs], dtype=np.int32)
    np.testing.assert_array_equal(got, exp)


def test_c4_synthetic_pairs(gpu):
    """C4 batches generated on the device: batched andCardinality == oracle per pair."""
    from roaringbitmap_amd import Engine
    e = Engine(0)
    n = 3000
    b = e.synth(3, 0xC4, n)
    st = e.batch_stats(b)
    assert st["bitmaps"] == 2 * n and st["array"] == st["containers"]
    e.batch_and_card(b)
    got = e.cards(n)
    bms = [e.batch_fetch(b, i).serialize() for i in range(2 * n)]
    exp = np.array([O.pairwise_card("and", bms[2 * i], bms[2 * i + 1]) for i in range(n)], dtype=np.int32)
    np.testing.assert_array_equal(got, exp)
    assert sum(O.stats(x)["card"] for x in bms) == st["cardinality"]
    matched, allb = e.pair_bytes(b)
    assert 0 < matched <= allb


def test_batch_and_card_large_and_mixed_pairs(gpu):
    """Pairs above the 64-key small-pair threshold (one wave per pair) mixed with small
    ones (one thread per pair aligns keys, one wave per matched key), every container
    family, empty bitmaps included."""
    import roaringbitmap_amd as rb
    rng = np.random.default_rng(4242)
    pairs = []
    for i in range(120):
        if i % 4 == 0:
            ka = np.sort(rng.choice(200, size=int(rng.integers(40, 120)), replace=False))
            kb = np.sort(rng.choice(200, size=int(rng.integers(40, 120)), replace=False))
        elif i % 4 == 1:
            ka = np.sort(rng.choice(64, size=int(rng.integers(1, 30)), replace=False))
            kb = np.sort(rng.choice(64, size=int(rng.integers(1, 30)), replace=False))
        elif i % 4 == 2:
            ka, kb = np.array([], dtype=np.int64), np.sort(rng.choice(64, size=3, replace=False))
        else:
            ka = np.sort(rng.choice(8, size=int(rng.integers(1, 8)), replace=False))
            kb = ka
        a = _gen.bitmap(rng, ka, p_present=1.0) if ka.size else O.from_values([])
        b = _gen.bitmap(rng, kb, p_present=1.0) if kb.size else O.from_values([])
        pairs.append((a, b))
    got = rb.batch_and_cardinality([(rb.RoaringBitmap(a), rb.RoaringBitmap(b)) for a, b in pairs])
    exp = np.array([O.pairwise_card("and", a, b) for a, b in pairs], dtype=np.int32)
    np.testing.assert_array_equal(got, exp)


def test_batch_and_card_threshold_pairs(gpu):
    """Pairs at the small-pair bound (64 keys in all): 32 + 32 identical keys give the most
    matched keys a small pair can have (32, one count byte); 33 + 32 keys go the large
    path; many such pairs span several plan workgroups (256 pairs each)."""
    import roaringbitmap_amd as rb
    rng = np.random.default_rng(6464)
    pairs = []
    for i in range(700):
        m = i % 5
        if m == 0:
            ka = kb = np.arange(32) * 3
        elif m == 1:
            ka, kb = np.arange(33) * 2, np.arange(32) * 2
        elif m == 2:
            ka, kb = np.arange(40), np.arange(24) + 16
        elif m == 3:
            ka, kb = np.sort(rng.choice(100, size=31, replace=False)), np.sort(rng.choice(100, size=33, replace=False))
        else:
            ka, kb = np.array([7]), np.array([7])
        pairs.append((_gen.bitmap(rng, ka, modes=["a_tiny", "a_small"], p_present=1.0),
                      _gen.bitmap(rng, kb, modes=["a_tiny", "a_small"], p_present=1.0)))
    got = rb.batch_and_cardinality([(rb.RoaringBitmap(a), rb.RoaringBitmap(b)) for a, b in pairs])
    exp = np.array([O.pairwise_card("and", a, b) for a, b in pairs], dtype=np.int32)
    np.testing.assert_array_equal(got, exp)
