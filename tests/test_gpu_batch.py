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
