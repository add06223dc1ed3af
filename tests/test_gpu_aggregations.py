"""ParallelAggregation, BufferFastAggregation.or(Mutable...), horizontal_or / horizontal_xor and
priorityqueue_or / priorityqueue_xor on the GPU, byte-exact against the oracle's restatements (tests/test_aggregation_oracle.py pins
those to the reference's tests).

Inputs mix every container family of tests/_gen.py at few keys so that many keys hold
2..15 containers (the lazyIOR chain of ParallelAggregation.or, RB/ParallelAggregation.java:
200-206) and some hold 16+ (its lazy-bitmap branch :208-214), plus equal-cardinality
array / run containers at one key, whose chain order comes from the heap's tie order
(horizontal_*, RB/FastAggregation.java:124-289).  priorityqueue_* (:677-812) pair whole
bitmaps by getLongSizeInBytes, so their result types depend on the whole queue: equal-size
inputs exercise the heap's tie order, and run / bitmap / array mixes the lazy algebra
(lazyor, in-place lazyor, lazyorfromlazyinputs) and the final repairAfterLazy.
"""
import os
import numpy as np
import pytest

import _gen
import _oracle as O
from _fmt import A, B, R, encode

pytestmark = pytest.mark.gpu

OPS = ["parallel_or", "parallel_xor", "buffer_or_mutable", "horizontal_or", "horizontal_xor", "priorityqueue_or",
       "priorityqueue_xor"]
GOLD = os.path.join(os.path.dirname(__file__), "golden")


def _wide(op, bufs):
    import roaringbitmap_amd as rb
    from roaringbitmap_amd.roaring import _wide as w
    return w(op, [rb.RoaringBitmap(b) for b in bufs]).serialize()


@pytest.mark.parametrize("seed", range(6))
@pytest.mark.parametrize("n", [1, 2, 3, 7, 15, 16, 40])
def test_aggregations_random(gpu, seed, n):
    rng = np.random.default_rng(1000 * n + seed)
    keys = np.sort(rng.choice(65536, 12, replace=False))
    bufs = [_gen.bitmap(rng, keys, p_present=0.6) for _ in range(n)]
    for op in OPS:
        assert _wide(op, bufs) == O.wide(op, bufs), (op, n, seed)


@pytest.mark.parametrize("modes", [["a_tiny", "a_small"], ["a_small", "r_tiny", "r_single"], ["r_tie", "r_few", "a_32"],
                                   ["a_mid", "r_mid"], ["r_many", "a_small"], ["b_mid", "a_small", "r_tiny"]])
def test_aggregations_mode_mixes(gpu, modes):
    """Mixes that walk the chain's thresholds: 1024 values for A + A, 4096 runs for A + R,
    toEfficientContainer for R + R, empty XOR results (kept by horizontal_xor)."""
    rng = np.random.default_rng(len("".join(modes)))
    keys = np.arange(0, 8)
    for n in (2, 4, 9, 15):
        bufs = [_gen.bitmap(rng, keys, modes=modes, p_present=0.9) for _ in range(n)]
        bufs.append(bufs[0])  # identical containers: XOR chains reach empty results
        for op in OPS:
            assert _wide(op, bufs) == O.wide(op, bufs), (op, modes, n)


def test_horizontal_equal_cardinality_ties(gpu):
    """Array and run containers of equal cardinality at one key: the chain order is the
    reference heap's tie order."""
    rng = np.random.default_rng(3)
    bufs = []
    for i in range(9):
        card = 100 if i % 3 else 700
        if i % 2:
            s = int(rng.integers(0, 60000))
            ctr = (0, R, np.arange(s, s + card, dtype=np.uint16))
        else:
            ctr = (0, A, np.sort(rng.choice(65536, card, replace=False)).astype(np.uint16))
        bufs.append(encode([ctr, (1, A, np.array([i], dtype=np.uint16))]))
    for op in OPS:
        assert _wide(op, bufs) == O.wide(op, bufs), op


def test_chains_without_runs(gpu):
    """Keys without run containers take the order-free path of the chain modes (the type is
    BY_CARD of the union / symmetric difference, RunContainer.full at 65536).  Key 0: arrays
    whose cardinalities sum past 1024 over a union of at most 1024 values (ArrayContainer.
    lazyor's 1024 threshold may or may not fire, the repaired type is the same); key 1: arrays
    whose union passes 4096; key 2: arrays and a bitmap that fill the key; key 3: pairs of
    identical arrays (XOR chains end empty: dropped by ParallelAggregation.xor, kept by
    horizontal_xor); key 4: one bitmap among arrays."""
    rng = np.random.default_rng(77)
    pool = np.sort(rng.choice(65536, 900, replace=False)).astype(np.uint16)
    odd = np.arange(1, 65536, 2, dtype=np.uint16)  # 8 arrays of 4,096 cover them
    for n in (2, 3, 6, 17):
        bufs = []
        for i in range(n):
            ctrs = [(0, A, np.sort(rng.choice(pool, 400, replace=False)).astype(np.uint16)),
                    (1, A, np.sort(rng.choice(65536, 3000, replace=False)).astype(np.uint16))]
            if i == 0:
                ctrs.append((2, B, np.arange(0, 65536, 2, dtype=np.uint16)))  # the even values
            else:
                ctrs.append((2, A, odd[4096 * ((i - 1) % 8):4096 * ((i - 1) % 8 + 1)]))
            ctrs.append((3, A, np.arange(100 + (i // 2) * 10, 110 + (i // 2) * 10, dtype=np.uint16)))
            if i == n // 2:
                ctrs.append((4, B, np.sort(rng.choice(65536, 5000, replace=False)).astype(np.uint16)))
            else:
                ctrs.append((4, A, np.sort(rng.choice(65536, 50, replace=False)).astype(np.uint16)))
            bufs.append(encode(ctrs))
        for op in OPS:
            assert _wide(op, bufs) == O.wide(op, bufs), (op, n)


def test_aggregations_c3_slices(gpu):
    """C3-style inputs (many bitmaps, mostly small arrays per key) through the chain modes."""
    from roaringbitmap_amd import Engine
    e = Engine(0)
    for kind, lo, hi in ((1, 5000, 5040), (2, 0, 65536)):
        b = e.synth(kind, 0xC3000000, 40, lo, hi)
        bms = [x.serialize() for x in e.batch_fetch_range(b)]
        for op in OPS:
            e.wide(op, b)
            assert e.fetch().serialize() == O.wide(op, bms), (kind, op)
        e.release(b)


def test_host_api_names(gpu):
    import roaringbitmap_amd as rb
    rng = np.random.default_rng(11)
    keys = np.sort(rng.choice(4000, 20, replace=False))
    bufs = [_gen.bitmap(rng, keys, p_present=0.7) for _ in range(6)]
    bms = [rb.RoaringBitmap(b) for b in bufs]
    assert getattr(rb.ParallelAggregation, "or")(*bms).serialize() == O.wide("parallel_or", bufs)
    assert rb.ParallelAggregation.xor(*bms).serialize() == O.wide("parallel_xor", bufs)
    assert rb.BufferFastAggregation.or_mutable(*bms).serialize() == O.wide("buffer_or_mutable", bufs)
    assert rb.FastAggregation.horizontal_or(bms).serialize() == O.wide("horizontal_or", bufs)
    assert rb.FastAggregation.horizontal_or(*bms).serialize() == O.wide("horizontal_or", bufs)
    assert rb.FastAggregation.horizontal_or(iter(bms)).serialize() == O.wide("or", bufs)
    assert rb.FastAggregation.horizontal_xor(*bms).serialize() == O.wide("horizontal_xor", bufs)
    assert rb.FastAggregation.priorityqueue_or(*bms).serialize() == O.wide("priorityqueue_or", bufs)
    assert rb.FastAggregation.priorityqueue_or(iter(bms)).serialize() == O.wide("priorityqueue_or", bufs)
    assert rb.FastAggregation.priorityqueue_xor(*bms).serialize() == O.wide("priorityqueue_xor", bufs)
    assert rb.FastAggregation.priorityqueue_or().serialize() == O.wide("priorityqueue_or", [])
    assert rb.FastAggregation.priorityqueue_xor().serialize() == O.wide("priorityqueue_xor", [])


@pytest.mark.parametrize("seed", range(4))
def test_priorityqueue_equal_sizes_and_lazy_mix(gpu, seed):
    """Equal getLongSizeInBytes (tie order of the heap), temps meeting temps
    (lazyorfromlazyinputs), full run containers and bitmap + array chains."""
    rng = np.random.default_rng(500 + seed)
    bufs = []
    for i in range(11):
        ctrs = [(k, A, np.sort(rng.choice(65536, 300, replace=False)).astype(np.uint16)) for k in (0, 1)]
        if i % 3 == 0:
            ctrs.append((2, R, np.arange(0, 65536).astype(np.uint16)))  # full run
        elif i % 3 == 1:
            s = int(rng.integers(0, 30000))
            ctrs.append((2, R, np.arange(s, s + 20000, dtype=np.uint16)))
        else:
            ctrs.append((2, A, np.sort(rng.choice(65536, 5000, replace=False)).astype(np.uint16)))
        ctrs.append((3 + i % 4, A, np.array([i, 100 + i], dtype=np.uint16)))
        bufs.append(encode(ctrs))
    for op in ("priorityqueue_or", "priorityqueue_xor"):
        assert _wide(op, bufs) == O.wide(op, bufs), op


def _realdata(ds):
    z = np.load(os.path.join(GOLD, "realdata", ds + ".npz"))
    v, o = z["values"], z["offsets"]
    return [v[o[i]:o[i + 1]] for i in range(len(o) - 1)]


@pytest.mark.parametrize("run_opt", [False, True])
def test_priorityqueue_realdata(gpu, run_opt):
    """RealDataBenchmarkWideOrPqTest datasets: byte parity with the queue restatement and the
    known wide-OR cardinality."""
    import json
    known = json.load(open(os.path.join(GOLD, "known_answers.json")))["values"]
    for ds in ["census1881", "wikileaks-noquotes_srt"]:
        bufs = [O.from_values(s, run_opt) for s in _realdata(ds)]
        got = _wide("priorityqueue_or", bufs)
        assert got == O.wide("priorityqueue_or", bufs), ds
        assert len(O.to_values(got)) == known[ds]["wide_or"]
        assert _wide("priorityqueue_xor", bufs) == O.wide("priorityqueue_xor", bufs), ds


@pytest.mark.parametrize("n", [600, 3000])
def test_priorityqueue_many_bitmaps_wide_keys(gpu, n):
    """Many small bitmaps spread over most of the 65,536 keys (C3-shaped key space): the
    temps hold arena blocks only for their own keys, so the op completes (the dense
    per-temp layout needed n/2 x keys x 8 KiB) and matches the queue restatement."""
    rng = np.random.default_rng(n)
    bufs = []
    for i in range(n):
        keys = np.sort(rng.choice(65536, 40, replace=False))
        v = (keys[:, None].astype(np.int64) << 16) + rng.integers(0, 65536, (40, 6 if i % 5 else 3000))
        bufs.append(O.from_values(v.ravel(), i % 7 == 0))
    for op in ("priorityqueue_or", "priorityqueue_xor"):
        assert _wide(op, bufs) == O.wide(op, bufs), op
