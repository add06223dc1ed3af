"""Session-API lifecycle and malformed-input edge cases.

- A materialised result references unchanged (cloned) containers inside its operand
  batches until it is serialized; releasing an operand first must not corrupt it.
- A run container whose header cardinality disagrees with its runs: the reference
  builds the RunContainer from the runs and ignores the header card
  (RB/RoaringArray.java:583-597, RB/RunContainer.java:1003-1009), so pass-through
  clones, cardinalities and EFF decisions all use the runs' cardinality.
- Range fetches of a batch equal single fetches.
"""
import struct

import numpy as np
import pytest

import _gen
import _oracle as O

pytestmark = pytest.mark.gpu


def _engine():
    from roaringbitmap_amd import Engine
    return Engine(0)


@pytest.mark.parametrize("op", ["and", "or", "xor", "andnot"])
def test_release_operand_before_fetch(gpu, op):
    rng = np.random.default_rng(7)
    keys = np.sort(rng.choice(2000, 60, replace=False))
    a_buf = _gen.bitmap(rng, keys, p_present=0.7)
    b_buf = _gen.bitmap(rng, keys, p_present=0.7)
    e = _engine()
    a, b = e.load([a_buf]), e.load([b_buf])
    e.pairwise(op, a, b)
    e.release(a)
    c = e.load([b_buf])  # reuses freed memory
    e.release(b)
    assert e.fetch().serialize() == O.pairwise(op, a_buf, b_buf)
    e.release(c)


def test_release_wide_operand_before_fetch(gpu):
    rng = np.random.default_rng(8)
    keys = np.sort(rng.choice(5000, 50, replace=False))
    bufs = [_gen.bitmap(rng, keys, p_present=0.3) for _ in range(6)]
    e = _engine()
    w = e.load(bufs)
    e.wide("or", w)
    e.release(w)
    x = e.load(bufs[::-1])
    assert e.fetch().serialize() == O.wide("or", bufs)
    e.release(x)


def _bad_run_card(card_hdr):
    """One run container (key 3) holding [100, 199] and [1000, 1099] (card 200), with the
    header cardinality replaced by card_hdr; plus an array container at key 5."""
    runs = [(100, 99), (1000, 99)]
    pay_r = struct.pack("<H", len(runs)) + b"".join(struct.pack("<HH", s, l) for s, l in runs)
    vals = np.array([1, 2, 3], dtype="<u2").tobytes()
    size = 2
    out = struct.pack("<I", 12347 | ((size - 1) << 16)) + bytes([0b01])
    out += struct.pack("<HH", 3, card_hdr - 1) + struct.pack("<HH", 5, 2)
    return out + pay_r + vals  # size < 4: no offset table


@pytest.mark.parametrize("card_hdr", [1, 7, 200, 5000, 65536])
def test_run_card_from_runs(gpu, card_hdr):
    import roaringbitmap_amd as rb
    x = _bad_run_card(card_hdr)
    other = O.from_values([5 * 65536 + 2, 9 * 65536])
    assert rb.RoaringBitmap(x).getLongCardinality() == 203  # host parse: from the runs
    for op in ["and", "or", "xor", "andnot"]:
        assert rb.RoaringBitmap._pair(op, rb.RoaringBitmap(x), rb.RoaringBitmap(other)).serialize() == \
            O.pairwise(op, x, other), op
    assert rb.RoaringBitmap.orCardinality(rb.RoaringBitmap(x), rb.RoaringBitmap(other)) == \
        O.pairwise_card("or", x, other)
    assert rb.FastAggregation.or_(rb.RoaringBitmap(x)).serialize() == O.wide("or", [x])  # n = 1: EFF on the card
    assert rb.FastAggregation.or_(rb.RoaringBitmap(x), rb.RoaringBitmap(other)).serialize() == O.wide("or", [x, other])
    e = _engine()
    b = e.load([x, other])
    assert e.batch_stats(b)["cardinality"] == 203 + 2
    e.release(b)


def test_fetch_range_equals_single(gpu):
    rng = np.random.default_rng(9)
    keys = np.sort(rng.choice(65536, 80, replace=False))
    bufs = [_gen.bitmap(rng, keys, p_present=0.4) for _ in range(9)] + [O.from_values([])]
    e = _engine()
    b = e.load(bufs)
    got = [x.serialize() for x in e.batch_fetch_range(b)]
    assert got == [e.batch_fetch(b, i).serialize() for i in range(len(bufs))]
    assert got == [O.roundtrip(x)[1] for x in bufs]
    assert [x.serialize() for x in e.batch_fetch_range(b, 3, 4)] == got[3:7]
    e.release(b)


def test_pooled_buffers_released_when_memory_runs_out(gpu):
    """A released batch's device buffers stay pooled in its context (engine.cpp: pool_put); an
    allocation that runs out of device memory empties every context's pool and retries."""
    import torch
    e = _engine()
    b = e.synth(0, 0xC2A0, 1)  # a C2 operand: ~0.36 GB of payload
    e.release(b)  # its buffers go to the pool
    torch.cuda.empty_cache()
    free, _ = torch.cuda.mem_get_info(0)
    hog = torch.empty(max(free - (200 << 20), 0), dtype=torch.uint8, device="cuda:0")  # ~200 MB left
    try:
        b2 = e.synth(0, 0xC2B0, 1)  # fits only once the pooled buffers are freed
        assert e.batch_stats(b2)["containers"] == 65536
        e.release(b2)
    finally:
        del hog
        torch.cuda.empty_cache()
