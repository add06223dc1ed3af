"""Portable-format decode on the device (decode.hip) vs the reference's deserialize rules.

Valid inputs: every container family of tests/_gen.py, loaded as one key-major batch and
fetched back bitmap by bitmap, must give the input bytes back (canonical inputs), and
the batch statistics must match the oracle's.  Malformed inputs: every truncation point
of run / no-run bitmaps (with and without an offset table), bad cookies, oversized and
negative sizes, and unordered keys must raise the same exception class with the same
message as the host-side restatement of RoaringArray.deserialize (RB/RoaringArray.java:
547-629) used by RoaringBitmap.deserialize.  An offset table that disagrees with the
payload walk is ignored, as the reference ignores it.
"""
import re
import struct

import numpy as np
import pytest

import _gen
import _oracle as O

pytestmark = pytest.mark.gpu


def _host_error(buf):
    from roaringbitmap_amd import RoaringBitmap
    try:
        RoaringBitmap.deserialize(buf)
    except Exception as e:  # noqa: BLE001
        return type(e), re.sub(r"^status -?\d+: ", "", str(e))
    return None


def _gpu_error(e, bufs):
    try:
        b = e.load(bufs)
    except Exception as ex:  # noqa: BLE001
        return type(ex), re.sub(r"^status -?\d+: ", "", str(ex))
    e.release(b)
    return None


def _samples():
    rng = np.random.default_rng(31)
    out = [O.from_values([1, 2, 3]), O.from_values(np.arange(0, 300000, 7)),
           O.from_values(np.arange(1000, 5000), run_optimize=True),               # run cookie, size 1
           O.from_values(np.concatenate([np.arange(k << 16, (k << 16) + 500) for k in range(6)]),
                         run_optimize=True)]                                        # run cookie, size 6
    for _ in range(4):
        keys = np.sort(rng.choice(1 << 16, size=int(rng.integers(2, 7)), replace=False))
        out.append(_gen.bitmap(rng, keys))
    return out


def test_roundtrip_families(gpu):
    from roaringbitmap_amd import Engine
    e = Engine(0)
    rng = np.random.default_rng(8)
    bufs = [O.from_values([])]
    for _ in range(80):
        keys = np.sort(rng.choice(1 << 16, size=int(rng.integers(1, 20)), replace=False))
        bufs.append(_gen.bitmap(rng, keys))
    bufs += _samples()
    b = e.load(bufs)
    st = e.batch_stats(b)
    assert st["bitmaps"] == len(bufs)
    assert st["serialized_bytes"] == sum(len(x) for x in bufs)
    assert st["cardinality"] == sum(O.stats(x)["card"] for x in bufs)
    for k in ("array", "bitmap", "run"):
        assert st[k] == sum(O.stats(x)[k] for x in bufs)
    for i, x in enumerate(bufs):
        assert e.batch_fetch(b, i).serialize() == x
    # the key-major batch as a wide-op input
    e.wide("or", b)
    assert e.fetch().serialize() == O.wide("or", bufs)
    e.release(b)


def test_trailing_bytes_and_bad_offsets_are_ignored(gpu):
    from roaringbitmap_amd import Engine
    e = Engine(0)
    x = O.from_values(np.arange(0, 300000, 7))  # no-run cookie, offsets present
    size = struct.unpack_from("<I", x, 4)[0]
    y = bytearray(x)
    struct.pack_into("<I", y, 8 + 4 * size + 4, 12345)  # corrupt offset[1]: the walk is still valid
    b = e.load([bytes(y) + b"\x00" * 7, x + b"junk"])
    assert e.batch_fetch(b, 0).serialize() == x
    assert e.batch_fetch(b, 1).serialize() == x
    e.release(b)


def test_malformed_inputs_match_host_errors(gpu):
    from roaringbitmap_amd import Engine
    e = Engine(0)
    bad = []
    for x in _samples():
        for cut in range(0, len(x), max(1, len(x) // 97)):
            bad.append(x[:cut])
        bad.append(x[:-1])
    x = _samples()[1]
    bad.append(b"\x00\x00\x00\x00" + x[4:])                    # bad cookie
    bad.append(struct.pack("<II", 12346, 70000) + x[8:])       # Size too large
    bad.append(struct.pack("<Ii", 12346, -5) + x[8:])          # negative size
    y = bytearray(x)                                            # keys not increasing
    y[8:12], y[12:16] = x[12:16], x[8:12]
    bad.append(bytes(y))
    checked = 0
    for buf in bad:
        he = _host_error(buf)
        if he is None:
            continue
        ge = _gpu_error(e, [O.from_values([9]), buf])
        assert ge is not None, (len(buf), he)
        assert ge[0] is he[0] and ge[1] == "input 1: " + he[1], (len(buf), he, ge)
        checked += 1
    assert checked > 100


def test_multi_chunk_inputs(gpu):
    """Inputs of more than 1,024 containers span several decode waves: keys, cards and
    payload positions across chunk boundaries, with and without run containers, and an
    offset table corrupted in the second chunk (the serial walk takes over)."""
    from roaringbitmap_amd import Engine
    e = Engine(0)
    rng = np.random.default_rng(99)
    big = []
    for modes in (["a_tiny", "a_small", "b_edge"], ["a_tiny", "r_few", "r_mid", "a_32"]):
        keys = np.sort(rng.choice(1 << 16, size=3000, replace=False))
        big.append(_gen.bitmap(rng, keys, modes=modes, p_present=1.0))
    x = big[0]  # no run containers: offset table always present
    size = struct.unpack_from("<I", x, 4)[0]
    y = bytearray(x)
    struct.pack_into("<I", y, 8 + 4 * size + 4 * 1500, 7)  # offset of container 1500
    b = e.load(big + [bytes(y)])
    for i, want in enumerate(big + [x]):
        assert e.batch_fetch(b, i).serialize() == want
    st = e.batch_stats(b)
    assert st["cardinality"] == sum(O.stats(v)["card"] for v in big + [x])
    e.release(b)
    # truncation inside the second chunk
    ge = _gpu_error(e, [big[1][: len(big[1]) - 5]])
    assert ge is not None and ge == (_host_error(big[1][: len(big[1]) - 5])[0],
                                     "input 0: " + _host_error(big[1][: len(big[1]) - 5])[1])


def test_packed_decode_for_wide_ops(gpu):
    """rbg_ctx_load_packed: 1,000 C3-uniform bitmaps (2,048 keys) from their serialized bytes keep the
    portable format's packed array payloads (RB/RoaringArray.java:547-629) and every wide op that reads
    that layout is byte-exact against the oracle (RB/FastAggregation.java:356-414,586-666,823-836);
    the padded decode gives the same bytes; a packed batch refuses the slot-aligned paths, and a batch
    holding a bitmap container is decoded slot-aligned whatever the flag."""
    from roaringbitmap_amd import Engine
    from roaringbitmap_amd._lib import IllegalArgumentException
    from _fmt import A, B, encode
    e = Engine(0)
    n = 1000
    sb = e.synth(1, 0xC3000000, n, 3000, 3000 + 2048)
    bufs = [x.serialize() for x in e.batch_fetch_range(sb)]
    e.release(sb)
    packed, padded = e.load(bufs, packed=True), e.load(bufs)
    assert e.batch_stats(packed)["payload_bytes"] == e.batch_stats(padded)["payload_bytes"]
    for op in ("or", "xor", "and", "workshy_and", "priorityqueue_or", "horizontal_xor", "parallel_or"):
        exp = O.wide(op, bufs)
        for b in (packed, padded):
            e.wide(op, b)
            assert e.fetch().serialize() == exp, op
    e.wide_card("or", packed)
    assert e.card() == O.wide_card("or", bufs)
    assert [x.serialize() for x in e.batch_fetch_range(packed, 0, 5)] == bufs[:5]  # fetches read packed payloads
    with pytest.raises(IllegalArgumentException):  # naive_and's chain needs slots
        e.wide("naive_and", packed)
    one = e.load([bufs[0]], packed=True)
    with pytest.raises(IllegalArgumentException):  # pairwise operands need slots
        e.pairwise("and", one, one)
    mixed = encode([(1, A, np.arange(10, dtype=np.uint16)), (2, B, np.arange(0, 9000, 2, dtype=np.uint16))])
    m = e.load([mixed, bufs[1]], packed=True)  # a bitmap container: slot-aligned, every op allowed
    e.wide("naive_and", m)
    assert e.fetch().serialize() == O.wide("naive_and", [mixed, bufs[1]])
    for b in (packed, padded, one, m):
        e.release(b)
