"""Key-range sharded wide ops through the HIP engine, and the C3 synthetic batches.

The ranks of a sharded run are played one after another in this process, each on
its own key slice of one device-resident batch; shard.concat_serialized assembles
them. The result must equal the unsharded oracle result byte for byte. For
naive_and, the start input is chosen over the whole universe
(RB/FastAggregation.java:333-339).
"""
import numpy as np
import pytest

import _gen
import _oracle as O
from roaringbitmap_amd import shard

pytestmark = pytest.mark.gpu


def _engine():
    from roaringbitmap_amd import Engine
    return Engine(0)


def _key_bytes(bufs):
    from _fmt import decode
    kb = np.zeros(65536)
    for b in bufs:
        for k, _, card, _, _ in decode(b):
            kb[k] += 4 + 2 * card
    return kb


@pytest.mark.parametrize("world", [2, 3, 8])
def test_engine_key_shards(gpu, world):
    rng = np.random.default_rng(300 + world)
    keys = np.sort(rng.choice(65536, size=40, replace=False))
    bufs = [_gen.bitmap(rng, keys, p_present=0.85) for _ in range(12)] + [_gen.bitmap(rng, keys[:5], p_present=1.0)]
    e = _engine()
    batch = e.load(bufs)
    ranges = shard.key_ranges(_key_bytes(bufs), world)
    for op in ["or", "xor", "and", "workshy_and"]:
        parts = []
        for lo, hi in ranges:
            e.wide(op, batch, lo, hi)
            parts.append(e.fetch().serialize())
        assert shard.concat_serialized(parts) == O.wide(op, bufs), op
    # naive_and (N <= 10): the start input is the global smallest, not the slice's
    small = bufs[:7]
    b2 = e.load(small)
    counts = np.zeros(len(small), dtype=np.int64)
    per_rank = []
    for lo, hi in ranges:
        per_rank.append((lo, hi))
    from _fmt import decode
    counts = np.array([len(decode(b)) for b in small])
    start = int(np.argmin(counts))
    parts = []
    for lo, hi in per_rank:
        parts.append(shard.engine_shard(e, "and", b2, lo, hi, ids=list(range(len(small))))(start))
    assert shard.concat_serialized(parts) == O.wide("and", small, list(range(len(small))))


@pytest.mark.parametrize("world", [2, 5])
def test_pairwise_key_shards(gpu, world):
    """rbg_ctx_pairwise_range: each rank's key slice of a pairwise op (RB/RoaringBitmap.java:382-399
    on that slice), concatenated, equals the oracle's whole result -- run containers on both sides."""
    rng = np.random.default_rng(900 + world)
    keys = np.sort(rng.choice(4096, size=60, replace=False))
    a = _gen.bitmap(rng, keys, p_present=0.9)
    b = _gen.bitmap(rng, keys, p_present=0.9)
    e = _engine()
    ba, bb = e.load([a]), e.load([b])
    ranges = shard.key_ranges(_key_bytes([a, b]), world)
    for op in ["and", "or", "xor", "andnot"]:
        parts = []
        for lo, hi in ranges:
            e.pairwise(op, ba, bb, key_lo=lo, key_hi=hi)
            parts.append(e.fetch().serialize())
        assert shard.concat_serialized(parts) == O.pairwise(op, a, b), op


@pytest.mark.parametrize("kind", [1, 2])
def test_c3_synthetic_matches_oracle(gpu, kind):
    """C3 batches generated on the device: wide or/and/xor == oracle over the fetched bitmaps."""
    e = _engine()
    n = 24
    lo, hi = (1000, 1200) if kind == 1 else (0, 65536)
    batch = e.synth(kind, 0xC3000000, n, lo, hi)
    st = e.batch_stats(batch)
    assert st["bitmaps"] == n and st["containers"] > 0
    bms = [e.batch_fetch(batch, i).serialize() for i in range(n)]
    assert sum(O.stats(b)["card"] for b in bms) == st["cardinality"]
    for op in ["or", "xor", "and"]:
        e.wide(op, batch)
        exp = O.wide(op, bms)
        rs = e.result_stats()  # device-side result facts before serialization
        so = O.stats(exp)
        assert rs["cardinality"] == so["card"] and rs["payload_bytes"] == so["payload"], op
        assert rs["containers"] == so["array"] + so["bitmap"] + so["run"], op
        assert e.fetch().serialize() == exp, op
    # key-sliced generation: a slice equals the restriction of the full batch
    if kind == 2:
        ranges = shard.key_ranges(shard_key_bytes(kind, n), 3)
        parts = []
        for r0, r1 in ranges:
            b = e.synth(kind, 0xC3000000, n, r0, r1)
            e.wide("or", b, r0, r1)
            parts.append(e.fetch().serialize())
            e.release(b)
        assert shard.concat_serialized(parts) == O.wide("or", bms)


def shard_key_bytes(kind, n):
    from roaringbitmap_amd.engine import synth_key_bytes
    return synth_key_bytes(kind, 0xC3000000, n)


@pytest.mark.parametrize("case", ["wide_or", "run_and"])
def test_same_device_assembly(gpu, case):
    """shard.assemble with the fill and the output on the same GPU (the bench's RCCL path at rank 0):
    the engine writes descriptors, offsets, run-flag bytes and payload straight into views of the
    output tensor on its own stream.  run_and: a pairwise AND of run-container bitmaps, so the
    result holds run containers and the run-flag bitset must survive (no zero fill racing the
    engine's writes)."""
    import torch
    e = _engine()
    if case == "wide_or":
        batch = e.synth(1, 0xC3000000, 24, 0, 2048)
        e.wide("or", batch)
    else:
        rng = np.random.default_rng(77)
        keys = np.sort(rng.choice(65536, size=300, replace=False))
        a = _gen.bitmap(rng, keys, modes=["r_few", "r_mid", "r_many", "a_mid", "b_mid"], p_present=0.95)
        b = _gen.bitmap(rng, keys, modes=["r_few", "r_mid", "r_many", "a_mid", "b_mid"], p_present=0.95)
        ba, bb = e.load([a]), e.load([b])
        e.pairwise("and", ba, bb)
    rs = e.result_stats()
    lay = shard.GlobalLayout([[rs["containers"], rs["payload_bytes"], int(rs["has_run"])]])
    out = shard.assemble(shard.engine_fill(e), lay, 0, fill_device="cuda:0", comm_device="cuda:0", sync=e.sync)
    torch.cuda.synchronize()
    got = bytes(out.cpu().numpy().tobytes())
    assert got == e.fetch().serialize()
    if case == "run_and":
        assert rs["has_run"]
        assert got == O.pairwise("and", a, b)


@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_device_layout_shards(gpu, world):
    """The device-resident layout exchange (bench's N > 1 headline, shard.DeviceShard): each key
    shard's (containers, payload bytes, has_run) written to device memory by
    rbg_ctx_result_layout_device, then every shard placed by rbg_ctx_fetch_shard_device_dyn from
    that device layout into one buffer laid out as the global bitmap; with the run flags packed,
    the buffer equals the oracle's whole result (an empty shard included for world 8)."""
    import torch
    rng = np.random.default_rng(1200 + world)
    keys = np.sort(rng.choice(3000, size=70, replace=False))
    a = _gen.bitmap(rng, keys, p_present=0.9)
    b = _gen.bitmap(rng, keys, p_present=0.9)
    e = _engine()
    ba, bb = e.load([a]), e.load([b])
    ranges = shard.key_ranges(_key_bytes([a, b]), world)
    if world == 8:
        ranges[3] = (ranges[3][0], ranges[3][0])  # an empty key range
        ranges[4] = (ranges[3][0], ranges[4][1])
    dev = torch.device("cuda", 0)
    for op in ["and", "or", "xor", "andnot"]:
        lay = torch.zeros(3 * world, dtype=torch.int64, device=dev)
        torch.cuda.synchronize(dev)
        for r, (lo, hi) in enumerate(ranges):
            e.pairwise(op, ba, bb, key_lo=lo, key_hi=hi)
            e.result_layout_device(lay[3 * r: 3 * r + 3])
        e.sync()
        out = torch.zeros(shard.MAX_SERIALIZED, dtype=torch.uint8, device=dev)
        runb = torch.zeros(shard.KEYS, dtype=torch.uint8, device=dev)
        torch.cuda.synchronize(dev)  # the fills (torch's stream) before the engine's writes (its own stream)
        for r, (lo, hi) in enumerate(ranges):
            e.pairwise(op, ba, bb, key_lo=lo, key_hi=hi)
            e.fetch_shard_device_dyn(lay, r, world, out, runb)
        e.sync()
        gl = shard.GlobalLayout(lay.cpu().numpy().reshape(-1, 3))
        if gl.has_run and gl.total:
            out[4:4 + gl.flag_bytes] = shard._pack_flags(runb[:gl.total])
        got = bytes(out[:gl.nbytes].cpu().numpy().tobytes())
        assert got == O.pairwise(op, a, b), op
    e.release(ba)
    e.release(bb)
