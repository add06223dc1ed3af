"""Full-size parity and property checks at BASELINE.json's configs.

C2  the bench's own device-generated pair (raw, and runOptimize'd): and / or / xor / andNot
    and the five cardinalities, byte-exact against the oracle on the fetched operands
    (RB/RoaringBitmap.java:377-473,698-720,860-1118).
C3  10,000 bitmaps, uniform and clustered: the full wide op's result, restricted to a few
    random keys, equals the oracle's wide op over the same key generated as a slice
    (RB/FastAggregation.java:26-63,586-666,823-836); whole-result invariants (container
    count, orCardinality vs the materialised cardinality) at full size.
C4  1M pairs: batched andCardinality against the oracle on 10k random pairs plus the
    first 2,000.
C5  10^9 rows: compare(RANGE) + sum against the closed form of the generator, computed
    independently with torch on the GPU (bsi/.../RoaringBitmapSliceIndex.java:482-513,581-592).

Big byte strings are compared by length + digest (a pytest diff of 200 MB would hang).
"""
import hashlib

import numpy as np
import pytest

import _fmt
import _oracle as O

pytestmark = pytest.mark.gpu

C2_SEEDS = (0xC2A0, 0xC2B0)
C3_SEED = 0xC3000000
C3_N = 10000


def _same(got: bytes, exp: bytes, what: str):
    if got == exp:
        return
    n = min(len(got), len(exp))
    first = next((i for i in range(n) if got[i] != exp[i]), n)
    raise AssertionError(f"{what}: {len(got)} B (sha {hashlib.sha1(got).hexdigest()[:12]}) vs oracle {len(exp)} B "
                         f"(sha {hashlib.sha1(exp).hexdigest()[:12]}), first difference at byte {first}")


@pytest.fixture(scope="module")
def eng(gpu):
    from roaringbitmap_amd import Engine
    e = Engine(0)
    yield e
    e.close()


@pytest.fixture(scope="module")
def c2(eng):
    """{variant: (batch a, batch b, bytes a, bytes b)} for the raw bench pair and its runOptimize'd form."""
    a = eng.synth(0, C2_SEEDS[0])
    b = eng.synth(0, C2_SEEDS[1])
    oa, _ = eng.run_optimize(a)
    ob, _ = eng.run_optimize(b)
    out = {}
    for name, (x, y) in {"raw": (a, b), "runopt": (oa, ob)}.items():
        out[name] = (x, y, eng.batch_fetch(x).serialize(), eng.batch_fetch(y).serialize())
    yield out
    for x in (a, b, oa, ob):
        eng.release(x)


@pytest.mark.parametrize("variant", ["raw", "runopt"])
@pytest.mark.parametrize("op", ["and", "or", "xor", "andnot"])
def test_c2_pipelined_serialization(eng, c2, variant, op, monkeypatch):
    """rbg_ctx_pairwise_serialized (the bench's headline step): the op in K key ranges, each range's
    placement and payload copies on a second stream while the next range computes.  For every K
    (and thinned compute grids), the bytes equal the oracle's and the two-call form's."""
    x, y, xa, xb = c2[variant]
    exp = O.pairwise(op, xa, xb)
    for k, pw in ((1, None), (2, None), (3, None), (4, None), (7, "3"), (16, None), (64, "2")):
        monkeypatch.setenv("RBG_SER_PIPE", str(k))
        if pw:
            monkeypatch.setenv("RBG_PIPE_PW_WG", pw)
        else:
            monkeypatch.delenv("RBG_PIPE_PW_WG", raising=False)
        for _ in range(2):  # back to back: the second op reuses the records the first one's stream2 read
            eng.pairwise_serialized(op, x, y)
        rs = eng.result_stats()
        _same(eng.fetch().serialize(), exp, f"C2 {variant} {op} pipelined K={k}")
        so = O.stats(exp)
        assert rs["containers"] == so["array"] + so["bitmap"] + so["run"]


@pytest.mark.parametrize("variant", ["raw", "runopt"])
@pytest.mark.parametrize("op", ["and", "or", "xor", "andnot"])
def test_c2_full_pair(eng, c2, variant, op):
    x, y, xa, xb = c2[variant]
    st = eng.batch_stats(x)
    assert st["containers"] == 65536 and min(st["array"], st["bitmap"], st["run"]) > 20000
    eng.pairwise(op, x, y)
    rs = eng.result_stats()
    got = eng.fetch().serialize()
    exp = O.pairwise(op, xa, xb)
    so = O.stats(exp)
    assert rs["cardinality"] == so["card"] and rs["containers"] == so["array"] + so["bitmap"] + so["run"]
    _same(got, exp, f"C2 {variant} {op}")
    if op == "andnot":  # the other direction too (x2 \ x1)
        eng.pairwise(op, y, x)
        _same(eng.fetch().serialize(), O.pairwise(op, xb, xa), f"C2 {variant} andNot reversed")


@pytest.mark.parametrize("lo,hi", [(1000, 19000), (7, 65530), (40000, 65536)])
def test_c2_key_ranges(eng, c2, lo, hi):
    """Key-range shards of the C2 pair (the N > 1 headline's per-rank op) against the oracle on operands
    restricted to [lo, hi) by whole-key removes (RB/RoaringBitmap.java:382-399: a key's result depends on
    that key's containers only).  18,000 keys: the balanced list's last band is partial and the two
    lightest bands are k_pair_cu's shared tail; 65,523 keys: the tail with a one-key-short last band."""
    x, y, xa, xb = c2["raw"]

    def restrict(buf):
        if lo > 0:
            buf = O.range_mut("remove", buf, 0, lo << 16)
        if hi < 65536:
            buf = O.range_mut("remove", buf, hi << 16, 1 << 32)
        return buf

    ra, rb_ = restrict(xa), restrict(xb)
    for op in ("and", "or", "xor", "andnot"):
        eng.pairwise(op, x, y, key_lo=lo, key_hi=hi)
        _same(eng.fetch().serialize(), O.pairwise(op, ra, rb_), f"C2 {op} keys [{lo}, {hi})")


@pytest.mark.parametrize("variant", ["raw", "runopt"])
def test_c2_widened_ops(eng, c2, variant):
    """The round-5 rows at the C2 size, byte-exact against the oracle on the fetched operands:
    orNot over the whole universe and mid-key (static and in place, heap and buffer), the buffer
    package's and / andNot, the static flip / add / remove over ranges that cut keys, and addOffset."""
    x, y, xa, xb = c2[variant]
    for end, flags in (((1 << 32), 0), ((40000 << 16) + 123, 0), ((1 << 32), 1), ((40000 << 16) + 123, 3)):
        eng.ornot(x, y, end, inplace=bool(flags & 1), buffer=bool(flags & 2))
        _same(eng.fetch().serialize(), O.ornot(xa, xb, end, inplace=bool(flags & 1), buffer=bool(flags & 2)),
              f"C2 {variant} orNot end={end} flags={flags}")
    for op in ("and_buffer", "andnot_buffer"):
        eng.pairwise(op, x, y)
        _same(eng.fetch().serialize(), O.pairwise(op.replace("_buffer", "_buf"), xa, xb), f"C2 {variant} {op}")
    for op, st, en in (("flip", 0, 1 << 32), ("flip", (100 << 16) + 5, (60000 << 16) + 7),
                       ("add", (100 << 16) + 5, (60000 << 16) + 7), ("remove", (100 << 16) + 5, (60000 << 16) + 7)):
        eng.range_mut(op, x, st, en)
        _same(eng.fetch().serialize(), O.range_mut(op, xa, st, en), f"C2 {variant} {op} [{st}, {en})")
    for off in (12345, -(7 << 16) - 99, 3 << 16):
        eng.add_offset(x, off)
        _same(eng.fetch().serialize(), O.add_offset(xa, off), f"C2 {variant} addOffset {off}")


@pytest.mark.parametrize("variant", ["raw", "runopt"])
def test_c2_full_pair_cardinalities(eng, c2, variant):
    import roaringbitmap_amd as rb
    x, y, xa, xb = c2[variant]
    eng.and_cardinality(x, y)
    assert eng.card() == O.pairwise_card("and", xa, xb)
    ra, rb_ = rb.RoaringBitmap(xa), rb.RoaringBitmap(xb)
    for op, fn in [("and", rb.RoaringBitmap.andCardinality), ("or", rb.RoaringBitmap.orCardinality),
                   ("xor", rb.RoaringBitmap.xorCardinality), ("andnot", rb.RoaringBitmap.andNotCardinality),
                   ("intersects", rb.RoaringBitmap.intersects)]:
        exp = O.pairwise_card(op, xa, xb)
        assert int(fn(ra, rb_)) == exp, op


def _c3_keys(kind, rng):
    if kind == 1:
        return sorted(int(k) for k in rng.choice(65536, 5, replace=False)) + [65535]
    return sorted(int(k) for k in rng.choice(4096 + 16, 5, replace=False)) + [0]


@pytest.mark.parametrize("kind", [1, 2], ids=["uniform", "clustered"])
def test_c3_full_size(eng, kind):
    """FastAggregation.or / and / xor of the bench's 10,000 C3 bitmaps: for 6 keys, the full
    result's container equals the oracle's result over the key's 10,000 input containers
    (generated as a key slice and fetched); whole-result invariants at full size."""
    full = eng.synth(kind, C3_SEED, C3_N)
    st = eng.batch_stats(full)
    assert st["bitmaps"] == C3_N
    keys = _c3_keys(kind, np.random.default_rng(1234 + kind))
    slices = {}
    for k in keys:
        sb = eng.synth(kind, C3_SEED, C3_N, k, k + 1)
        slices[k] = [b.serialize() for b in eng.batch_fetch_range(sb)]
        eng.release(sb)
        assert len(slices[k]) == C3_N
    for op in ["or", "and", "xor"]:
        eng.wide(op, full)
        rs = eng.result_stats()
        got = eng.fetch().serialize()
        assert rs["containers"] == len(_fmt.container_table(got)[0]) if rs["containers"] else got == O.from_values([])
        if op == "or":
            eng.wide_card("or", full)
            assert eng.card() == np.int64(rs["cardinality"]).astype(np.int32)
            if kind == 1:
                assert rs["containers"] == 65536  # every key holds input values
        if op == "and":
            assert rs["containers"] == 0  # no key is common to all 10,000 bitmaps
        for k in keys:
            exp = O.wide(op, slices[k])
            _same(_fmt.sub_bitmap(got, [k]), exp, f"C3 kind {kind} {op} key {k}")
    eng.release(full)


def test_c4_full_size(eng):
    """Batched andCardinality over the bench's 1M C4 pairs."""
    n = 1_000_000
    b = eng.synth(3, 0xC4, n)
    eng.batch_and_card(b)
    got = eng.cards(n)
    rng = np.random.default_rng(44)
    pick = np.unique(np.concatenate([np.arange(2000), rng.choice(n, 10000, replace=False)]))
    head = [x.serialize() for x in eng.batch_fetch_range(b, 0, 4000)]
    for i in pick:
        if i < 2000:
            xa, xb = head[2 * i], head[2 * i + 1]
        else:
            xa, xb = (x.serialize() for x in eng.batch_fetch_range(b, 2 * int(i), 2))
        assert got[i] == O.pairwise_card("and", xa, xb), int(i)
    assert (got >= 0).all() and got.max() <= 4 * 512
    eng.release(b)


def _splitmix_torch(x):
    """splitmix64 finaliser on int64 tensors (wrapping arithmetic, logical shifts)."""
    import torch

    def s64(c):
        return c - (1 << 64) if c >= (1 << 63) else c

    def shr(v, k):
        return (v >> k) & ((1 << (64 - k)) - 1)

    x = x + s64(0x9E3779B97F4A7C15)
    x = (x ^ shr(x, 30)) * s64(0xBF58476D1CE4E5B9)
    x = (x ^ shr(x, 27)) * s64(0x94D049BB133111EB)
    return x ^ shr(x, 31)


def test_c5_full_size(eng):
    """C5 at 10^9 rows: compare(RANGE, 2^29, 2^30) + sum == the generator's closed form
    (value(row) = splitmix64(seed ^ row * golden) & 0x7FFFFFFF, csrc/synth.hip), computed
    here with torch in chunks, independently of the engine."""
    import torch
    rows, seed = 1_000_000_000, 0xC5
    b = eng.synth(4, seed, rows)
    mn, mx = eng.batch_minmax(b)
    lo, hi = 1 << 29, 1 << 30
    eng.bsi(b, "RANGE", 31, lo, hi, mn, mx, want_sum=True)
    s, cnt = eng.bsi_sums()
    rs = eng.result_stats()
    dev = torch.device("cuda", 0)
    golden = 0x9E3779B97F4A7C15 - (1 << 64)
    tot, tcnt, vmin, vmax = 0, 0, None, None
    step = 100_000_000
    for r0 in range(0, rows, step):
        r = torch.arange(r0, min(rows, r0 + step), dtype=torch.int64, device=dev)
        v = _splitmix_torch(torch.bitwise_xor(r * golden, seed)) & 0x7FFFFFFF
        m = (v >= lo) & (v <= hi)
        tot += int(v[m].sum())
        tcnt += int(m.sum())
        vmin = int(v.min()) if vmin is None else min(vmin, int(v.min()))
        vmax = int(v.max()) if vmax is None else max(vmax, int(v.max()))
        del r, v, m
    assert (mn, mx) == (vmin, vmax)
    assert (s, cnt) == (tot, tcnt)
    assert rs["cardinality"] == tcnt
    # result bytes: for 6 keys (the first, the partial last one and 4 random), the full
    # result's container equals tests/_bsi.py's compare(RANGE) over that key's ebM and 31
    # slice containers (generated as a key slice and fetched), with the global min / max
    import _bsi
    got = eng.fetch().serialize()
    nkeys = (rows + 65535) // 65536
    keys = sorted({0, nkeys - 1, *np.random.default_rng(55).choice(nkeys, 4, replace=False).tolist()})
    for k in keys:
        sb = eng.synth(4, seed, rows, k, k + 1)
        bms = [eng.batch_fetch(sb, i).serialize() for i in range(32)]
        eng.release(sb)
        exp = _bsi.BSI(bms[0], bms[1:], mn, mx).compare("RANGE", lo, hi)
        _same(_fmt.sub_bitmap(got, [k]), exp, f"C5 key {k}")
    eng.release(b)


def test_c5_buffer_full_size(eng):
    """C5 at 10^9 rows through the buffer package's circuit (BitSliceIndexBase.compare(RANGE):
    owenGreatEqual over horizontal_or and oNeilCompare(LE), bsi/.../bsi/buffer/BitSliceIndexBase.java:
    243-275,190-234,444-449): the same set as the heap query (the closed form checked above), and
    for 6 keys the result's container equals tests/_bsi.BufferBSI's over that key's inputs."""
    import _bsi
    rows, seed = 1_000_000_000, 0xC5
    b = eng.synth(4, seed, rows)
    mn, mx = eng.batch_minmax(b)
    lo, hi = 1 << 29, 1 << 30
    eng.bsi(b, "RANGE", 31, lo, hi, mn, mx)
    heap_card = eng.result_stats()["cardinality"]
    eng.bsi_buffer(b, "RANGE", 31, lo, hi, mn, mx)
    assert eng.result_stats()["cardinality"] == heap_card
    got = eng.fetch().serialize()
    nkeys = (rows + 65535) // 65536
    keys = sorted({0, nkeys - 1, *np.random.default_rng(56).choice(nkeys, 4, replace=False).tolist()})
    for k in keys:
        sb = eng.synth(4, seed, rows, k, k + 1)
        bms = [eng.batch_fetch(sb, i).serialize() for i in range(32)]
        eng.release(sb)
        exp = _bsi.BufferBSI(bms[0], bms[1:], mn, mx).compare("RANGE", lo, hi)
        _same(_fmt.sub_bitmap(got, [k]), exp, f"C5 buffer key {k}")
    eng.release(b)
