"""Pairwise static ops on the MI355X vs the CPU oracle: byte-identical output.

RB/RoaringBitmap.java and :377, or :860, xor :1071, andNot :444, andCardinality :413,
or/xor/andNotCardinality :916-985, intersects :698.
"""
import json
import os

import numpy as np
import pytest

import _gen
import _oracle as O
from _fmt import decode, encode, R

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
OPS = ["and", "or", "xor", "andnot"]
CARDS = ["and", "or", "xor", "andnot", "intersects"]


def _rb():
    import roaringbitmap_amd as rb
    return rb


def gpu_pair(op, a, b):
    rb = _rb()
    return rb.RoaringBitmap._pair(op, rb.RoaringBitmap(a), rb.RoaringBitmap(b)).serialize()


def gpu_card(op, a, b):
    rb = _rb()
    return rb.RoaringBitmap._card(op, rb.RoaringBitmap(a), rb.RoaringBitmap(b))


def check_all(a, b, label=""):
    for op in OPS:
        exp = O.pairwise(op, a, b)
        got = gpu_pair(op, a, b)
        if got != exp:
            de, dg = decode(exp), decode(got)
            diff = [(x[0], x[1], x[2], y[1], y[2]) for x, y in zip(de, dg) if x[:3] != y[:3]]
            raise AssertionError(f"{label} {op}: {len(de)} vs {len(dg)} containers; first (key, kind, card) "
                                 f"diffs exp/got: {diff[:5]}")
    for op in CARDS:
        assert gpu_card(op, a, b) == O.pairwise_card(op, a, b), (label, op)


def test_every_container_mode_pair(gpu):
    """All 18x18 container-mode combinations on one key (type thresholds)."""
    rng = np.random.default_rng(7)
    for m1 in _gen.MODES:
        for m2 in _gen.MODES:
            k1, v1 = _gen.container(rng, m1)
            k2, v2 = _gen.container(rng, m2)
            check_all(encode([(3, k1, v1)]), encode([(3, k2, v2)]), f"{m1}x{m2}")


@pytest.mark.parametrize("seed", range(12))
def test_random_bitmaps(gpu, seed):
    rng = np.random.default_rng(seed)
    keys = np.sort(rng.choice(64, size=int(rng.integers(1, 40)), replace=False))
    check_all(_gen.bitmap(rng, keys), _gen.bitmap(rng, keys), f"seed{seed}")


@pytest.mark.parametrize("form", ["planned", "balanced"])
def test_random_bitmaps_many_tiles(gpu, form):
    """Random container modes over thousands of keys, so results span many tiles of 64 records (the fused
    placement + serialization's tile sums, round 6): 2,500 random keys of every mode (planned list), or
    34,000 dense keys present in both operands (balanced list) of the lighter modes."""
    rng = np.random.default_rng(31 if form == "planned" else 32)
    if form == "planned":
        keys = np.sort(rng.choice(65536, size=2500, replace=False))
        a, b = _gen.bitmap(rng, keys), _gen.bitmap(rng, keys)
    else:
        modes = ["a_tiny", "a_small", "r_tiny", "r_single", "r_tie", "r_few"]
        keys = np.arange(34000)
        a, b = _gen.bitmap(rng, keys, modes, p_present=1.0), _gen.bitmap(rng, keys, modes, p_present=1.0)
    check_all(a, b, form)


@pytest.mark.parametrize("seed", range(8))
def test_perturbed_pairs(gpu, seed):
    rng = np.random.default_rng(100 + seed)
    keys = np.sort(rng.choice(1 << 16, size=30, replace=False))
    a, b = _gen.perturbed_pair(rng, keys)
    check_all(a, b, f"pert{seed}")
    check_all(b, a, f"pert{seed}r")


def _sparse_result_pair(keys):
    """Operands whose AND is empty on most keys, a run container on every 211th and an array on every 97th:
    the result's run-flag bytes span tiles of 64 records with empty tiles between them."""
    ra = np.concatenate([np.arange(0, 100), np.arange(200, 300)]).astype(np.uint16)
    rb = np.arange(50, 150, dtype=np.uint16)
    a, b = [], []
    for k in keys:
        k = int(k)
        if k % 211 == 0:
            a.append((k, R, ra))
            b.append((k, R, rb))
        elif k % 97 == 0:
            a.append((k, 0, np.array([1, 2, 3, 10 + k % 1000], dtype=np.uint16)))
            b.append((k, 0, np.array([2, 3, 4], dtype=np.uint16)))
        else:
            a.append((k, 0, np.array([5, 6, 7], dtype=np.uint16)))
            b.append((k, 0, np.array([8, 9], dtype=np.uint16)))
    return encode(a), encode(b)


@pytest.mark.parametrize("form", ["balanced", "planned"])
def test_serialize_from_tile_sums_sparse_runs(gpu, form):
    """k_serialize_agg (placement + serialization from the compute kernel's per-tile sums, round 6): a sparse
    result with run containers, so a flag byte's tail is read from later tiles across empty ones; dense keys
    take the balanced form (k_pair_cu), every third key the planned one (k_pair_wave)
    (RB/RoaringArray.java:896-940)."""
    keys = np.arange(40000) if form == "balanced" else np.arange(0, 65536, 3)
    a, b = _sparse_result_pair(keys)
    check_all(a, b, form)
    got = decode(gpu_pair("and", a, b))
    assert sum(1 for c in got if c[1] == R) > 50 and len(got) > 200


def test_fused_serialization_and_placement_users(gpu):
    """k_serialize_agg places the records as k_place does: after it, the result statistics, the key-shard fetch
    (which reads the records' placement) and the fetch agree with the oracle; and the same op with the
    statistics first (k_place, then k_serialize) gives the same bytes (RB/RoaringArray.java:896-940)."""
    import struct
    from roaringbitmap_amd import Engine
    a, b = _sparse_result_pair(np.arange(40000))
    exp = O.pairwise("and", a, b)
    n = len(decode(exp))
    has_run = int((struct.unpack("<I", exp[:4])[0] & 0xFFFF) == 12347)
    desc_base = 4 + (n + 7) // 8 if has_run else 8
    offsets = not has_run or n >= 4
    head = desc_base + 4 * n + (4 * n if offsets else 0)
    e = Engine(0)
    try:
        x, y = e.load_pair(a, b)
        e.pairwise("and", x, y)
        e.serialize()
        st = e.result_stats()
        assert (st["containers"], st["has_run"]) == (n, has_run)
        assert st["cardinality"] == O.pairwise_card("and", a, b)
        assert e.fetch().serialize() == exp
        d, o, p = e.fetch_shard(n, has_run, 0, 0)
        assert d == exp[desc_base:desc_base + 4 * n]
        if offsets:
            assert o == exp[desc_base + 4 * n:head]
        assert p == exp[head:]
        e.pairwise("and", x, y)
        assert e.result_stats() == st
        e.serialize()
        assert e.fetch().serialize() == exp
    finally:
        e.close()


def test_run_and_above_lds_limit(gpu):
    """R AND R whose run lists do not fit one wave's LDS together (na + nb + 2 > 2558: the bitmap path;
    RB/RunContainer.java:381-456), beside pairs that do: runs that straddle 32768 in one or both operands,
    overlaps that end or start exactly there, pairs skewed into one half of the key's values, a result
    that is not a run container (EFF picks an array), and 2,047 runs per list.  (The same pairs pinned a
    two-value-window run merge for the large pairs, measured slower and not kept:
    profiles/r06/experiments/rr_value_windows.txt.)"""
    rng = np.random.default_rng(2558)
    H = 32768

    def runs(nr, span=65536, lo=0):
        return (lo + _gen._runs(rng, nr, span=span).astype(np.int64)).astype(np.uint16)

    def u(*xs):
        return np.unique(np.concatenate([np.asarray(x, dtype=np.int64) for x in xs])).astype(np.uint16)

    pairs = [
        (runs(1800), runs(1700)),                                           # C2-like
        (u(runs(1500), np.arange(H - 90, H + 110)), u(runs(1400), np.arange(H - 40, H + 300))),  # both straddle
        (u(runs(1500), np.arange(H - 90, H + 110)), runs(1400)),            # A straddles
        (runs(1500), u(runs(1400), np.arange(H - 7, H + 3))),               # B straddles
        (runs(1500, span=H), runs(1500, span=H)),                           # skewed: window 0 too big
        (u(runs(1400), np.arange(H - 8, H)), u(runs(1300), np.arange(H, H + 40))),  # touch at the edge
        (u(runs(1400), np.arange(H - 8, H)), u(runs(1300), np.arange(H - 1, H + 40))),  # overlap = {H - 1}
        (u(runs(1400), np.arange(H, H + 9)), u(runs(1300), np.arange(H - 30, H + 1))),  # overlap = {H}
        (np.arange(0, 4094, 2), np.arange(0, 4094, 2)),                     # 2047 singletons: an array result
        (runs(2047), runs(2047)),                                           # the most runs per list
        (runs(1300, span=H, lo=H), runs(1300, span=H, lo=H)),               # all runs in the upper window
    ]
    for i, (va, vb) in enumerate(pairs):
        a, b = encode([(7, R, va)]), encode([(7, R, vb)])
        check_all(a, b, f"rr{i}")
        check_all(b, a, f"rr{i}r")
    # all of them in one bitmap pair (one task per key, the balanced list mixes them)
    a = encode([(k, R, va) for k, (va, _) in enumerate(pairs)])
    b = encode([(k, R, vb) for k, (_, vb) in enumerate(pairs)])
    check_all(a, b, "rr-all")


def test_empty_and_disjoint(gpu):
    empty = encode([])
    rng = np.random.default_rng(5)
    x = _gen.bitmap(rng, np.arange(10))
    y = _gen.bitmap(rng, np.arange(100, 110))
    check_all(empty, empty, "empty")
    check_all(empty, x, "empty-x")
    check_all(x, empty, "x-empty")
    check_all(x, y, "disjoint")
    check_all(x, x, "self")


def test_golden_files(gpu):
    a = open(os.path.join(GOLD, "testdata", "bitmapwithruns.bin"), "rb").read()
    b = open(os.path.join(GOLD, "testdata", "bitmapwithoutruns.bin"), "rb").read()
    check_all(a, b, "golden")
    check_all(b, a, "golden-r")


def test_header_variants(gpu):
    """size < 4 with runs omits the offset table (RB/RoaringArray.java:927-933)."""
    full = np.arange(65536, dtype=np.uint16)
    for n in range(1, 6):
        a = encode([(k, R, full[: 100 + k]) for k in range(n)])
        b = encode([(k, R, full[50 + k: 300]) for k in range(n)])
        check_all(a, b, f"runs{n}")


def _realdata(ds):
    z = np.load(os.path.join(GOLD, "realdata", ds + ".npz"))
    v, o = z["values"], z["offsets"]
    return [v[o[i]:o[i + 1]] for i in range(len(o) - 1)]


@pytest.mark.parametrize("ds", ["census1881", "census1881_srt", "wikileaks-noquotes", "uscensus2000"])
@pytest.mark.parametrize("run_opt", [False, True])
def test_realdata_known_answers(gpu, ds, run_opt):
    rb = _rb()
    known = json.load(open(os.path.join(GOLD, "known_answers.json")))["values"][ds]
    bms = [rb.RoaringBitmap.from_values(s, run_opt) for s in _realdata(ds)]
    sums = {op: 0 for op in OPS}
    for k in range(len(bms) - 1):
        for op in OPS:
            got = rb.RoaringBitmap._pair(op, bms[k], bms[k + 1])
            sums[op] += got.getLongCardinality()
            if k % 20 == 0:
                assert got.serialize() == O.pairwise(op, bms[k].serialize(), bms[k + 1].serialize())
        assert rb.RoaringBitmap.andCardinality(bms[k], bms[k + 1]) == O.pairwise_card(
            "and", bms[k].serialize(), bms[k + 1].serialize())
    for op in OPS:
        assert sums[op] == known[op], op


def test_java_int_wrap(gpu):
    full = encode([(k, R, np.arange(65536, dtype=np.uint16)) for k in range(32768)])
    assert gpu_card("and", full, full) == -(1 << 31)
    assert gpu_card("or", full, full) == -(1 << 31)
    assert gpu_card("intersects", full, full) == 1


@pytest.mark.parametrize("i", range(1, 8))
def test_bad_inputs_raise_ioerror(gpu, i):
    rb = _rb()
    bad = open(os.path.join(GOLD, "testdata", f"crashproneinput{i}.bin"), "rb").read()
    good = encode([])
    with pytest.raises(OSError):
        rb.RoaringBitmap._pair("and", rb.RoaringBitmap(bad), rb.RoaringBitmap(good))


def _run_vals(rng, nruns, lo=0, hi=65536, min_len=1, max_len=None):
    """Sorted values forming exactly `nruns` disjoint, non-adjacent runs inside [lo, hi)."""
    span = hi - lo
    seg = span // nruns
    vals = []
    for i in range(nruns):
        s0 = lo + i * seg
        ml = max_len if max_len else max(1, seg // 2)
        ln = int(rng.integers(min_len, max(min_len, min(ml, seg - 1)) + 1))
        st = s0 + int(rng.integers(0, max(1, seg - ln)))
        vals.append(np.arange(st, min(st + ln, s0 + seg - 1)))
    return np.unique(np.concatenate(vals))


@pytest.mark.parametrize("na,nb", [(1, 1), (1, 2000), (2000, 1), (1279, 1281), (1280, 1280), (1281, 1280),
                                   (2047, 2047), (700, 900), (2, 3)])
def test_run_and_run_domain_boundaries(gpu, na, nb):
    """R AND R: the run-domain merge (na + nb <= 2560 runs) and the bitmap fallback
    above it give the oracle's bytes; also full containers, runs touching 0 and 65535,
    and results that EFF turns into arrays or bitmaps."""
    import roaringbitmap_amd as rb
    from _fmt import R, encode
    rng = np.random.default_rng(na * 7919 + nb)
    cases = []
    a = _run_vals(rng, na)
    b = _run_vals(rng, nb)
    cases.append((a, b))
    cases.append((np.arange(65536), b))                                  # full container
    cases.append((np.concatenate([np.arange(0, 10), np.arange(65500, 65536)]), a))  # edges
    if na == nb:
        cases.append((a, a))                                             # identical
        cases.append((a, np.setdiff1d(np.arange(65536), a)))             # disjoint: empty
    for x, y in cases:
        bx = encode([(5, R, x), (9, R, y)])
        by = encode([(5, R, y), (9, R, x)])
        got = rb.RoaringBitmap.and_(rb.RoaringBitmap(bx), rb.RoaringBitmap(by)).serialize()
        assert got == O.pairwise("and", bx, by)
        assert rb.RoaringBitmap.andCardinality(rb.RoaringBitmap(bx), rb.RoaringBitmap(by)) == \
            O.pairwise_card("and", bx, by)


@pytest.mark.parametrize("na,nb", [(1, 1), (1, 2000), (1279, 1281), (1281, 1280), (700, 900), (2, 3)])
def test_run_or_run(gpu, na, nb):
    """R OR R: overlapping, adjacent (coalescing) and nested runs, full containers,
    identical operands, many-run operands."""
    import roaringbitmap_amd as rb
    from _fmt import R, encode
    rng = np.random.default_rng(na * 31 + nb)
    a = _run_vals(rng, na)
    b = _run_vals(rng, nb)
    adj = np.concatenate([np.arange(0, 100), np.arange(300, 400)])
    adj2 = np.concatenate([np.arange(100, 300), np.arange(400, 401), np.arange(65000, 65536)])
    for x, y in [(a, b), (a, a), (np.arange(65536), b), (adj, adj2), (adj2, adj), (a, np.arange(10, 20))]:
        bx = encode([(5, R, x), (9, R, y)])
        by = encode([(5, R, y), (9, R, x)])
        got = rb.RoaringBitmap.or_(rb.RoaringBitmap(bx), rb.RoaringBitmap(by)).serialize()
        assert got == O.pairwise("or", bx, by)
        assert rb.RoaringBitmap.orCardinality(rb.RoaringBitmap(bx), rb.RoaringBitmap(by)) == \
            O.pairwise_card("or", bx, by)


def _split_cases(rng):
    """R AND R operand pairs whose run lists together exceed one wave's LDS
    (2558 < na + nb <= 5116): the two-window run-domain path, its junction at
    32767 / 32768, and its fallbacks (a window that does not fit, a result that is
    not R)."""
    lo_hi = lambda n1, n2: np.concatenate([_run_vals(rng, n1, 0, 32768), _run_vals(rng, n2, 32768, 65536)])
    a, b = _run_vals(rng, 2000), _run_vals(rng, 1900)
    cases = [("spread", a, b), ("spread_same", a, a)]
    # one run of each operand spans 32767 / 32768: the result run is split and merged
    cross_a = np.union1d(_run_vals(rng, 1100, 0, 32000), np.arange(32100, 33000))
    cross_a = np.union1d(cross_a, _run_vals(rng, 1100, 33100, 65536))
    cross_b = np.union1d(_run_vals(rng, 1100, 0, 32000), np.arange(32500, 34000))
    cross_b = np.union1d(cross_b, _run_vals(rng, 1100, 34100, 65536))
    cases.append(("junction", cross_a, cross_b))
    cases.append(("junction_exact", np.union1d(lo_hi(1200, 1200), [32767, 32768]),
                  np.union1d(lo_hi(1100, 1100), [32767, 32768])))
    # only A crosses; B has a run ending at 32767 and one starting at 32769
    b_edge = np.union1d(lo_hi(1100, 1100), np.concatenate([np.arange(32700, 32768), np.arange(32769, 32800)]))
    cases.append(("cross_a_only", cross_a, b_edge))
    # the result ends window 0 at 32767 without a junction
    cases.append(("end_at_32767", np.union1d(lo_hi(1200, 1200), np.arange(32600, 32768)),
                  np.union1d(lo_hi(1200, 1200), np.arange(32650, 32768))))
    # every run in the low half: window 0 does not fit, bitmap path
    cases.append(("low_half", _run_vals(rng, 1500, 0, 32768), _run_vals(rng, 1500, 0, 32768)))
    # interleaved short runs: the intersection has > 2047 runs (bitmap result) ...
    s3 = np.arange(0, 65536 - 3, 26)
    cases.append(("many_result_runs", np.unique(np.concatenate([s3, s3 + 1, s3 + 2])),
                  np.unique(np.concatenate([s3 + 1, s3 + 2, s3 + 3]))))
    # ... or single values (array result by EFF)
    s2 = np.arange(0, 65536 - 2, 40)
    cases.append(("array_result", np.unique(np.concatenate([s2, s2 + 1])), np.unique(np.concatenate([s2 + 1, s2 + 2]))))
    cases.append(("disjoint", a, np.setdiff1d(np.arange(65536), a)))
    return cases


def test_run_and_run_split_windows(gpu):
    """R AND R above the one-window LDS capacity (RB/RunContainer.java and(RunContainer)):
    byte-identical AND / andCardinality / intersects."""
    import roaringbitmap_amd as rb
    from _fmt import R, encode
    rng = np.random.default_rng(2558)
    for label, x, y in _split_cases(rng):
        bx = encode([(5, R, x), (9, R, y), (11, R, x)])
        by = encode([(5, R, y), (9, R, x), (11, R, x)])
        got = rb.RoaringBitmap.and_(rb.RoaringBitmap(bx), rb.RoaringBitmap(by)).serialize()
        assert got == O.pairwise("and", bx, by), label
        for op in ("and", "intersects"):
            assert gpu_card(op, bx, by) == O.pairwise_card(op, bx, by), (label, op)


@pytest.mark.parametrize("nruns", [3000, 9000, 32768])
def test_many_run_inputs_all_ops(gpu, nruns):
    """Input run containers with far more than 2047 runs (the deserializer accepts up to
    32768: alternating bits) against arrays, bitmaps and run containers, every op and
    cardinality: the run lists stream past the per-lane vectors and the R maps / bitmap
    materialisation take them whole."""
    from _fmt import A, B, R, encode
    rng = np.random.default_rng(nruns)
    if nruns == 32768:
        many = np.arange(0, 65536, 2)
    else:
        many = _run_vals(rng, nruns)
    others = [
        (A, np.sort(rng.choice(65536, size=3000, replace=False))),
        (A, np.sort(rng.choice(65536, size=40, replace=False))),
        (B, np.sort(rng.choice(65536, size=30000, replace=False))),
        (R, _run_vals(rng, 700)),
        (R, _run_vals(rng, 2500)),
        (R, np.arange(1, 65536, 2)),
    ]
    for kind, vals in others:
        x = encode([(2, R, many), (4, kind, vals), (6, R, many)])
        y = encode([(2, kind, vals), (4, R, many), (5, kind, vals)])
        check_all(x, y, f"R{nruns} x {kind}")
        check_all(y, x, f"{kind} x R{nruns}")


@pytest.mark.parametrize("seed", range(4))
def test_dense_key_range_direct_mode(gpu, seed):
    """Dense key ranges run without the plan launch (the compute kernel resolves key key_lo + t
    itself, csrc/pairwise.hip direct mode): every op and cardinality over a key range where each
    operand holds most keys, some keys in one operand only (empty records for AND / ANDNOT), and
    keys absent from both, against the oracle (RB/RoaringBitmap.java:382-400, :449-471, :864-896,
    :1076-1113)."""
    from roaringbitmap_amd import Engine
    rng = np.random.default_rng(4000 + seed)
    lo = int(rng.integers(0, 60000))
    n = int(rng.integers(40, 300))
    keys = np.arange(lo, lo + n)
    a = _gen.bitmap(rng, keys, p_present=0.85)
    b = _gen.bitmap(rng, keys, p_present=0.85)
    e = Engine(0)
    ba, bb = e.load([a]), e.load([b])
    for op in OPS:
        e.pairwise(op, ba, bb, key_lo=lo, key_hi=lo + n)
        assert e.fetch().serialize() == O.pairwise(op, a, b), (seed, op)
    e.and_cardinality(ba, bb)  # the whole key space: planned form
    assert e.card() == O.pairwise_card("and", a, b)
    e.release(ba)
    e.release(bb)


@pytest.mark.parametrize("balance", ["0", "1"])
@pytest.mark.parametrize("seed", range(3))
def test_dense_range_task_orders(gpu, seed, balance, monkeypatch):
    """Dense key ranges in both task orders: key order (RBG_PW_BALANCE=0, the direct form) and binned by
    estimated cost (k_plan_balanced: the task list out of key order, records still at key positions,
    empty records / zero counts for keys without a task) claimed per CU (k_pair_cu).  Every op, the
    key-range form and andCardinality over a range that covers every key, against the oracle."""
    from roaringbitmap_amd import Engine
    monkeypatch.setenv("RBG_PW_BALANCE", balance)
    rng = np.random.default_rng(4100 + seed)
    n = int(rng.integers(300, 1500))
    keys = np.arange(n)
    a = _gen.bitmap(rng, keys, p_present=0.8)
    b = _gen.bitmap(rng, keys, p_present=0.8)
    e = Engine(0)
    ba, bb = e.load([a]), e.load([b])
    for op in OPS:
        e.pairwise(op, ba, bb, key_lo=0, key_hi=n)
        assert e.fetch().serialize() == O.pairwise(op, a, b), (seed, op)
        lo, hi = n // 3, n // 3 + n // 2
        e.pairwise(op, ba, bb, key_lo=lo, key_hi=hi)
        rs = e.result_stats()
        exp = O.pairwise(op, a, b)
        want = sum(1 for c in decode(exp) if lo <= c[0] < hi)
        assert rs["containers"] == want, (seed, op)
    e.and_cardinality(ba, bb)
    assert e.card() == O.pairwise_card("and", a, b)
    e.release(ba)
    e.release(bb)
    for op in OPS:  # one-shot path (rbg_pairwise) with a dense pair
        assert gpu_pair(op, a, b) == O.pairwise(op, a, b), (seed, op)
