"""FastAggregation wide ops on the MI355X vs the CPU oracle (byte-identical).

RB/FastAggregation.java: and :37-42 (workShyAnd :356-414 for N>10, naive_and
:328-346 otherwise), and(Iterator) :26-28, or :664-666 (naive_or :603-610),
xor :834-836 (naive_xor :637-644), andCardinality :71-82, orCardinality :90-101.
"""
import os

import numpy as np
import pytest

import _gen
import _oracle as O
from _fmt import decode

pytestmark = pytest.mark.gpu
GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _rb():
    import roaringbitmap_amd as rb
    return rb


def gpu_wide(op, bufs, ids=None):
    rb = _rb()
    from roaringbitmap_amd.roaring import _wide
    return _wide(op, [rb.RoaringBitmap(b) for b in bufs], ids).serialize()


def gpu_wide_card(op, bufs):
    rb = _rb()
    from roaringbitmap_amd.roaring import _wide_card
    return _wide_card(op, [rb.RoaringBitmap(b) for b in bufs])


def _cmp(op, bufs, ids=None):
    exp = O.wide(op, bufs, ids)
    got = gpu_wide(op, bufs, ids)
    if got != exp:
        de, dg = decode(exp), decode(got)
        diff = [(x[0], x[1], x[2], y[1], y[2]) for x, y in zip(de, dg) if x[:3] != y[:3]]
        raise AssertionError(f"{op} N={len(bufs)}: {len(de)} vs {len(dg)} containers; diffs {diff[:5]}")


@pytest.mark.parametrize("n", [0, 1, 2, 3, 5, 10, 11, 16])
def test_wide_random(gpu, n):
    rng = np.random.default_rng(50 + n)
    keys = np.arange(10)
    bufs = [_gen.bitmap(rng, keys, p_present=0.9) for _ in range(n)]
    for op in ["or", "xor", "and", "and_iter", "naive_and"]:
        _cmp(op, bufs, list(range(n)))
    if n:
        _cmp("workshy_and", bufs)
    for op in ["and", "or"]:
        assert gpu_wide_card(op, bufs) == O.wide_card(op, bufs), op


@pytest.mark.parametrize("seed", range(6))
def test_wide_dense_overlap(gpu, seed):
    """inputs restricted to modes whose intersections stay non-empty"""
    rng = np.random.default_rng(900 + seed)
    modes = ["b_dense", "full_b", "full_r", "r_dense", "r_few", "b_mid"]
    n = [2, 4, 7, 10, 12, 20][seed]
    bufs = [_gen.bitmap(rng, np.arange(6), modes=modes, p_present=1.0) for _ in range(n)]
    for op in ["or", "xor", "and", "and_iter", "naive_and", "workshy_and"]:
        _cmp(op, bufs, list(range(n)))
    assert gpu_wide_card("and", bufs) == O.wide_card("and", bufs)
    assert gpu_wide_card("or", bufs) == O.wide_card("or", bufs)


def test_wide_identity_skip(gpu):
    """naive_and skips inputs that are the smallest object (RB/FastAggregation.java:341)"""
    rng = np.random.default_rng(3)
    small = _gen.bitmap(rng, np.arange(3), modes=["r_few", "r_tie", "r_many"], p_present=1.0)
    big = _gen.bitmap(rng, np.arange(8), modes=["r_dense", "full_r"], p_present=1.0)
    bufs = [big, small, big, small]
    _cmp("and", bufs, [0, 1, 0, 1])
    _cmp("and", bufs, [0, 1, 2, 3])


def _realdata(ds):
    z = np.load(os.path.join(GOLD, "realdata", ds + ".npz"))
    v, o = z["values"], z["offsets"]
    return [v[o[i]:o[i + 1]] for i in range(len(o) - 1)]


@pytest.mark.parametrize("run_opt", [False, True])
def test_wide_realdata(gpu, run_opt):
    import json
    known = json.load(open(os.path.join(GOLD, "known_answers.json")))["values"]
    for ds in ["census1881", "census1881_srt", "wikileaks-noquotes_srt"]:
        bufs = [O.from_values(s, run_opt) for s in _realdata(ds)]
        _cmp("or", bufs)
        _cmp("and", bufs)
        _cmp("xor", bufs)
        rb = _rb()
        got = rb.FastAggregation.or_(*[rb.RoaringBitmap(b) for b in bufs])
        assert got.getLongCardinality() == known[ds]["wide_or"]
        got = rb.FastAggregation.and_(iter([rb.RoaringBitmap(b) for b in bufs]))
        assert got.getLongCardinality() == known[ds]["wide_and"]


def test_parallel_and_horizontal_aggregation_sets(gpu):
    """ParallelAggregation.or/xor and FastAggregation.horizontal_*/priorityqueue_* give the
    reference's sets (RBT/ParallelAggregationTest compares sets); horizontal_or(Iterator)
    is naive_or itself, byte for byte."""
    import numpy as np
    import roaringbitmap_amd as rb
    import _gen
    import _oracle as O
    rng = np.random.default_rng(77)
    bufs = [_gen.bitmap(rng, np.sort(rng.choice(40, size=int(rng.integers(1, 12)), replace=False)))
            for _ in range(9)]
    bms = [rb.RoaringBitmap(b) for b in bufs]
    union = set(O.to_values(O.wide("or", bufs)).tolist())
    sym = set(O.to_values(O.wide("xor", bufs)).tolist())
    for got in (getattr(rb.ParallelAggregation, "or")(*bms), rb.FastAggregation.horizontal_or(bms),
                rb.FastAggregation.horizontal_or(*bms), rb.FastAggregation.priorityqueue_or(*bms)):
        assert set(got.toArray().tolist()) == union
    for got in (rb.ParallelAggregation.xor(*bms), rb.FastAggregation.horizontal_xor(*bms),
                rb.FastAggregation.priorityqueue_xor(*bms)):
        assert set(got.toArray().tolist()) == sym
    assert rb.FastAggregation.horizontal_or(iter(bms)).serialize() == O.wide("or", bufs)


@pytest.mark.parametrize("n", [0, 1, 2, 5, 10, 11, 14])
def test_buffer_fast_aggregation_dispatch(gpu, n):
    """RB/buffer/BufferFastAggregation.java: and(Iterator) :66-89 and and(Mutable...)
    :100-102 run workShyAnd for every N (FastAggregation's Iterator form runs
    naive_and); naive_and(Mutable...) :407-416 chains from the first bitmap; the
    varargs forms dispatch like FastAggregation (workShyAnd above 10 inputs).  The and
    chains are the buffer package's (run AND run keeps the merged runs)."""
    import roaringbitmap_amd as rb
    rng = np.random.default_rng(900 + n)
    bufs = [_gen.bitmap(rng, np.arange(8), p_present=0.85) for _ in range(n)]
    bms = [rb.RoaringBitmap(b) for b in bufs]
    B = rb.BufferFastAggregation
    empty = rb.RoaringBitmap().serialize()
    ws = O.wide("workshy_and", bufs) if n else empty
    assert B.and_(iter(bms)).serialize() == ws
    assert B.and_mutable(*bms).serialize() == ws
    assert getattr(B, "and")(*bms).serialize() == O.wide("buffer_and", bufs, list(range(n)))
    assert B.naive_and(*bms).serialize() == O.wide("buffer_naive_and", bufs, list(range(n)))
    assert B.naive_and(iter(bms)).serialize() == O.wide("buffer_and_iter", bufs)
    assert B.naive_and_mutable(*bms).serialize() == O.wide("buffer_and_iter", bufs)
    assert B.or_(*bms).serialize() == O.wide("or", bufs)
    assert B.or_(iter(bms)).serialize() == O.wide("or", bufs)
    assert B.xor(*bms).serialize() == O.wide("xor", bufs)
    assert B.andCardinality(*bms) == O.wide_card("and", bufs)
    assert B.orCardinality(*bms) == O.wide_card("or", bufs)
    if n > 10:
        buf = np.zeros(1024, dtype=np.int64)
        assert B.and_(buf, *bms).serialize() == ws
        with pytest.raises(rb.IllegalArgumentException):
            B.and_(np.zeros(10, dtype=np.int64), *bms)


@pytest.mark.parametrize("n", [1, 2, 3, 11])
def test_wide_many_run_inputs(gpu, n):
    """Wide ops over inputs whose run containers hold 2,500 - 32,768 runs (beyond any
    per-lane staging), mixed with arrays and bitmaps on the same keys: naive_or's single
    input pass-through (R -> EFF), the lazy OR, the naive_xor chain replay with runs,
    workShyAnd / naive_and."""
    from _fmt import A, B, R, encode
    rng = np.random.default_rng(900 + n)

    def runs(k):
        seg = 65536 // k
        st = np.arange(k) * seg + rng.integers(0, max(1, seg // 2), k)
        return np.unique(np.concatenate([np.arange(s, min(s + 1 + int(rng.integers(0, max(1, seg // 2))), 65536))
                                         for s in st]))
    bufs = []
    for i in range(n):
        ctrs = []
        for key in (1, 3, 8):
            m = (i + key) % 4
            if m == 0:
                ctrs.append((key, R, np.arange(i % 2, 65536, 2)))  # 32,768 runs
            elif m == 1:
                ctrs.append((key, R, runs(2500 + 1000 * i)))
            elif m == 2:
                ctrs.append((key, A, np.sort(rng.choice(65536, size=2000, replace=False))))
            else:
                ctrs.append((key, B, np.sort(rng.choice(65536, size=20000, replace=False))))
        bufs.append(encode(ctrs))
    for op in ["or", "xor", "and", "and_iter", "naive_and"]:
        _cmp(op, bufs, list(range(n)))
    _cmp("workshy_and", bufs)
    for op in ["and", "or"]:
        assert gpu_wide_card(op, bufs) == O.wide_card(op, bufs), op


@pytest.mark.parametrize("case", ["all_bitmaps", "array_first", "run_middle", "gap"])
def test_wide_or_in_place_bitmaps(gpu, case):
    """Wide OR writes a bitmap result of task t straight to payload offset 8192 t (OutCtx::spec);
    it is in place only while every earlier key kept an 8 KiB container, else k_spec_fix moves it
    to its slot before the serialization.  Byte-identical to the oracle in every case."""
    rb = _rb()
    rng = np.random.default_rng(7)
    nk = 40
    per = [[] for _ in range(6)]
    for k in range(nk):
        for i in range(6):
            if case == "gap" and k == 17:
                continue  # no input has key 17: no task for it, so the later bitmaps stay in place
            if case == "array_first" and k == 0:
                v = rng.choice(65536, 300, replace=False)  # a small array result for key 0
            elif case == "run_middle" and k == 20:
                s = int(rng.integers(0, 30000))
                v = np.arange(s, s + 20000)  # one long run: a run container result
            else:
                v = rng.choice(65536, 2000, replace=False)  # six of these: ~11,000 values, a bitmap
            per[i].append((k << 16) + v)
    bufs = [rb.RoaringBitmap.from_values(np.concatenate(p), run_optimize=True).serialize() for p in per]
    _cmp("or", bufs, list(range(6)))


def test_workshy_bytes_read(gpu):
    """rbg_ctx_profile_bytes (the bench's C3 AND roofline): payload + 4 B per container that the
    early-exit workShyAnd read.  Identical inputs never empty, so every container is read;
    pairwise-disjoint ones are empty after two inputs, where the chain stops (it tests the
    intersection after every input)."""
    from roaringbitmap_amd import Engine
    e = Engine(0)

    def read(bufs):
        b = e.load(bufs)
        e.profile(1)
        e.wide("workshy_and", b)
        e.profile_read()
        v = e.profile_bytes()
        e.profile(0)
        e.release(b)
        return v

    rng = np.random.default_rng(9)
    base = _gen.bitmap(rng, np.arange(6), p_present=1.0)
    st = O.stats(base)
    assert read([base] * 12) == 12 * (st["payload"] + 4 * (st["array"] + st["bitmap"] + st["run"]))
    disjoint = [O.from_values(np.concatenate([k * 65536 + 100 * i + np.arange(50) for k in range(6)]))
                for i in range(12)]
    assert read(disjoint) == 6 * 2 * (4 + 2 * 50)


@pytest.mark.parametrize("n", [2, 3, 6])
def test_buffer_and_chain_run_pairs(gpu, n):
    """BufferFastAggregation's and chains keep a run AND run result as the merged run container
    (RB/buffer/MappeableRunContainer.java:474-536 via iand :1106-1108), including results of more
    than 2,047 runs (16,384 one-value runs on key 2), where FastAggregation's heap chain converts
    (RB/RunContainer.java:381-456): heap and buffer bytes differ, each byte-exact to its oracle."""
    from _fmt import A, R, encode
    rb = _rb()
    rng = np.random.default_rng(40 + n)
    bufs = []
    for i in range(n):
        ph = i % 2  # alternate {4k, 4k+1} and {4k+1, 4k+2}: every AND leaves the one-value runs {4k+1}
        ctrs = [(1, R, np.sort(np.concatenate([np.arange(ph, 4000, 4), np.arange(1 + ph, 4000, 4)]))),
                (2, R, np.sort(np.concatenate([np.arange(ph, 65536, 4), np.arange(1 + ph, 65536, 4)]))),
                (3, R, np.arange(100 + 50 * i, 30000 + 1000 * i)),
                (5, A, np.sort(rng.choice(65536, 3000, replace=False)))]
        if i % 3 == 2:
            ctrs.append((4, R, np.arange(0, 65536, 2)))  # 32,768 runs against the others' absence
        bufs.append(encode(ctrs))
    bms = [rb.RoaringBitmap(b) for b in bufs]
    ids = list(range(n))
    B = rb.BufferFastAggregation
    for got, op, i in ((getattr(B, "and")(*bms), "buffer_and", ids), (B.naive_and(*bms), "buffer_naive_and", ids),
                       (B.naive_and(iter(bms)), "buffer_and_iter", None),
                       (B.naive_and_mutable(*bms), "buffer_and_iter", None)):
        exp = O.wide(op, bufs, i)
        assert got.serialize() == exp, op
        assert exp != O.wide(op.replace("buffer_", ""), bufs, i)
    kinds = [c[:2] for c in decode(B.naive_and(*bms).serialize())]
    assert (2, R) in kinds and (1, R) in kinds
    # FastAggregation's chains on the same inputs stay the heap's
    _cmp("naive_and", bufs, ids)
    _cmp("and_iter", bufs)


@pytest.mark.parametrize("seed", range(3))
def test_workshy_forms(gpu, seed):
    """FastAggregation.workShyAnd (RB/FastAggregation.java:356-414) per key, through every form of the
    wave-per-key kernel's running intersection: small arrays kept in lanes (identical, partly
    overlapping), array AND bitmap (bit gathers), array AND large array (LDS binary search), array
    AND run (to a bitmap), run / bitmap AND small array (back to lanes), large arrays as bitmaps,
    a full result (RunContainer.full), and chains that empty.  Bytes and cardinality vs the oracle."""
    from _fmt import A, B, R, encode
    rng = np.random.default_rng(300 + seed)
    n = 12
    base1 = np.sort(rng.choice(65536, 40, replace=False))
    small = np.sort(rng.choice(5000, 30, replace=False))
    big_sup = np.unique(np.concatenate([small, rng.choice(65536, 1970, replace=False)]))
    mids = np.sort(rng.choice(65536, 3000, replace=False))
    per = [[] for _ in range(n)]
    for i in range(n):
        per[i].append((0, A, small))
        per[i].append((1, A, np.sort(rng.choice(base1, 36, replace=False))))
        per[i].append((2, A, small) if i == 0 else (2, B, np.unique(np.concatenate([small, rng.choice(65536, 6000)]))))
        per[i].append((3, R, np.arange(0, 5000)) if i == 0 else (3, A, np.sort(rng.choice(small, 28, replace=False)))
                      if i == 1 else (3, A, small))
        per[i].append((4, A, np.sort(rng.choice(mids, 2900, replace=False))))
        per[i].append((5, R, np.arange(65536)))
        per[i].append((6, A, small) if i % 2 == 0 else (6, R, np.arange(0, 6000)))
        per[i].append((7, A, small) if i % 3 else (7, A, big_sup))
        per[i].append((8, A, np.arange(100 * i, 100 * i + 50)))  # empty after two inputs
        per[i].append((9, B, np.sort(rng.choice(65536, 20000, replace=False))))
    bufs = [encode(p) for p in per]
    _cmp("workshy_and", bufs)
    _cmp("and", bufs, list(range(n)))  # N > 10: workShyAnd
    assert gpu_wide_card("and", bufs) == O.wide_card("and", bufs)
    kinds = {c[0]: c[1] for c in decode(O.wide("workshy_and", bufs))}
    assert kinds[5] == R and kinds[0] == A and 8 not in kinds


def test_work_and_memory_shy_and(gpu):
    """FastAggregation.workAndMemoryShyAnd (RB/FastAggregation.java:522-576): workShyAnd's result with a
    zeroed buffer; a nonzero buffer adds its bits to the first bitmap's keys (a key the first bitmap
    lacks is skipped per bitmap, i.e. it acts as a full container); afterwards the buffer holds the last
    key's lazy intersection (the per-key fill with ones, then each container ANDed in place)."""
    from roaringbitmap_amd.roaring import _full_containers
    from roaringbitmap_amd._lib import ArrayIndexOutOfBoundsException
    rb = _rb()
    rng = np.random.default_rng(21)
    bufs = [_gen.bitmap(rng, np.arange(10), p_present=0.9) for _ in range(4)]
    bms = [rb.RoaringBitmap(b) for b in bufs]

    def last_key_and(keys_alive, inputs):
        """the buffer the reference leaves: the AND of the last surviving key's containers, as 1,024 words"""
        k = max(keys_alive)
        m = np.ones(65536, dtype=bool)
        for x in inputs:
            v = O.to_values(x)
            if (v >> 16 == k).any():
                bits = np.zeros(65536, dtype=bool)
                bits[(v[v >> 16 == k] & 0xFFFF).astype(np.int64)] = True
                m &= bits
        return np.packbits(m, bitorder="little").view(np.int64)

    keysets = [set((O.to_values(b) >> 16).tolist()) for b in bufs]
    buf = np.zeros(1024, dtype=np.int64)
    assert rb.FastAggregation.workAndMemoryShyAnd(buf, *bms).serialize() == O.wide("workshy_and", bufs)
    assert (buf == last_key_and(set.intersection(*keysets), bufs)).all()
    # a dirty buffer: keys 20 and 3 set; key 20 is in no input, so it cannot survive (n > 1)
    keys0 = keysets[0]
    common = set.intersection(*keysets[1:])
    extra = sorted(k for k in common if k not in keys0)
    buf = np.zeros(1024, dtype=np.int64)
    for k in [20] + extra:
        buf[k >> 6] |= np.int64(1) << np.int64(k & 63)
    exp_first = O.pairwise("or", bufs[0], _full_containers(extra)) if extra else bufs[0]
    got = rb.FastAggregation.workAndMemoryShyAnd(buf, *bms).serialize()
    assert got == O.wide("workshy_and", [exp_first] + bufs[1:])
    # one input and a dirty buffer: the key array is sized by the first bitmap's containers (:540-548)
    buf = np.zeros(1024, dtype=np.int64)
    buf[1] = 1  # key 64, not a key of bms[0]
    with pytest.raises(ArrayIndexOutOfBoundsException):
        rb.FastAggregation.workAndMemoryShyAnd(buf, bms[0])
    # one input, a dirty bit on one of its own keys: no extra key
    buf = np.zeros(1024, dtype=np.int64)
    k0 = min(keys0)
    buf[k0 >> 6] |= np.int64(1) << np.int64(k0 & 63)
    assert rb.FastAggregation.workAndMemoryShyAnd(buf, bms[0]).serialize() == O.wide("workshy_and", [bufs[0]])
    # an empty first bitmap: an empty result, the buffer untouched (:532, :537-539)
    buf = np.full(1024, 7, dtype=np.int64)
    assert rb.FastAggregation.workAndMemoryShyAnd(buf, rb.RoaringBitmap.bitmapOf(), *bms).isEmpty()
    assert (buf == 7).all()
    # an empty later bitmap: intersectArrayIntoBitmap with no keys leaves word 0 and zeroes the rest
    buf = np.zeros(1024, dtype=np.int64)
    buf[5] = 3
    a = rb.RoaringBitmap.bitmapOf(1, 2, 3 << 16)
    assert rb.FastAggregation.workAndMemoryShyAnd(buf, a, rb.RoaringBitmap.bitmapOf()).isEmpty()
    assert buf[0] == 0b1001 and (buf[1:] == 0).all()
    # disjoint keys: nothing survives, the buffer is left zero
    a, b = rb.RoaringBitmap.bitmapOf(1, 2), rb.RoaringBitmap.bitmapOf(1 << 16)
    buf = np.zeros(1024, dtype=np.int64)
    assert rb.FastAggregation.workAndMemoryShyAnd(buf, a, b).isEmpty() and (buf == 0).all()
    # a longer buffer: the fills and the key intersection run over its whole length
    buf = np.zeros(1100, dtype=np.int64)
    x, y = rb.RoaringBitmap.bitmapOf(1, 5, 9), rb.RoaringBitmap.bitmapOf(5, 9, 12)
    assert rb.FastAggregation.workAndMemoryShyAnd(buf, x, y).serialize() == rb.RoaringBitmap.bitmapOf(5, 9).serialize()
    assert buf[0] == (1 << 5) | (1 << 9) and (buf[1:] == 0).all()
