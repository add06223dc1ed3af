"""Pins the oracle's alternative aggregations (oracle/rbcpu.cpp: ParallelAggregation,
horizontal_*, priorityqueue_*, BufferFastAggregation over Mutable bitmaps) to the
reference's own tests.  No GPU.

Java's RoaringBitmap.equals is what those tests assert: keys equal, and per key
ArrayContainer vs BitmapContainer is type-sensitive (RB/ArrayContainer.java:371-379,
RB/BitmapContainer.java:416-428) while RunContainer compares sets with anything
(RB/RunContainer.java:929-949).  `java_equals` restates it.

Sources:
  RBT/ParallelAggregationTest.java:41-240      Parallel == FastAggregation (or, xor)
  RBT/TestFastAggregation.java:21-70           horizontal_or / priorityqueue_or small cases
  RBT/TestRoaringBitmap.java:3176-3320         massive or / xor vs chained pairwise ops
  jmh/src/test/.../RealDataBenchmarkWideOrPqTest.java:14-19  priorityqueue_or known answers
"""
import json
import os

import numpy as np
import pytest

import _oracle as O
from _fmt import A, B, R, decode, encode

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def java_equals(x: bytes, y: bytes) -> bool:
    dx, dy = decode(x), decode(y)
    if [c[0] for c in dx] != [c[0] for c in dy]:
        return False
    for (_, kx, _, vx, _), (_, ky, _, vy, _) in zip(dx, dy):
        if kx != ky and R not in (kx, ky):
            return False  # array vs bitmap: never equal
        if not np.array_equal(np.asarray(vx, np.int64), np.asarray(vy, np.int64)):
            return False
    return True


def _values(buf):
    return O.to_values(buf)


# ---- SeededTestData-style builders (RBT/SeededTestData.java:95-173) ------------------
def _case(rng, spec):
    """spec: [(key, 'A'|'B'|'R')] -> a bitmap with one container of that type per key."""
    ctrs = []
    for key, t in spec:
        if t == "A":
            n = int(rng.integers(1, 4096))
            ctrs.append((key, A, np.sort(rng.choice(65536, n, replace=False)).astype(np.uint16)))
        elif t == "B":
            n = int(rng.integers(4097, 65536))
            ctrs.append((key, B, np.sort(rng.choice(65536, n, replace=False)).astype(np.uint16)))
        else:  # rleRegion: 1..2047 runs from sorted random u16 (:95-102)
            nr = int(rng.integers(1, 2048))
            b = np.unique(rng.integers(0, 65536, 2 * nr))
            if b.size % 2:
                b = b[:-1]
            vals = np.concatenate([np.arange(b[i], b[i + 1]) for i in range(0, b.size, 2)] or [np.zeros(0)])
            vals = np.unique(vals.astype(np.int64))
            if vals.size == 0:
                vals = np.array([7])
            ctrs.append((key, R, vals.astype(np.uint16)))
    return O.run_optimize(encode(ctrs)) if any(t == "R" for _, t in spec) else encode(ctrs)


PARALLEL_OR_CASES = {
    "singleContainerOR": [[(0, "R")], [(0, "B")], [(0, "A")]],
    "twoContainerOR": [[(0, "R"), (1, "A")], [(1, "B")], [(1, "A")]],
    "disjointOR": [[(0, "R"), (2, "A")], [(1, "B")], [(3, "A")]],
    "disjointBigKeysOR": [[(0, "R"), (2, "A"), ((1 << 15) | 1, "B")], [(1, "B"), ((1 << 15) | 2, "R")],
                          [(3, "A"), ((1 << 15) | 3, "R")]],
}
PARALLEL_XOR_CASES = {
    "singleContainerXOR": [[(0, "R")], [(0, "B")], [(0, "A")]],
    "missingMiddleContainerXOR": [[(0, "R"), (1, "B"), (2, "A")], [(0, "B"), (2, "A")],
                                  [(0, "A"), (1, "B"), (2, "A")]],
    "twoContainerXOR": [[(0, "R"), (1, "A")], [(1, "B")], [(1, "A")]],
    "disjointXOR": [[(0, "R"), (2, "A")], [(1, "B")], [(3, "A")]],
}


@pytest.mark.parametrize("name", sorted(PARALLEL_OR_CASES))
def test_parallel_or_small_cases(name):
    rng = np.random.default_rng(len(name))
    bms = [_case(rng, spec) for spec in PARALLEL_OR_CASES[name]]
    assert java_equals(O.wide("or", bms), O.wide("parallel_or", bms))


@pytest.mark.parametrize("name", sorted(PARALLEL_XOR_CASES))
def test_parallel_xor_small_cases(name):
    rng = np.random.default_rng(len(name) + 100)
    bms = [_case(rng, spec) for spec in PARALLEL_XOR_CASES[name]]
    assert java_equals(O.wide("xor", bms), O.wide("parallel_xor", bms))


@pytest.mark.parametrize("n", [20, 513, 1999])
def test_parallel_wide_and_huge_or(n):
    """wideOr (20), hugeOr1/2 (513, 1999): B at 0, A at 1, R at 2 in every input."""
    rng = np.random.default_rng(n)
    bms = [_case(rng, [(0, "B"), (1, "A"), (2, "R")]) for _ in range(n)]
    got = O.wide("parallel_or", bms)
    assert java_equals(O.wide("or", bms), got)
    # n >= 16 per key: the lazy-bitmap branch, which is FastAggregation's type rule
    assert got == O.wide("or", bms)


def test_horizontal_and_priorityqueue_small():
    """RBT/TestFastAggregation.java:21-70"""
    rb1, rb2, rb3 = O.from_values([0, 1, 2]), O.from_values([0, 5, 6]), O.from_values([1 << 16, 2 << 16])
    exp = O.from_values([0, 1, 2, 5, 6, 1 << 16, 2 << 16])
    for op in ["or", "horizontal_or", "priorityqueue_or", "parallel_or", "buffer_or_mutable"]:
        assert java_equals(exp, O.wide(op, [rb1, rb2, rb3])), op


def _massive(howmany, big):
    """RBT/TestRoaringBitmap.java:3176-3320 inputs: k -> ewah[|k + 2k^2| % 128], then every
    third bitmap flipped on [13, howmany / 2) (bitmapOf / flip results are BY_CARD)."""
    N = 128
    sets = [set() for _ in range(N)]
    base = (1 << 31) if big else 0
    for k in range(howmany):
        sets[abs(k + 2 * k * k) % N].add(base + k)
    for k in range(3, N, 3):
        sets[k] ^= set(range(base + 13, base + howmany // 2))
    return [O.from_values(sorted(s)) for s in sets]


@pytest.mark.parametrize("howmany", [512, 4096, 65536, 262144])
@pytest.mark.parametrize("big", [False, True])
def test_massive_or_xor(howmany, big):
    ewah = _massive(howmany, big)
    ans_or, ans_xor = ewah[0], ewah[0]
    for b in ewah[1:]:
        ans_or = O.pairwise("or", ans_or, b)
        ans_xor = O.pairwise("xor", ans_xor, b)
    assert java_equals(ans_or, O.wide("or", ewah))
    assert java_equals(ans_or, O.wide("horizontal_or", ewah))
    assert java_equals(ans_xor, O.wide("xor", ewah))
    assert java_equals(ans_xor, O.wide("horizontal_xor", ewah))
    rng = np.random.default_rng(howmany)
    rb1 = O.from_values(rng.integers(0, 1 << 22, 5000))
    rb2 = O.from_values(rng.integers(0, 1 << 22, 5000))
    rbor = O.pairwise("or", rb1, rb2)
    assert java_equals(rbor, O.wide("horizontal_or", [rb1, rb2]))
    assert java_equals(rbor, O.wide("priorityqueue_or", [rb1, rb2]))
    assert java_equals(O.wide("xor", [rb1, rb2]), O.wide("priorityqueue_xor", [rb1, rb2]))


def _realdata(ds):
    z = np.load(os.path.join(GOLD, "realdata", ds + ".npz"))
    v, o = z["values"], z["offsets"]
    return [v[o[i]:o[i + 1]] for i in range(len(o) - 1)]


KNOWN = json.load(open(os.path.join(GOLD, "known_answers.json")))["values"]


@pytest.mark.parametrize("ds", sorted(KNOWN))
@pytest.mark.parametrize("run_opt", [False, True])
def test_realdata_wide_or_variants(ds, run_opt):
    """RealDataBenchmarkWideOrPqTest: priorityqueue_or cardinality == the wide-OR answer;
    every OR variant gives that set; every XOR variant gives naive_xor's set."""
    bms = [O.from_values(s, run_opt) for s in _realdata(ds)]
    ref = _values(O.wide("or", bms))
    assert ref.size == KNOWN[ds]["wide_or"]
    for op in ["priorityqueue_or", "horizontal_or", "parallel_or", "buffer_or_mutable"]:
        assert np.array_equal(_values(O.wide(op, bms)), ref), op
    xref = _values(O.wide("xor", bms))
    for op in ["priorityqueue_xor", "horizontal_xor", "parallel_xor"]:
        assert np.array_equal(_values(O.wide(op, bms)), xref), op


def test_chain_variants_agree_where_the_reference_says_so():
    """Internal consistency of the restatement: ParallelAggregation.or below 16 containers per
    key is the lazyIOR chain of BufferFastAggregation.or(Mutable...) (both clone the first and
    repair at the end, RB/ParallelAggregation.java:200-206, RB/buffer/BufferFastAggregation.java:
    810-817); at 16 and more it is FastAggregation.or's type rule."""
    import _gen
    rng = np.random.default_rng(5)
    keys = np.sort(rng.choice(3000, 30, replace=False))
    for n in (2, 5, 15):
        bms = [_gen.bitmap(rng, keys, p_present=0.9) for _ in range(n)]
        assert O.wide("parallel_or", bms) == O.wide("buffer_or_mutable", bms)
    bms = [_gen.bitmap(rng, keys, p_present=1.0) for _ in range(16)]
    assert O.wide("parallel_or", bms) == O.wide("or", bms)


def _rr_inputs(extra_arrays=False):
    """Two run-container bitmaps whose run ANDs give one-value runs: keys 1 (1,000 runs of one value,
    toEfficientContainer -> array), 2 (16,384 runs of one value -> bitmap, and more than 2,047 runs)
    and 3 (a few long runs, which stay runs either way)."""
    a = [(1, R, np.sort(np.concatenate([np.arange(0, 4000, 4), np.arange(1, 4000, 4)]))),
         (2, R, np.sort(np.concatenate([np.arange(0, 65536, 4), np.arange(1, 65536, 4)]))),
         (3, R, np.arange(100, 30000))]
    b = [(1, R, np.sort(np.concatenate([np.arange(1, 4000, 4), np.arange(2, 4000, 4)]))),
         (2, R, np.sort(np.concatenate([np.arange(1, 65536, 4), np.arange(2, 65536, 4)]))),
         (3, R, np.arange(20000, 50000))]
    if extra_arrays:
        a.append((4, A, np.arange(0, 4000, 3)))
        b.append((4, A, np.arange(0, 4000, 2)))
    return encode(a), encode(b)


def test_buffer_and_chain_keeps_merged_runs():
    """BufferFastAggregation's and chains run MutableRoaringBitmap.and in place
    (RB/buffer/MutableRoaringBitmap.java:886-910); MappeableRunContainer.iand(R) = and(R)
    (RB/buffer/MappeableRunContainer.java:1106-1108, :474-536) keeps the merged run container,
    where the heap's RunContainer.and(R) ends in toEfficientContainer (RB/RunContainer.java:381-456).
    Same sets, other bytes."""
    a, b = _rr_inputs(extra_arrays=True)
    for heap_op, buf_op, ids in (("naive_and", "buffer_naive_and", [0, 1]), ("and", "buffer_and", [0, 1]),
                                 ("and_iter", "buffer_and_iter", None)):
        heap, buf = O.wide(heap_op, [a, b], ids), O.wide(buf_op, [a, b], ids)
        assert heap != buf, buf_op
        assert java_equals(heap, buf)  # RunContainer.equals compares sets: the reference's tests pass either way
        dh, db = decode(heap), decode(buf)
        assert [c[:3] for c in dh] == [(1, A, 1000), (2, B, 16384), (3, R, 10000), (4, A, 667)]
        assert [c[:3] for c in db] == [(1, R, 1000), (2, R, 16384), (3, R, 10000), (4, A, 667)]
    # the static ImmutableRoaringBitmap.and (RB/buffer/ImmutableRoaringBitmap.java:299-325) types alike
    assert O.pairwise("and_buf", a, b) == O.wide("buffer_naive_and", [a, b], [0, 1])
    # above 10 inputs and(Immutable...) is workShyAnd, which types as the heap's
    many = [a, b] + [a] * 9
    assert O.wide("buffer_and", many, list(range(11))) == O.wide("workshy_and", many)


def test_buffer_and_chain_without_run_pairs_is_heap():
    """Without a run AND run step the buffer chain's types are the heap chain's."""
    rng = np.random.default_rng(5)
    from _gen import bitmap
    bufs = [bitmap(rng, np.arange(6), modes=["a_small", "b_dense", "b_mid"], p_present=1.0) for _ in range(4)]
    assert O.wide("buffer_naive_and", bufs, [0, 1, 2, 3]) == O.wide("naive_and", bufs, [0, 1, 2, 3])
    assert O.wide("buffer_and_iter", bufs) == O.wide("and_iter", bufs)
