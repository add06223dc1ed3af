"""Pins the CPU oracle (oracle/rbcpu.cpp) to the reference's own fixtures.

No GPU.  Sources of truth (all committed under tests/golden/, see make_fixtures.py):
  * RBT/TestAdversarialInputs.java:32-55 - golden serialized files and crash inputs
  * jmh/src/test/java/org/roaringbitmap/realdata/*Test.java - known-answer constants
  * RBT/TestContainer.java:890-979, RBT/TestRunContainer.java:2635-2661 - type assertions
  * fuzz-tests/src/test/java/org/roaringbitmap/Fuzzer.java:252-365 - invariants
"""
import json
import os

import numpy as np
import pytest

import _oracle as O
from _fmt import A, B, R, decode, encode, kinds
import _gen

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def _read(name):
    with open(os.path.join(GOLD, "testdata", name), "rb") as f:
        return f.read()


@pytest.mark.parametrize("name,mix", [("bitmapwithruns.bin", (3, 5, 3)), ("bitmapwithoutruns.bin", (3, 8, 0))])
def test_golden_roundtrip_bytes(name, mix):
    buf = _read(name)
    st, out, used = O.roundtrip(buf)
    assert st == 0 and used == len(buf)
    assert out == buf  # deserialize -> serialize reproduces the reference bytes
    s = O.stats(buf)
    assert s["card"] == 200100  # TestAdversarialInputs.java:37,45
    assert (s["array"], s["bitmap"], s["run"]) == mix


@pytest.mark.parametrize("i", range(1, 8))
def test_crashprone_inputs_rejected(i):
    st, _, _ = O.roundtrip(_read(f"crashproneinput{i}.bin"))
    assert st in (-1, -2)  # IOException: InvalidRoaringFormat (-1) or EOF (-2)


def _realdata(ds):
    z = np.load(os.path.join(GOLD, "realdata", ds + ".npz"))
    v, o = z["values"], z["offsets"]
    return [v[o[i]:o[i + 1]] for i in range(len(o) - 1)]


KNOWN = json.load(open(os.path.join(GOLD, "known_answers.json")))["values"]


@pytest.mark.parametrize("ds", sorted(KNOWN))
@pytest.mark.parametrize("run_opt", [False, True])
def test_realdata_known_answers(ds, run_opt):
    bms = [O.from_values(s, run_opt) for s in _realdata(ds)]
    exp = KNOWN[ds]
    for op in ["or", "and", "xor", "andnot"]:
        got = sum(O.stats(O.pairwise(op, bms[k], bms[k + 1]))["card"] for k in range(len(bms) - 1))
        assert got == exp[op], (ds, op)
    nocard = 0
    for k in range(len(bms) - 1):
        vals = O.to_values(O.pairwise("or", bms[k], bms[k + 1]))
        if vals.size:
            nocard += int(vals[0])
    assert np.int64(nocard).astype(np.int32) == exp["or_nocard"]
    assert O.stats(O.wide("or", bms))["card"] == exp["wide_or"]
    assert O.stats(O.wide("and_iter", bms))["card"] == exp["wide_and"]


def _one(kind, vals, key=0):
    return encode([(key, kind, np.asarray(vals, dtype=np.uint16))])


@pytest.mark.parametrize("vals,kind,expect", [
    ([1, 2, 3, 4, 5, 6, 7, 8, 9, 50000, 50001], A, R),          # testRunOptimize1
    ([1, 2, 3, 4, 6, 8, 9, 50000, 50003], A, A),                 # testRunOptimize1A
    (list(range(40000)), B, R),                                  # testRunOptimize2
    (list(range(0, 40000, 2)), B, B),                            # testRunOptimize2A
    ([1, 2, 3, 4, 5, 6, 7, 8, 9, 50000, 50001], R, R),          # testRunOptimize3
    ([1, 3, 5, 7, 9, 11, 17, 21, 50000, 50002], R, A),           # testRunOptimize3A
    (list(range(100, 30000, 2)), R, B),                          # testRunOptimize3B
])
def test_run_optimize_types(vals, kind, expect):
    assert kinds(O.run_optimize(_one(kind, vals))) == [expect]


@pytest.mark.parametrize("c1,c2", [
    ((R, range(0, 1 << 15)), (B, range(1 << 15, 1 << 16))),                   # orFullToRunContainer
    ((R, range((1 << 10) - 200, 1 << 16)), (A, range(0, 1 << 10))),           # orFullToRunContainer2
    ((R, range(0, 1 << 15)), (R, range((1 << 15) - 200, 1 << 16))),          # orFullToRunContainer3
])
def test_or_full_is_run(c1, c2):
    out = O.pairwise("or", _one(c1[0], list(c1[1])), _one(c2[0], list(c2[1])))
    d = decode(out)
    assert len(d) == 1 and d[0][1] == R and d[0][2] == 65536 and d[0][4] == 1


def test_transition_4096():
    # RBT/TestContainer.java transitionTest: 4096 values stay an array, 4097 become a bitmap
    assert kinds(O.from_values(np.arange(4096))) == [A]
    assert kinds(O.from_values(np.arange(4097))) == [B]


def _set(buf):
    return set(O.to_values(buf).tolist())


@pytest.mark.parametrize("seed", range(6))
def test_fuzz_invariants(seed):
    rng = np.random.default_rng(1000 + seed)
    keys = np.arange(12)
    l = _gen.bitmap(rng, keys)
    r = _gen.bitmap(rng, keys)
    sl, sr = _set(l), _set(r)
    a, o, x, n = (O.pairwise(op, l, r) for op in ["and", "or", "xor", "andnot"])
    assert _set(a) == sl & sr and _set(o) == sl | sr and _set(x) == sl ^ sr and _set(n) == sl - sr
    assert O.pairwise_card("and", l, r) == len(sl & sr)             # Fuzzer.java:252-257
    assert O.pairwise_card("or", l, r) == len(sl | sr)              # :259-264
    assert O.pairwise_card("xor", l, r) == len(sl ^ sr)             # :266-271
    assert O.pairwise_card("andnot", l, r) == len(sl - sr)
    assert O.pairwise_card("intersects", l, r) == int(bool(sl & sr))
    assert _set(O.pairwise("or", l, a)) == sl                       # :347-351
    # workShyAnd == naive_and (RBT/TestFastAggregation.java:245-281), set level
    bms = [_gen.bitmap(rng, keys, p_present=0.95) for _ in range(12)]
    inter = set.intersection(*[_set(b) for b in bms])
    assert _set(O.wide("workshy_and", bms)) == inter
    assert _set(O.wide("naive_and", bms)) == inter
    assert O.wide_card("and", bms) == len(inter)
    union = set.union(*[_set(b) for b in bms])
    assert O.wide_card("or", bms) == len(union)
    sx = set()
    for b in bms:
        sx ^= _set(b)
    assert _set(O.wide("xor", bms)) == sx


def test_java_int_wrap():
    full = encode([(k, R, np.arange(65536, dtype=np.uint16)) for k in range(32768)])
    # 2^31 values: the Java int cardinality wraps to -2^31
    assert O.pairwise_card("and", full, full) == -(1 << 31)
