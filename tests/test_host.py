"""Host-side checks that need no GPU: the C-ABI library loads and exports every
entry point include/roaring_mi355x.h declares, the host format helpers match the
oracle byte for byte, error behaviour mirrors the reference's, and compute calls
fail loudly (no CPU fallback) when no gfx950 device is present.
"""
import ctypes
import os
import re

import numpy as np
import pytest

from roaringbitmap_amd import _lib as L
from roaringbitmap_amd import RoaringBitmap, FastAggregation
from roaringbitmap_amd._lib import DeviceError, InvalidRoaringFormat, TruncatedInput, IllegalArgumentException

import _oracle as O
from _gen import MODES, container


def bitmap_values(rng, mode, n_keys):
    """Values of a bitmap whose n_keys containers all come from generator mode `mode`."""
    keys = np.sort(rng.choice(65536, size=n_keys, replace=False)).astype(np.uint32)
    return np.concatenate([(k << 16) | container(rng, mode)[1].astype(np.uint32) for k in keys])

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "roaring_mi355x.h")
TESTDATA = os.path.join(ROOT, "tests", "golden", "testdata")


def _declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    src = re.sub(r"//[^\n]*", "", src)
    return sorted(set(re.findall(r"\b(rbg_\w+)\s*\(", src)))


def test_header_declares_entry_points():
    names = _declared()
    assert "rbg_pairwise" in names and "rbg_wide" in names and "rbg_ctx_fetch_shard" in names
    assert len(names) >= 30


def test_library_exports_every_declared_symbol():
    lib = ctypes.CDLL(L.LIB_PATH)
    missing = [n for n in _declared() if not hasattr(lib, n)]
    assert not missing, missing


def test_python_binding_covers_header():
    assert sorted(L.EXPORTED) == sorted(n for n in _declared() if n in L.EXPORTED)
    assert set(_declared()) <= set(L.EXPORTED)


def test_version():
    assert L.lib().rbg_version() >= 1


@pytest.mark.parametrize("mode", MODES)
@pytest.mark.parametrize("run_opt", [False, True])
def test_from_values_matches_oracle(mode, run_opt):
    rng = np.random.default_rng(hash(mode) & 0xFFFF)
    vals = bitmap_values(rng, mode, n_keys=4)
    got = RoaringBitmap.from_values(vals, run_optimize=run_opt).serialize()
    assert got == O.from_values(vals, run_optimize=run_opt)


@pytest.mark.parametrize("mode", MODES)
def test_run_optimize_and_to_values(mode):
    # construction with runOptimize (bitmapOf + runOptimize on the host); the
    # RoaringBitmap.runOptimize() op itself runs on the GPU (test_gpu_runopt.py)
    rng = np.random.default_rng(7 + (hash(mode) & 0xFF))
    vals = bitmap_values(rng, mode, n_keys=3)
    rb = RoaringBitmap.from_values(vals)
    rb2 = RoaringBitmap.from_values(vals, run_optimize=True)
    assert rb2.serialize() == O.run_optimize(rb.serialize())
    assert np.array_equal(rb2.toArray(), np.unique(np.asarray(vals, dtype=np.uint32)))
    assert rb2.getLongCardinality() == len(np.unique(vals))


@pytest.mark.parametrize("name", ["bitmapwithruns.bin", "bitmapwithoutruns.bin"])
def test_deserialize_reference_files(name):
    data = open(os.path.join(TESTDATA, name), "rb").read()
    rb = RoaringBitmap.deserialize(data)
    st = O.stats(data)
    assert rb.getLongCardinality() == st["card"]
    assert np.array_equal(rb.toArray(), O.to_values(data))


@pytest.mark.parametrize("i", range(1, 9))
def test_crashprone_inputs_raise_like_reference(i):
    """TestAdversarialInputs.java:50-54: deserialize of the crashprone inputs must
    throw an IOException (both our errors are OSError) and never crash.  The
    engine also rejects non-increasing keys (which Java leaves unchecked), so
    the exact subclass may differ from the oracle's first failure."""
    data = open(os.path.join(TESTDATA, f"crashproneinput{i}.bin"), "rb").read()
    st, _, _ = O.roundtrip(data)
    assert st != 0
    with pytest.raises(OSError):
        RoaringBitmap.deserialize(data)


def test_truncated_and_bad_cookie():
    data = RoaringBitmap.bitmapOf(1, 2, 3, 70000).serialize()
    with pytest.raises(TruncatedInput):
        RoaringBitmap.deserialize(data[:-1])
    with pytest.raises(InvalidRoaringFormat):
        RoaringBitmap.deserialize(b"\x00\x00\x00\x00" + data[4:])


def test_java_int_cardinality_wraps():
    rb = RoaringBitmap.from_values(np.arange(0, 1 << 31, 1 << 10, dtype=np.uint32))
    assert rb.getLongCardinality() == 1 << 21
    assert rb.getCardinality() == 1 << 21


def _have_gpu():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.mark.skipif(_have_gpu(), reason="checks the no-device failure mode")
def test_compute_fails_loudly_without_device():
    a = RoaringBitmap.bitmapOf(1, 2, 3)
    b = RoaringBitmap.bitmapOf(2, 3, 4)
    with pytest.raises(DeviceError):
        RoaringBitmap.and_(a, b)
    with pytest.raises(DeviceError):
        RoaringBitmap.andCardinality(a, b)
    with pytest.raises(DeviceError):
        FastAggregation.or_(a, b)
    with pytest.raises(DeviceError):  # RoaringBitmap.runOptimize runs the device pass
        a.runOptimize()


def test_illegal_argument_type():
    assert issubclass(IllegalArgumentException, ValueError)
    with pytest.raises(IllegalArgumentException):
        L.check(L.RBG_ERR_ILLEGAL_ARGUMENT)


@pytest.mark.parametrize("n_keys", [1, 3, 4, 9])
@pytest.mark.parametrize("run_opt", [False, True])
def test_contains_reads_serialized_bytes(n_keys, run_opt):
    """RoaringBitmap.contains (RB/RoaringBitmap.java:1693-1701) on the serialized bytes: every
    container kind, run bitmaps below 4 containers (no offset table) and above, members and
    non-members, against the value list."""
    rng = np.random.default_rng(n_keys * 2 + run_opt)
    vals = np.concatenate([bitmap_values(rng, m, n_keys) for m in ("a_small", "b_dense", "r_few")])
    vals = np.unique(vals.astype(np.uint32))
    rb = RoaringBitmap.from_values(vals, run_optimize=run_opt)
    members = set(vals.tolist())
    probes = np.concatenate([rng.choice(vals, 300), rng.integers(0, 1 << 32, 300, dtype=np.uint64),
                             vals[:50] + 1, vals[-50:] - 1]).astype(np.uint32)
    for x in probes.tolist():
        assert rb.contains(x) == (x in members), x
    assert not RoaringBitmap().contains(5)


def test_bsi_get_value_uses_contains():
    """BSI getValue (bsi/.../RoaringBitmapSliceIndex.java:181-196): ebM.contains, then valueAt."""
    from roaringbitmap_amd import RoaringBitmapSliceIndex
    rng = np.random.default_rng(3)
    cols = np.unique(rng.integers(0, 1 << 20, 5000))
    vals = rng.integers(0, 1 << 12, cols.size)
    bsi = RoaringBitmapSliceIndex.from_columns(cols, vals, run_optimize=True)
    for c, v in list(zip(cols.tolist(), vals.tolist()))[:200]:
        assert bsi.getValue(c) == (v, True)
    assert bsi.getValue(int(cols.max()) + 1) == (0, False)


def test_inplace_same_object_needs_no_device():
    """x1.and(x1) / x1.or(x1) return at once and x1.xor(x1) / x1.andNot(x1) clear it
    (RB/RoaringBitmap.java:1273, 2482, 3297-3300, 1347-1350): no device call, so this runs without a
    GPU.  The C ABI hands x1's own bytes back (validated; trailing bytes past the bitmap dropped)."""
    from _fmt import R, encode
    x = encode([(k, R, np.arange(10 * k, 10 * k + 500)) for k in range(5)])  # run bitmap, offset table
    rb = RoaringBitmap(x)
    rb.and_(rb)
    assert rb.serialize() == x
    rb.or_(rb)
    assert rb.serialize() == x
    for op in (0, 1):
        out = L.rbg_buffer()
        L.check(L.lib().rbg_pairwise_inplace(op, x + b"tail", len(x) + 4, x, len(x), 1, ctypes.byref(out)))
        assert L.take(out) == x
    for op in (2, 3):
        out = L.rbg_buffer()
        L.check(L.lib().rbg_pairwise_inplace(op, x, len(x), x, len(x), 1, ctypes.byref(out)))
        assert L.take(out) == bytes.fromhex("3a30000000000000")
    with pytest.raises(InvalidRoaringFormat):
        out = L.rbg_buffer()
        L.check(L.lib().rbg_pairwise_inplace(0, b"\x00" * 12, 12, x, len(x), 1, ctypes.byref(out)))
    L.lib().rbg_trim()
    assert L.lib().rbg_pool_evictions() == 0


def test_work_and_memory_shy_and_buffer_check():
    """FastAggregation.workAndMemoryShyAnd checks the buffer before anything (RB/FastAggregation.java:523-525)."""
    x = RoaringBitmap.bitmapOf(1, 2, 3)
    with pytest.raises(IllegalArgumentException):
        FastAggregation.workAndMemoryShyAnd(np.zeros(100, dtype=np.int64), x, x)


def test_work_and_memory_shy_and_key_bitset():
    """workAndMemoryShyAnd's key-bitset steps on the caller's buffer, which end before any container work
    (RB/FastAggregation.java:527-548; RB/Util.java:531-555): an empty first bitmap returns at once with the
    buffer untouched; an empty later bitmap leaves word 0 and zeroes the rest; one input with a dirty bit
    outside its keys overruns the key array (ArrayIndexOutOfBoundsException)."""
    from roaringbitmap_amd._lib import ArrayIndexOutOfBoundsException
    x = RoaringBitmap.bitmapOf(1, 2, 3 << 16)
    buf = np.full(1024, 7, dtype=np.int64)
    assert FastAggregation.workAndMemoryShyAnd(buf, RoaringBitmap.bitmapOf(), x).isEmpty()
    assert (buf == 7).all()
    buf = np.zeros(1024, dtype=np.int64)
    buf[5] = 3
    assert FastAggregation.workAndMemoryShyAnd(buf, x, RoaringBitmap.bitmapOf()).isEmpty()
    assert buf[0] == 0b1001 and (buf[1:] == 0).all()
    buf = np.zeros(1024, dtype=np.int64)
    buf[1] = 1
    with pytest.raises(ArrayIndexOutOfBoundsException):
        FastAggregation.workAndMemoryShyAnd(buf, x)
    with pytest.raises(IllegalArgumentException):  # not a long[]
        FastAggregation.workAndMemoryShyAnd(np.zeros(1024, dtype=np.int32), x, x)


def test_pairwise_op_codes_match_header():
    """_lib.OP (the Python mirror's rbg_pairwise codes) equals the header's enum, including the buffer
    package's and / andNot (RBG_AND_BUFFER / RBG_ANDNOT_BUFFER)."""
    src = open(HEADER).read()
    names = {"and": "RBG_AND", "or": "RBG_OR", "xor": "RBG_XOR", "andnot": "RBG_ANDNOT", "ior": "RBG_OR_INPLACE",
             "and_buffer": "RBG_AND_BUFFER", "andnot_buffer": "RBG_ANDNOT_BUFFER"}
    for k, c in names.items():
        m = re.search(r"\b" + c + r"\s*=\s*(\d+)", src)
        assert m and int(m.group(1)) == L.OP[k], k
    for k, c in {"and_buffer": "RBG_RANGE_BUFFER_AND", "or_buffer": "RBG_RANGE_BUFFER_OR",
                 "xor_buffer": "RBG_RANGE_BUFFER_XOR", "andnot_buffer": "RBG_RANGE_BUFFER_ANDNOT",
                 "and": "RBG_RANGE_AND", "andnot": "RBG_RANGE_ANDNOT"}.items():  # rbg_range_op
        m = re.search(r"\b" + c + r"\s*=\s*(\d+)", src)
        assert m and int(m.group(1)) == L.RANGE_OP[k], k
    for k, c in {"add": "RBG_RMUT_ADD", "remove": "RBG_RMUT_REMOVE", "flip": "RBG_RMUT_FLIP"}.items():
        m = re.search(r"\b" + c + r"\s*=\s*(\d+)", src)
        assert m and int(m.group(1)) == L.RMUT_OP[k], k
    for c in ("RBG_ORNOT_INPLACE", "RBG_ORNOT_BUFFER", "RBG_RMUT_BUFFER"):  # rbg_ornot's / rbg_range_mut's flags
        m = re.search(r"\b" + c + r"\s*=\s*(\d+)", src)
        assert m and int(m.group(1)) == getattr(L, c), c


def test_ornot_self_and_arguments_need_no_device():
    """x1.orNot(x1, end) is the reference's UnsupportedOperationException (RB/RoaringBitmap.java:1432-1434,
    RB/buffer/MutableRoaringBitmap.java:963-965), raised before any device call; ImmutableRoaringBitmap
    has the static form only."""
    from roaringbitmap_amd import ImmutableRoaringBitmap, MutableRoaringBitmap, RoaringBitmap
    buf = O.from_values(np.arange(10))
    for cls in (RoaringBitmap, MutableRoaringBitmap):
        x = cls(buf)
        with pytest.raises(NotImplementedError):
            x.orNot(x, 5)
    with pytest.raises(TypeError):
        ImmutableRoaringBitmap.orNot(ImmutableRoaringBitmap(buf), 5)


def test_mutable_same_object_needs_no_device():
    """MutableRoaringBitmap x1.and(x1) leaves x1, x1.andNot(x1) clears it
    (RB/buffer/MutableRoaringBitmap.java:887, 919-922): answered on the host."""
    from roaringbitmap_amd import MutableRoaringBitmap
    buf = O.from_values(np.arange(0, 100000, 3))
    x = MutableRoaringBitmap(buf)
    getattr(x, "and")(x)
    assert x.serialize() == buf
    x.andNot(x)
    assert x.isEmpty() and x.serialize() == bytes.fromhex("3a30000000000000")
    with pytest.raises(NotImplementedError):
        x.or_(x)


def test_in_place_range_forms_dispatch():
    """x.add(start, end) in place maps to RBG_RMUT_ADD_INPLACE; single-value forms are refused"""
    import roaringbitmap_amd as rb
    import roaringbitmap_amd._lib as L
    assert L.RMUT_OP["add_inplace"] == 3
    with pytest.raises(NotImplementedError):
        rb.RoaringBitmap().add(5)


def test_contains_subset_op_code():
    import roaringbitmap_amd._lib as L
    assert L.CARD_OP["contains"] == 5
