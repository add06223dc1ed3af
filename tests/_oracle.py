"""ctypes binding to the CPU ORACLE (oracle/build/librbcpu.so) — test infrastructure.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this.
"""
import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(ROOT, "oracle", "build", "librbcpu.so")

_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "oracle")])
        L = ctypes.CDLL(LIB_PATH)
        u8p = ctypes.POINTER(ctypes.c_uint8)
        L.rbo_free.argtypes = [ctypes.c_void_p]
        L.rbo_pairwise.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p,
                                   ctypes.c_size_t, ctypes.POINTER(u8p),
                                   ctypes.POINTER(ctypes.c_size_t)]
        L.rbo_pairwise_card.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t,
                                        ctypes.c_char_p, ctypes.c_size_t,
                                        ctypes.POINTER(ctypes.c_int32)]
        L.rbo_wide.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_char_p),
                               ctypes.POINTER(ctypes.c_size_t), ctypes.c_size_t,
                               ctypes.POINTER(ctypes.c_int), ctypes.POINTER(u8p),
                               ctypes.POINTER(ctypes.c_size_t)]
        L.rbo_wide_card.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_char_p),
                                    ctypes.POINTER(ctypes.c_size_t), ctypes.c_size_t,
                                    ctypes.POINTER(ctypes.c_int32)]
        L.rbo_from_values.argtypes = [ctypes.POINTER(ctypes.c_uint32), ctypes.c_size_t, ctypes.c_int,
                                      ctypes.POINTER(u8p), ctypes.POINTER(ctypes.c_size_t)]
        L.rbo_run_optimize.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(u8p),
                                       ctypes.POINTER(ctypes.c_size_t)]
        L.rbo_to_values.argtypes = [ctypes.c_char_p, ctypes.c_size_t,
                                    ctypes.POINTER(ctypes.POINTER(ctypes.c_uint32)),
                                    ctypes.POINTER(ctypes.c_size_t)]
        L.rbo_roundtrip.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(u8p),
                                    ctypes.POINTER(ctypes.c_size_t),
                                    ctypes.POINTER(ctypes.c_size_t)]
        L.rbo_stats.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(ctypes.c_int64)]
        L.rbo_time_pairwise.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t,
                                        ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int]
        L.rbo_time_pairwise.restype = ctypes.c_double
        L.rbo_time_wide.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_char_p),
                                    ctypes.POINTER(ctypes.c_size_t), ctypes.c_size_t, ctypes.c_int]
        L.rbo_time_wide.restype = ctypes.c_double
        L.rbo_time_wide_parallel.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_char_p),
                                             ctypes.POINTER(ctypes.c_size_t), ctypes.c_size_t, ctypes.c_int,
                                             ctypes.c_int]
        L.rbo_time_wide_parallel.restype = ctypes.c_double
        L.rbo_time_and_parallel.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t,
                                            ctypes.c_int, ctypes.c_int]
        L.rbo_time_and_parallel.restype = ctypes.c_double
        L.rbo_time_pairs.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_size_t),
                                     ctypes.c_size_t, ctypes.c_int, ctypes.c_int]
        L.rbo_time_pairs.restype = ctypes.c_double
        L.rbo_time_bsi_range_sum.argtypes = [ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_size_t),
                                             ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int,
                                             ctypes.POINTER(ctypes.c_int64)]
        L.rbo_time_bsi_range_sum.restype = ctypes.c_double
        L.rbo_time_bsi_range_sum_parallel.argtypes = [ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_size_t),
                                                      ctypes.c_int, ctypes.c_uint32, ctypes.c_uint32, ctypes.c_int,
                                                      ctypes.c_int, ctypes.POINTER(ctypes.c_int64)]
        L.rbo_time_bsi_range_sum_parallel.restype = ctypes.c_double
        L.rbo_range_op.argtypes = [ctypes.c_int, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_size_t),
                                   ctypes.c_size_t, ctypes.c_int64, ctypes.c_int64,
                                   ctypes.POINTER(ctypes.POINTER(ctypes.c_uint8)), ctypes.POINTER(ctypes.c_size_t)]
        L.rbo_ornot.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int64,
                                ctypes.c_int, ctypes.POINTER(ctypes.c_int), ctypes.POINTER(u8p),
                                ctypes.POINTER(ctypes.c_size_t)]
        L.rbo_range_mut.argtypes = [ctypes.c_int, ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int64, ctypes.c_int64,
                                    ctypes.POINTER(u8p), ctypes.POINTER(ctypes.c_size_t)]
        L.rbo_add_offset.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int64, ctypes.POINTER(u8p),
                                     ctypes.POINTER(ctypes.c_size_t)]
        L.rbo_remove_run_compression.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.POINTER(u8p),
                                                 ctypes.POINTER(ctypes.c_size_t)]
        L.rbo_limit.argtypes = [ctypes.c_char_p, ctypes.c_size_t, ctypes.c_int32, ctypes.POINTER(u8p),
                                ctypes.POINTER(ctypes.c_size_t)]
        L.rbo_bitmap_of_range.argtypes = [ctypes.c_int64, ctypes.c_int64, ctypes.POINTER(u8p),
                                          ctypes.POINTER(ctypes.c_size_t)]
        L.rbo_long_size.argtypes = [ctypes.c_char_p, ctypes.c_size_t]
        L.rbo_long_size.restype = ctypes.c_int64
        _lib = L
    return _lib


class OracleError(Exception):
    def __init__(self, status):
        super().__init__(f"oracle status {status}")
        self.status = status


def _take(p, n):
    out = ctypes.string_at(p, n.value)
    lib().rbo_free(p)
    return out


def _check(st):
    if st != 0:
        raise OracleError(st)


OPS = {"and": 0, "or": 1, "xor": 2, "andnot": 3, "and_buf": 4, "andnot_buf": 5,  # *_buf: ImmutableRoaringBitmap ops
       "ior": 6}  # x1.or(x2) in place
CARD_OPS = {"and": 0, "or": 1, "xor": 2, "andnot": 3, "intersects": 4}
WIDE_OPS = {"and": 0, "or": 1, "xor": 2, "and_iter": 3, "naive_and": 4, "workshy_and": 5,
            "parallel_or": 6, "parallel_xor": 7, "buffer_or_mutable": 8, "horizontal_or": 9, "horizontal_xor": 10,
            "priorityqueue_or": 11, "priorityqueue_xor": 12, "buffer_and": 13, "buffer_naive_and": 14,
            "buffer_and_iter": 15}


def pairwise(op, a: bytes, b: bytes) -> bytes:
    p = ctypes.POINTER(ctypes.c_uint8)()
    n = ctypes.c_size_t()
    _check(lib().rbo_pairwise(OPS[op], a, len(a), b, len(b), ctypes.byref(p), ctypes.byref(n)))
    return _take(p, n)


def pairwise_card(op, a: bytes, b: bytes) -> int:
    out = ctypes.c_int32()
    _check(lib().rbo_pairwise_card(CARD_OPS[op], a, len(a), b, len(b), ctypes.byref(out)))
    return out.value


def _bufs(bufs):
    arr = (ctypes.c_char_p * max(len(bufs), 1))(*bufs)
    lens = (ctypes.c_size_t * max(len(bufs), 1))(*[len(b) for b in bufs])
    return arr, lens


def wide(op, bufs, ids=None) -> bytes:
    arr, lens = _bufs(bufs)
    idp = None
    if ids is not None:
        idp = (ctypes.c_int * len(ids))(*ids)
    p = ctypes.POINTER(ctypes.c_uint8)()
    n = ctypes.c_size_t()
    _check(lib().rbo_wide(WIDE_OPS[op], arr, lens, len(bufs), idp, ctypes.byref(p),
                          ctypes.byref(n)))
    return _take(p, n)


def wide_card(op, bufs) -> int:
    arr, lens = _bufs(bufs)
    out = ctypes.c_int32()
    _check(lib().rbo_wide_card({"and": 0, "or": 1}[op], arr, lens, len(bufs), ctypes.byref(out)))
    return out.value


def from_values(values, run_optimize=False) -> bytes:
    v = np.ascontiguousarray(np.asarray(values, dtype=np.uint32))
    p = ctypes.POINTER(ctypes.c_uint8)()
    n = ctypes.c_size_t()
    _check(lib().rbo_from_values(v.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), v.size,
                                 int(run_optimize), ctypes.byref(p), ctypes.byref(n)))
    return _take(p, n)


def run_optimize(buf: bytes) -> bytes:
    p = ctypes.POINTER(ctypes.c_uint8)()
    n = ctypes.c_size_t()
    _check(lib().rbo_run_optimize(buf, len(buf), ctypes.byref(p), ctypes.byref(n)))
    return _take(p, n)


def to_values(buf: bytes) -> np.ndarray:
    p = ctypes.POINTER(ctypes.c_uint32)()
    n = ctypes.c_size_t()
    _check(lib().rbo_to_values(buf, len(buf), ctypes.byref(p), ctypes.byref(n)))
    out = np.ctypeslib.as_array(p, shape=(n.value,)).copy() if n.value else np.zeros(0, np.uint32)
    lib().rbo_free(p)
    return out


def roundtrip(buf: bytes):
    """Returns (status, bytes, consumed)."""
    p = ctypes.POINTER(ctypes.c_uint8)()
    n = ctypes.c_size_t()
    used = ctypes.c_size_t()
    st = lib().rbo_roundtrip(buf, len(buf), ctypes.byref(p), ctypes.byref(n), ctypes.byref(used))
    if st != 0:
        return st, None, 0
    return 0, _take(p, n), used.value


def stats(buf: bytes):
    s = (ctypes.c_int64 * 5)()
    _check(lib().rbo_stats(buf, len(buf), s))
    return {"array": s[0], "bitmap": s[1], "run": s[2], "card": s[3], "payload": s[4]}


def time_pairwise(op, a, b, reps):
    code = {"and": 0, "or": 1, "xor": 2, "andnot": 3, "and_card": 4}[op]
    return lib().rbo_time_pairwise(code, a, len(a), b, len(b), reps)


def time_wide(op, bufs, reps):
    arr, lens = _bufs(bufs)
    return lib().rbo_time_wide({"and": 0, "or": 1, "xor": 2}[op], arr, lens, len(bufs), reps)


def time_wide_parallel(op, bufs, threads, reps):
    """ParallelAggregation.or / xor semantics, key groups over `threads` workers; seconds for reps runs."""
    arr, lens = _bufs(bufs)
    return lib().rbo_time_wide_parallel({"or": 0, "xor": 1}[op], arr, lens, len(bufs), threads, reps)


def time_and_parallel(a, b, threads, reps):
    """Key-parallel RoaringBitmap.and over `threads` key ranges; seconds for reps runs."""
    return lib().rbo_time_and_parallel(a, len(a), b, len(b), threads, reps)


def time_pairs(op, bufs, threads, reps):
    """Loop of RoaringBitmap.and(...).getCardinality() (op "and") or andCardinality (op "and_card")
    over the pairs (bufs[2i], bufs[2i+1]) on `threads` workers; seconds for reps passes."""
    arr, lens = _bufs(bufs)
    return lib().rbo_time_pairs({"and": 0, "and_card": 4}[op], arr, lens, len(bufs) // 2, threads, reps)


def time_bsi_range_sum(ebm, slices, lo, hi, reps):
    """RoaringBitmapSliceIndex.compare(RANGE, lo, hi, null) + sum on the heap BSI (one thread);
    -> (seconds for reps queries, (sum, count))."""
    arr, lens = _bufs([ebm] + list(slices))
    out = (ctypes.c_int64 * 2)()
    t = lib().rbo_time_bsi_range_sum(arr, lens, len(slices), lo, hi, reps, out)
    return t, (int(out[0]), int(out[1]))


def time_bsi_range_sum_parallel(ebm, slices, lo, hi, threads, reps):
    """The same query key-parallel over `threads` workers (per-key sums added before sum's int cast);
    -> (seconds for reps queries, (sum, count))."""
    arr, lens = _bufs([ebm] + list(slices))
    out = (ctypes.c_int64 * 2)()
    t = lib().rbo_time_bsi_range_sum_parallel(arr, lens, len(slices), lo, hi, threads, reps, out)
    return t, (int(out[0]), int(out[1]))


def range_op(op, bufs, start, end) -> bytes:
    """RoaringBitmap.and / or / xor(Iterator, start, end) ("and" / "or" / "xor") and andNot(x1, x2, start,
    end) ("andnot", two inputs): RB/RoaringBitmap.java:1308-1336, 2536-2557, 3359-3379, 1396-1423; "*_buf":
    ImmutableRoaringBitmap's (RB/buffer/ImmutableRoaringBitmap.java:261, 992, 1048, 402)."""
    arr, lens = _bufs(bufs)
    p = ctypes.POINTER(ctypes.c_uint8)()
    n = ctypes.c_size_t()
    _check(lib().rbo_range_op({"and": 0, "or": 1, "xor": 2, "andnot": 3, "select": 4, "and_buf": 5, "or_buf": 6,
                               "xor_buf": 7, "andnot_buf": 8, "select_buf": 9}[op], arr, lens, len(bufs), start, end,
                              ctypes.byref(p), ctypes.byref(n)))
    return _take(p, n)


class NegativeArraySize(OracleError):
    """The reference's orNot sizes its key array with a negative maxSize (NegativeArraySizeException)."""


def ornot(a, b, range_end, inplace=False, buffer=False) -> bytes:
    """RoaringBitmap.orNot(x1, x2, rangeEnd) (RB/RoaringBitmap.java:1521-1603) or, inplace, x1.orNot(x2,
    rangeEnd) (:1431-1506); buffer: ImmutableRoaringBitmap.orNot / MutableRoaringBitmap.orNot
    (RB/buffer/ImmutableRoaringBitmap.java:484-548, MutableRoaringBitmap.java:962-1030)."""
    p = ctypes.POINTER(ctypes.c_uint8)()
    n = ctypes.c_size_t()
    neg = ctypes.c_int()
    st = lib().rbo_ornot(a, len(a), b, len(b), range_end, int(inplace) | (2 if buffer else 0), ctypes.byref(neg), ctypes.byref(p),
                         ctypes.byref(n))
    if neg.value:
        raise NegativeArraySize(st)
    _check(st)
    return _take(p, n)


def range_mut(op, buf, start, end, buffer=False) -> bytes:
    """static RoaringBitmap.add / remove / flip(rb, start, end) ("add" / "remove" / "flip",
    RB/RoaringBitmap.java:298, 995, 626); buffer: MutableRoaringBitmap's."""
    p = ctypes.POINTER(ctypes.c_uint8)()
    n = ctypes.c_size_t()
    code = {"add": 0, "remove": 1, "flip": 2, "add_inplace": 3}[op] | (4 if buffer else 0)
    _check(lib().rbo_range_mut(code, buf, len(buf), start, end, ctypes.byref(p), ctypes.byref(n)))
    return _take(p, n)


def add_offset(buf, offset) -> bytes:
    """RoaringBitmap.addOffset(x, offset) (RB/RoaringBitmap.java:230-288; MutableRoaringBitmap's alike)."""
    p = ctypes.POINTER(ctypes.c_uint8)()
    n = ctypes.c_size_t()
    _check(lib().rbo_add_offset(buf, len(buf), int(offset), ctypes.byref(p), ctypes.byref(n)))
    return _take(p, n)


def remove_run_compression(buf) -> bytes:
    """x.removeRunCompression() (RB/RoaringBitmap.java:2738-2749), x's bytes afterwards."""
    p = ctypes.POINTER(ctypes.c_uint8)()
    n = ctypes.c_size_t()
    _check(lib().rbo_remove_run_compression(buf, len(buf), ctypes.byref(p), ctypes.byref(n)))
    return _take(p, n)


def limit(buf, maxcard) -> bytes:
    """x.limit(maxcardinality) (RB/RoaringBitmap.java:2457-2476)."""
    p = ctypes.POINTER(ctypes.c_uint8)()
    n = ctypes.c_size_t()
    _check(lib().rbo_limit(buf, len(buf), int(maxcard), ctypes.byref(p), ctypes.byref(n)))
    return _take(p, n)


def bitmap_of_range(lo, hi) -> bytes:
    """RoaringBitmap.bitmapOfRange(min, max) (RB/RoaringBitmap.java:588-615)."""
    p = ctypes.POINTER(ctypes.c_uint8)()
    n = ctypes.c_size_t()
    _check(lib().rbo_bitmap_of_range(int(lo), int(hi), ctypes.byref(p), ctypes.byref(n)))
    return _take(p, n)


def long_size(buf) -> int:
    """RoaringBitmap.getLongSizeInBytes (RB/RoaringBitmap.java:2212-2219)."""
    return int(lib().rbo_long_size(buf, len(buf)))
