"""ctypes binding of libroaring_mi355x.so (include/roaring_mi355x.h).

The library is built in-tree (roaringbitmap_amd/_build.py).  There is no CPU
fallback: if the shared object is missing this module raises at import time,
and every compute call returns RBG_ERR_DEVICE when no gfx950 device is present.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("RBG_LIB") or os.path.join(HERE, "lib", "libroaring_mi355x.so")

RBG_OK = 0
RBG_ERR_INVALID_FORMAT = -1
RBG_ERR_TRUNCATED = -2
RBG_ERR_ILLEGAL_ARGUMENT = -3
RBG_ERR_DEVICE = -4
RBG_ERR_OUT_OF_MEMORY = -5

OP = {"and": 0, "or": 1, "xor": 2, "andnot": 3, "ior": 4,  # ior: x1.or(x2) in place (Container.ior types)
      "and_buffer": 5, "andnot_buffer": 6}  # the buffer package's and / andNot (ImmutableRoaringBitmap)
CARD_OP = {"and": 0, "or": 1, "xor": 2, "andnot": 3, "intersects": 4, "contains": 5}
WIDE_OP = {"and": 0, "or": 1, "xor": 2, "and_iter": 3, "naive_and": 4, "workshy_and": 5, "parallel_or": 6,
           "parallel_xor": 7, "buffer_or_mutable": 8, "horizontal_or": 9, "horizontal_xor": 10,
           "priorityqueue_or": 11, "priorityqueue_xor": 12, "buffer_and": 13, "buffer_naive_and": 14,
           "buffer_and_iter": 15}
WIDE_CARD_OP = {"and": 0, "or": 1}
RANGE_OP = {"and": 0, "or": 1, "xor": 2, "andnot": 3,
            "and_buffer": 4, "or_buffer": 5, "xor_buffer": 6, "andnot_buffer": 7}  # ImmutableRoaringBitmap's
RBG_ORNOT_INPLACE, RBG_ORNOT_BUFFER = 1, 2
RMUT_OP = {"add": 0, "remove": 1, "flip": 2, "add_inplace": 3}  # rbg_range_mut (| RBG_RMUT_BUFFER: MutableRoaringBitmap's)
RBG_RMUT_BUFFER = 4


class rbg_buffer(ctypes.Structure):
    _fields_ = [("data", ctypes.POINTER(ctypes.c_uint8)), ("len", ctypes.c_size_t)]


EXPORTED = [
    "rbg_pairwise", "rbg_pairwise_card", "rbg_wide", "rbg_wide_card", "rbg_range_op", "rbg_ctx_select_range", "rbg_batch_and_card", "rbg_free",
    "rbg_set_devices", "rbg_last_error", "rbg_version", "rbg_trim", "rbg_pool_evictions", "rbg_from_values", "rbg_run_optimize",
    "rbg_to_values", "rbg_inspect", "rbg_ctx_create", "rbg_ctx_destroy", "rbg_ctx_stream", "rbg_ctx_sync",
    "rbg_ctx_load", "rbg_ctx_synth", "rbg_ctx_release", "rbg_ctx_batch_stats", "rbg_ctx_batch_fetch",
    "rbg_ctx_pairwise", "rbg_ctx_pairwise_serialized", "rbg_ctx_pairwise_range", "rbg_ctx_pairwise_card", "rbg_ctx_wide", "rbg_ctx_wide_card",
    "rbg_ctx_batch_and_card", "rbg_ctx_card", "rbg_ctx_cards", "rbg_ctx_result_stats", "rbg_ctx_fetch",
    "rbg_ctx_fetch_shard", "rbg_ctx_profile", "rbg_ctx_profile_compute", "rbg_ctx_profile_read", "rbg_ctx_profile_bytes", "rbg_ctx_serialize", "rbg_ctx_wide_start",
    "rbg_ctx_batch_counts", "rbg_synth_key_bytes", "rbg_ctx_pair_bytes", "rbg_debug_stamps",
    "rbg_bsi_compare", "rbg_bsi_sum", "rbg_ctx_bsi", "rbg_ctx_bsi_sums", "rbg_ctx_bsi_sums_device", "rbg_ctx_bsi_sums_target", "rbg_ctx_batch_minmax",
    "rbg_ctx_run_optimize", "rbg_run_optimize_many", "rbg_ctx_batch_fetch_range",
    "rbg_ctx_fetch_shard_device", "rbg_bsi_compare_buffer", "rbg_ctx_bsi_buffer",
    "rbg_ctx_result_layout_device", "rbg_ctx_fetch_shard_device_dyn", "rbg_pairwise_inplace",
    "rbg_ctx_load_separate", "rbg_ctx_load_packed", "rbg_ornot", "rbg_ctx_ornot", "rbg_range_mut", "rbg_ctx_range_mut", "rbg_add_offset", "rbg_ctx_add_offset", "rbg_select_range", "rbg_remove_run_compression", "rbg_limit", "rbg_bitmap_of_range",
]

_lib = None


def _declare(L):
    P = ctypes.POINTER
    u8p = ctypes.c_char_p
    sz = ctypes.c_size_t
    buf = P(rbg_buffer)
    i32 = ctypes.c_int32
    vp = ctypes.c_void_p
    L.rbg_pairwise.argtypes = [ctypes.c_int, u8p, sz, u8p, sz, buf]
    L.rbg_trim.argtypes = []
    L.rbg_trim.restype = None
    L.rbg_pool_evictions.argtypes = []
    L.rbg_pool_evictions.restype = ctypes.c_uint64
    L.rbg_pairwise_card.argtypes = [ctypes.c_int, u8p, sz, u8p, sz, P(i32)]
    L.rbg_pairwise_inplace.argtypes = [ctypes.c_int, u8p, sz, u8p, sz, ctypes.c_int, buf]
    L.rbg_wide.argtypes = [ctypes.c_int, P(ctypes.c_char_p), P(sz), P(i32), sz, buf]
    L.rbg_wide_card.argtypes = [ctypes.c_int, P(ctypes.c_char_p), P(sz), sz, P(i32)]
    L.rbg_range_op.argtypes = [ctypes.c_int, P(ctypes.c_char_p), P(sz), sz, ctypes.c_int64, ctypes.c_int64, buf]
    L.rbg_ornot.argtypes = [u8p, sz, u8p, sz, ctypes.c_int64, ctypes.c_int, buf]
    L.rbg_ctx_ornot.argtypes = [vp, i32, sz, i32, sz, ctypes.c_int64, ctypes.c_int]
    L.rbg_range_mut.argtypes = [ctypes.c_int, u8p, sz, ctypes.c_int64, ctypes.c_int64, buf]
    L.rbg_ctx_range_mut.argtypes = [vp, ctypes.c_int, i32, sz, ctypes.c_int64, ctypes.c_int64]
    L.rbg_add_offset.argtypes = [u8p, sz, ctypes.c_int64, buf]
    L.rbg_remove_run_compression.argtypes = [u8p, sz, buf]
    L.rbg_limit.argtypes = [u8p, sz, ctypes.c_int32, buf]
    L.rbg_bitmap_of_range.argtypes = [ctypes.c_int64, ctypes.c_int64, buf]
    L.rbg_select_range.argtypes = [u8p, sz, ctypes.c_int64, ctypes.c_int64, ctypes.c_int, buf]
    L.rbg_ctx_add_offset.argtypes = [vp, i32, sz, ctypes.c_int64]
    L.rbg_ctx_select_range.argtypes = [vp, i32, ctypes.c_int64, ctypes.c_int64, P(i32)]
    L.rbg_batch_and_card.argtypes = [sz, P(ctypes.c_char_p), P(sz), P(ctypes.c_char_p), P(sz), P(i32)]
    L.rbg_free.argtypes = [buf]
    L.rbg_free.restype = None
    L.rbg_set_devices.argtypes = [ctypes.c_uint64]
    L.rbg_last_error.restype = ctypes.c_char_p
    L.rbg_from_values.argtypes = [P(ctypes.c_uint32), sz, ctypes.c_int, buf]
    L.rbg_run_optimize.argtypes = [u8p, sz, buf]
    L.rbg_to_values.argtypes = [u8p, sz, buf]
    L.rbg_inspect.argtypes = [u8p, sz, P(sz), P(ctypes.c_int64), P(ctypes.c_int64)]
    L.rbg_ctx_create.argtypes = [ctypes.c_int, P(vp)]
    L.rbg_ctx_destroy.argtypes = [vp]
    L.rbg_ctx_destroy.restype = None
    L.rbg_ctx_stream.argtypes = [vp]
    L.rbg_ctx_stream.restype = vp
    L.rbg_ctx_sync.argtypes = [vp]
    L.rbg_ctx_load.argtypes = [vp, P(ctypes.c_char_p), P(sz), sz, P(i32)]
    L.rbg_ctx_load_separate.argtypes = [vp, P(ctypes.c_char_p), P(sz), sz, P(i32)]
    L.rbg_ctx_load_packed.argtypes = [vp, P(ctypes.c_char_p), P(sz), sz, P(i32)]
    L.rbg_ctx_synth.argtypes = [vp, ctypes.c_int, ctypes.c_uint64, sz, ctypes.c_int, ctypes.c_int, P(i32)]
    L.rbg_ctx_release.argtypes = [vp, i32]
    L.rbg_ctx_batch_stats.argtypes = [vp, i32, P(ctypes.c_int64)]
    L.rbg_ctx_batch_fetch.argtypes = [vp, i32, sz, buf]
    L.rbg_ctx_batch_fetch_range.argtypes = [vp, i32, sz, sz, vp]
    L.rbg_ctx_pairwise.argtypes = [vp, ctypes.c_int, i32, sz, i32, sz]
    L.rbg_ctx_pairwise_serialized.argtypes = [vp, ctypes.c_int, i32, sz, i32, sz]
    L.rbg_ctx_pairwise_range.argtypes = [vp, ctypes.c_int, i32, sz, i32, sz, ctypes.c_int, ctypes.c_int]
    L.rbg_ctx_pairwise_card.argtypes = [vp, ctypes.c_int, i32, sz, i32, sz]
    L.rbg_ctx_wide.argtypes = [vp, ctypes.c_int, i32, ctypes.c_int, ctypes.c_int, P(i32)]
    L.rbg_ctx_wide_card.argtypes = [vp, ctypes.c_int, i32, ctypes.c_int, ctypes.c_int]
    L.rbg_ctx_wide_start.argtypes = [vp, ctypes.c_int, i32, ctypes.c_int, ctypes.c_int, P(i32), i32]
    L.rbg_ctx_batch_counts.argtypes = [vp, i32, P(ctypes.c_uint32), sz]
    L.rbg_bsi_compare.argtypes = [ctypes.c_int, i32, i32, u8p, sz, P(ctypes.c_char_p), P(sz), sz, i32, i32, u8p, sz,
                                  buf]
    L.rbg_bsi_compare_buffer.argtypes = L.rbg_bsi_compare.argtypes
    L.rbg_ctx_bsi_buffer.argtypes = [vp, i32, ctypes.c_int, ctypes.c_int, ctypes.c_int, i32, i32, i32, i32]
    L.rbg_bsi_sum.argtypes = [u8p, sz, P(ctypes.c_char_p), P(sz), sz, u8p, sz, P(ctypes.c_int64)]
    L.rbg_ctx_bsi.argtypes = [vp, i32, ctypes.c_int, ctypes.c_int, ctypes.c_int, i32, i32, i32, i32, ctypes.c_int]
    L.rbg_ctx_bsi_sums.argtypes = [vp, P(ctypes.c_int64)]
    L.rbg_ctx_bsi_sums_device.argtypes = [vp, vp]
    L.rbg_ctx_bsi_sums_target.argtypes = [vp, vp]
    L.rbg_ctx_batch_minmax.argtypes = [vp, i32, P(i32)]
    L.rbg_ctx_run_optimize.argtypes = [vp, i32, P(i32), P(ctypes.c_uint8)]
    L.rbg_run_optimize_many.argtypes = [vp, P(sz), sz, vp, P(ctypes.c_uint8)]
    L.rbg_debug_stamps.argtypes = [P(ctypes.c_uint64), ctypes.c_int]
    L.rbg_ctx_pair_bytes.argtypes = [vp, i32, P(ctypes.c_int64)]
    L.rbg_synth_key_bytes.argtypes = [ctypes.c_int, ctypes.c_uint64, sz, P(ctypes.c_uint64)]
    L.rbg_ctx_batch_and_card.argtypes = [vp, i32]
    L.rbg_ctx_serialize.argtypes = [vp]
    L.rbg_ctx_card.argtypes = [vp, P(i32)]
    L.rbg_ctx_cards.argtypes = [vp, P(i32), sz]
    L.rbg_ctx_result_stats.argtypes = [vp, P(ctypes.c_int64)]
    L.rbg_ctx_fetch.argtypes = [vp, buf]
    L.rbg_ctx_profile.argtypes = [vp, ctypes.c_int]
    L.rbg_ctx_profile_compute.argtypes = [vp, ctypes.c_int]
    L.rbg_ctx_profile_read.argtypes = [vp, P(ctypes.c_double), P(ctypes.c_int)]
    L.rbg_ctx_profile_bytes.argtypes = [vp, P(ctypes.c_int64)]
    L.rbg_ctx_fetch_shard_device.argtypes = [vp, ctypes.c_int64, ctypes.c_int, ctypes.c_int64, vp, vp, vp, vp]
    L.rbg_ctx_result_layout_device.argtypes = [vp, vp]
    L.rbg_ctx_fetch_shard_device_dyn.argtypes = [vp, vp, ctypes.c_int, ctypes.c_int, vp, vp]
    L.rbg_ctx_fetch_shard.argtypes = [vp, ctypes.c_int64, ctypes.c_int, ctypes.c_int64, ctypes.c_int64, buf, buf,
                                      buf]


def lib():
    """Load the engine library; raises if it has not been built (no fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(
                f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
                "(the engine has no CPU fallback)")
        L = ctypes.CDLL(LIB_PATH)
        _declare(L)
        _lib = L
    return _lib


class RoaringError(Exception):
    pass


class InvalidRoaringFormat(RoaringError, OSError):
    """RB/InvalidRoaringFormat.java surfaced as IOException (RB/RoaringBitmap.java:1779-1811)."""


class TruncatedInput(RoaringError, OSError):
    """EOFException / BufferUnderflowException on a truncated buffer."""


class IllegalArgumentException(RoaringError, ValueError):
    pass


class ArrayIndexOutOfBoundsException(RoaringError, IndexError):
    """java.lang.ArrayIndexOutOfBoundsException, where the reference's own control flow throws it on
    caller-supplied input (FastAggregation.workAndMemoryShyAnd with a dirty buffer, RB/FastAggregation.java:541-548)"""


class DeviceError(RoaringError, RuntimeError):
    pass


def check(status):
    if status >= 0:
        return status
    msg = lib().rbg_last_error().decode(errors="replace")
    cls = {RBG_ERR_INVALID_FORMAT: InvalidRoaringFormat, RBG_ERR_TRUNCATED: TruncatedInput,
           RBG_ERR_ILLEGAL_ARGUMENT: IllegalArgumentException}.get(status, DeviceError)
    raise cls(f"status {status}: {msg}")


def take(b: rbg_buffer) -> bytes:
    out = ctypes.string_at(b.data, b.len) if b.len else b""
    lib().rbg_free(ctypes.byref(b))
    return out


def buf_array(bufs):
    n = len(bufs)
    arr = (ctypes.c_char_p * max(n, 1))(*bufs)
    lens = (ctypes.c_size_t * max(n, 1))(*[len(b) for b in bufs])
    return arr, lens
