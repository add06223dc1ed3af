"""Device-resident session API (rbg_ctx_*): one HIP stream + workspace per context.

Used by bench.py (HIP-event timing on `stream_ptr`) and by multi-GPU sharding
(`fetch_shard`).  All op calls enqueue asynchronously; `sync()` waits.
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import check, lib, take
from .roaring import RoaringBitmap

SYNTH_C2, SYNTH_C3_UNIFORM, SYNTH_C3_CLUSTERED, SYNTH_C4_PAIRS, SYNTH_C5_BSI = 0, 1, 2, 3, 4


def synth_key_bytes(kind, seed, n) -> np.ndarray:
    """Per-key algorithmic input bytes of a synthetic C3 workload (host, for key-range partitioning)."""
    out = np.zeros(65536, dtype=np.uint64)
    check(lib().rbg_synth_key_bytes(int(kind), int(seed), int(n),
                                    out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint64))))
    return out


class Engine:
    def __init__(self, device=0):
        self._ctx = ctypes.c_void_p()
        check(lib().rbg_ctx_create(int(device), ctypes.byref(self._ctx)))
        self.device = device
        self._bsi_target = None  # device tensor the BSI sum kernels write into (bsi_sums_target)

    def close(self):
        if self._ctx:
            lib().rbg_ctx_destroy(self._ctx)
            self._ctx = ctypes.c_void_p()
        self._bsi_target = None  # the BSI sums target is released with the context that wrote it

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def stream_ptr(self) -> int:
        return lib().rbg_ctx_stream(self._ctx)

    def sync(self):
        check(lib().rbg_ctx_sync(self._ctx))

    def profile(self, max_ops, compute_only=False):
        """Enable HIP-event phase timing for the next `max_ops` ops (0 disables); compute_only: two events
        per op around the container compute kernel (only compute_ms is read)."""
        f = lib().rbg_ctx_profile_compute if compute_only else lib().rbg_ctx_profile
        check(f(self._ctx, int(max_ops)))

    def profile_read(self):
        """-> (n_ops, [plan_ms, compute_ms, assemble_ms]) summed over the recorded ops."""
        ms = (ctypes.c_double * 3)()
        n = ctypes.c_int()
        check(lib().rbg_ctx_profile_read(self._ctx, ms, ctypes.byref(n)))
        return n.value, list(ms)

    def profile_bytes(self) -> int:
        """Bytes the early-exit wide AND (workShyAnd) read since profiling was enabled."""
        v = ctypes.c_int64()
        check(lib().rbg_ctx_profile_bytes(self._ctx, ctypes.byref(v)))
        return v.value

    # ---- batches ------------------------------------------------------------
    def load(self, bitmaps, packed=False) -> int:
        """Upload + device decode of serialized bitmaps as one key-major batch.  packed: for a batch
        that feeds wide ops -- a batch of arrays alone keeps the portable format's packed array
        payloads (rbg_ctx_load_packed), the wide kernels' fastest layout."""
        bufs = [b.serialize() if isinstance(b, RoaringBitmap) else bytes(b) for b in bitmaps]
        arr, lens = _lib.buf_array(bufs)
        out = ctypes.c_int32()
        f = lib().rbg_ctx_load_packed if packed else lib().rbg_ctx_load
        check(f(self._ctx, arr, lens, len(bufs), ctypes.byref(out)))
        return out.value

    def load_pair(self, *bitmaps):
        """Upload several serialized bitmaps at once, each decoded into a batch of its own
        (rbg_ctx_load_separate): the operands of pairwise ops.  -> list of batch ids."""
        bufs = [b.serialize() if isinstance(b, RoaringBitmap) else bytes(b) for b in bitmaps]
        arr, lens = _lib.buf_array(bufs)
        ids = (ctypes.c_int32 * max(len(bufs), 1))()
        check(lib().rbg_ctx_load_separate(self._ctx, arr, lens, len(bufs), ids))
        return list(ids)[:len(bufs)]

    def synth(self, kind, seed, n=0, key_lo=0, key_hi=65536) -> int:
        out = ctypes.c_int32()
        check(lib().rbg_ctx_synth(self._ctx, int(kind), int(seed), int(n), int(key_lo), int(key_hi),
                                  ctypes.byref(out)))
        return out.value

    def release(self, batch):
        check(lib().rbg_ctx_release(self._ctx, int(batch)))

    def batch_stats(self, batch) -> dict:
        s = (ctypes.c_int64 * 8)()
        check(lib().rbg_ctx_batch_stats(self._ctx, int(batch), s))
        keys = ["bitmaps", "containers", "array", "bitmap", "run", "payload_bytes", "cardinality", "serialized_bytes"]
        return dict(zip(keys, list(s)))

    def batch_fetch(self, batch, i=0) -> RoaringBitmap:
        b = _lib.rbg_buffer()
        check(lib().rbg_ctx_batch_fetch(self._ctx, int(batch), int(i), ctypes.byref(b)))
        return RoaringBitmap(take(b))

    def batch_fetch_range(self, batch, first=0, count=None) -> list:
        """Bitmaps [first, first + count) of a batch (default: all), one device gather + one copy."""
        if count is None:
            count = self.batch_stats(batch)["bitmaps"] - first
        outs = (_lib.rbg_buffer * max(count, 1))()
        check(lib().rbg_ctx_batch_fetch_range(self._ctx, int(batch), int(first), int(count), outs))
        return [RoaringBitmap(take(outs[k])) for k in range(count)]

    # ---- ops (asynchronous) -------------------------------------------------------
    def pairwise(self, op, a, b, ia=0, ib=0, key_lo=0, key_hi=65536):
        """A pairwise op; key_lo / key_hi restrict it to one key-range shard (shard.py assembles shards)."""
        if key_lo == 0 and key_hi == 65536:
            check(lib().rbg_ctx_pairwise(self._ctx, _lib.OP[op], int(a), int(ia), int(b), int(ib)))
        else:
            check(lib().rbg_ctx_pairwise_range(self._ctx, _lib.OP[op], int(a), int(ia), int(b), int(ib), int(key_lo),
                                               int(key_hi)))

    def ornot(self, a, b, range_end, inplace=False, buffer=False, ia=0, ib=0):
        """RoaringBitmap.orNot(x1, x2, rangeEnd) (inplace: x1.orNot(x2, rangeEnd); buffer: the buffer
        package's) of two resident bitmaps; the result pending like pairwise's (rbg_ctx_ornot)."""
        flags = (_lib.RBG_ORNOT_INPLACE if inplace else 0) | (_lib.RBG_ORNOT_BUFFER if buffer else 0)
        check(lib().rbg_ctx_ornot(self._ctx, int(a), int(ia), int(b), int(ib), int(range_end), flags))

    def range_mut(self, op, a, range_start, range_end, buffer=False, ia=0):
        """static RoaringBitmap.add / remove / flip(rb, start, end) ("add" / "remove" / "flip"; buffer:
        MutableRoaringBitmap's) of a resident bitmap; the result pending like pairwise's (rbg_ctx_range_mut)."""
        code = _lib.RMUT_OP[op] | (_lib.RBG_RMUT_BUFFER if buffer else 0)
        check(lib().rbg_ctx_range_mut(self._ctx, code, int(a), int(ia), int(range_start), int(range_end)))

    def add_offset(self, a, offset, ia=0):
        """RoaringBitmap.addOffset(x, offset) of a resident bitmap; the result pending like pairwise's
        (rbg_ctx_add_offset)."""
        check(lib().rbg_ctx_add_offset(self._ctx, int(a), int(ia), int(offset)))

    def pairwise_serialized(self, op, a, b, ia=0, ib=0):
        """pairwise(op) + serialize() as one pipeline (rbg_ctx_pairwise_serialized): the result's
        placement and payload copies for one key range overlap the next range's compute."""
        check(lib().rbg_ctx_pairwise_serialized(self._ctx, _lib.OP[op], int(a), int(ia), int(b), int(ib)))

    def and_cardinality(self, a, b, ia=0, ib=0):
        check(lib().rbg_ctx_pairwise_card(self._ctx, 0, int(a), int(ia), int(b), int(ib)))

    def wide(self, op, batch, key_lo=0, key_hi=65536, ids=None):
        idp = None
        if ids is not None:
            idp = (ctypes.c_int32 * len(ids))(*ids)
        check(lib().rbg_ctx_wide(self._ctx, _lib.WIDE_OP[op], int(batch), int(key_lo), int(key_hi), idp))

    def wide_start(self, op, batch, key_lo, key_hi, start_bm, ids=None):
        """wide op whose naive_and chain starts from input `start_bm` (key-range shards)."""
        idp = None
        if ids is not None:
            idp = (ctypes.c_int32 * len(ids))(*ids)
        check(lib().rbg_ctx_wide_start(self._ctx, _lib.WIDE_OP[op], int(batch), int(key_lo), int(key_hi), idp,
                                       int(start_bm)))

    def pair_bytes(self, batch):
        """(matched payload + descriptors, all payload + descriptors) of a batch of pairs (C4)."""
        out = (ctypes.c_int64 * 2)()
        check(lib().rbg_ctx_pair_bytes(self._ctx, int(batch), out))
        return int(out[0]), int(out[1])

    def run_optimize(self, batch, answers=True):
        """RoaringBitmap.runOptimize (RB/RoaringBitmap.java:2764-2774) of every bitmap of a batch, on the
        device -> (new batch id, [runOptimize's boolean per bitmap]).  The booleans need a read-back
        (synchronous); answers=False returns (id, None) with nothing read back: the new batch's
        statistics stay on the device until a host-side use needs them."""
        out = ctypes.c_int32()
        if not answers:
            check(lib().rbg_ctx_run_optimize(self._ctx, int(batch), ctypes.byref(out), None))
            return int(out.value), None
        n = self.batch_stats(batch)["bitmaps"]
        ans = (ctypes.c_uint8 * max(n, 1))()
        check(lib().rbg_ctx_run_optimize(self._ctx, int(batch), ctypes.byref(out), ans))
        return int(out.value), [bool(x) for x in ans[:n]]

    def select_range(self, batch, start, end):
        """selectRangeWithoutCopy (RB/RoaringBitmap.java:3160-3214) of every bitmap of a batch, on the device
        -> new batch id (rbg_ctx_select_range)."""
        out = ctypes.c_int32()
        check(lib().rbg_ctx_select_range(self._ctx, int(batch), int(start), int(end), ctypes.byref(out)))
        return int(out.value)

    def batch_minmax(self, batch):
        out = (ctypes.c_int32 * 2)()
        check(lib().rbg_ctx_batch_minmax(self._ctx, int(batch), out))
        return int(out[0]), int(out[1])

    def bsi(self, batch, op, nbits, start, end=0, min_value=0, max_value=0, has_found=False, want_sum=False):
        """RoaringBitmapSliceIndex.compare (op in BitmapSliceIndex.Operation order; 8 = sum alone) over a
        key-major batch [ebM, bA[0..nbits-1], foundSet?]; want_sum fuses sum(result)."""
        from .bsi import OPERATIONS
        code = OPERATIONS.index(op) if isinstance(op, str) else int(op)
        check(lib().rbg_ctx_bsi(self._ctx, int(batch), code, int(nbits), int(bool(has_found)), int(start), int(end),
                                int(min_value), int(max_value), int(bool(want_sum))))

    def bsi_buffer(self, batch, op, nbits, start, end=0, min_value=0, max_value=0, has_found=False):
        """The buffer package's BitSliceIndexBase.compare (bsi/.../bsi/buffer/BitSliceIndexBase.java:422-453;
        op 7 = rangeNEQ called directly) over a key-major batch [ebM, bA[0..nbits-1], foundSet?]."""
        from .bsi import OPERATIONS
        code = OPERATIONS.index(op) if isinstance(op, str) else int(op)
        check(lib().rbg_ctx_bsi_buffer(self._ctx, int(batch), code, int(nbits), int(bool(has_found)), int(start),
                                       int(end), int(min_value), int(max_value)))

    def bsi_sums(self):
        out = (ctypes.c_int64 * 2)()
        check(lib().rbg_ctx_bsi_sums(self._ctx, out))
        return int(out[0]), int(out[1])

    def bsi_sums_device(self, dst):
        """(sum, count) of the last BSI call into a device int64 tensor of two elements, enqueued on
        the engine stream (no host synchronisation)."""
        check(lib().rbg_ctx_bsi_sums_device(self._ctx, ctypes.c_void_p(dst.data_ptr())))

    def bsi_sums_target(self, dst):
        """From now on every BSI sum also writes its (sum, count) into the int64 device tensor `dst`
        (two elements) from the kernel that computes it; None stops it (rbg_ctx_bsi_sums_target).

        The engine keeps a reference to `dst` until it is replaced, cleared with None or the engine is
        closed, so the kernels never write into memory the caller's allocator has handed on."""
        if dst is not None:
            import torch
            if not isinstance(dst, torch.Tensor) or dst.dtype != torch.int64 or not dst.is_contiguous() \
                    or dst.numel() < 2 or dst.device.type != "cuda" or dst.device.index != self.device:
                raise ValueError("bsi_sums_target: a contiguous int64 CUDA tensor of at least 2 elements on "
                                 f"device {self.device} is required")
        check(lib().rbg_ctx_bsi_sums_target(self._ctx, None if dst is None else ctypes.c_void_p(dst.data_ptr())))
        self._bsi_target = dst

    def batch_counts(self, batch) -> np.ndarray:
        """containers per input bitmap of a batch"""
        n = self.batch_stats(batch)["bitmaps"]
        out = np.zeros(n, dtype=np.uint32)
        check(lib().rbg_ctx_batch_counts(self._ctx, int(batch), out.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)),
                                         n))
        return out

    def wide_card(self, op, batch, key_lo=0, key_hi=65536):
        check(lib().rbg_ctx_wide_card(self._ctx, _lib.WIDE_CARD_OP[op], int(batch), int(key_lo), int(key_hi)))

    def batch_and_card(self, batch):
        check(lib().rbg_ctx_batch_and_card(self._ctx, int(batch)))

    # ---- results (synchronous) -------------------------------------------------
    def card(self) -> int:
        out = ctypes.c_int32()
        check(lib().rbg_ctx_card(self._ctx, ctypes.byref(out)))
        return out.value

    def cards(self, n) -> np.ndarray:
        out = np.zeros(n, dtype=np.int32)
        check(lib().rbg_ctx_cards(self._ctx, out.ctypes.data_as(ctypes.POINTER(ctypes.c_int32)), n))
        return out

    def result_stats(self) -> dict:
        s = (ctypes.c_int64 * 4)()
        check(lib().rbg_ctx_result_stats(self._ctx, s))
        return {"containers": s[0], "payload_bytes": s[1], "has_run": s[2], "cardinality": s[3]}

    def serialize(self):
        """Enqueue the on-device portable serialization of the last result."""
        check(lib().rbg_ctx_serialize(self._ctx))

    def fetch(self) -> RoaringBitmap:
        b = _lib.rbg_buffer()
        check(lib().rbg_ctx_fetch(self._ctx, ctypes.byref(b)))
        return RoaringBitmap(take(b))

    def fetch_shard_device(self, total_containers, has_run, payload_base, desc, offsets, runflags, payload):
        """Enqueue the pending result as a key shard of a global bitmap, written straight into
        device memory (torch tensors or raw pointers; offsets / runflags may be None when the
        global layout has no offset table / no run container).  Asynchronous: sync() before use."""
        def ptr(t):
            if t is None:
                return None
            return int(t) if isinstance(t, int) else int(t.data_ptr())
        check(lib().rbg_ctx_fetch_shard_device(self._ctx, int(total_containers), int(bool(has_run)), int(payload_base),
                                               ptr(desc), ptr(offsets), ptr(runflags), ptr(payload)))

    def result_layout_device(self, dst3):
        """Enqueue (containers, payload bytes, has_run) of the pending result into a device int64
        tensor of 3 elements on the engine stream (the input of a device all-gather)."""
        check(lib().rbg_ctx_result_layout_device(self._ctx, ctypes.c_void_p(dst3.data_ptr())))

    def fetch_shard_device_dyn(self, layout, rank, world, out, runb=None):
        """Enqueue this rank's slice of the global bitmap, placed by a device-resident layout
        (world x 3 int64 tensor, key-range order), into `out` (a uint8 tensor laid out as the whole
        global bitmap) and one run byte per global container into runb.  No host synchronisation."""
        check(lib().rbg_ctx_fetch_shard_device_dyn(self._ctx, ctypes.c_void_p(layout.data_ptr()), int(rank),
                                                   int(world), ctypes.c_void_p(out.data_ptr()),
                                                   ctypes.c_void_p(runb.data_ptr()) if runb is not None else None))

    def fetch_shard(self, total_containers, has_run, first_container, payload_base):
        d, o, p = _lib.rbg_buffer(), _lib.rbg_buffer(), _lib.rbg_buffer()
        check(lib().rbg_ctx_fetch_shard(self._ctx, int(total_containers), int(has_run), int(first_container),
                                        int(payload_base), ctypes.byref(d), ctypes.byref(o), ctypes.byref(p)))
        return take(d), take(o), take(p)
