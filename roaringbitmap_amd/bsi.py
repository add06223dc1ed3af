"""Host-side mirror of the bit-sliced indexes' query path.

Mirrors bsi/src/main/java/org/roaringbitmap/bsi/RoaringBitmapSliceIndex.java (BSI/):
compare(Operation, startOrValue, end, foundSet) (BSI/:482-513) and
sum(foundSet) (BSI/:581-592), and the buffer package's ImmutableBitSliceIndex /
MutableBitSliceIndex (bsi/src/main/java/org/roaringbitmap/bsi/buffer/BitSliceIndexBase.java,
BBSI/): compare (BBSI/:422-453), rangeEQ / rangeNEQ / rangeLT / rangeLE / rangeGT / rangeGE /
range (BBSI/:351-408) and sum (BBSI/:521-532).  Every query runs on the MI355X
(csrc/bsi.hip) and the results are the reference's bytes, container types included.
Construction (setValue) is host-side.
"""
import ctypes

import numpy as np

from . import _lib
from ._lib import IllegalArgumentException, check, lib, take
from .roaring import RoaringBitmap, run_optimize_many

OPERATIONS = ("EQ", "NEQ", "LE", "LT", "GE", "GT", "RANGE")  # BitmapSliceIndex.Operation order


class RoaringBitmapSliceIndex:
    """ebM (existence bitmap), bA (slices, bit 0 first), minValue, maxValue (BSI/:16-38)."""

    def __init__(self, ebm=None, slices=(), min_value=0, max_value=0):
        self.ebM = ebm if ebm is not None else RoaringBitmap()
        self.bA = list(slices)
        self.minValue = int(min_value)
        self.maxValue = int(max_value)
        self.runOptimized = False

    @classmethod
    def from_columns(cls, columns, values, run_optimize=False):
        """setValue(c, v) for each pair, in order (BSI/:320-347); runOptimize() if asked (BSI/:141-150)."""
        columns = np.asarray(columns, dtype=np.int64)
        values = np.asarray(values, dtype=np.int64)
        if columns.shape != values.shape:
            raise IllegalArgumentException("columns and values differ in length")
        if (values < 0).any():
            raise IllegalArgumentException("Values should be non-negative")
        mn = mx = 0
        if values.size:  # ensureCapacityInternal: first value sets both, then min or else max
            mn = mx = int(values[0])
            for v in values[1:]:
                v = int(v)
                if mn > v:
                    mn = v
                elif mx < v:
                    mx = v
        nbits = (len(bin(mx)) - 2) if values.size else 0
        ebm = RoaringBitmap.from_values(columns, run_optimize)
        ba = [RoaringBitmap.from_values(columns[(values >> i) & 1 == 1], run_optimize) for i in range(nbits)]
        obj = cls(ebm, ba, mn, mx)
        obj.runOptimized = bool(run_optimize)
        return obj

    def merge(self, otherBsi):
        """BSI/:379-405 ("designed for distributed computing"; the two indexes hold disjoint
        columns): slice-wise RoaringBitmap.or, runOptimize when either side was run-optimized
        (one device pass over all slices), the existence bitmaps united in place (x1.or(x2),
        Container.ior types) and min / max widened.  The buffer MutableBitSliceIndex.merge is the
        same steps over MutableRoaringBitmap (bsi/.../buffer/MutableBitSliceIndex.java:270-298)."""
        if otherBsi is None or otherBsi.ebM.isEmpty():
            return
        if RoaringBitmap.intersects(self.ebM, otherBsi.ebM):
            raise IllegalArgumentException("merge can be used only in bsiA  bsiB  is null")
        depth = max(self.bitCount(), otherBsi.bitCount())
        new = []
        for i in range(depth):
            cur = self.bA[i] if i < len(self.bA) else RoaringBitmap()
            other = otherBsi.bA[i] if i < len(otherBsi.bA) else RoaringBitmap()
            new.append(RoaringBitmap.or_(cur, other))
        if self.runOptimized or otherBsi.runOptimized:
            run_optimize_many(new)
        self.bA = new
        self.ebM.or_(otherBsi.ebM)  # in place
        self.runOptimized = self.runOptimized or otherBsi.runOptimized
        self.maxValue = max(self.maxValue, otherBsi.maxValue)
        self.minValue = min(self.minValue, otherBsi.minValue)

    def getValue(self, columnId):
        """BSI/:181-196 getValue(columnId) -> (value, exists): ebM.contains, then one contains per slice
        (RoaringBitmap.contains on the serialized bitmaps, on the host)"""
        if not self.ebM.contains(columnId):
            return 0, False
        v = 0
        for i, b in enumerate(self.bA):
            if b.contains(columnId):
                v |= 1 << i
        return v, True

    def runOptimize(self):
        """BSI/:141-150: runOptimize of ebM and of every slice (one device pass over all of them)."""
        run_optimize_many([self.ebM] + self.bA)
        self.runOptimized = True

    def bitCount(self):
        return len(self.bA)

    def getExistenceBitmap(self):
        return self.ebM

    def getLongCardinality(self):
        return self.ebM.getLongCardinality()

    def _slices(self):
        bufs = [b.serialize() for b in self.bA]
        return _lib.buf_array(bufs)

    def compare(self, operation, startOrValue, end=0, foundSet=None):
        """BSI/:482-513 -> RoaringBitmap"""
        op = OPERATIONS.index(operation) if isinstance(operation, str) else int(operation)
        arr, lens = self._slices()
        e = self.ebM.serialize()
        f = foundSet.serialize() if foundSet is not None else None
        out = _lib.rbg_buffer()
        check(lib().rbg_bsi_compare(op, int(startOrValue), int(end), e, len(e), arr, lens, len(self.bA),
                                    self.minValue, self.maxValue, f, len(f) if f else 0, ctypes.byref(out)))
        return RoaringBitmap(take(out))

    def sum(self, foundSet):
        """BSI/:581-592 -> (sum, count) as Java longs"""
        arr, lens = self._slices()
        e = self.ebM.serialize()
        f = foundSet.serialize() if foundSet is not None else None
        out = (ctypes.c_int64 * 2)()
        check(lib().rbg_bsi_sum(e, len(e), arr, lens, len(self.bA), f, len(f) if f else 0, out))
        return int(out[0]), int(out[1])


class BitSliceIndexBase(RoaringBitmapSliceIndex):
    """The buffer package's index (BBSI/): the same fields, its own compare circuit
    (owenGreatEqual for GE and RANGE's lower bound, rangeEQ from and(ebM, foundSet), rangeNEQ
    against ebM) and ImmutableRoaringBitmap's result types (csrc/bsi.hip, k_bsi_buf)."""

    RANGE_NEQ_DIRECT = 7  # RBG_BSI_RANGE_NEQ_DIRECT

    def _compare(self, op, start, end, foundSet):
        arr, lens = self._slices()
        e = self.ebM.serialize()
        f = foundSet.serialize() if foundSet is not None else None
        out = _lib.rbg_buffer()
        check(lib().rbg_bsi_compare_buffer(op, int(start), int(end), e, len(e), arr, lens, len(self.bA),
                                           self.minValue, self.maxValue, f, len(f) if f else 0, ctypes.byref(out)))
        return RoaringBitmap(take(out))

    def compare(self, operation, startOrValue, end=0, foundSet=None):
        """BBSI/:422-453 -> ImmutableRoaringBitmap (as RoaringBitmap bytes)"""
        op = OPERATIONS.index(operation) if isinstance(operation, str) else int(operation)
        return self._compare(op, startOrValue, end, foundSet)

    def rangeEQ(self, foundSet, predicate):  # BBSI/:351-375 (== compare(EQ))
        return self._compare(0, predicate, 0, foundSet)

    def rangeNEQ(self, foundSet, predicate):  # BBSI/:384-387
        return self._compare(self.RANGE_NEQ_DIRECT, predicate, 0, foundSet)

    def rangeLT(self, foundSet, predicate):  # BBSI/:389-391
        return self.compare("LT", predicate, 0, foundSet)

    def rangeLE(self, foundSet, predicate):  # BBSI/:393-395
        return self.compare("LE", predicate, 0, foundSet)

    def rangeGT(self, foundSet, predicate):  # BBSI/:397-399
        return self.compare("GT", predicate, 0, foundSet)

    def rangeGE(self, foundSet, predicate):  # BBSI/:401-403
        return self.compare("GE", predicate, 0, foundSet)

    def range(self, foundSet, start, end):  # BBSI/:405-408
        return self.compare("RANGE", start, end, foundSet)

    def sum(self, foundSet):
        """BBSI/:521-532 (the heap index's sum, BSI/:581-592); None or empty -> (0, 0)"""
        if foundSet is None or foundSet.isEmpty():
            return 0, 0
        return RoaringBitmapSliceIndex.sum(self, foundSet)


ImmutableBitSliceIndex = BitSliceIndexBase
MutableBitSliceIndex = BitSliceIndexBase
