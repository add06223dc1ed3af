"""CPU ORACLE of the bit-sliced index query path (test infrastructure only).

Restates bsi/src/main/java/org/roaringbitmap/bsi/RoaringBitmapSliceIndex.java
(BSI/ below) on top of the container-exact oracle's pairwise ops (tests/_oracle.py),
so every intermediate and final bitmap has the reference's container types:
  compareUsingMinMax  BSI/:515-579     oNeilCompare  BSI/:432-468
  compare             BSI/:482-513     sum           BSI/:581-592
  construction        setValue / ensureCapacityInternal BSI/:320-347 (bitmapOf-typed slices)
Bitmaps are portable serialized bytes.
"""
import numpy as np

import _oracle as O

EMPTY = bytes.fromhex("3a30000000000000")
OPS = ("EQ", "NEQ", "LE", "LT", "GE", "GT", "RANGE")


class BSI:
    """ebM, bA (slice 0 = least significant bit), minValue, maxValue."""

    def __init__(self, ebm, slices, min_value, max_value, run_optimized=False):
        self.ebm, self.ba, self.min, self.max = ebm, list(slices), int(min_value), int(max_value)
        self.run_optimized = bool(run_optimized)

    @classmethod
    def from_columns(cls, columns, values, run_optimize=False):
        """setValue(c, v) for every (c, v): slices are set-equal to the bits of the values
        and typed like bitmapOf (only adds, BSI/:320-331); min/max as ensureCapacityInternal
        (BSI/:333-347, values set in the given order)."""
        columns = np.asarray(columns, dtype=np.int64)
        values = np.asarray(values, dtype=np.int64)
        if (values < 0).any():
            raise ValueError("Values should be non-negative")
        mn = mx = 0
        for i, v in enumerate(values):
            v = int(v)
            if i == 0:
                mn = mx = v
            elif mn > v:
                mn = v
            elif mx < v:
                mx = v
        nbits = len(bin(mx)) - 2 if len(values) else 0
        ebm = O.from_values(columns, run_optimize)
        ba = [O.from_values(columns[(values >> i) & 1 == 1], run_optimize) for i in range(nbits)]
        return cls(ebm, ba, mn, mx, run_optimize)

    # BSI/:379-405 (the buffer MutableBitSliceIndex.merge, BBSI mutable :270-298, is the same steps over
    # MutableRoaringBitmap.or (static types as the heap's), runOptimize and the in-place ebM.or)
    def merge(self, other):
        if other is None or O.stats(other.ebm)["card"] == 0:
            return
        if O.pairwise_card("intersects", self.ebm, other.ebm):
            raise ValueError("merge can be used only in bsiA  bsiB  is null")
        depth = max(self.bit_count(), other.bit_count())
        new = []
        for i in range(depth):
            cur = self.ba[i] if i < len(self.ba) else EMPTY
            oth = other.ba[i] if i < len(other.ba) else EMPTY
            x = O.pairwise("or", cur, oth)  # RoaringBitmap.or(current, other)
            if self.run_optimized or other.run_optimized:
                x = O.run_optimize(x)
            new.append(x)
        self.ba = new
        self.ebm = O.pairwise("ior", self.ebm, other.ebm)  # this.ebM.or(otherBsi.ebM), in place
        self.run_optimized = self.run_optimized or other.run_optimized
        self.max = max(self.max, other.max)
        self.min = min(self.min, other.min)

    def get_value(self, column):
        """BSI/ getValue: (value, exists)"""
        if column not in set(O.to_values(self.ebm).tolist()):
            return 0, False
        v = 0
        for i, b in enumerate(self.ba):
            if column in set(O.to_values(b).tolist()):
                v |= 1 << i
        return v, True

    def bit_count(self):
        return len(self.ba)

    # BSI/:432-468
    def _oneil(self, op, predicate, found):
        fixed = self.ebm if found is None else found
        gt, lt, eq = EMPTY, EMPTY, self.ebm
        for i in range(self.bit_count() - 1, -1, -1):
            if (predicate >> i) & 1:
                lt = O.pairwise("or", lt, O.pairwise("andnot", eq, self.ba[i]))
                eq = O.pairwise("and", eq, self.ba[i])
            else:
                gt = O.pairwise("or", gt, O.pairwise("and", eq, self.ba[i]))
                eq = O.pairwise("andnot", eq, self.ba[i])
        eq = O.pairwise("and", fixed, eq)
        if op == "EQ":
            return eq
        if op == "NEQ":
            return O.pairwise("andnot", fixed, eq)
        if op == "GT":
            return O.pairwise("and", gt, fixed)
        if op == "LT":
            return O.pairwise("and", lt, fixed)
        if op == "LE":
            return O.pairwise("or", lt, eq)
        if op == "GE":
            return O.pairwise("or", gt, eq)
        raise ValueError(op)

    # BSI/:515-579 -> bytes, or None to run the circuit
    def _minmax(self, op, start, end, found):
        all_ = self.ebm if found is None else O.pairwise("and", self.ebm, found)
        lo, hi = self.min, self.max
        if op == "LT":
            return all_ if start > hi else EMPTY if start <= lo else None
        if op == "LE":
            return all_ if start >= hi else EMPTY if start < lo else None
        if op == "GT":
            return all_ if start < lo else EMPTY if start >= hi else None
        if op == "GE":
            return all_ if start <= lo else EMPTY if start > hi else None
        if op == "EQ":
            if lo == hi and lo == start:
                return all_
            return EMPTY if (start < lo or start > hi) else None
        if op == "NEQ":
            if lo == hi:
                return EMPTY if lo == start else all_
            return None
        if op == "RANGE":
            if start <= lo and end >= hi:
                return all_
            return EMPTY if (start > hi or end < lo) else None
        return None

    # BSI/:482-513
    def compare(self, op, start, end=0, found=None):
        r = self._minmax(op, start, end, found)
        if r is not None:
            return r
        if op == "RANGE":
            left = self._oneil("GE", start, found)
            right = self._oneil("LE", end, found)
            return O.pairwise("and", left, right)
        return self._oneil(op, start, found)

    # BSI/:581-592 -> (sum, count) as Java longs
    def sum(self, found):
        if found is None or O.stats(found)["card"] == 0:
            return 0, 0
        count = O.stats(found)["card"]
        s = 0
        for x in range(self.bit_count()):
            shift = np.int64(np.int32(np.uint32(1) << np.uint32(x)))  # (long) (1 << x), Java int shift
            s += int(shift) * O.pairwise_card("and", self.ba[x], found)
        return int(np.int64(np.uint64(s % (1 << 64)))), count


def _i32(x):
    return int(np.int64(x).astype(np.int32))


class BufferBSI(BSI):
    """The buffer package's bit-sliced index, ImmutableBitSliceIndex / MutableBitSliceIndex:
    bsi/src/main/java/org/roaringbitmap/bsi/buffer/BitSliceIndexBase.java (BBSI/ below).

    Its compare dispatches differently from the heap one (BBSI/:422-453):
      EQ    rangeEQ (BBSI/:351-375): the chain starts from and(ebM, foundSet), not from ebM
      NEQ   rangeNEQ (BBSI/:384-387): andNot(ebM, rangeEQ(...)) -- ebM, not the found set
      GE    owenGreatEqual (BBSI/:243-275): BufferFastAggregation.horizontal_or over spine ANDs
      GT/LT/LE  oNeilCompare (BBSI/:190-234), tracking only the needed GT / LT
      RANGE and(owenGreatEqual(start), oNeilCompare(LE, end)) (BBSI/:444-449)
    and every pairwise step is ImmutableRoaringBitmap's (O "and_buf" / "andnot_buf": a run AND /
    ANDNOT run keeps the merged run container, RB/buffer/MappeableRunContainer.java:474-536,600-663).
    horizontal_or over ImmutableRoaringBitmaps (RB/buffer/BufferFastAggregation.java:187-235) is the
    heap FastAggregation.horizontal_or loop (RB/FastAggregation.java:183-231) over the same container
    pointers (compareTo: RB/buffer/ImmutableRoaringArray.java:242-247 = RB/RoaringArray.java:708-713),
    lazyOR / lazyIOR dispatch (RB/buffer/MappeableContainer.java:639-696 = RB/Container.java:717-774)
    and repairAfterLazy, so O.wide("horizontal_or") gives its bytes.  sum is BBSI/:521-532 = BSI/:581-592.
    """

    def _and(self, a, b):
        return O.pairwise("and_buf", a, b)

    def _andnot(self, a, b):
        return O.pairwise("andnot_buf", a, b)

    # BBSI/:455-519 (all = ebM.clone() or ImmutableRoaringBitmap.and(ebM, foundSet))
    def _minmax(self, op, start, end, found):
        if found is None:
            return BSI._minmax(self, op, start, end, None)
        r = BSI._minmax(self, op, start, end, None)
        if r is self.ebm:
            return self._and(self.ebm, found)
        return r

    # BBSI/:190-234
    def _oneil_buf(self, op, predicate, found):
        fixed = self.ebm if found is None else found
        gt = EMPTY if op in ("GT", "GE") else None
        lt = EMPTY if op in ("LT", "LE") else None
        eq = self.ebm
        for i in range(self.bit_count() - 1, -1, -1):
            if (predicate >> i) & 1:
                if lt is not None:
                    lt = O.pairwise("or", lt, self._andnot(eq, self.ba[i]))
                eq = self._and(eq, self.ba[i])
            else:
                if gt is not None:
                    gt = O.pairwise("or", gt, self._and(eq, self.ba[i]))
                eq = self._andnot(eq, self.ba[i])
        if op not in ("LT", "GT"):
            eq = self._and(fixed, eq)
        if op == "EQ":
            return eq
        if op == "GT":
            return self._and(gt, fixed)
        if op == "LT":
            return self._and(lt, fixed)
        if op == "LE":
            return O.pairwise("or", lt, eq)
        if op == "GE":
            return O.pairwise("or", gt, eq)
        raise ValueError(op)

    def owen_inputs(self, predicate):
        """owenGreatEqual's orInputs (BBSI/:245-264) as (kind, w) in order: "slice" = bA[w] itself,
        "and" = and(spine, bA[w]); Java int / long arithmetic of beGtrThan and leastSignifZero."""
        b = _i32(predicate - 1)
        nb = _i32(~b)
        lsz = 64 if nb == 0 else ((nb & 0xFFFFFFFF) & -(nb & 0xFFFFFFFF)).bit_length() - 1
        spine, out = False, []
        for w in range(self.bit_count() - 1, lsz - 1, -1):
            if (b & (1 << w)) == 0:
                out.append(("and" if spine else "slice", w))
            else:
                spine = True
        return out

    # BBSI/:243-275
    def _owen_ge(self, predicate, found):
        b = _i32(predicate - 1)
        nb = _i32(~b)
        lsz = 64 if nb == 0 else ((nb & 0xFFFFFFFF) & -(nb & 0xFFFFFFFF)).bit_length() - 1
        spine, inputs = None, []
        for w in range(self.bit_count() - 1, lsz - 1, -1):
            if (b & (1 << w)) == 0:
                inputs.append(self.ba[w] if spine is None else self._and(spine, self.ba[w]))
            else:
                spine = self.ba[w] if spine is None else self._and(spine, self.ba[w])
        res = O.wide("horizontal_or", inputs) if inputs else EMPTY
        return res if found is None else self._and(res, found)

    # BBSI/:351-375
    def range_eq(self, found, predicate):
        eq = self.ebm if found is None else self._and(self.ebm, found)
        r = self._minmax("EQ", predicate, 0, found)
        if r is not None:
            return r
        for i in range(self.bit_count() - 1, -1, -1):
            eq = self._and(eq, self.ba[i]) if (predicate >> i) & 1 else self._andnot(eq, self.ba[i])
        return eq

    # BBSI/:422-453
    def compare(self, op, start, end=0, found=None):
        r = self._minmax(op, start, end, found)
        if r is not None:
            return r
        if op == "EQ":
            return self.range_eq(found, start)
        if op == "NEQ":  # BBSI/:384-387
            return self._andnot(self.ebm, self.range_eq(found, start))
        if op == "GE":
            return self._owen_ge(start, found)
        if op == "RANGE":
            return self._and(self._owen_ge(start, found), self._oneil_buf("LE", end, found))
        return self._oneil_buf(op, start, found)
