"""Host-side mirror of the reference's static-op interface for the hot path.

Mirrors (RB/ = RoaringBitmap/src/main/java/org/roaringbitmap/):
  * RoaringBitmap static ops and/or/xor/andNot, and/or/xor/andNotCardinality,
    intersects, or(RoaringBitmap...)        RB/RoaringBitmap.java:377-473,698-720,844,860-1118
  * FastAggregation and/or/xor (+ Iterator and long[] buffer overloads),
    andCardinality/orCardinality, naive_and/naive_or/naive_xor, workShyAnd
                                            RB/FastAggregation.java:26-101,304-414,586-666,823-836
A RoaringBitmap here is an immutable value holding its portable serialized bytes
(RB/RoaringArray.java:896-940); every op runs on the MI355X through the C ABI of
include/roaring_mi355x.h and returns the bytes the reference would serialize.
Java names that are Python keywords are exposed with a trailing underscore and
also registered under the Java name (getattr(RoaringBitmap, "and")).
"""
import ctypes
import itertools
from collections.abc import Iterator

import numpy as np

from . import _lib
from ._lib import ArrayIndexOutOfBoundsException, IllegalArgumentException, check, lib, take

EMPTY = bytes.fromhex("3a30000000000000")


def _int32(x):
    return int(np.int64(x).astype(np.int32)) if -(1 << 63) <= x < (1 << 63) else int(x)


class _StaticOrInPlace:
    """Java overloads one name with a static op and an in-place instance op: RoaringBitmap.and(x1, x2)
    (RB/RoaringBitmap.java:377) and x1.and(x2) (:1272).  On the class this is the static form; on an
    instance with one argument it modifies the instance (with two, Java calls the static one)."""

    def __init__(self, static, op):
        self.static, self.op = static, op
        self.__doc__ = static.__doc__

    def __get__(self, obj, objtype=None):
        if obj is None:
            return self.static

        def call(*args):
            if len(args) != 1:
                return self.static(*args)
            obj._inplace(self.op, args[0])

        call.__doc__ = self.static.__doc__
        return call


def _range_op(op, bitmaps, start, end, cls=None):
    """RB/RoaringBitmap.java range-restricted forms: every input through selectRangeWithoutCopy
    (:3160-3214), then FastAggregation.and / or / xor(Iterator) or andNot (rbg_range_op); "*_buffer":
    ImmutableRoaringBitmap's (MutableRoaringBitmap results)."""
    bufs = [b._buf for b in bitmaps]
    arr, lens = _lib.buf_array(bufs)
    b = _lib.rbg_buffer()
    check(lib().rbg_range_op(_lib.RANGE_OP[op], arr, lens, len(bufs), int(start), int(end), ctypes.byref(b)))
    return (cls or RoaringBitmap)(take(b))


def _is_range(args):
    return len(args) == 3 and isinstance(args[0], Iterator) and all(isinstance(x, (int, np.integer)) for x in args[1:])


def _s_and(*args):
    """static and(x1, x2), RB/RoaringBitmap.java:377-401; and(Iterator, rangeStart, rangeEnd) :1308-1316;
    x1.and(x2) in place :1272-1296"""
    if _is_range(args):
        return _range_op("and", list(args[0]), args[1], args[2])
    x1, x2 = args
    return RoaringBitmap._pair("and", x1, x2)


def _s_or(*bitmaps):
    """static or(x1, x2) (:860-902); or(Iterator, rangeStart, rangeEnd) :2536-2543; any other arity is
    or(RoaringBitmap...) (:844) = FastAggregation.or; x1.or(x2) in place :2481-2523 (Container.ior's types)"""
    if _is_range(bitmaps):
        return _range_op("or", list(bitmaps[0]), bitmaps[1], bitmaps[2])
    if len(bitmaps) == 2:
        return RoaringBitmap._pair("or", bitmaps[0], bitmaps[1])
    return FastAggregation.or_(*bitmaps)


def _s_xor(*args):
    """static xor(x1, x2), :1071-1118; xor(Iterator, rangeStart, rangeEnd) :3359-3365; x1.xor(x2) in place
    :3296-3348"""
    if _is_range(args):
        return _range_op("xor", list(args[0]), args[1], args[2])
    x1, x2 = args
    return RoaringBitmap._pair("xor", x1, x2)


def _s_andnot(*args):
    """static andNot(x1, x2), :444-473; andNot(x1, x2, rangeStart, rangeEnd) :1396-1404; x1.andNot(x2) in
    place :1346-1382"""
    if len(args) == 4:
        return _range_op("andnot", [args[0], args[1]], args[2], args[3])
    x1, x2 = args
    return RoaringBitmap._pair("andnot", x1, x2)


class _OrNot:
    """RoaringBitmap.orNot(x1, x2, rangeEnd) (static, RB/RoaringBitmap.java:1521-1603) on the class or with
    three arguments; x1.orNot(x2, rangeEnd) in place (:1431-1506) on an instance with two.  buffer: the
    buffer package's (MutableRoaringBitmap.orNot, RB/buffer/MutableRoaringBitmap.java:962-1030)."""

    def __init__(self, static, buffer=False):
        self.static, self.buffer = static, buffer
        self.__doc__ = static.__doc__

    def __get__(self, obj, objtype=None):
        if obj is None:
            return self.static

        def call(*args):
            if len(args) == 3:
                return self.static(*args)
            other, range_end = args
            if other is obj:
                raise NotImplementedError("orNot between a bitmap and itself?")  # UnsupportedOperationException
            obj._buf = _ornot(obj, other, range_end, True, self.buffer)
            obj._lcard = None

        call.__doc__ = self.static.__doc__
        return call


def _ornot(x1, x2, range_end, inplace, buffer=False):
    b = _lib.rbg_buffer()
    flags = (_lib.RBG_ORNOT_INPLACE if inplace else 0) | (_lib.RBG_ORNOT_BUFFER if buffer else 0)
    check(lib().rbg_ornot(x1._buf, len(x1._buf), x2._buf, len(x2._buf), int(range_end), flags, ctypes.byref(b)))
    return take(b)


def _s_ornot(x1, x2, range_end):
    """static orNot(x1, x2, rangeEnd), RB/RoaringBitmap.java:1521-1603: per key up to (rangeEnd - 1) >>> 16,
    x1 | ~x2 within the range (Container.orNot, x2's complement alone, full containers where neither
    holds the key), then x1's keys above; x1.orNot(x2, rangeEnd) in place :1431-1506.  rangeEnd outside
    [0, 2^32] -> IllegalArgumentException.  x1 is not modified (the reference's static form updates x1's
    container at maxKey in place)."""
    return RoaringBitmap(_ornot(x1, x2, range_end, False))


class _RangeMut:
    """The static range mutations RoaringBitmap.add / remove / flip(rb, rangeStart, rangeEnd)
    (RB/RoaringBitmap.java:298-345, 995-1040, 626-668) on the class or with three arguments; buffer:
    MutableRoaringBitmap's (RB/buffer/MutableRoaringBitmap.java:152-205, 649-700, 455-505), results of
    class `cls`.  With two arguments on an instance of `cls`: x.add / remove / flip(rangeStart, rangeEnd) in
    place (RB/RoaringBitmap.java:1181-1206, 2656-2710, 1893-1925; RB/buffer/MutableRoaringBitmap.java
    :831-858, 1489, 1195): the in-place add runs Container.iadd on every key of the range (its own
    typing, RBG_RMUT_ADD_INPLACE), the in-place remove / flip end in the static forms' containers.  The
    single-value forms x.add(int) / remove(int) / flip(int) are not on this path."""

    def __init__(self, op, buffer=False, cls=None):
        self.op, self.buffer, self.cls = op, buffer, cls

    def _run(self, op, rb, range_start, range_end):
        b = _lib.rbg_buffer()
        code = _lib.RMUT_OP[op] | (_lib.RBG_RMUT_BUFFER if self.buffer else 0)
        check(lib().rbg_range_mut(code, rb._buf, len(rb._buf), int(range_start), int(range_end), ctypes.byref(b)))
        return take(b)

    def static(self, rb, range_start, range_end):
        return (self.cls or RoaringBitmap)(self._run(self.op, rb, range_start, range_end))

    def __get__(self, obj, objtype=None):
        if obj is None:
            return self.static

        def call(*args):
            if len(args) == 3:
                return self.static(*args)
            if len(args) == 2 and isinstance(obj, self.cls or RoaringBitmap):
                obj._buf = self._run("add_inplace" if self.op == "add" else self.op, obj, *args)
                obj._lcard = None
                return None
            raise NotImplementedError(f"{type(obj).__name__}.{self.op}{args}: the range forms "
                                      f"{self.op}(rb, rangeStart, rangeEnd) and x.{self.op}(rangeStart, rangeEnd)")
        return call


class RoaringBitmap:
    __slots__ = ("_buf", "_lcard")

    def __init__(self, serialized: bytes = None):
        self._buf = EMPTY if serialized is None else bytes(serialized)
        self._lcard = None

    # ---- construction -----------------------------------------------------
    @classmethod
    def bitmapOf(cls, *values):
        """RoaringBitmap.bitmapOf(int...) (RB/RoaringBitmap.java:566-570); ints taken as unsigned 32-bit."""
        if len(values) == 1 and not isinstance(values[0], (int, np.integer)):
            values = values[0]
        return cls.from_values(values)

    @classmethod
    def from_values(cls, values, run_optimize=False):
        v = np.ascontiguousarray(np.asarray(values, dtype=np.int64).astype(np.uint32))
        b = _lib.rbg_buffer()
        check(lib().rbg_from_values(v.ctypes.data_as(ctypes.POINTER(ctypes.c_uint32)), v.size, int(run_optimize),
                                    ctypes.byref(b)))
        return cls(take(b))

    @classmethod
    def deserialize(cls, data: bytes):
        """RoaringBitmap.deserialize: raises InvalidRoaringFormat / TruncatedInput (both OSError)."""
        consumed = ctypes.c_size_t()
        card = ctypes.c_int64()
        stats = (ctypes.c_int64 * 3)()
        data = bytes(data)
        check(lib().rbg_inspect(data, len(data), ctypes.byref(consumed), ctypes.byref(card), stats))
        out = cls(data[:consumed.value])
        out._lcard = card.value
        return out

    def runOptimize(self) -> bool:
        """In-place runOptimize (RB/RoaringBitmap.java:2764-2774); True if a run container results."""
        b = _lib.rbg_buffer()
        check(lib().rbg_run_optimize(self._buf, len(self._buf), ctypes.byref(b)))
        self._buf = take(b)
        return self.container_stats()[2] > 0

    def limit(self, maxcardinality):
        """x.limit(maxcardinality) (RB/RoaringBitmap.java:2457-2476) on the GPU: a new bitmap of the first
        maxcardinality values (the cut container through Container.limit).  ImmutableRoaringBitmap.limit
        (RB/buffer/ImmutableRoaringBitmap.java:1658-1677, the same types) returns a MutableRoaringBitmap."""
        b = _lib.rbg_buffer()
        check(lib().rbg_limit(self._buf, len(self._buf), _int32(maxcardinality), ctypes.byref(b)))
        return (MutableRoaringBitmap if isinstance(self, ImmutableRoaringBitmap) else RoaringBitmap)(take(b))

    def removeRunCompression(self) -> bool:
        """In-place removeRunCompression (RB/RoaringBitmap.java:2738-2749; MutableRoaringBitmap's alike): every
        run container as an array or bitmap by cardinality, on the GPU; True if there was one."""
        had = self.container_stats()[2] > 0
        b = _lib.rbg_buffer()
        check(lib().rbg_remove_run_compression(self._buf, len(self._buf), ctypes.byref(b)))
        self._buf = take(b)
        return had

    def clone(self):
        return RoaringBitmap(self._buf)

    # ---- inspection ---------------------------------------------------------
    def serialize(self) -> bytes:
        return self._buf

    def serializedSizeInBytes(self) -> int:
        return len(self._buf)

    def getLongCardinality(self) -> int:
        if self._lcard is None:
            card = ctypes.c_int64()
            check(lib().rbg_inspect(self._buf, len(self._buf), None, ctypes.byref(card), None))
            self._lcard = card.value
        return self._lcard

    def getCardinality(self) -> int:
        """Java int cast of the long cardinality (RB/RoaringBitmap.java:1966-1968)."""
        return _int32(self.getLongCardinality())

    def isEmpty(self) -> bool:
        return self.getLongCardinality() == 0

    def container_stats(self):
        """(#array, #bitmap, #run) containers, as RB/insights/BitmapAnalyser reports."""
        stats = (ctypes.c_int64 * 3)()
        check(lib().rbg_inspect(self._buf, len(self._buf), None, None, stats))
        return tuple(stats)

    def toArray(self) -> np.ndarray:
        b = _lib.rbg_buffer()
        check(lib().rbg_to_values(self._buf, len(self._buf), ctypes.byref(b)))
        raw = take(b)
        return np.frombuffer(raw, dtype=np.uint32).copy()

    def contains(self, x) -> bool:
        """RoaringBitmap.contains(int) (RB/RoaringBitmap.java:1693-1701): the key's container through
        a binary search of the descriptor table (RoaringArray.getContainer), then the container's own
        contains (ArrayContainer binary search, BitmapContainer bit test, RunContainer binary search
        of the run starts), read straight from the serialized bytes.  With a bitmap: contains(subset)
        (:2781-2802; ImmutableRoaringBitmap.contains :1242), on the GPU (rbg_pairwise_card RBG_CONTAINS)."""
        if isinstance(x, RoaringBitmap):
            return RoaringBitmap._card("contains", self, x) != 0
        x = int(x) & 0xFFFFFFFF
        key, low = x >> 16, x & 0xFFFF
        ctr = _find_container(self._buf, key)
        if ctr is None:
            return False
        kind, pay = ctr
        if kind == 0:
            i = int(np.searchsorted(pay, low))
            return i < pay.size and int(pay[i]) == low
        if kind == 1:
            return bool((int(pay[low >> 6]) >> (low & 63)) & 1)
        starts = pay[0::2]
        i = int(np.searchsorted(starts, low, side="right")) - 1
        return i >= 0 and low <= int(starts[i]) + int(pay[2 * i + 1])

    def selectRange(self, range_start, range_end):
        """x.selectRange(rangeStart, rangeEnd) (RB/RoaringBitmap.java:3095-3147) on the GPU: the values in
        [rangeStart, rangeEnd), the cut keys through Container.remove.  ImmutableRoaringBitmap.selectRange
        (RB/buffer/ImmutableRoaringBitmap.java:701-757) keeps the buffer package's types and returns a
        MutableRoaringBitmap."""
        buffer = isinstance(self, ImmutableRoaringBitmap)
        b = _lib.rbg_buffer()
        check(lib().rbg_select_range(self._buf, len(self._buf), int(range_start), int(range_end), int(buffer),
                                     ctypes.byref(b)))
        return (MutableRoaringBitmap if buffer else RoaringBitmap)(take(b))

    def isHammingSimilar(self, other, tolerance) -> bool:
        """RoaringBitmap.isHammingSimilar(other, tolerance) (RB/RoaringBitmap.java:1831-1863): the budget
        walk ends true iff |self XOR other| <= tolerance (tolerance < 0: false).  The XOR count is
        |self| + |other| - 2 |self AND other| from the GPU's and-cardinality, in 64 bits (the int
        and-cardinality wraps only when both bitmaps hold all 2^32 values)."""
        tolerance = int(tolerance)
        if tolerance < 0:
            return False
        ca, cb = self.getLongCardinality(), other.getLongCardinality()
        a = RoaringBitmap._card("and", self, other) & 0xFFFFFFFF
        if a == 0 and ca == cb == 1 << 32:
            a = 1 << 32
        return ca + cb - 2 * a <= tolerance

    def __contains__(self, x):
        return self.contains(x)

    def __len__(self):
        return self.getLongCardinality()

    def __eq__(self, other):
        return isinstance(other, RoaringBitmap) and self._buf == other._buf

    def __hash__(self):
        return hash(self._buf)

    def __repr__(self):
        a, b, r = self.container_stats()
        return f"RoaringBitmap(card={self.getLongCardinality()}, containers=A{a}/B{b}/R{r}, bytes={len(self._buf)})"

    # ---- static pairwise ops (RB/RoaringBitmap.java) --------------------------
    @staticmethod
    def _pair(op, x1, x2):
        b = _lib.rbg_buffer()
        check(lib().rbg_pairwise(_lib.OP[op], x1._buf, len(x1._buf), x2._buf, len(x2._buf), ctypes.byref(b)))
        return RoaringBitmap(take(b))

    @staticmethod
    def _card(op, x1, x2):
        out = ctypes.c_int32()
        check(lib().rbg_pairwise_card(_lib.CARD_OP[op], x1._buf, len(x1._buf), x2._buf, len(x2._buf),
                                      ctypes.byref(out)))
        return out.value

    and_ = _StaticOrInPlace(_s_and, "and")
    or_ = _StaticOrInPlace(_s_or, "or")
    xor = _StaticOrInPlace(_s_xor, "xor")
    andNot = _StaticOrInPlace(_s_andnot, "andnot")
    orNot = _OrNot(_s_ornot)
    add = _RangeMut("add")
    remove = _RangeMut("remove")
    flip = _RangeMut("flip")

    @classmethod
    def bitmapOfRange(cls, range_min, range_max):
        """RoaringBitmap.bitmapOfRange(min, max) (RB/RoaringBitmap.java:588-615) on the GPU: [min, max) as
        run containers (RunContainer.rangeOfOnes, even for one or two values)."""
        b = _lib.rbg_buffer()
        check(lib().rbg_bitmap_of_range(int(range_min), int(range_max), ctypes.byref(b)))
        return cls(take(b))

    @classmethod
    def addOffset(cls, x, offset):
        """RoaringBitmap.addOffset(x, offset) (RB/RoaringBitmap.java:230-288): every value plus `offset`
        (a long in [-2^32, 2^32]; values leaving [0, 2^32) dropped).  The buffer package's
        MutableRoaringBitmap.addOffset(ImmutableRoaringBitmap, long) (RB/buffer/MutableRoaringBitmap.java
        :84-142) gives the same bytes, as a MutableRoaringBitmap."""
        b = _lib.rbg_buffer()
        check(lib().rbg_add_offset(x._buf, len(x._buf), int(offset), ctypes.byref(b)))
        return cls(take(b))

    def _inplace(self, op, x2):
        """x1.and / or / xor / andNot(x2) in place (rbg_pairwise_inplace); x2 may be x1 itself"""
        if x2 is self and op in ("and", "or"):
            return  # x1.and(x1) / x1.or(x1) return at once (RB/RoaringBitmap.java:1273, 2482)
        b = _lib.rbg_buffer()
        check(lib().rbg_pairwise_inplace(_lib.OP[op], self._buf, len(self._buf), x2._buf, len(x2._buf),
                                         int(x2 is self), ctypes.byref(b)))
        self._buf = take(b)
        self._lcard = None

    @staticmethod
    def andCardinality(x1, x2) -> int:
        """:413-434 (Java int, wraps)"""
        return RoaringBitmap._card("and", x1, x2)

    @staticmethod
    def orCardinality(x1, x2) -> int:
        """:916-920"""
        return RoaringBitmap._card("or", x1, x2)

    @staticmethod
    def xorCardinality(x1, x2) -> int:
        """:931-933"""
        return RoaringBitmap._card("xor", x1, x2)

    @staticmethod
    def andNotCardinality(x1, x2) -> int:
        """:944-985"""
        return RoaringBitmap._card("andnot", x1, x2)

    @staticmethod
    def intersects(x1, x2) -> bool:
        """:698-720"""
        return RoaringBitmap._card("intersects", x1, x2) != 0


setattr(RoaringBitmap, "and", RoaringBitmap.__dict__["and_"])
setattr(RoaringBitmap, "or", RoaringBitmap.__dict__["or_"])


def _find_container(buf, key):
    """(kind, payload view) of `key`'s container in a portable serialized bitmap (RB/RoaringArray.java
    :547-629 layout: cookie, run flags, (key, card - 1) descriptors, offsets unless a run bitmap of
    fewer than 4 containers), or None.  kind 0 = array (u16 values), 1 = bitmap (u64 words), 2 = run
    (u16 start, length - 1 pairs)."""
    cookie = int.from_bytes(buf[0:4], "little")
    if (cookie & 0xFFFF) == 12347:
        size = (cookie >> 16) + 1
        flags = buf[4:4 + (size + 7) // 8]
        dpos = 4 + (size + 7) // 8
        has_off = size >= 4
    else:
        size = int.from_bytes(buf[4:8], "little")
        flags = None
        dpos = 8
        has_off = True
    if size == 0:
        return None
    desc = np.frombuffer(buf, dtype="<u2", count=2 * size, offset=dpos)
    keys = desc[0::2]
    i = int(np.searchsorted(keys, key))
    if i >= size or int(keys[i]) != key:
        return None

    def kind_of(j):
        if flags is not None and (flags[j >> 3] >> (j & 7)) & 1:
            return 2
        return 1 if int(desc[2 * j + 1]) + 1 > 4096 else 0

    def length(j, pos):
        k = kind_of(j)
        if k == 2:
            return 2 + 4 * int.from_bytes(buf[pos:pos + 2], "little")
        return 8192 if k == 1 else 2 * (int(desc[2 * j + 1]) + 1)

    if has_off:
        pos = int.from_bytes(buf[dpos + 4 * size + 4 * i:dpos + 4 * size + 4 * i + 4], "little")
    else:  # no offset table: walk the (at most 3) payloads before it
        pos = dpos + 4 * size
        for j in range(i):
            pos += length(j, pos)
    k = kind_of(i)
    if k == 0:
        return 0, np.frombuffer(buf, dtype="<u2", count=int(desc[2 * i + 1]) + 1, offset=pos)
    if k == 1:
        return 1, np.frombuffer(buf, dtype="<u8", count=1024, offset=pos)
    nr = int.from_bytes(buf[pos:pos + 2], "little")
    return 2, np.frombuffer(buf, dtype="<u2", count=2 * nr, offset=pos + 2)


def _intersect_array_into_bitmap(words, keys) -> int:
    """Util.intersectArrayIntoBitmap(long[] bitmap, char[] array, int length) (RB/Util.java:531-555) on a
    uint64 word array in place, with its edge behaviour: an empty array leaves word 0 untouched and zeroes
    the rest; the words past the array's last word are zeroed to the buffer's end.  -> the bits left."""
    keys = np.asarray(keys, dtype=np.int64)
    if len(keys) == 0:
        words[1:] = 0
        return 0
    mask = np.zeros(len(words), dtype=np.uint64)
    np.bitwise_or.at(mask, keys >> 6, np.uint64(1) << (keys & 63).astype(np.uint64))
    words &= mask
    return int(np.unpackbits(words.view(np.uint8)).sum())


def _keys_of(buf) -> np.ndarray:
    """the container keys of a portable serialized bitmap (its descriptor table, RB/RoaringArray.java:547-588)"""
    cookie = int.from_bytes(buf[0:4], "little")
    if (cookie & 0xFFFF) == 12347:
        size = (cookie >> 16) + 1
        dpos = 4 + (size + 7) // 8
    else:
        size = int.from_bytes(buf[4:8], "little")
        dpos = 8
    return np.frombuffer(buf, dtype="<u2", count=2 * size, offset=dpos)[0::2].astype(np.int64)


def _full_containers(keys) -> bytes:
    """the portable bytes of a bitmap with a full run container (RunContainer.full(), one run 0..65535)
    at each of the sorted `keys` (RB/RoaringArray.java:896-940 layout)"""
    import struct
    n = len(keys)
    out = bytearray(struct.pack("<I", 12347 | ((n - 1) << 16)))
    out += bytes([0xFF] * (n // 8)) + (bytes([(1 << (n % 8)) - 1]) if n % 8 else b"")
    for k in keys:
        out += struct.pack("<HH", k, 0xFFFF)
    header = len(out) + (4 * n if n >= 4 else 0)
    if n >= 4:
        for i in range(n):
            out += struct.pack("<I", header + 6 * i)
    for _ in keys:
        out += struct.pack("<HHH", 1, 0, 0xFFFF)
    return bytes(out)


def _identity_ids(bitmaps):
    seen = {}
    return [seen.setdefault(id(b), len(seen)) for b in bitmaps]


def _wide(op, bitmaps, ids=None):
    bufs = [b._buf for b in bitmaps]
    arr, lens = _lib.buf_array(bufs)
    idp = None
    if ids is not None and bitmaps:
        idp = (ctypes.c_int32 * len(ids))(*ids)
    b = _lib.rbg_buffer()
    check(lib().rbg_wide(_lib.WIDE_OP[op], arr, lens, idp, len(bufs), ctypes.byref(b)))
    return RoaringBitmap(take(b))


def _wide_card(op, bitmaps):
    bufs = [b._buf for b in bitmaps]
    arr, lens = _lib.buf_array(bufs)
    out = ctypes.c_int32()
    check(lib().rbg_wide_card(_lib.WIDE_CARD_OP[op], arr, lens, len(bufs), ctypes.byref(out)))
    return out.value


def _split_args(args):
    """Java overloads: (Iterator) vs (RoaringBitmap...) vs (long[] buffer, RoaringBitmap...)."""
    if len(args) == 1 and isinstance(args[0], Iterator):
        return "iter", None, list(args[0])
    if args and isinstance(args[0], np.ndarray):
        return "buffer", args[0], list(args[1:])
    if len(args) == 1 and isinstance(args[0], (list, tuple)):
        return "varargs", None, list(args[0])
    return "varargs", None, list(args)


class FastAggregation:
    """RB/FastAggregation.java static methods."""

    @staticmethod
    def and_(*args):
        """and(RoaringBitmap...) :37-42, and(long[], RoaringBitmap...) :51-63, and(Iterator) :26-28"""
        kind, buf, bms = _split_args(args)
        if kind == "iter":
            return _wide("and_iter", bms)
        if kind == "buffer" and len(bms) > 10:
            if buf.size < 1024:
                raise IllegalArgumentException("buffer should have at least 1024 elements.")
            try:
                return _wide("and", bms, _identity_ids(bms))
            finally:
                buf[...] = 0  # Arrays.fill(aggregationBuffer, 0L)
        return _wide("and", bms, _identity_ids(bms))

    @staticmethod
    def or_(*args):
        """or(RoaringBitmap...) :664-666 and or(Iterator) :653-655 -> naive_or"""
        _, _, bms = _split_args(args)
        return _wide("or", bms)

    @staticmethod
    def xor(*args):
        """xor(RoaringBitmap...) :834-836 and xor(Iterator) :823-825 -> naive_xor"""
        _, _, bms = _split_args(args)
        return _wide("xor", bms)

    @staticmethod
    def naive_or(*args):
        _, _, bms = _split_args(args)
        return _wide("or", bms)

    @staticmethod
    def naive_xor(*args):
        _, _, bms = _split_args(args)
        return _wide("xor", bms)

    @staticmethod
    def naive_and(*args):
        """naive_and(RoaringBitmap...) :328-346 for any N, naive_and(Iterator) :304-313"""
        kind, _, bms = _split_args(args)
        if kind == "iter":
            return _wide("and_iter", bms)
        return _wide("naive_and", bms, _identity_ids(bms))

    @staticmethod
    def workShyAnd(buffer, *bitmaps):
        """workShyAnd(long[] buffer, RoaringBitmap...) :356-414"""
        bms = list(bitmaps[0]) if len(bitmaps) == 1 and isinstance(bitmaps[0], (list, tuple)) else list(bitmaps)
        return _wide("workshy_and", bms)

    @staticmethod
    def workAndMemoryShyAnd(buffer, *bitmaps):
        """workAndMemoryShyAnd(long[] buffer, RoaringBitmap...) (RB/FastAggregation.java:522-576), following
        the reference's control flow on the caller's buffer, which it uses as the key bitset without
        clearing it first:

        - the first bitmap's keys are OR-ed into the buffer (:527-531) and the count starts at its size
          (:532): an empty first bitmap returns an empty result and leaves the buffer as it was;
        - every further bitmap's keys are intersected into it with Util.intersectArrayIntoBitmap over the
          buffer's whole length while the count is nonzero (:533-536; RB/Util.java:531-555, whose word 0
          survives an empty key array);
        - the surviving bits are the keys (:540-548): with a single bitmap the key array is sized by its
          container count, so a dirty bit outside its keys throws ArrayIndexOutOfBoundsException; with
          more, a dirty bit that survives is a key the first bitmap lacks, skipped by the per-key
          getIndex (:561-564), i.e. a full container there;
        - per key the buffer is filled with ones (its whole length) and becomes a lazy bitmap that each
          container ANDs in place (:557-569), so afterwards it holds the last key's lazy intersection.
          The result containers are workShyAnd's (computed on the device).

        A buffer longer than 1,024 words reaches the per-key chain as a bitmap of that length: a bitmap
        container there throws ArrayIndexOutOfBoundsException in the reference (BitmapContainer.iand's
        loop runs to the buffer's length, RB/BitmapContainer.java:535-538), and so it does here."""
        if buffer is None or len(buffer) < 1024:
            raise IllegalArgumentException("buffer should have at least 1024 elements.")
        bms = list(bitmaps[0]) if len(bitmaps) == 1 and isinstance(bitmaps[0], (list, tuple)) else list(bitmaps)
        if not isinstance(buffer, np.ndarray) or buffer.dtype.itemsize != 8 or buffer.ndim != 1:
            raise IllegalArgumentException("buffer must be a one-dimensional numpy array of 64-bit words")
        words = buffer.view(np.uint64)  # the caller's memory: the reference writes its long[] in place
        nw = len(words)
        fk = _keys_of(bms[0]._buf)
        np.bitwise_or.at(words, fk >> 6, np.uint64(1) << (fk & 63).astype(np.uint64))  # :527-531
        num = len(fk)
        for b in bms[1:]:  # :533-536
            if num == 0:
                break
            num = _intersect_array_into_bitmap(words, _keys_of(b._buf))
        if num == 0:  # :537-539
            return RoaringBitmap()
        bits = np.nonzero(np.unpackbits(words.view(np.uint8), bitorder="little"))[0]
        if len(bits) > num:  # keys[pos++] past numContainers (:540-548)
            raise ArrayIndexOutOfBoundsException(f"Index {num} out of bounds for length {num}")
        keys = (bits & 0xFFFF).astype(np.int64)  # (char)(base + tz)
        in_first = np.isin(keys, fk)
        first = bms[0]
        if not in_first.all():  # the first bitmap lacks these keys: skipped there, a full container for AND
            first = RoaringBitmap._pair("or", bms[0], RoaringBitmap(_full_containers(sorted(keys[~in_first].tolist()))))
        chains = [[_find_container(b._buf, int(k)) for b in bms] for k in keys]
        if nw > 1024 and any(c is not None and c[0] == 1 for ch in chains for c in ch):
            raise ArrayIndexOutOfBoundsException("Index 1024 out of bounds for length 1024")
        out = _wide("workshy_and", [first] + bms[1:])
        # the buffer after the last key's chain (:557-569): ones, then each present container ANDed in place
        words[:] = np.uint64(0xFFFFFFFFFFFFFFFF)
        for c in chains[-1]:
            if c is None:
                continue
            kind, pay = c
            if kind == 0:  # BitmapContainer.iand(ArrayContainer), lazy: intersectArrayIntoBitmap (:523-527)
                _intersect_array_into_bitmap(words, pay.astype(np.int64))
            elif kind == 1:  # lazy iand(BitmapContainer) (:535-538)
                words[:1024] &= pay
            else:  # lazy iand(RunContainer): the ranges between runs reset (:557-590)
                m = np.zeros(65536, dtype=bool)
                for s, ln in zip(pay[0::2].astype(np.int64), pay[1::2].astype(np.int64)):
                    m[s:s + ln + 1] = True
                words[:1024] &= np.packbits(m, bitorder="little").view(np.uint64)
        return out

    @staticmethod
    def andCardinality(*args) -> int:
        """:71-82"""
        _, _, bms = _split_args(args)
        return _wide_card("and", bms)

    @staticmethod
    def orCardinality(*args) -> int:
        """:90-101"""
        _, _, bms = _split_args(args)
        return _wide_card("or", bms)


    # The horizontal / priority-queue variants (RB/FastAggregation.java:110-300, 677-822) compute
    # the same sets as or / xor, but each fixes its own result container types through its
    # own chain; every form below reproduces those types (byte parity with the reference).
    @staticmethod
    def horizontal_or(*args):
        """horizontal_or(Iterator) :110-112 is naive_or; horizontal_or(List) :124-175 and
        horizontal_or(RoaringBitmap...) :185-231 run the container-pointer priority queue"""
        if len(args) == 1 and isinstance(args[0], Iterator):
            return _wide("or", list(args[0]))
        bms = list(args[0]) if len(args) == 1 and isinstance(args[0], (list, tuple)) else list(args)
        return _wide("horizontal_or", bms)

    @staticmethod
    def horizontal_xor(*bitmaps):
        """horizontal_xor(RoaringBitmap...) :243-289 (empty results are kept as empty containers)"""
        bms = list(bitmaps[0]) if len(bitmaps) == 1 and isinstance(bitmaps[0], (list, tuple)) else list(bitmaps)
        return _wide("horizontal_xor", bms)

    @staticmethod
    def priorityqueue_or(*args):
        """priorityqueue_or(Iterator) :677-727 and priorityqueue_or(RoaringBitmap...) :737-781: a
        queue of whole bitmaps by getLongSizeInBytes, lazy unions, repairAfterLazy at the end"""
        if len(args) == 1 and isinstance(args[0], Iterator):
            return _wide("priorityqueue_or", list(args[0]))
        bms = list(args[0]) if len(args) == 1 and isinstance(args[0], (list, tuple)) else list(args)
        return _wide("priorityqueue_or", bms)

    @staticmethod
    def priorityqueue_xor(*bitmaps):
        """priorityqueue_xor(RoaringBitmap...) :794-812: RoaringBitmap.xor of the two smallest"""
        bms = list(bitmaps[0]) if len(bitmaps) == 1 and isinstance(bitmaps[0], (list, tuple)) else list(bitmaps)
        return _wide("priorityqueue_xor", bms)


class ParallelAggregation:
    """RB/ParallelAggregation.java: or (:161-175, per key :197-223) and xor (:182-195).

    The reference reduces each key's containers on the ForkJoin pool; the engine reduces
    every key in parallel on the GPU with the reference's per-key algorithm, so the result
    container types are ParallelAggregation's own: below 16 containers a key is a lazyIOR
    chain from a clone of the first (repairAfterLazy at the end), from 16 on a lazy bitmap;
    xor is a clone + ixor chain without FastAggregation's restart, empty keys dropped."""

    @staticmethod
    def or_(*bitmaps):
        bms = list(bitmaps[0]) if len(bitmaps) == 1 and isinstance(bitmaps[0], (list, tuple)) else list(bitmaps)
        return _wide("parallel_or", bms)

    @staticmethod
    def xor(*bitmaps):
        bms = list(bitmaps[0]) if len(bitmaps) == 1 and isinstance(bitmaps[0], (list, tuple)) else list(bitmaps)
        return _wide("parallel_xor", bms)


class BufferFastAggregation:
    """RB/buffer/BufferFastAggregation.java over ImmutableRoaringBitmap inputs.

    An ImmutableRoaringBitmap is a mapped portable-format buffer, which is exactly
    what RoaringBitmap(serialized) holds, so every form takes the same objects.
    The or / xor algorithms are FastAggregation's (naive_or :774-781 is naivelazyor +
    repairAfterLazy like :603-610; naive_xor :827-833 is the xor chain of :637-644), and
    buffer workShyAnd :426-494 is FastAggregation.workShyAnd :356-414 over Mappeable
    containers.  The and chains are the buffer package's own: they run the in-place
    MutableRoaringBitmap.and (RB/buffer/MutableRoaringBitmap.java:886-910), whose run AND run
    keeps the merged run container (MappeableRunContainer.iand(R) = and(R), :1106-1108,
    :474-536) where the heap chain's RunContainer.and(R) ends in toEfficientContainer.  So
    these forms give other bytes than FastAggregation's whenever two run containers meet.
    The dispatch also differs:
      - and(Iterator) :66-89 always runs workShyAnd (FastAggregation's runs
        naive_and, :26-28);
      - and(MutableRoaringBitmap...) :100-102 goes through convertToImmutable,
        i.e. the Iterator form, so workShyAnd too;
      - naive_and(MutableRoaringBitmap...) :407-416 chains from a clone of the
        first bitmap (no smallest-first choice, like naive_and(Iterator) :383-396).
    """

    @staticmethod
    def and_(*args):
        """and(ImmutableRoaringBitmap...) :28-33, and(long[], ...) :43-58 (N > 10: workShyAnd, else the
        buffer naive_and), and(Iterator) :66-89"""
        kind, buf, bms = _split_args(args)
        if kind == "iter":
            return _wide("workshy_and", bms) if bms else RoaringBitmap()
        if kind == "buffer" and len(bms) > 10:
            if buf.size < 1024:
                raise IllegalArgumentException("buffer should have at least 1024 elements.")
            try:
                return _wide("workshy_and", bms)
            finally:
                buf[...] = 0  # Arrays.fill(aggregationBuffer, 0L)
        return _wide("buffer_and", bms, _identity_ids(bms))

    @staticmethod
    def and_mutable(*bitmaps):
        """and(MutableRoaringBitmap...) :100-102 -> and(convertToImmutable(...)) -> workShyAnd"""
        return BufferFastAggregation.and_(iter(list(bitmaps)))

    @staticmethod
    def naive_and(*args):
        """naive_and(ImmutableRoaringBitmap...) :347-369 (smallest first, identity skip),
        naive_and(Iterator) :383-396 (from the first)"""
        kind, _, bms = _split_args(args)
        if kind == "iter":
            return _wide("buffer_and_iter", bms)
        return _wide("buffer_naive_and", bms, _identity_ids(bms))

    @staticmethod
    def naive_and_mutable(*bitmaps):
        """naive_and(MutableRoaringBitmap...) :407-416: clone of the first, then the and chain"""
        bms = list(bitmaps[0]) if len(bitmaps) == 1 and isinstance(bitmaps[0], (list, tuple)) else list(bitmaps)
        return _wide("buffer_and_iter", bms)

    @staticmethod
    def workShyAnd(buffer, *bitmaps):
        """workShyAnd(long[], ImmutableRoaringBitmap...) :426-494"""
        return FastAggregation.workShyAnd(buffer, *bitmaps)

    @staticmethod
    def or_(*args):
        """or(ImmutableRoaringBitmap...) :875-877, or(Iterator) :886-888, or(Mutable...) :896-898 -> naive_or"""
        return FastAggregation.or_(*args)

    @staticmethod
    def xor(*args):
        """xor(ImmutableRoaringBitmap...) :1061-1063, xor(Iterator) :1072-1074 -> naive_xor"""
        return FastAggregation.xor(*args)

    @staticmethod
    def naive_or(*args):
        """naive_or(ImmutableRoaringBitmap...) :774-781 / (Iterator) :791-798: naivelazyor chain"""
        return FastAggregation.naive_or(*args)

    @staticmethod
    def or_mutable(*bitmaps):
        """or(MutableRoaringBitmap...) :896-898 -> naive_or(MutableRoaringBitmap...) :810-817:
        MutableRoaringBitmap.lazyor per input (RB/buffer/MutableRoaringBitmap.java:1309-1351),
        i.e. a lazyIOR chain per key, then repairAfterLazy"""
        bms = list(bitmaps[0]) if len(bitmaps) == 1 and isinstance(bitmaps[0], (list, tuple)) else list(bitmaps)
        return _wide("buffer_or_mutable", bms)

    naive_or_mutable = or_mutable

    @staticmethod
    def naive_xor(*args):
        return FastAggregation.naive_xor(*args)

    @staticmethod
    def andCardinality(*args) -> int:
        """:110-121 (0 -> 0, 1 -> card, 2 -> pairwise, else workShyAndCardinality)"""
        return FastAggregation.andCardinality(*args)

    @staticmethod
    def orCardinality(*args) -> int:
        """:129-140"""
        return FastAggregation.orCardinality(*args)

    horizontal_or = staticmethod(FastAggregation.horizontal_or)
    horizontal_xor = staticmethod(FastAggregation.horizontal_xor)
    priorityqueue_or = staticmethod(FastAggregation.priorityqueue_or)
    priorityqueue_xor = staticmethod(FastAggregation.priorityqueue_xor)


class ImmutableRoaringBitmap(RoaringBitmap):
    """RB/buffer/ImmutableRoaringBitmap.java: the mapped portable-format buffer (the same bytes a
    RoaringBitmap here holds).  Its static pairwise ops return MutableRoaringBitmap and type their
    containers as the buffer package does: and / andNot (:299-325, :441-471) per key c1.and(c2) /
    c1.andNot(c2), where run AND / ANDNOT run keep the merged run container
    (RB/buffer/MappeableRunContainer.java:474-536, 600-663: no toEfficientContainer, more than 2047
    runs possible); or / xor (:927-977, :1087-1134) type like the heap's."""
    __slots__ = ()

    @staticmethod
    def _bpair(op, x1, x2):
        b = _lib.rbg_buffer()
        check(lib().rbg_pairwise(_lib.OP[op], x1._buf, len(x1._buf), x2._buf, len(x2._buf), ctypes.byref(b)))
        return MutableRoaringBitmap(take(b))

    @staticmethod
    def _s_and(*args):
        """and(x1, x2) :299-325; and(Iterator, rangeStart, rangeEnd) :261-267 (selectRangeWithoutCopy, then
        BufferFastAggregation.and(Iterator) = workShyAnd)"""
        if _is_range(args):
            return _range_op("and_buffer", list(args[0]), args[1], args[2], MutableRoaringBitmap)
        x1, x2 = args
        return ImmutableRoaringBitmap._bpair("and_buffer", x1, x2)

    @staticmethod
    def _s_andnot(*args):
        """andNot(x1, x2) :441-471; andNot(x1, x2, rangeStart, rangeEnd) :402-408"""
        if len(args) == 4:
            return _range_op("andnot_buffer", [args[0], args[1]], args[2], args[3], MutableRoaringBitmap)
        x1, x2 = args
        return ImmutableRoaringBitmap._bpair("andnot_buffer", x1, x2)

    @staticmethod
    def _s_or(*args):
        """or(x1, x2) :927-977; or(Iterator, rangeStart, rangeEnd) :992-998; or(ImmutableRoaringBitmap...)
        :911 and or(Iterator) :979 = BufferFastAggregation.or = naive_or"""
        if _is_range(args):
            return _range_op("or_buffer", list(args[0]), args[1], args[2], MutableRoaringBitmap)
        if len(args) == 2 and not isinstance(args[0], Iterator):
            return ImmutableRoaringBitmap._bpair("or", args[0], args[1])
        bms = list(args[0]) if len(args) == 1 and isinstance(args[0], Iterator) else list(args)
        return MutableRoaringBitmap(_wide("or", bms)._buf)

    @staticmethod
    def _s_xor(*args):
        """xor(x1, x2) :1087-1134; xor(Iterator, rangeStart, rangeEnd) :1048-1053 (naive_xor)"""
        if _is_range(args):
            return _range_op("xor_buffer", list(args[0]), args[1], args[2], MutableRoaringBitmap)
        x1, x2 = args
        return ImmutableRoaringBitmap._bpair("xor", x1, x2)

    @staticmethod
    def orNot(x1, x2, range_end):
        """orNot(x1, x2, rangeEnd) :484-548 -> MutableRoaringBitmap (the buffer package's container types)"""
        return MutableRoaringBitmap(_ornot(x1, x2, range_end, False, True))

    and_ = _s_and
    andNot = _s_andnot
    or_ = _s_or
    xor = _s_xor
    add = remove = None  # no static add / remove on ImmutableRoaringBitmap (MutableRoaringBitmap's: below)
    addOffset = None  # MutableRoaringBitmap.addOffset(ImmutableRoaringBitmap, long): below
    removeRunCompression = None  # in place: MutableRoaringBitmap's (RB/buffer/MutableRoaringBitmap.java:1568)
    andCardinality = RoaringBitmap.__dict__["andCardinality"]  # :336-359, a set-level count
    intersects = RoaringBitmap.__dict__["intersects"]


class MutableRoaringBitmap(ImmutableRoaringBitmap):
    """RB/buffer/MutableRoaringBitmap.java: the static and / andNot (:235-301) are ImmutableRoaringBitmap's
    per-key code; the in-place x1.and(x2) (:886-910) and x1.andNot(x2) (:918-954) run
    MappeableContainer.iand / iandNot, which type like the static ops (MappeableRunContainer.iand /
    iandNot = and / andNot, :1106-1123; MappeableArrayContainer.iandNot :703-749 keeps an array,
    MappeableBitmapContainer.iandNot :680-760 by cardinality).  x1.and(x1) leaves x1, x1.andNot(x1)
    clears it (:887, :919-922).  The in-place or / xor (Container.ior / ixor of the buffer package) are
    not on this path."""
    __slots__ = ()

    and_ = _StaticOrInPlace(ImmutableRoaringBitmap._s_and, "and_buffer")
    andNot = _StaticOrInPlace(ImmutableRoaringBitmap._s_andnot, "andnot_buffer")
    or_ = _StaticOrInPlace(ImmutableRoaringBitmap._s_or, "or")
    xor = _StaticOrInPlace(ImmutableRoaringBitmap._s_xor, "xor")
    orNot = _OrNot(ImmutableRoaringBitmap.__dict__["orNot"].__func__, buffer=True)  # x1.orNot in place :962-1030
    addOffset = RoaringBitmap.__dict__["addOffset"]  # RB/buffer/MutableRoaringBitmap.java:84-142, the same bytes
    removeRunCompression = RoaringBitmap.removeRunCompression

    def _inplace(self, op, x2):
        if op not in ("and_buffer", "andnot_buffer"):
            raise NotImplementedError("MutableRoaringBitmap.or / xor in place")
        if x2 is self:
            if op == "andnot_buffer":
                self._buf = EMPTY
                self._lcard = 0
            return
        self._buf = ImmutableRoaringBitmap._bpair(op, self, x2)._buf
        self._lcard = None


setattr(ImmutableRoaringBitmap, "and", ImmutableRoaringBitmap.__dict__["and_"])
setattr(ImmutableRoaringBitmap, "or", ImmutableRoaringBitmap.__dict__["or_"])
setattr(MutableRoaringBitmap, "and", MutableRoaringBitmap.__dict__["and_"])
setattr(MutableRoaringBitmap, "or", MutableRoaringBitmap.__dict__["or_"])
# the buffer package's static range mutations: ImmutableRoaringBitmap.flip (RB/buffer/ImmutableRoaringBitmap
# .java:592-640), MutableRoaringBitmap.add / remove / flip (RB/buffer/MutableRoaringBitmap.java:152, 649, 455)
ImmutableRoaringBitmap.flip = _RangeMut("flip", True, MutableRoaringBitmap)
for _op in ("add", "remove", "flip"):
    setattr(MutableRoaringBitmap, _op, _RangeMut(_op, True, MutableRoaringBitmap))

setattr(BufferFastAggregation, "and", BufferFastAggregation.and_)
setattr(BufferFastAggregation, "or", BufferFastAggregation.or_)
setattr(ParallelAggregation, "or", ParallelAggregation.or_)
setattr(FastAggregation, "and", FastAggregation.and_)
setattr(FastAggregation, "or", FastAggregation.or_)


def batch_and_cardinality(pairs):
    """out[i] = RoaringBitmap.andCardinality(a_i, b_i) for (a_i, b_i) in pairs (config C4)."""
    pairs = list(pairs)
    n = len(pairs)
    if n == 0:
        return np.zeros(0, dtype=np.int32)
    a_arr, a_lens = _lib.buf_array([p[0]._buf for p in pairs])
    b_arr, b_lens = _lib.buf_array([p[1]._buf for p in pairs])
    out = np.zeros(n, dtype=np.int32)
    check(lib().rbg_batch_and_card(n, a_arr, a_lens, b_arr, b_lens,
                                   out.ctypes.data_as(ctypes.POINTER(ctypes.c_int32))))
    return out


def run_optimize_many(bitmaps):
    """RoaringBitmap.runOptimize() (RB/RoaringBitmap.java:2764-2774) applied in place to every bitmap,
    as one device pass over all their containers; returns runOptimize's boolean per bitmap."""
    bitmaps = list(bitmaps)
    n = len(bitmaps)
    if n == 0:
        return []
    arr, lens = _lib.buf_array([b._buf for b in bitmaps])
    outs = (_lib.rbg_buffer * n)()
    ans = (ctypes.c_uint8 * n)()
    check(lib().rbg_run_optimize_many(arr, lens, n, outs, ans))
    for b, o in zip(bitmaps, outs):
        b._buf = take(o)
        b._lcard = None
    return [bool(x) for x in ans]


def _chain(*its):
    return itertools.chain(*its)
