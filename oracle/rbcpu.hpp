// rbcpu — CPU ORACLE for the Roaring set-algebra hot path.
//
// TEST INFRASTRUCTURE ONLY.  This is a C++17 restatement of the Java reference
// (luvk1412/RoaringBitmap @ 2025-02-27, read at /root/reference) used as the
// parity checker.  Only tests/, __graft_entry__.smoke() and bench.py's
// cpu_baseline leg may load it.  The product engine (roaringbitmap_amd/) never
// links, loads or calls anything in oracle/.
//
// Path prefixes used in citations:
//   RB/  = RoaringBitmap/src/main/java/org/roaringbitmap/
//
// The Java reference cannot be compiled or run in this image (no JDK, see
// DESIGN.md §Oracle).  Parity of this restatement is pinned by the reference's
// own fixtures: the golden serialized files (testdata/bitmapwith{,out}runs.bin,
// crashproneinput1..7.bin), the realdata known-answer constants
// (jmh/src/test/.../realdata/*Test.java) and the container-type assertions of
// RBT/TestContainer.java / TestRunContainer.java.  See tests/test_oracle_*.py.
//
// Every container operation restates the Java control flow of the cited
// method, because the *result container type* (array / bitmap / run) and the
// run layout are part of the serialized bytes and therefore of parity.
#pragma once
#include <cstdint>
#include <cstddef>
#include <string>
#include <vector>

namespace rbcpu {

enum Kind : uint8_t { ARRAY = 0, BITMAP = 1, RUN = 2 };

constexpr int kArrayMax = 4096;          // RB/ArrayContainer.java:27 DEFAULT_MAX_SIZE
constexpr int kArrayLazyLowerBound = 1024;  // RB/ArrayContainer.java:25
constexpr int kWords = 1024;             // RB/BitmapContainer.java:28 (1<<16)/64
constexpr int kMaxCapacity = 1 << 16;    // RB/BitmapContainer.java:24
constexpr int kRunVsArrayThreshold = 32; // RB/RunContainer.java:576,2412 "arbitrary_threshold"

// One container.  A: `vals` sorted u16, `card` = size.  B: `words` (1024 u64),
// `card` cached cardinality, -1 = lazy (RB/BitmapContainer.java:648-676).
// R: `vals` interleaved (start, length-1) pairs (RB/RunContainer.java:92-99).
struct Ctr {
  Kind kind = ARRAY;
  int card = 0;
  std::vector<uint16_t> vals;
  std::vector<uint64_t> words;

  int nruns() const { return (int)(vals.size() / 2); }
  int cardinality() const;                 // R: RB/RunContainer.java:1003-1009
  bool empty() const;
  bool full() const;                       // RB/RunContainer.java:1659-1661, BitmapContainer isFull
  int array_size_bytes() const;            // getArraySizeInBytes (payload bytes)
};

// ---- container constructors / conversions ---------------------------------
Ctr make_array(std::vector<uint16_t> v);
Ctr make_bitmap_zero();
Ctr run_full();                                      // RB/RunContainer.java:1663
Ctr to_bitmap(const Ctr& c);                         // toBitmapContainer()
Ctr bitmap_to_array(const Ctr& b);                   // BitmapContainer.toArrayContainer
Ctr to_efficient(const Ctr& r);                      // RB/RunContainer.java:2326-2335
Ctr to_bitmap_or_array(const Ctr& r, int card);      // RB/RunContainer.java:2300-2323
Ctr repair_after_lazy(const Ctr& c);                 // A: this, B: :1205-1215, R: EFF
Ctr run_optimize(const Ctr& c);                      // A :1085-1099, B :1218-1237, R :2083
int number_of_runs(const Ctr& c);                    // exact run count of the set

// ---- pairwise container ops (Container.and/or/xor/andNot dispatch) --------
Ctr c_and(const Ctr& a, const Ctr& b);               // RB/Container.java:81-88
Ctr c_or(const Ctr& a, const Ctr& b);                // RB/Container.java:822-829
Ctr c_xor(const Ctr& a, const Ctr& b);               // RB/Container.java:964-971
Ctr c_andnot(const Ctr& a, const Ctr& b);            // RB/Container.java:164-171
int c_and_card(const Ctr& a, const Ctr& b);          // RB/Container.java:113-126
// buffer package: run AND / ANDNOT run keep the merged run container (RB/buffer/MappeableRunContainer.java:474-536,600-663)
Ctr c_and_buf(const Ctr& a, const Ctr& b);
Ctr c_andnot_buf(const Ctr& a, const Ctr& b);
bool c_intersects(const Ctr& a, const Ctr& b);
// in-place variants used by the FastAggregation chains
Ctr c_iand(const Ctr& a, const Ctr& b);              // RB/Container.java:459-466
Ctr c_ixor(const Ctr& a, const Ctr& b);              // RB/Container.java:688-695
Ctr b_ilazyor(const Ctr& lazy_bitmap, const Ctr& x); // RB/BitmapContainer.java:648-676
Ctr b_lazy_iand(const Ctr& lazy_bitmap, const Ctr& x); // RB/BitmapContainer.java:523-599 lazy branches

// ---- bitmaps ---------------------------------------------------------------
struct Bitmap {
  std::vector<uint16_t> keys;
  std::vector<Ctr> ctrs;
  size_t size() const { return keys.size(); }
  int64_t long_card() const;
  int32_t card() const { return (int32_t)(uint32_t)(uint64_t)long_card(); }
};

Bitmap bitmap_of(const uint32_t* vals, size_t n);    // RoaringBitmap.bitmapOf via addN (BY_CARD)
void bitmap_run_optimize(Bitmap& b);                 // RB/RoaringBitmap.java:2764-2774
std::vector<uint32_t> bitmap_values(const Bitmap& b);

// static pairwise ops, RB/RoaringBitmap.java
Bitmap op_and(const Bitmap& x1, const Bitmap& x2);        // :377-401
Bitmap op_or(const Bitmap& x1, const Bitmap& x2);         // :860-902
Bitmap op_ior(const Bitmap& x1, const Bitmap& x2);        // x1.or(x2) in place, :2481-2523
Ctr c_ior(const Ctr& a, const Ctr& b);                    // Container.ior
Bitmap op_xor(const Bitmap& x1, const Bitmap& x2);        // :1071-1118
Bitmap op_andnot(const Bitmap& x1, const Bitmap& x2);     // :444-473
int32_t op_and_card(const Bitmap& x1, const Bitmap& x2);  // :413-434
int32_t op_or_card(const Bitmap& x1, const Bitmap& x2);   // :916-920
int32_t op_xor_card(const Bitmap& x1, const Bitmap& x2);  // :931-933
int32_t op_andnot_card(const Bitmap& x1, const Bitmap& x2); // :944-985
bool op_intersects(const Bitmap& x1, const Bitmap& x2);   // :698-720
// ImmutableRoaringBitmap.and / andNot, RB/buffer/ImmutableRoaringBitmap.java:299-325, 441-471
Bitmap op_and_buf(const Bitmap& x1, const Bitmap& x2);
Bitmap op_andnot_buf(const Bitmap& x1, const Bitmap& x2);

// FastAggregation, RB/FastAggregation.java.  `ids` carries Java object
// identity (naive_and skips `bitmaps[k] != smallest` by reference, :341):
// two inputs with equal id are the same object.  nullptr = all distinct.
Bitmap fa_or(const std::vector<const Bitmap*>& bms);                        // :653-666 -> naive_or :603-610
Bitmap fa_and(const std::vector<const Bitmap*>& bms, const int* ids);       // :37-42
Bitmap fa_and_iter(const std::vector<const Bitmap*>& bms);                  // :26-28 -> naive_and(Iterator) :304-313
Bitmap fa_xor(const std::vector<const Bitmap*>& bms);                       // :823-836 -> naive_xor :621-644
Bitmap fa_naive_and(const std::vector<const Bitmap*>& bms, const int* ids); // :328-346
Bitmap fa_workshy_and(const std::vector<const Bitmap*>& bms);               // :356-414
int32_t fa_and_card(const std::vector<const Bitmap*>& bms);                 // :71-82
int32_t fa_or_card(const std::vector<const Bitmap*>& bms);                  // :90-101

// lazy OR algebra, RB/Container.java:717-774
Ctr c_lazy_ior(const Ctr& cur, const Ctr& x);  // lazyIOR
Ctr c_lazy_or(const Ctr& a, const Ctr& x);     // lazyOR
// alternative aggregations (their result container types follow their own chains)
Bitmap pa_or(const std::vector<const Bitmap*>& bms);                 // ParallelAggregation.or :161-175
Bitmap pa_xor(const std::vector<const Bitmap*>& bms);                // ParallelAggregation.xor :182-195
Ctr pa_or_key(const std::vector<const Ctr*>& cs);                    // :197-223
Ctr pa_xor_key(const std::vector<const Ctr*>& cs);                   // :189-195
Bitmap buf_or_mutable(const std::vector<const Bitmap*>& bms);        // BufferFastAggregation.naive_or(Mutable...)
// BufferFastAggregation's and chains (RB/buffer/BufferFastAggregation.java:28-56,347-416): the in-place
// MutableRoaringBitmap.and, whose run AND run keeps the merged run container
Bitmap buf_and(const std::vector<const Bitmap*>& bms, const int* ids);        // and(Immutable...) :28-56
Bitmap buf_naive_and(const std::vector<const Bitmap*>& bms, const int* ids);  // naive_and(Immutable...) :347-369
Bitmap buf_and_iter(const std::vector<const Bitmap*>& bms);  // naive_and(Iterator) :383-396, (Mutable...) :407-416
// range-restricted aggregations, RB/RoaringBitmap.java (selectRangeWithoutCopy, then the op)
Bitmap select_range(const Bitmap& b, uint64_t start, uint64_t end, bool buf = false);
Bitmap range_aggregate(int op, const std::vector<const Bitmap*>& bms, uint64_t start, uint64_t end);  // 0 and 1 or 2 xor
Bitmap op_andnot_range(const Bitmap& x1, const Bitmap& x2, uint64_t start, uint64_t end);  // :1396-1423
// the buffer package's (ImmutableRoaringBitmap): 0 and (workShyAnd), 1 or, 2 xor, 3 andNot (n == 2)
Bitmap range_aggregate_buf(int op, const std::vector<const Bitmap*>& bms, uint64_t start, uint64_t end);
// RoaringBitmap.orNot(x1, x2, rangeEnd) (static, RB/RoaringBitmap.java:1521-1603; inplace = false) and
// x1.orNot(x2, rangeEnd) (:1431-1506; inplace = true).  *neg = true where the reference's maxSize is
// negative (new char[maxSize] throws NegativeArraySizeException).  buf: ImmutableRoaringBitmap.orNot
// (RB/buffer/ImmutableRoaringBitmap.java:484-548) / MutableRoaringBitmap.orNot (RB/buffer/
// MutableRoaringBitmap.java:962-1030), the same loop with the buffer package's container types.
Bitmap op_ornot(const Bitmap& x1, const Bitmap& x2, uint64_t range_end, bool inplace, bool* neg, bool buf = false);
Ctr c_not_prefix(const Ctr& c, int end);  // Container.not(0, end)
// static add / remove / flip(rb, rangeStart, rangeEnd): op 0 / 1 / 2 (RB/RoaringBitmap.java:298, 995, 626);
// buf: MutableRoaringBitmap's (RB/buffer/MutableRoaringBitmap.java:152, 649, 455)
Bitmap op_range_mut(int op, const Bitmap& b, uint64_t start, uint64_t end, bool buf = false);
// RoaringBitmap.addOffset(x, offset) (RB/RoaringBitmap.java:230-288; MutableRoaringBitmap's :84-142)
Bitmap op_add_offset(const Bitmap& x, int64_t offset);
Bitmap op_remove_run_compression(const Bitmap& x);  // RB/RoaringBitmap.java:2738-2749
Bitmap op_limit(const Bitmap& x, int32_t maxcard);   // RB/RoaringBitmap.java:2457-2476
Bitmap op_bitmap_of_range(uint64_t min, uint64_t max);  // RB/RoaringBitmap.java:588-615
Bitmap fa_horizontal_or(const std::vector<const Bitmap*>& bms);      // FastAggregation.horizontal_or :124-231
Bitmap fa_horizontal_xor(const std::vector<const Bitmap*>& bms);     // :243-289
Bitmap fa_priorityqueue_or(const std::vector<const Bitmap*>& bms);   // :733-781
Bitmap fa_priorityqueue_xor(const std::vector<const Bitmap*>& bms);  // :790-812
int64_t long_size_in_bytes(const Bitmap& b);                         // RoaringBitmap.getLongSizeInBytes

// ---- portable format, RB/RoaringArray.java ---------------------------------
enum Status : int { OK = 0, ERR_FORMAT = -1, ERR_TRUNCATED = -2, ERR_ARG = -3 };
std::vector<uint8_t> serialize(const Bitmap& b);                            // :896-940
int deserialize(const uint8_t* p, size_t n, Bitmap* out, size_t* consumed); // :547-629

}  // namespace rbcpu
