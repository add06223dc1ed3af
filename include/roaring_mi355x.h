/*
 * roaring_mi355x.h — C ABI of the MI355X Roaring set-algebra engine.
 *
 * Drop-in boundary for the reference's data-parallel hot path
 * (luvk1412/RoaringBitmap, Java; RB/ = RoaringBitmap/src/main/java/org/roaringbitmap/).
 * The reference has no native boundary, so each entry point below is what a
 * JNI shim for the cited static Java method binds.
 *
 * Data contract
 *   - Bitmaps cross the boundary in the portable serialized format
 *     (RB/RoaringArray.java:896-940 serialize, :547-629 deserialize), exactly the
 *     bytes of RoaringBitmap.serialize(ByteBuffer) or an ImmutableRoaringBitmap's
 *     mapped buffer.  Outputs are the bytes RoaringBitmap.serialize would write
 *     for the reference's result object, including its array/bitmap/run
 *     container choice, so RoaringBitmap.deserialize(out) == reference result.
 *   - Inputs are borrowed, read-only, caller-owned, valid for the call.
 *   - Outputs (rbg_buffer) are allocated by the library; release with rbg_free.
 *   - All calls are reentrant.  Concurrent calls from different threads each use
 *     their own HIP stream and workspace (thread-local device context).
 *   - Every compute entry point runs on the GPU.  If no HIP device is usable the
 *     call returns RBG_ERR_DEVICE; there is no CPU fallback.
 *
 * Status codes map 1:1 to the reference's exceptions.
 */
#ifndef ROARING_MI355X_H
#define ROARING_MI355X_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RBG_OK 0
/* InvalidRoaringFormat -> IOException: bad cookie or size > 65536
 * (RB/RoaringArray.java:279-288,553-566; RB/RoaringBitmap.java:1779-1811).
 * Also returned for a negative container count (Java NegativeArraySizeException)
 * and for keys that are not strictly increasing (the reference does not check
 * this; such input is outside the format spec). */
#define RBG_ERR_INVALID_FORMAT (-1)
/* EOFException / BufferUnderflowException on truncated input
 * (RBT/TestAdversarialInputs.java:50-55). */
#define RBG_ERR_TRUNCATED (-2)
/* IllegalArgumentException (e.g. aggregation buffer < 1024 longs,
 * RB/FastAggregation.java:52-54) or a bad op code / null pointer. */
#define RBG_ERR_ILLEGAL_ARGUMENT (-3)
/* HIP runtime failure or no usable gfx950 device. */
#define RBG_ERR_DEVICE (-4)
#define RBG_ERR_OUT_OF_MEMORY (-5)

typedef struct rbg_buffer {
  uint8_t* data;
  size_t len;
} rbg_buffer;

/* pairwise ops: RB/RoaringBitmap.java and :377, or :860, xor :1071, andNot :444;
 * RBG_OR_INPLACE: x1.or(x2) in place (:2481-2523), Container.ior's result types;
 * RBG_AND_BUFFER / RBG_ANDNOT_BUFFER: the buffer package's static and / andNot,
 * RB/buffer/ImmutableRoaringBitmap.java:299-325, 441-471 (= MutableRoaringBitmap.and / andNot
 * static, RB/buffer/MutableRoaringBitmap.java:235-301): run AND / ANDNOT run keep the merged run
 * container (RB/buffer/MappeableRunContainer.java:474-536, 600-663), results above 2047 runs
 * included; every other container pair types like the heap's.  Synchronous (the run arena is checked).
 * The buffer or / xor type like the heap's: RBG_OR / RBG_XOR. */
enum { RBG_AND = 0, RBG_OR = 1, RBG_XOR = 2, RBG_ANDNOT = 3, RBG_OR_INPLACE = 4, RBG_AND_BUFFER = 5,
       RBG_ANDNOT_BUFFER = 6 };
/* cardinality ops: andCardinality :413, orCardinality :916, xorCardinality :931,
 * andNotCardinality :944 (all Java int, wrapping mod 2^32), intersects :698 (0/1);
 * RBG_CONTAINS: a.contains(b), b a subset of a (RB/RoaringBitmap.java:2781-2802; ImmutableRoaringBitmap
 * :1242), 0/1, from the 64-bit and-cardinality (|a AND b| == |b|) */
enum { RBG_CARD_AND = 0, RBG_CARD_OR = 1, RBG_CARD_XOR = 2, RBG_CARD_ANDNOT = 3, RBG_INTERSECTS = 4,
       RBG_CONTAINS = 5 };
/* wide ops, RB/FastAggregation.java:
 *   RBG_WIDE_AND      and(RoaringBitmap...)  :37-42  (N>10 workShyAnd, else naive_and)
 *   RBG_WIDE_OR       or(RoaringBitmap...)   :664-666 (naive_or); also RoaringBitmap.or(...) :844
 *   RBG_WIDE_XOR      xor(RoaringBitmap...)  :834-836 (naive_xor)
 *   RBG_WIDE_AND_ITER and(Iterator)          :26-28  (naive_and over an iterator)
 *   RBG_WIDE_NAIVE_AND   naive_and(RoaringBitmap...) :328-346 for any N
 *   RBG_WIDE_WORKSHY_AND workShyAnd(long[], RoaringBitmap...) :356-414 for any N >= 1 */
enum { RBG_WIDE_AND = 0, RBG_WIDE_OR = 1, RBG_WIDE_XOR = 2, RBG_WIDE_AND_ITER = 3, RBG_WIDE_NAIVE_AND = 4,
       RBG_WIDE_WORKSHY_AND = 5,
/* alternative aggregations, each with its own result container types:
 *   RBG_WIDE_PARALLEL_OR        ParallelAggregation.or(RoaringBitmap...)  RB/ParallelAggregation.java:161-175,197-223
 *   RBG_WIDE_PARALLEL_XOR       ParallelAggregation.xor(RoaringBitmap...) :182-195
 *   RBG_WIDE_BUFFER_OR_MUTABLE  BufferFastAggregation.or / naive_or(MutableRoaringBitmap...)
 *                               RB/buffer/BufferFastAggregation.java:810-817,896-898 (lazyor chain)
 *   RBG_WIDE_HORIZONTAL_OR      FastAggregation.horizontal_or(List / RoaringBitmap...) RB/FastAggregation.java:124-231
 *   RBG_WIDE_HORIZONTAL_XOR     FastAggregation.horizontal_xor(RoaringBitmap...) :243-289
 *   RBG_WIDE_PQ_OR              FastAggregation.priorityqueue_or(Iterator / RoaringBitmap...) :677-781
 *   RBG_WIDE_PQ_XOR             FastAggregation.priorityqueue_xor(RoaringBitmap...) :790-812
 * The horizontal_* chain order is the poll order of the reference's container-pointer
 * priority queue, planned from the container table (keys and cardinalities).  The
 * priorityqueue_* ops replay the reference's bitmap queue ordered by getLongSizeInBytes:
 * N - 1 dependent whole-bitmap steps, one device pass over the union keys each (full key
 * range only: the queue order depends on every key). */
       RBG_WIDE_PARALLEL_OR = 6, RBG_WIDE_PARALLEL_XOR = 7, RBG_WIDE_BUFFER_OR_MUTABLE = 8,
       RBG_WIDE_HORIZONTAL_OR = 9, RBG_WIDE_HORIZONTAL_XOR = 10, RBG_WIDE_PQ_OR = 11, RBG_WIDE_PQ_XOR = 12,
/* BufferFastAggregation's and chains, RB/buffer/BufferFastAggregation.java.  They chain the buffer
 * package's in-place MutableRoaringBitmap.and (RB/buffer/MutableRoaringBitmap.java:886-910), whose
 * run AND run keeps the merged run container (MappeableRunContainer.iand(R) = and(R), :1106-1108,
 * :474-536) where the heap's converts it (RunContainer.and(R) ends in toEfficientContainer):
 *   RBG_WIDE_BUFFER_AND         and(ImmutableRoaringBitmap...) / and(long[], ...) :28-56 (N>10 workShyAnd)
 *   RBG_WIDE_BUFFER_NAIVE_AND   naive_and(ImmutableRoaringBitmap...) :347-369 (smallest first)
 *   RBG_WIDE_BUFFER_AND_ITER    naive_and(Iterator) :383-396, naive_and(MutableRoaringBitmap...) :407-416
 * A result container of more than 2047 runs is kept as such; these calls synchronise the stream
 * (the run arena is checked after the op). */
       RBG_WIDE_BUFFER_AND = 13, RBG_WIDE_BUFFER_NAIVE_AND = 14, RBG_WIDE_BUFFER_AND_ITER = 15 };
/* range-restricted aggregations, RB/RoaringBitmap.java: every input through selectRangeWithoutCopy
 * (:3160-3214: keys outside [rangeStart >> 16, (rangeEnd - 1) >> 16] dropped, the first / last key's
 * container cut by Container.remove -- A stays A, B becomes A at <= 4096 values, R stays R with its runs
 * clipped -- and emptied ones dropped), then
 *   RBG_RANGE_AND     and(Iterator, rangeStart, rangeEnd) :1308-1316 -> FastAggregation.and(Iterator)
 *   RBG_RANGE_OR      or(Iterator, rangeStart, rangeEnd) :2536-2543 -> FastAggregation.or(Iterator)
 *   RBG_RANGE_XOR     xor(Iterator, rangeStart, rangeEnd) :3359-3365 -> FastAggregation.xor(Iterator)
 *   RBG_RANGE_ANDNOT  andNot(x1, x2, rangeStart, rangeEnd) :1396-1404 (n == 2)
 * rangeSanityCheck (:204-213): rangeStart in [0, 2^32 - 1], rangeEnd in [0, 2^32], else
 * RBG_ERR_ILLEGAL_ARGUMENT; rangeEnd <= rangeStart gives the empty bitmap. */
/* The buffer package's forms, RB/buffer/ImmutableRoaringBitmap.java (MutableRoaringBitmap results):
 *   RBG_RANGE_BUFFER_AND     and(Iterator, rangeStart, rangeEnd) :261-267 -> BufferFastAggregation.and
 *                            (Iterator) = workShyAnd for any input count (RB/buffer/BufferFastAggregation.java
 *                            :66-89, 505-576)
 *   RBG_RANGE_BUFFER_OR      or(Iterator, rangeStart, rangeEnd) :992-998 -> naive_or
 *   RBG_RANGE_BUFFER_XOR     xor(Iterator, rangeStart, rangeEnd) :1048-1053 -> naive_xor
 *   RBG_RANGE_BUFFER_ANDNOT  andNot(x1, x2, rangeStart, rangeEnd) :402-408 -> ImmutableRoaringBitmap.andNot
 *                            (RBG_ANDNOT_BUFFER's types)
 * whose selectRangeWithoutCopy (:768-820) cuts through MappeableContainer.remove: a bitmap becomes an
 * array only below 4096 values (RB/buffer/MappeableBitmapContainer.java:1597-1612).  The buffer xor has
 * no rangeSanityCheck in the reference; here every form checks the range. */
enum { RBG_RANGE_AND = 0, RBG_RANGE_OR = 1, RBG_RANGE_XOR = 2, RBG_RANGE_ANDNOT = 3, RBG_RANGE_BUFFER_AND = 4,
       RBG_RANGE_BUFFER_OR = 5, RBG_RANGE_BUFFER_XOR = 6, RBG_RANGE_BUFFER_ANDNOT = 7 };
int rbg_range_op(int op, const uint8_t* const* bufs, const size_t* lens, size_t n, int64_t range_start,
                 int64_t range_end, rbg_buffer* out);
/* orNot: flags 0 = RoaringBitmap.orNot(x1, x2, rangeEnd) (RB/RoaringBitmap.java:1521-1603);
 * RBG_ORNOT_INPLACE = x1.orNot(x2, rangeEnd) (:1431-1506, the new bytes of x1; the caller rejects x2 == x1 as
 * the reference's UnsupportedOperationException); | RBG_ORNOT_BUFFER = the buffer package's
 * ImmutableRoaringBitmap.orNot (RB/buffer/ImmutableRoaringBitmap.java:484-548) / MutableRoaringBitmap.orNot
 * (RB/buffer/MutableRoaringBitmap.java:962-1030), whose MappeableBitmapContainer.iremove keeps a
 * 4096-value bitmap (:1003-1017 of MappeableBitmapContainer.java).  Per key <= maxKey = (rangeEnd - 1) >>> 16: x1.orNot(x2) / iorNot
 * (RB/Container.java:191-196, 536-541), full / x1.ior(rangeOfOnes) at maxKey for x1 alone, x2.not(0, end)
 * for x2 alone (not clipped at rangeEnd), full / rangeOfOnes for neither; the key loop bounded by the
 * reference's maxSize estimate; x1's keys above maxKey appended.  rangeEnd in [0, 2^32] (rangeSanityCheck,
 * :204-213) and a negative maxSize (NegativeArraySizeException) -> RBG_ERR_ILLEGAL_ARGUMENT.  x1 is not
 * modified (the reference's static form updates x1's maxKey container through Container.ior, see
 * DESIGN.md §7). */
enum { RBG_ORNOT_INPLACE = 1, RBG_ORNOT_BUFFER = 2 };
int rbg_ornot(const uint8_t* a, size_t a_len, const uint8_t* b, size_t b_len, int64_t range_end, int flags,
              rbg_buffer* out);
/* static range mutations of one bitmap: RBG_RMUT_ADD = RoaringBitmap.add(rb, rangeStart, rangeEnd)
 * (RB/RoaringBitmap.java:298-345: Container.add on the first / last key, full run containers between,
 * rangeOfOnes where a key is missing), RBG_RMUT_REMOVE = remove(rb, ...) (:995-1040: Container.remove on
 * the first / last key unless the cut covers the whole key, the keys between dropped), RBG_RMUT_FLIP =
 * flip(rb, ...) (:626-668: Container.not on every key of the range, rangeOfOnes where a key is missing);
 * empty containers dropped, keys outside the range cloned.  | RBG_RMUT_BUFFER: MutableRoaringBitmap's
 * (RB/buffer/MutableRoaringBitmap.java:152-205, 649-700, 455-505; ImmutableRoaringBitmap.flip :592),
 * whose MappeableBitmapContainer.remove keeps a 4096-value bitmap.  rangeSanityCheck (:204-213) ->
 * RBG_ERR_ILLEGAL_ARGUMENT; rangeEnd <= rangeStart: the input's bytes.  Synchronises the stream (a run
 * result above 2047 runs, from an input run container that large, is checked for in the run arena).
 * RBG_RMUT_ADD_INPLACE = x.add(rangeStart, rangeEnd) (RB/RoaringBitmap.java:1181-1206,
 * RB/buffer/MutableRoaringBitmap.java:831-858): Container.iadd on every key of the range, so an array
 * between the first and last key becomes a full bitmap where the static add puts a full run container.
 * The in-place remove / flip (:2656, :1893) give the static forms' bytes: use RBG_RMUT_REMOVE / FLIP. */
enum { RBG_RMUT_ADD = 0, RBG_RMUT_REMOVE = 1, RBG_RMUT_FLIP = 2, RBG_RMUT_ADD_INPLACE = 3, RBG_RMUT_BUFFER = 4 };
int rbg_range_mut(int op, const uint8_t* a, size_t a_len, int64_t range_start, int64_t range_end, rbg_buffer* out);
/* RoaringBitmap.addOffset(x, offset) (RB/RoaringBitmap.java:230-288; MutableRoaringBitmap.addOffset,
 * RB/buffer/MutableRoaringBitmap.java:84-142, gives the same bytes): every value plus offset, values
 * leaving [0, 2^32) dropped.  The container chain's types (Util.addOffset's parts, Container.ior of a
 * low part into the previous high part, repairAfterLazy).  A whole-key offset clones the containers;
 * where the reference's (char) cast would wrap keys out of [0, 65535] into an unsorted key list, those
 * containers are dropped. */
int rbg_add_offset(const uint8_t* a, size_t a_len, int64_t offset, rbg_buffer* out);
/* x.removeRunCompression() (RB/RoaringBitmap.java:2738-2749; MutableRoaringBitmap's alike): out = x's
 * bytes afterwards, every run container as an array (<= 4096 values) or a bitmap
 * (RunContainer.toBitmapOrArrayContainer, RB/RunContainer.java:2300-2323), the rest unchanged */
int rbg_remove_run_compression(const uint8_t* a, size_t a_len, rbg_buffer* out);
/* x.limit(maxcardinality) (RB/RoaringBitmap.java:2457-2476): the first maxcardinality values; whole
 * containers while they fit, the next one through Container.limit (an array stays an array, a bitmap
 * becomes an array at <= 4096 values, a run container keeps its runs up to the cut); maxcardinality <= 0:
 * the empty bitmap */
int rbg_limit(const uint8_t* a, size_t a_len, int32_t maxcard, rbg_buffer* out);
/* RoaringBitmap.bitmapOfRange(min, max) (RB/RoaringBitmap.java:588-615): every container a run container
 * (RunContainer.rangeOfOnes, even for one or two values; static add over an empty bitmap would write
 * arrays there).  rangeSanityCheck -> RBG_ERR_ILLEGAL_ARGUMENT; max <= min: the empty bitmap. */
int rbg_bitmap_of_range(int64_t min, int64_t max, rbg_buffer* out);
/* x.selectRange(rangeStart, rangeEnd) (RB/RoaringBitmap.java:3095-3147): the values in the range, the
 * first / last key's container cut by Container.remove (A stays A, B becomes A at <= 4096 values, R stays
 * R with its runs clipped), the keys between cloned; buffer != 0: ImmutableRoaringBitmap.selectRange
 * (RB/buffer/ImmutableRoaringBitmap.java:701-757), whose bitmaps become arrays below 4096 values.  The
 * reference only asserts the range; here rangeSanityCheck's bounds apply (RBG_ERR_ILLEGAL_ARGUMENT).
 * rangeEnd <= rangeStart: the empty bitmap. */
int rbg_select_range(const uint8_t* a, size_t a_len, int64_t range_start, int64_t range_end, int buffer,
                     rbg_buffer* out);
/* wide cardinalities: andCardinality(RoaringBitmap...) :71-82, orCardinality :90-101 */
enum { RBG_WIDE_CARD_AND = 0, RBG_WIDE_CARD_OR = 1 };

/* static RoaringBitmap.and/or/xor/andNot(RoaringBitmap, RoaringBitmap) -> RoaringBitmap */
int rbg_pairwise(int op, const uint8_t* a, size_t a_len, const uint8_t* b, size_t b_len,
                 rbg_buffer* out);

/* In-place instance ops x1.and(x2) / x1.or(x2) / x1.xor(x2) / x1.andNot(x2) (op RBG_AND..RBG_ANDNOT;
 * RB/RoaringBitmap.java:1272-1296, 2481-2523, 3296-3348, 1346-1382): out = x1's bytes afterwards.
 * same_object != 0 when x2 is x1 itself (and / or leave it unchanged, xor / andNot clear it).
 * and / xor / andNot give the static ops' bytes (iand / ixor / iandNot type alike); or follows
 * Container.ior, whose bitmap | array keeps a full bitmap. */
int rbg_pairwise_inplace(int op, const uint8_t* a, size_t a_len, const uint8_t* b, size_t b_len, int same_object,
                         rbg_buffer* out);

/* static RoaringBitmap.{and,or,xor,andNot}Cardinality / intersects -> int */
int rbg_pairwise_card(int op, const uint8_t* a, size_t a_len, const uint8_t* b, size_t b_len,
                      int32_t* out);

/* FastAggregation.and/or/xor.  `ids` (may be NULL) carries Java object identity:
 * inputs with equal id are the same RoaringBitmap object (naive_and skips
 * `bitmaps[k] != smallest` by reference, RB/FastAggregation.java:341).
 * n == 0 yields the empty bitmap (:329-331). */
int rbg_wide(int op, const uint8_t* const* bufs, const size_t* lens, const int32_t* ids, size_t n,
             rbg_buffer* out);

/* FastAggregation.andCardinality / orCardinality(RoaringBitmap...) -> int */
int rbg_wide_card(int op, const uint8_t* const* bufs, const size_t* lens, size_t n, int32_t* out);

/* Batched andCardinality: out[i] = RoaringBitmap.andCardinality(a_i, b_i).  No reference
 * signature; defined as a loop of RB/RoaringBitmap.java:413-434 (config C4). */
int rbg_batch_and_card(size_t n_pairs, const uint8_t* const* a_bufs, const size_t* a_lens,
                       const uint8_t* const* b_bufs, const size_t* b_lens, int32_t* out);

/* ---- bit-sliced index (bsi/src/main/java/org/roaringbitmap/bsi/RoaringBitmapSliceIndex.java) ----
 * A BSI crosses the boundary as its fields: the serialized existence bitmap ebM, the
 * serialized slices bA[0..nbits-1] (bit 0 first) and minValue / maxValue.
 * op is BitmapSliceIndex.Operation's ordinal (BitmapSliceIndex.java:23-38). */
enum { RBG_BSI_EQ = 0, RBG_BSI_NEQ = 1, RBG_BSI_LE = 2, RBG_BSI_LT = 3, RBG_BSI_GE = 4, RBG_BSI_GT = 5,
       RBG_BSI_RANGE = 6 };
/* compare(op, startOrValue, end, foundSet) -> RoaringBitmap (RoaringBitmapSliceIndex.java:482-513);
 * found may be NULL (foundSet == null). */
int rbg_bsi_compare(int op, int32_t start, int32_t end, const uint8_t* ebm, size_t ebm_len,
                    const uint8_t* const* slices, const size_t* slice_lens, size_t nbits, int32_t min_value,
                    int32_t max_value, const uint8_t* found, size_t found_len, rbg_buffer* out);
/* The buffer package's index, ImmutableBitSliceIndex / MutableBitSliceIndex
 * (bsi/src/main/java/org/roaringbitmap/bsi/buffer/BitSliceIndexBase.java, BBSI/): the same fields,
 * its own compare circuit and ImmutableRoaringBitmap's result types.
 *   op RBG_BSI_EQ .. RBG_BSI_RANGE: compare(op, startOrValue, end, foundSet)   BBSI/:422-453
 *       (rangeEQ / rangeLT / rangeLE / rangeGT / rangeGE / range are compare, BBSI/:351-408)
 *   op RBG_BSI_RANGE_NEQ_DIRECT: rangeNEQ(foundSet, value) called directly      BBSI/:384-387
 *       (it skips compare's NEQ shortcut of compareUsingMinMax, :500-503)
 * sum(foundSet) of this index is rbg_bsi_sum (BBSI/:521-532 is RoaringBitmapSliceIndex.java:581-592). */
#define RBG_BSI_RANGE_NEQ_DIRECT 7
int rbg_bsi_compare_buffer(int op, int32_t start, int32_t end, const uint8_t* ebm, size_t ebm_len,
                           const uint8_t* const* slices, const size_t* slice_lens, size_t nbits, int32_t min_value,
                           int32_t max_value, const uint8_t* found, size_t found_len, rbg_buffer* out);
/* sum(foundSet) -> Pair<Long, Long> (RoaringBitmapSliceIndex.java:581-592): out2 = {sum, count}. */
int rbg_bsi_sum(const uint8_t* ebm, size_t ebm_len, const uint8_t* const* slices, const size_t* slice_lens,
                size_t nbits, const uint8_t* found, size_t found_len, int64_t* out2);

/* Releases an output.  Large results (>= 8 MiB, 2 MiB-aligned huge-page buffers) are kept for
 * reuse by the next large result, at most two of them, so a caller's steady stream of big results
 * does not fault and zero fresh pages every call. */
void rbg_free(rbg_buffer* buf);

/* Select the HIP devices the one-shot calls may use (bit i = device i).  Returns the
 * number of usable devices selected, or RBG_ERR_DEVICE. */
int rbg_set_devices(uint64_t mask);

/* Human-readable message for the last error on this thread. */
const char* rbg_last_error(void);
int rbg_version(void);
/* Result buffers of 8 MiB and more are kept for reuse after rbg_free (at most two, 1 GiB in all, so a
 * repeated large fetch does not fault fresh pages); rbg_trim frees them. */
void rbg_trim(void);
/* Pooled device buffers freed to satisfy an out-of-memory allocation since the library loaded
 * (first the calling context's pool, then the other contexts' on the device). */
uint64_t rbg_pool_evictions(void);

/* ---- host-side format utilities (construction, not the hot path) ----------------
 * RoaringBitmap.bitmapOf(int...) (RB/RoaringBitmap.java:566-570) optionally followed
 * by runOptimize() (:2764-2774); values need not be sorted or distinct. */
int rbg_from_values(const uint32_t* values, size_t n, int run_optimize, rbg_buffer* out);
/* RoaringBitmap.runOptimize() on a serialized bitmap (RB/RoaringBitmap.java:2764-2774),
 * computed on the GPU: the device runOptimize pass of rbg_run_optimize_many over a
 * one-bitmap batch.  Without a usable device it returns RBG_ERR_DEVICE. */
int rbg_run_optimize(const uint8_t* buf, size_t len, rbg_buffer* out);
/* RoaringBitmap.toArray(): ascending values (unsigned); out->data holds n*4 bytes. */
int rbg_to_values(const uint8_t* buf, size_t len, rbg_buffer* out);
/* Validate a serialized bitmap; returns bytes consumed, long cardinality and the
 * container mix (stats[0..2] = #array, #bitmap, #run). */
int rbg_inspect(const uint8_t* buf, size_t len, size_t* consumed, int64_t* cardinality,
                int64_t* stats3);

/* ---- device-resident session API (bench.py, torch integration) ------------------
 * A context owns one HIP stream and a workspace on one device.  Batches are
 * device-resident sets of bitmaps in the engine's key-major arena layout
 * (DESIGN.md §Data layout).  Ops on a context are enqueued asynchronously on its
 * stream; rbg_ctx_sync waits. */
typedef struct rbg_ctx rbg_ctx;
int rbg_ctx_create(int device, rbg_ctx** out);
void rbg_ctx_destroy(rbg_ctx* ctx);
/* hipStream_t of the context, for HIP-event timing by the caller */
void* rbg_ctx_stream(rbg_ctx* ctx);
int rbg_ctx_sync(rbg_ctx* ctx);
/* HIP-event phase timing on the context stream: enable for up to max_ops ops (0 disables).
 * rbg_ctx_profile_read returns the summed device time of the recorded ops in three phases:
 * ms3[0] = key plan + compaction, ms3[1] = container compute kernel, ms3[2] = result
 * assembly (finalize + emit / reduction), and resets the record. */
int rbg_ctx_profile(rbg_ctx* ctx, int max_ops);
/* The same with two events per op, around the container compute kernel only (ms3[1]; ms3[0] and
 * ms3[2] read 0): the least added to a timed loop of back-to-back ops. */
int rbg_ctx_profile_compute(rbg_ctx* ctx, int max_ops);
int rbg_ctx_profile_read(rbg_ctx* ctx, double* ms3, int* n_ops);
/* Bytes read by the early-exit wide AND (workShyAnd stops reading a key's inputs once the
 * intersection is empty: payload + 4 B per container it read) over the ops run since
 * rbg_ctx_profile enabled profiling; the algorithmic input of that kernel. */
int rbg_ctx_profile_bytes(rbg_ctx* ctx, int64_t* bytes);

/* n serialized bitmaps in one upload, each decoded into a single-bitmap batch of its own
 * (ids[i]): the operands of pairwise ops, staged and copied to the device together. */
int rbg_ctx_load_separate(rbg_ctx* ctx, const uint8_t* const* bufs, const size_t* lens, size_t n, int32_t* ids);
/* Parse + upload n serialized bitmaps as one batch; returns a batch id >= 0. */
int rbg_ctx_load(rbg_ctx* ctx, const uint8_t* const* bufs, const size_t* lens, size_t n,
                 int32_t* batch);
/* The same for a batch that feeds wide ops: when every container is an array, the array payloads
 * stay packed back to back at 2 B granularity as in the portable format (RB/RoaringArray.java:547-629)
 * instead of 16 B slots -- the layout FastAggregation.or / xor / workShyAnd (and the queue, horizontal
 * and parallel forms) read fastest.  Such a batch serves those wide ops, the wide cardinalities and
 * fetches; pairwise, BSI, runOptimize, naive_and chains and batched andCardinality refuse it
 * (RBG_ERR_ILLEGAL_ARGUMENT).  A batch holding bitmap or run containers is decoded as rbg_ctx_load does.
 * Replaces nothing in the reference: its deserializer keeps each container's own array (same bytes). */
int rbg_ctx_load_packed(rbg_ctx* ctx, const uint8_t* const* bufs, const size_t* lens, size_t n,
                        int32_t* batch);
/* Synthetic batches generated on the device (bench configs).
 *   kind 0: C2 operand: one bitmap, all 65536 keys, per key A/B/R with p=1/3 (seed)
 *   kind 1: C3 uniform: n bitmaps x keys [key_lo,key_hi), ~15.26 values per (bitmap,key)
 *   kind 2: C3 clustered: n bitmaps, 16 dense bitmap keys each, restricted to [key_lo,key_hi)
 *   kind 4: C5 bit-sliced index over n rows (value = hash & 0x7FFFFFFF, 31 slices) as the batch
 *           [ebM, bA[0..30]] of rbg_ctx_bsi (runOptimize'd types); min / max: rbg_ctx_batch_minmax
 *   kind 3: C4 pairs: n pairs = 2n bitmaps, bitmap-major (pairs adjacent), 1-4 array keys in
 *           [0,64) each, card 16..512 (key_lo / key_hi ignored) */
int rbg_ctx_synth(rbg_ctx* ctx, int kind, uint64_t seed, size_t n, int key_lo, int key_hi,
                  int32_t* batch);
/* Drops a batch.  Its device buffers (up to 2 GiB per context, none above 1 GiB) are kept for
 * reuse by later batches of the context and freed with it (rbg_ctx_destroy). */
int rbg_ctx_release(rbg_ctx* ctx, int32_t batch);
/* selectRangeWithoutCopy of every bitmap of a key-major batch into a new batch (the first step of the
 * RBG_RANGE_* ops, on the device; synchronous: one read-back of the new batch's container counts). */
int rbg_ctx_select_range(rbg_ctx* ctx, int32_t batch, int64_t range_start, int64_t range_end, int32_t* out_batch);
/* RoaringBitmap.runOptimize() (RB/RoaringBitmap.java:2764-2774) applied on the device to
 * every bitmap of a batch; the result is a new batch (same bitmaps, keys and order).
 * answers (n bitmaps, nullable) receives runOptimize's boolean per bitmap.  Also backs
 * RoaringBitmapSliceIndex.runOptimize (bsi/.../RoaringBitmapSliceIndex.java:141-150). */
int rbg_ctx_run_optimize(rbg_ctx* ctx, int32_t batch, int32_t* out_batch, uint8_t* answers);
/* One-shot form: runOptimize each of n serialized bitmaps on the device; outs[i] receives
 * the optimized bytes (free each with rbg_free), answers[i] (nullable) the boolean. */
int rbg_run_optimize_many(const uint8_t* const* bufs, const size_t* lens, size_t n, rbg_buffer* outs,
                          uint8_t* answers);
/* min / max of the values of a synthetic C5 batch (out2). */
int rbg_ctx_batch_minmax(rbg_ctx* ctx, int32_t batch, int32_t* out2);
/* Batch facts: stats[0..7] = bitmaps, containers, #array, #bitmap, #run, payload bytes,
 * long cardinality, serialized bytes. (synchronous) */
int rbg_ctx_batch_stats(rbg_ctx* ctx, int32_t batch, int64_t* stats8);
/* Download bitmap i of a batch as serialized bytes (synchronous). */
int rbg_ctx_batch_fetch(rbg_ctx* ctx, int32_t batch, size_t i, rbg_buffer* out);
/* Download bitmaps [first, first + count) of a batch: outs[k] receives bitmap first + k
 * (free each with rbg_free).  One device gather and one copy for the whole range. */
int rbg_ctx_batch_fetch_range(rbg_ctx* ctx, int32_t batch, size_t first, size_t count, rbg_buffer* outs);

/* Enqueue a pairwise op between bitmap ia of batch a and bitmap ib of batch b.  The
 * result is materialised on the device (containers in slots + a compacted
 * container table, the counterpart of the Java result object); it is turned into
 * the portable format only by rbg_ctx_serialize / rbg_ctx_fetch. */
int rbg_ctx_pairwise(rbg_ctx* ctx, int op, int32_t a, size_t ia, int32_t b, size_t ib);
/* rbg_ctx_pairwise followed by rbg_ctx_serialize (RoaringBitmap.and/or/xor/andNot, then serialize,
 * RB/RoaringBitmap.java:377-473,3017-3019), as one pipeline: the key universe is cut into
 * RBG_SER_PIPE (default 4) ranges and range r's placement and payload copies run on a second stream
 * while range r + 1 computes.  The same bytes as the two calls. */
int rbg_ctx_pairwise_serialized(rbg_ctx* ctx, int op, int32_t a, size_t ia, int32_t b, size_t ib);
/* rbg_ctx_pairwise restricted to keys [key_lo, key_hi): one key-range shard of the op (each
 * key's result depends on that key's containers only, RB/RoaringBitmap.java:382-399); the
 * shards of a partition are assembled with rbg_ctx_fetch_shard(_device). */
int rbg_ctx_pairwise_range(rbg_ctx* ctx, int op, int32_t a, size_t ia, int32_t b, size_t ib, int key_lo, int key_hi);
/* rbg_ornot over device-resident single-bitmap batches; the result pending like rbg_ctx_pairwise's */
int rbg_ctx_ornot(rbg_ctx* ctx, int32_t a, size_t ia, int32_t b, size_t ib, int64_t range_end, int flags);
/* rbg_range_mut over a device-resident single-bitmap batch; the result pending like rbg_ctx_pairwise's */
int rbg_ctx_range_mut(rbg_ctx* ctx, int op, int32_t batch, size_t i, int64_t range_start, int64_t range_end);
/* rbg_add_offset over a device-resident single-bitmap batch; the result pending like rbg_ctx_pairwise's */
int rbg_ctx_add_offset(rbg_ctx* ctx, int32_t batch, size_t i, int64_t offset);
/* Enqueue a cardinality op; the int32 lands in device memory, read by rbg_ctx_card. */
int rbg_ctx_pairwise_card(rbg_ctx* ctx, int op, int32_t a, size_t ia, int32_t b, size_t ib);
/* Enqueue a wide op over every bitmap of a batch, restricted to keys [key_lo, key_hi)
 * (key-range sharding; use 0, 65536 for the whole universe).  The chain-order
 * decisions of FastAggregation (smallest input, identity skips) use `ids` as in
 * rbg_wide (may be NULL). */
int rbg_ctx_wide(rbg_ctx* ctx, int op, int32_t batch, int key_lo, int key_hi, const int32_t* ids);
int rbg_ctx_wide_card(rbg_ctx* ctx, int op, int32_t batch, int key_lo, int key_hi);
/* rbg_ctx_wide with the naive_and start input given by the caller (start_bm >= 0).
 * A key-range shard passes the input with the fewest containers over the whole
 * universe (RB/FastAggregation.java:333-339), which its key slice cannot see. */
int rbg_ctx_wide_start(rbg_ctx* ctx, int op, int32_t batch, int key_lo, int key_hi, const int32_t* ids,
                       int32_t start_bm);
/* Algorithmic input bytes of batched andCardinality over the pairs of a bitmap-major
 * batch (array / bitmap payloads; synthetic C4 batches have no run containers):
 * out2[0] = matched payload + 4 B per descriptor, out2[1] = all of it. */
int rbg_ctx_pair_bytes(rbg_ctx* ctx, int32_t batch, int64_t* out2);
/* BSI over a device-resident key-major batch [ebM, bA[0..nbits-1], foundSet if has_found]:
 * op = RBG_BSI_* (compare; min/max decide compareUsingMinMax's shortcuts) or 8 = sum(foundSet)
 * alone; want_sum fuses sum(result) into the compare pass.  The result is fetched like any
 * other (rbg_ctx_fetch); rbg_ctx_bsi_sums returns {sum, count} of the last BSI call. */
int rbg_ctx_bsi(rbg_ctx* ctx, int32_t batch, int op, int nbits, int has_found, int32_t start, int32_t end,
                int32_t min_value, int32_t max_value, int want_sum);
int rbg_ctx_bsi_sums(rbg_ctx* ctx, int64_t* out2);
/* rbg_bsi_compare_buffer over a device-resident batch (op as there); synchronous (the result's
 * run containers above 2047 runs have an arena whose size is checked after the op). */
int rbg_ctx_bsi_buffer(rbg_ctx* ctx, int32_t batch, int op, int nbits, int has_found, int32_t start, int32_t end,
                       int32_t min_value, int32_t max_value);
/* The same {sum, count} (two int64) copied to device memory dst2, enqueued on the context
 * stream (no host synchronisation: the sum stays on the device, e.g. for an all-reduce). */
int rbg_ctx_bsi_sums_device(rbg_ctx* ctx, void* dst2);
/* From now on every rbg_ctx_bsi with want_sum also writes its {sum, count} (two int64) to device
 * memory dst2, in the kernel that computes them (no copy launch); null stops it. */
int rbg_ctx_bsi_sums_target(rbg_ctx* ctx, void* dst2);
/* Retired diagnostic (the per-phase clock builds of rounds 2-5 are gone; their results are in
 * profiles/): writes 20 zeros.  Kept so bindings of earlier rounds still link. */
int rbg_debug_stamps(uint64_t* out20, int reset);
/* Containers per input bitmap of a batch (out has n == bitmaps entries). */
int rbg_ctx_batch_counts(rbg_ctx* ctx, int32_t batch, uint32_t* out, size_t n);
/* Algorithmic input bytes per key (payload + 4 B descriptor per container) of the
 * synthetic C3 workloads (kind 1 uniform, 2 clustered), for key-range partitioning
 * by equal bytes; out has 65536 entries.  Host only. */
int rbg_synth_key_bytes(int kind, uint64_t seed, size_t n, uint64_t* out);
/* Enqueue batched andCardinality over pairs (2i, 2i+1) of a batch; results stay on device. */
int rbg_ctx_batch_and_card(rbg_ctx* ctx, int32_t batch);

/* Result access (synchronous). */
int rbg_ctx_card(rbg_ctx* ctx, int32_t* out);
int rbg_ctx_cards(rbg_ctx* ctx, int32_t* out, size_t n);
/* stats[0..3] = containers, payload bytes, has_run, long cardinality of the last
 * result (before header).  Used for the cross-shard allgather. */
int rbg_ctx_result_stats(rbg_ctx* ctx, int64_t* stats4);
/* Enqueue the portable serialization of the last result on the device
 * (RoaringBitmap.serialize, RB/RoaringArray.java:896-940); idempotent.  Fetch
 * calls it implicitly. */
int rbg_ctx_serialize(rbg_ctx* ctx);
/* Serialized bytes of the last result (a standalone portable bitmap). */
int rbg_ctx_fetch(rbg_ctx* ctx, rbg_buffer* out);
/* Key-range shard assembly: write this shard's descriptors / offsets / payloads into
 * a global serialized bitmap whose header is described by (total containers,
 * has_run, this shard's first container index, this shard's payload byte offset
 * within the global payload region).  Returns this shard's byte slices:
 * out_desc (descriptors), out_offsets (offset table, may be empty), out_payload. */
int rbg_ctx_fetch_shard(rbg_ctx* ctx, int64_t total_containers, int has_run,
                        int64_t first_container, int64_t payload_base, rbg_buffer* out_desc,
                        rbg_buffer* out_offsets, rbg_buffer* out_payload);
/* Device form of rbg_ctx_fetch_shard, enqueued on the context stream (no host copy): the
 * pending result's n containers are written as a key shard of the global bitmap straight
 * into device memory -- desc_dst (4n bytes), offsets_dst (4n bytes of the global offset
 * table; required iff the global bitmap has one: !has_run || total_containers >= 4),
 * runflag_dst (n bytes, 1 = run container; used iff has_run, nullable otherwise) and
 * payload_dst (this shard's payload bytes).  Any byte alignment.  Destinations may be
 * views into the final global bitmap (each shard writes its slice at its
 * global offset); the run-flag bytes are packed into the header by the assembler. */
int rbg_ctx_fetch_shard_device(rbg_ctx* ctx, int64_t total_containers, int has_run, int64_t payload_base,
                               void* desc_dst, void* offsets_dst, void* runflag_dst, void* payload_dst);
/* The layout exchange without host synchronisation (SURVEY §8(e) steps 1-2 on the device):
 * rbg_ctx_result_layout_device writes the pending result's (containers, payload bytes, has_run) as
 * three int64 into device memory dst3, enqueued on the context stream -- the input of a device
 * all-gather (RCCL).  rbg_ctx_fetch_shard_device_dyn then reads the gathered layout from device
 * memory (world x 3 int64, ranks in key-range order) and writes this rank's slice into `out`, a
 * buffer laid out as the whole global bitmap (descriptors, offset-table entries and payload at
 * their global places; rank 0 also the cookie), and one run byte per global container into runb
 * (needed when any shard has run containers; packed into the header by the assembler).  `out`
 * must hold header + all payload bytes of the global bitmap: 8 + 8 * 65536 + 8194 * 65536 bytes
 * bound any layout. */
int rbg_ctx_result_layout_device(rbg_ctx* ctx, void* dst3);
int rbg_ctx_fetch_shard_device_dyn(rbg_ctx* ctx, const void* layout, int rank, int world, void* out, void* runb);

#ifdef __cplusplus
}
#endif
#endif /* ROARING_MI355X_H */
