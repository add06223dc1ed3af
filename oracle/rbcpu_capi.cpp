// C entry points of the CPU ORACLE (test infrastructure only; see rbcpu.hpp).
// Loaded through ctypes by tests/ and by bench.py's cpu_baseline leg.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <cstdlib>
#include <cstring>
#include <map>
#include <thread>
#include <vector>

#include "rbcpu.hpp"

using namespace rbcpu;

namespace {
int emit(const Bitmap& b, uint8_t** out, size_t* out_len) {
  std::vector<uint8_t> s = serialize(b);
  uint8_t* p = (uint8_t*)std::malloc(s.size() ? s.size() : 1);
  if (!p) return ERR_ARG;
  std::memcpy(p, s.data(), s.size());
  *out = p;
  *out_len = s.size();
  return OK;
}
int load(const uint8_t* p, size_t n, Bitmap* b) {
  size_t used = 0;
  return deserialize(p, n, b, &used);
}
int load_many(const uint8_t* const* bufs, const size_t* lens, size_t n, std::vector<Bitmap>* bms,
              std::vector<const Bitmap*>* ptrs) {
  bms->resize(n);
  for (size_t i = 0; i < n; i++) {
    int st = load(bufs[i], lens[i], &(*bms)[i]);
    if (st != OK) return st;
  }
  ptrs->clear();
  for (size_t i = 0; i < n; i++) ptrs->push_back(&(*bms)[i]);
  return OK;
}
double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
}  // namespace

extern "C" {

void rbo_free(void* p) { std::free(p); }

// op: 0 and, 1 or, 2 xor, 3 andNot   (RB/RoaringBitmap.java:377,860,1071,444);
// 4 and, 5 andNot of the buffer package (ImmutableRoaringBitmap.and :299, andNot :441);
// 6 x1.or(x2) in place (RB/RoaringBitmap.java:2481)
int rbo_pairwise(int op, const uint8_t* a, size_t an, const uint8_t* b, size_t bn, uint8_t** out,
                 size_t* out_len) {
  Bitmap x, y;
  int st = load(a, an, &x);
  if (st) return st;
  if ((st = load(b, bn, &y))) return st;
  switch (op) {
    case 0: return emit(op_and(x, y), out, out_len);
    case 1: return emit(op_or(x, y), out, out_len);
    case 2: return emit(op_xor(x, y), out, out_len);
    case 3: return emit(op_andnot(x, y), out, out_len);
    case 4: return emit(op_and_buf(x, y), out, out_len);
    case 5: return emit(op_andnot_buf(x, y), out, out_len);
    case 6: return emit(op_ior(x, y), out, out_len);
  }
  return ERR_ARG;
}

// op: 0 andCardinality, 1 orCardinality, 2 xorCardinality, 3 andNotCardinality, 4 intersects
int rbo_pairwise_card(int op, const uint8_t* a, size_t an, const uint8_t* b, size_t bn, int32_t* out) {
  Bitmap x, y;
  int st = load(a, an, &x);
  if (st) return st;
  if ((st = load(b, bn, &y))) return st;
  switch (op) {
    case 0: *out = op_and_card(x, y); return OK;
    case 1: *out = op_or_card(x, y); return OK;
    case 2: *out = op_xor_card(x, y); return OK;
    case 3: *out = op_andnot_card(x, y); return OK;
    case 4: *out = op_intersects(x, y) ? 1 : 0; return OK;
  }
  return ERR_ARG;
}

// op: 0 FastAggregation.and(varargs), 1 or, 2 xor, 3 and(Iterator), 4 naive_and, 5 workShyAnd,
//     6 ParallelAggregation.or, 7 ParallelAggregation.xor, 8 BufferFastAggregation.or(Mutable...),
//     9 FastAggregation.horizontal_or(varargs/List), 10 horizontal_xor, 11 priorityqueue_or,
//     12 priorityqueue_xor, 13 BufferFastAggregation.and(Immutable...), 14 BufferFastAggregation.naive_and
//     (Immutable...), 15 BufferFastAggregation.naive_and(Iterator / Mutable...)
int rbo_wide(int op, const uint8_t* const* bufs, const size_t* lens, size_t n, const int* ids,
             uint8_t** out, size_t* out_len) {
  std::vector<Bitmap> bms;
  std::vector<const Bitmap*> ptrs;
  int st = load_many(bufs, lens, n, &bms, &ptrs);
  if (st) return st;
  switch (op) {
    case 0: return emit(fa_and(ptrs, ids), out, out_len);
    case 1: return emit(fa_or(ptrs), out, out_len);
    case 2: return emit(fa_xor(ptrs), out, out_len);
    case 3: return emit(fa_and_iter(ptrs), out, out_len);
    case 4: return emit(fa_naive_and(ptrs, ids), out, out_len);
    case 5: return emit(n ? fa_workshy_and(ptrs) : Bitmap(), out, out_len);
    case 6: return emit(pa_or(ptrs), out, out_len);
    case 7: return emit(pa_xor(ptrs), out, out_len);
    case 8: return emit(buf_or_mutable(ptrs), out, out_len);
    case 9: return emit(fa_horizontal_or(ptrs), out, out_len);
    case 10: return emit(fa_horizontal_xor(ptrs), out, out_len);
    case 11: return emit(fa_priorityqueue_or(ptrs), out, out_len);
    case 12: return emit(fa_priorityqueue_xor(ptrs), out, out_len);
    case 13: return emit(buf_and(ptrs, ids), out, out_len);
    case 14: return emit(buf_naive_and(ptrs, ids), out, out_len);
    case 15: return emit(buf_and_iter(ptrs), out, out_len);
  }
  return ERR_ARG;
}

// RoaringBitmap.and / or / xor(Iterator, rangeStart, rangeEnd) (op 0 / 1 / 2) and andNot(x1, x2,
// rangeStart, rangeEnd) (op 3, n == 2): RB/RoaringBitmap.java:1308-1336, 2536-2557, 3359-3379, 1396-1423.
// op 4: selectRangeWithoutCopy alone; ops 5-8: ImmutableRoaringBitmap's and / or / xor / andNot range
// forms (RB/buffer/ImmutableRoaringBitmap.java:261, 992, 1048, 402); op 9: the buffer selection alone.
// rangeSanityCheck (:204-213) -> ERR_ARG.
int rbo_range_op(int op, const uint8_t* const* bufs, const size_t* lens, size_t n, int64_t start, int64_t end,
                 uint8_t** out, size_t* out_len) {
  if (start < 0 || start > 0xFFFFFFFFll || end < 0 || end > 0x100000000ll) return ERR_ARG;
  std::vector<Bitmap> bms;
  std::vector<const Bitmap*> ptrs;
  int st = load_many(bufs, lens, n, &bms, &ptrs);
  if (st) return st;
  if (op == 3) {
    if (n != 2) return ERR_ARG;
    return emit(op_andnot_range(bms[0], bms[1], (uint64_t)start, (uint64_t)end), out, out_len);
  }
  if (op == 4 || op == 9) {  // selectRangeWithoutCopy alone (n == 1)
    if (n != 1) return ERR_ARG;
    return emit(select_range(bms[0], (uint64_t)start, (uint64_t)end, op == 9), out, out_len);
  }
  if (op >= 5 && op <= 8) {
    if (op == 8 && n != 2) return ERR_ARG;
    return emit(range_aggregate_buf(op - 5, ptrs, (uint64_t)start, (uint64_t)end), out, out_len);
  }
  if (op < 0 || op > 2) return ERR_ARG;
  return emit(range_aggregate(op, ptrs, (uint64_t)start, (uint64_t)end), out, out_len);
}

// RoaringBitmap.orNot(x1, x2, rangeEnd) (flags 0, RB/RoaringBitmap.java:1521-1603) and
// x1.orNot(x2, rangeEnd) (flags 1, :1431-1506); flags | 2: the buffer package's (ImmutableRoaringBitmap /
// MutableRoaringBitmap.orNot, RB/buffer/ImmutableRoaringBitmap.java:484-548, MutableRoaringBitmap.java:962).
// rangeSanityCheck(0, rangeEnd) -> ERR_ARG; a negative maxSize (the reference's NegativeArraySizeException) -> ERR_ARG with *neg = 1.
int rbo_ornot(const uint8_t* a, size_t an, const uint8_t* b, size_t bn, int64_t range_end, int flags,
              int* neg, uint8_t** out, size_t* out_len) {
  *neg = 0;
  if (range_end < 0 || range_end > 0x100000000ll) return ERR_ARG;
  Bitmap x, y;
  int st = load(a, an, &x);
  if (st) return st;
  if ((st = load(b, bn, &y))) return st;
  bool ng = false;
  Bitmap r = op_ornot(x, y, (uint64_t)range_end, (flags & 1) != 0, &ng, (flags & 2) != 0);
  if (ng) {
    *neg = 1;
    return ERR_ARG;
  }
  return emit(r, out, out_len);
}

// static add / remove / flip(rb, rangeStart, rangeEnd) (op 0 / 1 / 2, RB/RoaringBitmap.java:298, 995, 626);
// op 3: x.add(rangeStart, rangeEnd) in place (:1181);
// op | 4: MutableRoaringBitmap's (RB/buffer/MutableRoaringBitmap.java:152, 649, 455).  rangeSanityCheck -> ERR_ARG.
int rbo_range_mut(int op, const uint8_t* a, size_t an, int64_t start, int64_t end, uint8_t** out, size_t* out_len) {
  if (start < 0 || start > 0xFFFFFFFFll || end < 0 || end > 0x100000000ll || op < 0 || op > 7) return ERR_ARG;
  Bitmap x;
  int st = load(a, an, &x);
  if (st) return st;
  return emit(op_range_mut(op & 3, x, (uint64_t)start, (uint64_t)end, (op & 4) != 0), out, out_len);
}

// RoaringBitmap.addOffset(x, offset) (RB/RoaringBitmap.java:230-288)
int rbo_add_offset(const uint8_t* a, size_t an, int64_t offset, uint8_t** out, size_t* out_len) {
  Bitmap x;
  int st = load(a, an, &x);
  if (st) return st;
  return emit(op_add_offset(x, offset), out, out_len);
}

// RoaringBitmap.bitmapOfRange(min, max) (RB/RoaringBitmap.java:588-615); rangeSanityCheck -> ERR_ARG
int rbo_bitmap_of_range(int64_t min, int64_t max, uint8_t** out, size_t* out_len) {
  if (min < 0 || min > 0xFFFFFFFFll || max < 0 || max > 0x100000000ll) return ERR_ARG;
  return emit(op_bitmap_of_range((uint64_t)min, (uint64_t)max), out, out_len);
}

// x.limit(maxcardinality) (RB/RoaringBitmap.java:2457-2476)
int rbo_limit(const uint8_t* a, size_t an, int32_t maxcard, uint8_t** out, size_t* out_len) {
  Bitmap x;
  int st = load(a, an, &x);
  if (st) return st;
  return emit(op_limit(x, maxcard), out, out_len);
}

// x.removeRunCompression() (RB/RoaringBitmap.java:2738-2749)
int rbo_remove_run_compression(const uint8_t* a, size_t an, uint8_t** out, size_t* out_len) {
  Bitmap x;
  int st = load(a, an, &x);
  if (st) return st;
  return emit(op_remove_run_compression(x), out, out_len);
}

// RoaringBitmap.getLongSizeInBytes of a serialized bitmap (RB/RoaringBitmap.java:2212-2219)
int64_t rbo_long_size(const uint8_t* a, size_t an) {
  Bitmap b;
  if (load(a, an, &b)) return -1;
  return long_size_in_bytes(b);
}

// op: 0 andCardinality(varargs), 1 orCardinality(varargs)
int rbo_wide_card(int op, const uint8_t* const* bufs, const size_t* lens, size_t n, int32_t* out) {
  std::vector<Bitmap> bms;
  std::vector<const Bitmap*> ptrs;
  int st = load_many(bufs, lens, n, &bms, &ptrs);
  if (st) return st;
  if (op == 0) { *out = fa_and_card(ptrs); return OK; }
  if (op == 1) { *out = fa_or_card(ptrs); return OK; }
  return ERR_ARG;
}

int rbo_from_values(const uint32_t* vals, size_t n, int run_optimize, uint8_t** out, size_t* out_len) {
  Bitmap b = bitmap_of(vals, n);
  if (run_optimize) bitmap_run_optimize(b);
  return emit(b, out, out_len);
}

int rbo_run_optimize(const uint8_t* a, size_t an, uint8_t** out, size_t* out_len) {
  Bitmap b;
  int st = load(a, an, &b);
  if (st) return st;
  bitmap_run_optimize(b);
  return emit(b, out, out_len);
}

int rbo_to_values(const uint8_t* a, size_t an, uint32_t** out, size_t* n) {
  Bitmap b;
  int st = load(a, an, &b);
  if (st) return st;
  std::vector<uint32_t> v = bitmap_values(b);
  uint32_t* p = (uint32_t*)std::malloc((v.size() ? v.size() : 1) * 4);
  std::memcpy(p, v.data(), v.size() * 4);
  *out = p;
  *n = v.size();
  return OK;
}

// deserialize then serialize (byte round trip); *consumed = bytes read
int rbo_roundtrip(const uint8_t* a, size_t an, uint8_t** out, size_t* out_len, size_t* consumed) {
  Bitmap b;
  int st = deserialize(a, an, &b, consumed);
  if (st) return st;
  return emit(b, out, out_len);
}

// stats[0..4] = #array, #bitmap, #run, cardinality(long), payload bytes
int rbo_stats(const uint8_t* a, size_t an, int64_t* stats) {
  Bitmap b;
  int st = load(a, an, &b);
  if (st) return st;
  std::memset(stats, 0, 5 * sizeof(int64_t));
  for (const Ctr& c : b.ctrs) {
    stats[c.kind]++;
    stats[4] += c.array_size_bytes();
  }
  stats[3] = b.long_card();
  return OK;
}

// ---- timing helpers for bench.py's cpu_baseline (inputs parsed outside the clock) ----
// Runs `reps` pairwise ops (op as rbo_pairwise, 4 = andCardinality); returns seconds.
double rbo_time_pairwise(int op, const uint8_t* a, size_t an, const uint8_t* b, size_t bn, int reps) {
  Bitmap x, y;
  if (load(a, an, &x) || load(b, bn, &y)) return -1.0;
  volatile int64_t sink = 0;
  double t0 = now_s();
  for (int r = 0; r < reps; r++) {
    switch (op) {
      case 0: sink += (int64_t)op_and(x, y).size(); break;
      case 1: sink += (int64_t)op_or(x, y).size(); break;
      case 2: sink += (int64_t)op_xor(x, y).size(); break;
      case 3: sink += (int64_t)op_andnot(x, y).size(); break;
      case 4: sink += op_and_card(x, y); break;
    }
  }
  return now_s() - t0;
}

// Runs `reps` wide ops (op as rbo_wide 0..2) over n inputs; returns seconds.
double rbo_time_wide(int op, const uint8_t* const* bufs, const size_t* lens, size_t n, int reps) {
  std::vector<Bitmap> bms;
  std::vector<const Bitmap*> ptrs;
  if (load_many(bufs, lens, n, &bms, &ptrs)) return -1.0;
  volatile int64_t sink = 0;
  double t0 = now_s();
  for (int r = 0; r < reps; r++) {
    switch (op) {
      case 0: sink += (int64_t)fa_and(ptrs, nullptr).size(); break;
      case 1: sink += (int64_t)fa_or(ptrs).size(); break;
      case 2: sink += (int64_t)fa_xor(ptrs).size(); break;
    }
  }
  return now_s() - t0;
}

// ---- multi-threaded legs (key-parallel, like ParallelAggregation's ForkJoin stream over
// keys, RB/ParallelAggregation.java:171-173): `threads` workers take key groups from a
// shared counter.  op 0: ParallelAggregation.or, 1: ParallelAggregation.xor.  Returns
// seconds for `reps` runs (inputs parsed outside the clock; groupByKey inside, as in Java).
double rbo_time_wide_parallel(int op, const uint8_t* const* bufs, const size_t* lens, size_t n, int threads,
                              int reps) {
  std::vector<Bitmap> bms;
  std::vector<const Bitmap*> ptrs;
  if (load_many(bufs, lens, n, &bms, &ptrs)) return -1.0;
  volatile int64_t sink = 0;
  double t0 = now_s();
  for (int r = 0; r < reps; r++) {
    std::map<uint16_t, std::vector<const Ctr*>> g;  // groupByKey :137-153
    for (const Bitmap* b : ptrs)
      for (size_t i = 0; i < b->size(); i++) g[b->keys[i]].push_back(&b->ctrs[i]);
    std::vector<const std::vector<const Ctr*>*> slices;
    std::vector<uint16_t> keys;
    for (auto& kv : g) {
      keys.push_back(kv.first);
      slices.push_back(&kv.second);
    }
    std::vector<Ctr> vals(slices.size());
    std::atomic<size_t> next{0};
    std::vector<std::thread> th;
    for (int t = 0; t < std::max(1, threads); t++)
      th.emplace_back([&]() {
        for (size_t k; (k = next.fetch_add(16)) < slices.size();)
          for (size_t j = k; j < std::min(slices.size(), k + 16); j++)
            vals[j] = op == 0 ? pa_or_key(*slices[j]) : pa_xor_key(*slices[j]);
      });
    for (auto& x : th) x.join();
    Bitmap ans;
    for (size_t j = 0; j < vals.size(); j++)
      if (op == 0 || !vals[j].empty()) {
        ans.keys.push_back(keys[j]);
        ans.ctrs.push_back(std::move(vals[j]));
      }
    sink += (int64_t)ans.size();
  }
  return now_s() - t0;
}

// Key-parallel RoaringBitmap.and(x1, x2) (the per-key container AND of :377-401 over
// `threads` contiguous key ranges); seconds for `reps` runs.
double rbo_time_and_parallel(const uint8_t* a, size_t an, const uint8_t* b, size_t bn, int threads, int reps) {
  Bitmap x, y;
  if (load(a, an, &x) || load(b, bn, &y)) return -1.0;
  const int T = std::max(1, threads);
  volatile int64_t sink = 0;
  double t0 = now_s();
  for (int r = 0; r < reps; r++) {
    std::vector<Bitmap> part(T);
    std::vector<std::thread> th;
    for (int t = 0; t < T; t++)
      th.emplace_back([&, t]() {
        const int klo = (65536 * t) / T, khi = (65536 * (t + 1)) / T;
        size_t p1 = std::lower_bound(x.keys.begin(), x.keys.end(), (uint16_t)klo) - x.keys.begin();
        size_t p2 = std::lower_bound(y.keys.begin(), y.keys.end(), (uint16_t)klo) - y.keys.begin();
        Bitmap& o = part[t];
        while (p1 < x.size() && p2 < y.size() && x.keys[p1] < khi && y.keys[p2] < khi) {
          if (x.keys[p1] == y.keys[p2]) {
            Ctr c = c_and(x.ctrs[p1], y.ctrs[p2]);
            if (!c.empty()) {
              o.keys.push_back(x.keys[p1]);
              o.ctrs.push_back(std::move(c));
            }
            p1++;
            p2++;
          } else if (x.keys[p1] < y.keys[p2]) {
            p1++;
          } else {
            p2++;
          }
        }
      });
    for (auto& z : th) z.join();
    for (auto& p : part) sink += (int64_t)p.size();
  }
  return now_s() - t0;
}

// C1 / C4 legs: a loop of RoaringBitmap.and(x1, x2).getCardinality() (op 0, :377-401) or
// RoaringBitmap.andCardinality (op 4, :413-434) over the pairs (bufs[2i], bufs[2i+1]),
// split into `threads` contiguous ranges; seconds for `reps` passes (inputs parsed outside
// the clock).
double rbo_time_pairs(int op, const uint8_t* const* bufs, const size_t* lens, size_t n_pairs, int threads, int reps) {
  std::vector<Bitmap> bms;
  std::vector<const Bitmap*> ptrs;
  if (load_many(bufs, lens, 2 * n_pairs, &bms, &ptrs)) return -1.0;
  const int T = std::max(1, threads);
  std::vector<int64_t> sinks(T, 0);
  double t0 = now_s();
  for (int r = 0; r < reps; r++) {
    std::vector<std::thread> th;
    for (int t = 0; t < T; t++)
      th.emplace_back([&, t]() {
        const size_t lo = n_pairs * t / T, hi = n_pairs * (t + 1) / T;
        int64_t s = 0;
        for (size_t i = lo; i < hi; i++)
          s += op == 4 ? op_and_card(bms[2 * i], bms[2 * i + 1]) : op_and(bms[2 * i], bms[2 * i + 1]).long_card();
        sinks[t] += s;
      });
    for (auto& x : th) x.join();
  }
  const double dt = now_s() - t0;
  volatile int64_t sink = 0;
  for (int64_t v : sinks) sink += v;
  return dt;
}

// C5 leg: RoaringBitmapSliceIndex.compare(RANGE, lo, hi, null) + sum(result) on the heap
// BSI (bsi/src/main/java/org/roaringbitmap/bsi/RoaringBitmapSliceIndex.java): the O'Neil
// circuit oNeilCompare (:432-468) for GE lo and LE hi, their and (:508-511), then
// sum = sum over slices of (1 << x) * andCardinality(bA[x], found) (:581-592).  bufs[0] = ebM,
// bufs[1..nbits] = bA; single thread, as the heap BSI is; seconds for `reps` queries.
static Bitmap oneil(const Bitmap& ebm, const std::vector<Bitmap>& ba, bool ge, uint32_t predicate) {
  Bitmap gt, lt, eq = ebm;
  for (int i = (int)ba.size() - 1; i >= 0; i--) {
    if ((predicate >> i) & 1) {
      lt = op_or(lt, op_andnot(eq, ba[i]));
      eq = op_and(eq, ba[i]);
    } else {
      gt = op_or(gt, op_and(eq, ba[i]));
      eq = op_andnot(eq, ba[i]);
    }
  }
  eq = op_and(ebm, eq);                  // fixedFoundSet = ebM
  return ge ? op_or(gt, eq) : op_or(lt, eq);
}
double rbo_time_bsi_range_sum(const uint8_t* const* bufs, const size_t* lens, int nbits, uint32_t lo, uint32_t hi,
                              int reps, int64_t* out2) {
  std::vector<Bitmap> bms;
  std::vector<const Bitmap*> ptrs;
  if (load_many(bufs, lens, (size_t)nbits + 1, &bms, &ptrs)) return -1.0;
  const Bitmap& ebm = bms[0];
  std::vector<Bitmap> ba(bms.begin() + 1, bms.end());
  int64_t sum = 0, count = 0;
  double t0 = now_s();
  for (int r = 0; r < reps; r++) {
    const Bitmap found = op_and(oneil(ebm, ba, true, lo), oneil(ebm, ba, false, hi));
    count = found.long_card();
    uint64_t s = 0;
    for (int x = 0; x < nbits; x++) s += (uint64_t)((int64_t)(int32_t)(1u << x) * (int64_t)op_and_card(ba[x], found));
    sum = (int64_t)s;
  }
  const double dt = now_s() - t0;
  if (out2) {
    out2[0] = sum;
    out2[1] = count;
  }
  return dt;
}

// The same query key-parallel (compare and the per-slice andCardinality are per-key sums, BSI/:482-513,
// 581-592): every bitmap is cut into `threads` contiguous key ranges outside the clock (ranges of equal
// ebM container counts), each worker runs the circuit on its ranges, and the per-slice cardinalities are
// added over the workers before sum's Java int cast.  Seconds for reps queries.
double rbo_time_bsi_range_sum_parallel(const uint8_t* const* bufs, const size_t* lens, int nbits, uint32_t lo,
                                       uint32_t hi, int threads, int reps, int64_t* out2) {
  std::vector<Bitmap> bms;
  std::vector<const Bitmap*> ptrs;
  if (load_many(bufs, lens, (size_t)nbits + 1, &bms, &ptrs)) return -1.0;
  const int T = std::max(1, threads);
  const Bitmap& e0 = bms[0];
  auto cut = [&](const Bitmap& b, uint32_t klo, uint32_t khi) {
    Bitmap o;
    for (size_t i = 0; i < b.size(); i++)
      if (b.keys[i] >= klo && b.keys[i] < khi) {
        o.keys.push_back(b.keys[i]);
        o.ctrs.push_back(b.ctrs[i]);
      }
    return o;
  };
  std::vector<std::vector<Bitmap>> part(T);  // part[t] = [ebM, bA...] restricted to worker t's keys
  for (int t = 0; t < T; t++) {
    const size_t i0 = e0.size() * t / T, i1 = e0.size() * (t + 1) / T;
    const uint32_t klo = i0 < e0.size() ? e0.keys[i0] : 65536u, khi = i1 < e0.size() ? e0.keys[i1] : 65536u;
    for (const Bitmap& b : bms) part[t].push_back(cut(b, klo, khi));
  }
  std::vector<int64_t> cards((size_t)T * nbits), counts(T);
  int64_t sum = 0, count = 0;
  double t0 = now_s();
  for (int r = 0; r < reps; r++) {
    std::vector<std::thread> th;
    for (int t = 0; t < T; t++)
      th.emplace_back([&, t]() {
        const Bitmap& ebm = part[t][0];
        std::vector<Bitmap> ba(part[t].begin() + 1, part[t].end());
        const Bitmap found = op_and(oneil(ebm, ba, true, lo), oneil(ebm, ba, false, hi));
        counts[t] = found.long_card();
        for (int x = 0; x < nbits; x++) cards[(size_t)t * nbits + x] = op_and_card(ba[x], found);
      });
    for (auto& x : th) x.join();
    count = 0;
    for (int t = 0; t < T; t++) count += counts[t];
    uint64_t s = 0;
    for (int x = 0; x < nbits; x++) {
      int64_t c = 0;
      for (int t = 0; t < T; t++) c += cards[(size_t)t * nbits + x];
      s += (uint64_t)((int64_t)(int32_t)(1u << x) * (int64_t)(int32_t)(uint32_t)(uint64_t)c);
    }
    sum = (int64_t)s;
  }
  const double dt = now_s() - t0;
  if (out2) {
    out2[0] = sum;
    out2[1] = count;
  }
  return dt;
}

}  // extern "C"
