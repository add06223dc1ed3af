// C entry points of the CPU ORACLE (test infrastructure only; see rbcpu.hpp).
// Loaded through ctypes by tests/ and by bench.py's cpu_baseline leg.
#include <chrono>
#include <cstdlib>
#include <cstring>
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

// op: 0 and, 1 or, 2 xor, 3 andNot   (RB/RoaringBitmap.java:377,860,1071,444)
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

// op: 0 FastAggregation.and(varargs), 1 or, 2 xor, 3 and(Iterator), 4 naive_and, 5 workShyAnd
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
  }
  return ERR_ARG;
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

}  // extern "C"
