// rbcpu — CPU ORACLE (test infrastructure only; see rbcpu.hpp header).
// Restates the Java reference's container algebra with its exact result-type
// control flow.  Citations are file:line into /root/reference (RB/ prefix =
// RoaringBitmap/src/main/java/org/roaringbitmap/).
#include "rbcpu.hpp"

#include <map>

#include <algorithm>
#include <cstring>
#include <stdexcept>

namespace rbcpu {

// ============================================================================
// small bit helpers (RB/Util.java:366-430, 505-522, 616-633)
// ============================================================================
static inline int popc(uint64_t w) { return __builtin_popcountll(w); }
static inline int bit_value(const Ctr& b, int v) { return (int)((b.words[v >> 6] >> (v & 63)) & 1); }

static int card_in_range(const std::vector<uint64_t>& w, int start, int end) {
  // Util.cardinalityInBitmapRange, [start, end)
  if (start >= end) return 0;
  int fw = start / 64, ew = (end - 1) / 64;
  uint64_t lo = ~0ULL << (start & 63);
  uint64_t hi = ~0ULL >> ((64 - (end & 63)) & 63);
  if (fw == ew) return popc(w[fw] & lo & hi);
  int a = popc(w[fw] & lo);
  for (int i = fw + 1; i < ew; i++) a += popc(w[i]);
  a += popc(w[ew] & hi);
  return a;
}
template <int MODE>  // 0 set, 1 reset, 2 flip ; range [start, end)
static void range_apply(std::vector<uint64_t>& w, int start, int end) {
  if (start == end) return;
  int fw = start / 64, ew = (end - 1) / 64;
  uint64_t lo = ~0ULL << (start & 63);
  uint64_t hi = ~0ULL >> ((64 - (end & 63)) & 63);
  auto ap = [&](int i, uint64_t m) {
    if (MODE == 0) w[i] |= m; else if (MODE == 1) w[i] &= ~m; else w[i] ^= m;
  };
  if (fw == ew) { ap(fw, lo & hi); return; }
  ap(fw, lo);
  for (int i = fw + 1; i < ew; i++) ap(i, ~0ULL);
  ap(ew, hi);
}
static void set_range(std::vector<uint64_t>& w, int s, int e) { range_apply<0>(w, s, e); }
static void reset_range(std::vector<uint64_t>& w, int s, int e) { range_apply<1>(w, s, e); }
static void flip_range(std::vector<uint64_t>& w, int s, int e) { range_apply<2>(w, s, e); }

static int compute_card(const std::vector<uint64_t>& w) {
  int c = 0;
  for (uint64_t x : w) c += popc(x);
  return c;
}

// ============================================================================
// Ctr basics
// ============================================================================
int Ctr::cardinality() const {
  if (kind == RUN) {  // RB/RunContainer.java:1003-1009: nbrruns + sum(lengths)
    int s = nruns();
    for (size_t k = 1; k < vals.size(); k += 2) s += vals[k];
    return s;
  }
  return card;
}
bool Ctr::empty() const {
  if (kind == RUN) return nruns() == 0;
  if (kind == ARRAY) return card == 0;
  return cardinality() == 0;  // BitmapContainer.isEmpty: cardinality == 0
}
bool Ctr::full() const {
  if (kind == RUN) return nruns() == 1 && vals[0] == 0 && vals[1] == 0xFFFF;
  if (kind == BITMAP) return card == kMaxCapacity;
  return card == kMaxCapacity;  // ArrayContainer.isFull
}
int Ctr::array_size_bytes() const {
  if (kind == ARRAY) return 2 * card;          // RB/ArrayContainer.java:418-420
  if (kind == BITMAP) return 8192;             // RB/BitmapContainer.java:468-470
  return 2 + 4 * nruns();                      // RB/RunContainer.java:997-999
}

Ctr make_array(std::vector<uint16_t> v) {
  Ctr c;
  c.kind = ARRAY;
  c.card = (int)v.size();
  c.vals = std::move(v);
  return c;
}
Ctr make_bitmap_zero() {
  Ctr c;
  c.kind = BITMAP;
  c.card = 0;
  c.words.assign(kWords, 0);
  return c;
}
static Ctr make_run(std::vector<uint16_t> pairs, int n) {
  Ctr c;
  c.kind = RUN;
  pairs.resize(2 * (size_t)n);
  c.vals = std::move(pairs);
  c.card = 0;
  return c;
}
Ctr run_full() { return make_run({0, 0xFFFF}, 1); }  // RB/RunContainer.java:1663-1665

static void compute_card_inplace(Ctr& b) { b.card = compute_card(b.words); }

Ctr to_bitmap(const Ctr& c) {  // Container.toBitmapContainer()
  if (c.kind == BITMAP) return c;  // RB/BitmapContainer.java:1667-1669 returns this
  Ctr b = make_bitmap_zero();
  if (c.kind == ARRAY) {  // RB/ArrayContainer.java:1126-1129 loadData
    for (uint16_t v : c.vals) b.words[v >> 6] |= 1ULL << (v & 63);
    b.card = c.card;
  } else {  // RB/RunContainer.java:2634-2646
    int card = 0;
    for (int r = 0; r < c.nruns(); r++) {
      int s = c.vals[2 * r], e = s + c.vals[2 * r + 1] + 1;
      card += e - s;
      set_range(b.words, s, e);
    }
    b.card = card;
  }
  return b;
}

Ctr bitmap_to_array(const Ctr& b) {  // BitmapContainer.toArrayContainer
  std::vector<uint16_t> v;
  v.reserve(b.card > 0 ? b.card : 0);
  for (int i = 0; i < kWords; i++) {
    uint64_t w = b.words[i];
    while (w) {
      v.push_back((uint16_t)(i * 64 + __builtin_ctzll(w)));
      w &= w - 1;
    }
  }
  return make_array(std::move(v));
}

static std::vector<uint16_t> run_values(const Ctr& r) {
  std::vector<uint16_t> v;
  for (int k = 0; k < r.nruns(); k++) {
    int s = r.vals[2 * k], e = s + r.vals[2 * k + 1];
    for (int x = s; x <= e; x++) v.push_back((uint16_t)x);
  }
  return v;
}

Ctr to_bitmap_or_array(const Ctr& r, int card) {  // RB/RunContainer.java:2300-2323
  if (card <= kArrayMax) return make_array(run_values(r));
  Ctr b = make_bitmap_zero();
  for (int k = 0; k < r.nruns(); k++) {
    int s = r.vals[2 * k], e = s + r.vals[2 * k + 1] + 1;
    set_range(b.words, s, e);
  }
  b.card = card;
  return b;
}

Ctr to_efficient(const Ctr& r) {  // RB/RunContainer.java:2326-2335
  int size_run = 2 + 4 * r.nruns();
  int size_bmp = 8192;
  int card = r.cardinality();
  int size_arr = 2 + 2 * card;  // ArrayContainer.serializedSizeInBytes(card)
  if (size_run <= std::min(size_bmp, size_arr)) return r;
  return to_bitmap_or_array(r, card);
}

Ctr repair_after_lazy(const Ctr& c) {
  if (c.kind == ARRAY) return c;  // RB/ArrayContainer.java:1080-1082
  if (c.kind == RUN) return to_efficient(c);  // RB/RunContainer.java:2073-2075
  // RB/BitmapContainer.java:1205-1215
  Ctr b = c;
  if (b.card < 0) {
    compute_card_inplace(b);
    if (b.card <= kArrayMax) return bitmap_to_array(b);
    if (b.full()) return run_full();
  }
  return b;
}

int number_of_runs(const Ctr& c) {
  if (c.kind == RUN) return c.nruns();
  if (c.kind == ARRAY) {  // RB/ArrayContainer.java:931-946
    if (c.card == 0) return 0;
    int n = 1, old = c.vals[0];
    for (int i = 1; i < c.card; i++) {
      if (old + 1 != c.vals[i]) n++;
      old = c.vals[i];
    }
    return n;
  }
  // bitmap: count of run starts (exact; RB/BitmapContainer.java numberOfRuns)
  int n = 0;
  for (int i = 0; i < kWords; i++) {
    uint64_t w = c.words[i];
    uint64_t prev_top = i ? (c.words[i - 1] >> 63) : 0;
    n += popc(w & ~((w << 1) | prev_top));
  }
  return n;
}

// RunContainer(ArrayContainer, nbrRuns) / RunContainer(BitmapContainer, nbrRuns):
// both build the maximal-run representation of the set.
static Ctr runs_from_values(const std::vector<uint16_t>& v) {
  std::vector<uint16_t> p;
  int prev = -2, start = -1;
  for (uint16_t x : v) {
    if (x != prev + 1) {
      if (start >= 0) { p.push_back((uint16_t)start); p.push_back((uint16_t)(prev - start)); }
      start = x;
    }
    prev = x;
  }
  if (start >= 0) { p.push_back((uint16_t)start); p.push_back((uint16_t)(prev - start)); }
  int n = (int)(p.size() / 2);
  return make_run(std::move(p), n);
}

Ctr run_optimize(const Ctr& c) {
  if (c.kind == ARRAY) {  // RB/ArrayContainer.java:1085-1099
    int nr = number_of_runs(c);
    if (2 * c.card > 2 + 4 * nr) return runs_from_values(c.vals);
    return c;
  }
  if (c.kind == BITMAP) {  // RB/BitmapContainer.java:1218-1237 (lower bound + exact => nr-based)
    int nr = number_of_runs(c);
    if (8192 > 2 + 4 * nr) return runs_from_values(bitmap_to_array(c).vals);
    return c;
  }
  return to_efficient(c);  // RB/RunContainer.java:2083-2085
}

// ============================================================================
// run construction helpers, literal restatements of RunContainer.smartAppend*
// ============================================================================
struct RunBuf {
  std::vector<uint16_t> v;
  int n = 0;
  explicit RunBuf(size_t cap_runs) : v(2 * std::max<size_t>(cap_runs, 1) + 4, 0) {}
  int val(int i) const { return v[2 * i]; }
  int len(int i) const { return v[2 * i + 1]; }
  void ensure(int runs) { if ((int)v.size() < 2 * runs + 2) v.resize(2 * runs + 16); }
  void set_val(int i, int x) { v[2 * i] = (uint16_t)x; }
  void set_len(int i, int x) { v[2 * i + 1] = (uint16_t)x; }
  void push(int s, int l) { ensure(n + 1); v[2 * n] = (uint16_t)s; v[2 * n + 1] = (uint16_t)l; n++; }

  // RB/RunContainer.java:2175-2188
  void smart_append(int val_) {
    int oldend = 0;
    if (n == 0 || val_ > (oldend = val(n - 1) + len(n - 1)) + 1) { push(val_, 0); return; }
    if (val_ == (uint16_t)(oldend + 1)) v[2 * (n - 1) + 1]++;
  }
  // RB/RunContainer.java:2190-2205
  void smart_append(int start, int length) {
    int oldend = 0;
    if (n == 0 || start > (oldend = val(n - 1) + len(n - 1)) + 1) { push(start, length); return; }
    int newend = start + length + 1;
    if (newend > oldend) set_len(n - 1, newend - 1 - val(n - 1));
  }
  // RB/RunContainer.java:2207-2247
  void smart_append_excl(int val_) {
    int oldend = 0;
    if (n == 0 || val_ > (oldend = val(n - 1) + len(n - 1) + 1)) { push(val_, 0); return; }
    if (oldend == val_) { v[2 * (n - 1) + 1]++; return; }
    int newend = val_ + 1;
    if (val_ == val(n - 1)) {
      if (newend != oldend) {
        set_val(n - 1, newend);
        set_len(n - 1, oldend - newend - 1);
        return;
      } else {
        n--;
        return;
      }
    }
    set_len(n - 1, val_ - val(n - 1) - 1);
    if (newend < oldend) {
      ensure(n + 1);
      set_val(n, newend);
      set_len(n, oldend - newend - 1);
      n++;
    }
  }
  // RB/RunContainer.java:2249-2298
  void smart_append_excl(int start, int length) {
    int oldend = 0;
    if (n == 0 || start > (oldend = val(n - 1) + len(n - 1) + 1)) { push(start, length); return; }
    if (oldend == start) { v[2 * (n - 1) + 1] = (uint16_t)(v[2 * (n - 1) + 1] + length + 1); return; }
    int newend = start + length + 1;
    if (start == val(n - 1)) {
      if (newend < oldend) {
        set_val(n - 1, newend);
        set_len(n - 1, oldend - newend - 1);
        return;
      } else if (newend > oldend) {
        set_val(n - 1, oldend);
        set_len(n - 1, newend - oldend - 1);
        return;
      } else {
        n--;
        return;
      }
    }
    set_len(n - 1, start - val(n - 1) - 1);
    if (newend < oldend) {
      ensure(n + 1);
      set_val(n, newend);
      set_len(n, oldend - newend - 1);
      n++;
    } else if (newend > oldend) {
      ensure(n + 1);
      set_val(n, oldend);
      set_len(n, newend - oldend - 1);
      n++;
    }
  }
  Ctr build() { return make_run(v, n); }
};

// ============================================================================
// sorted u16 merges (RB/Util.java:717-1168)
// ============================================================================
static std::vector<uint16_t> v_inter(const std::vector<uint16_t>& a, const std::vector<uint16_t>& b) {
  std::vector<uint16_t> o;
  std::set_intersection(a.begin(), a.end(), b.begin(), b.end(), std::back_inserter(o));
  return o;
}
static std::vector<uint16_t> v_union(const std::vector<uint16_t>& a, const std::vector<uint16_t>& b) {
  std::vector<uint16_t> o;
  std::set_union(a.begin(), a.end(), b.begin(), b.end(), std::back_inserter(o));
  return o;
}
static std::vector<uint16_t> v_diff(const std::vector<uint16_t>& a, const std::vector<uint16_t>& b) {
  std::vector<uint16_t> o;
  std::set_difference(a.begin(), a.end(), b.begin(), b.end(), std::back_inserter(o));
  return o;
}
static std::vector<uint16_t> v_xor(const std::vector<uint16_t>& a, const std::vector<uint16_t>& b) {
  std::vector<uint16_t> o;
  std::set_symmetric_difference(a.begin(), a.end(), b.begin(), b.end(), std::back_inserter(o));
  return o;
}

// ============================================================================
// BitmapContainer ops
// ============================================================================
static Ctr B_and_A(const Ctr& b, const Ctr& a) {  // RB/BitmapContainer.java:162-171
  std::vector<uint16_t> o;
  for (uint16_t v : a.vals) if (bit_value(b, v)) o.push_back(v);
  return make_array(std::move(o));
}
static Ctr B_and_B(const Ctr& x, const Ctr& y) {  // :174-188
  Ctr r = make_bitmap_zero();
  for (int k = 0; k < kWords; k++) r.words[k] = x.words[k] & y.words[k];
  r.card = compute_card(r.words);
  if (r.card > kArrayMax) return r;
  return bitmap_to_array(r);  // Util.fillArrayAND
}
static Ctr B_andnot_A(const Ctr& b, const Ctr& a) {  // :221-236
  Ctr r = b;
  for (uint16_t v : a.vals) {
    uint64_t w = r.words[v >> 6], aft = w & ~(1ULL << (v & 63));
    r.words[v >> 6] = aft;
    r.card -= (int)((w ^ aft) >> (v & 63));
  }
  if (r.card <= kArrayMax) return bitmap_to_array(r);
  return r;
}
static Ctr B_andnot_B(const Ctr& x, const Ctr& y) {  // :239-256
  Ctr r = make_bitmap_zero();
  for (int k = 0; k < kWords; k++) r.words[k] = x.words[k] & ~y.words[k];
  r.card = compute_card(r.words);
  if (r.card > kArrayMax) return r;
  return bitmap_to_array(r);
}
static Ctr B_andnot_R(const Ctr& b, const Ctr& run) {  // :259-274
  Ctr r = b;
  for (int k = 0; k < run.nruns(); k++) {
    int s = run.vals[2 * k], e = s + run.vals[2 * k + 1] + 1;
    int prev = card_in_range(r.words, s, e);
    reset_range(r.words, s, e);
    r.card -= prev;
  }
  if (r.card > kArrayMax) return r;
  return bitmap_to_array(r);
}
// BitmapContainer.ior(ArrayContainer) (RB/BitmapContainer.java:740-757): the bits set in place and
// the bitmap returned as is -- a full result stays a bitmap (no RunContainer.full())
static Ctr B_ior_A(const Ctr& b, const Ctr& a) {
  Ctr r = b;
  for (uint16_t v : a.vals) {
    uint64_t w = r.words[v >> 6], aft = w | (1ULL << (v & 63));
    r.words[v >> 6] = aft;
    if (w != aft) r.card++;
  }
  return r;
}
static Ctr B_or_A(const Ctr& b, const Ctr& a) {  // :1064-1085
  Ctr r = B_ior_A(b, a);
  if (r.full()) return run_full();
  return r;
}
static Ctr B_ior_B(Ctr r, const Ctr& y) {  // :760-769
  for (int k = 0; k < kWords; k++) r.words[k] |= y.words[k];
  compute_card_inplace(r);
  if (r.full()) return run_full();
  return r;
}
static Ctr B_xor_A(const Ctr& b, const Ctr& a) {  // :1372-1388 (and ixor :828-843, same typing)
  Ctr r = b;
  for (uint16_t v : a.vals) {
    uint64_t m = 1ULL << (v & 63), val = r.words[v >> 6];
    r.card += 1 - 2 * (int)((val & m) >> (v & 63));
    r.words[v >> 6] = val ^ m;
  }
  if (r.card <= kArrayMax) return bitmap_to_array(r);
  return r;
}
static Ctr B_xor_B(const Ctr& x, const Ctr& y) {  // :1391-1408 (ixor :847-858 same typing)
  Ctr r = make_bitmap_zero();
  for (int k = 0; k < kWords; k++) r.words[k] = x.words[k] ^ y.words[k];
  r.card = compute_card(r.words);
  if (r.card > kArrayMax) return r;
  return bitmap_to_array(r);
}
static Ctr B_ixor_R(Ctr r, const Ctr& run) {  // :862-876
  for (int k = 0; k < run.nruns(); k++) {
    int s = run.vals[2 * k], e = s + run.vals[2 * k + 1] + 1;
    int prev = card_in_range(r.words, s, e);
    flip_range(r.words, s, e);
    r.card += (e - s - prev) - prev;
  }
  if (r.card > kArrayMax) return r;
  return bitmap_to_array(r);
}
static Ctr B_iandnot_A(Ctr r, const Ctr& a) {  // :602-610
  for (uint16_t v : a.vals) {
    uint64_t w = r.words[v >> 6], aft = w & ~(1ULL << (v & 63));
    if (w != aft) { r.words[v >> 6] = aft; r.card--; }
  }
  if (r.card <= kArrayMax) return bitmap_to_array(r);
  return r;
}

// ============================================================================
// RunContainer ops
// ============================================================================
static Ctr R_and_A(const Ctr& r, const Ctr& a) {  // RB/RunContainer.java:305-334
  std::vector<uint16_t> o;
  if (r.nruns() == 0) return make_array(o);
  int rlepos = 0, ap = 0;
  int rv = r.vals[0], rl = r.vals[1];
  while (ap < a.card) {
    int av = a.vals[ap];
    while (rv + rl < av) {
      ++rlepos;
      if (rlepos == r.nruns()) return make_array(std::move(o));
      rv = r.vals[2 * rlepos];
      rl = r.vals[2 * rlepos + 1];
    }
    if (rv > av) {
      // Util.advanceUntil: first index > ap with value >= rv
      while (ap < a.card && a.vals[ap] < rv) ap++;
    } else {
      o.push_back((uint16_t)av);
      ap++;
    }
  }
  return make_array(std::move(o));
}
static Ctr R_and_B(const Ctr& r, const Ctr& b) {  // :338-378
  int card = r.cardinality();
  if (card <= kArrayMax) {
    std::vector<uint16_t> o;
    for (int k = 0; k < r.nruns(); k++) {
      int s = r.vals[2 * k], e = s + r.vals[2 * k + 1];
      for (int x = s; x <= e; x++) if (bit_value(b, x)) o.push_back((uint16_t)x);
    }
    return make_array(std::move(o));
  }
  Ctr ans = b;
  int start = 0;
  for (int k = 0; k < r.nruns(); k++) {
    int end = r.vals[2 * k];
    int prev = card_in_range(ans.words, start, end);
    reset_range(ans.words, start, end);
    ans.card -= prev;
    start = end + r.vals[2 * k + 1] + 1;
  }
  int ones = card_in_range(ans.words, start, kMaxCapacity);
  reset_range(ans.words, start, kMaxCapacity);
  ans.card -= ones;
  if (ans.card > kArrayMax) return ans;
  return bitmap_to_array(ans);
}
// The run merge of RB/RunContainer.java:381-456 (no galloping: ENABLE_GALLOPING_AND=false) before its
// toEfficientContainer; the buffer package's MappeableRunContainer.and(MappeableRunContainer)
// (RB/buffer/MappeableRunContainer.java:474-536) returns exactly this merge.
static Ctr R_and_R_runs(const Ctr& t, const Ctr& x) {
  RunBuf ans(t.nruns() + x.nruns());
  if (t.empty()) return ans.build();
  int rp = 0, xp = 0;
  int start = t.vals[0], end = start + t.vals[1] + 1;
  int xstart = x.vals[0], xend = xstart + x.vals[1] + 1;
  const int tn = t.nruns(), xn = x.nruns();
  while (rp < tn && xp < xn) {
    if (end <= xstart) {
      ++rp;
      if (rp < tn) { start = t.vals[2 * rp]; end = start + t.vals[2 * rp + 1] + 1; }
    } else if (xend <= start) {
      ++xp;
      if (xp < xn) { xstart = x.vals[2 * xp]; xend = xstart + x.vals[2 * xp + 1] + 1; }
    } else {
      int latest = std::max(start, xstart), earliest;
      if (end == xend) {
        earliest = end;
        rp++;
        xp++;
        if (rp < tn) { start = t.vals[2 * rp]; end = start + t.vals[2 * rp + 1] + 1; }
        if (xp < xn) { xstart = x.vals[2 * xp]; xend = xstart + x.vals[2 * xp + 1] + 1; }
      } else if (end < xend) {
        earliest = end;
        rp++;
        if (rp < tn) { start = t.vals[2 * rp]; end = start + t.vals[2 * rp + 1] + 1; }
      } else {
        earliest = xend;
        xp++;
        if (xp < xn) { xstart = x.vals[2 * xp]; xend = xstart + x.vals[2 * xp + 1] + 1; }
      }
      ans.push(latest, earliest - latest - 1);
    }
  }
  return ans.build();
}
static Ctr R_and_R(const Ctr& t, const Ctr& x) { return to_efficient(R_and_R_runs(t, x)); }  // :381-456
static int R_and_card_A(const Ctr& r, const Ctr& a) {  // :459-486
  if (r.nruns() == 0) return a.card;
  int rp = 0, ap = 0, c = 0;
  int rv = r.vals[0], rl = r.vals[1];
  while (ap < a.card) {
    int av = a.vals[ap];
    while (rv + rl < av) {
      ++rp;
      if (rp == r.nruns()) return c;
      rv = r.vals[2 * rp];
      rl = r.vals[2 * rp + 1];
    }
    if (rv > av) {
      while (ap < a.card && a.vals[ap] < rv) ap++;
    } else {
      c++;
      ap++;
    }
  }
  return c;
}
static int R_and_card_B(const Ctr& r, const Ctr& b) {  // :490-499
  int c = 0;
  for (int k = 0; k < r.nruns(); k++) {
    int s = r.vals[2 * k], e = s + r.vals[2 * k + 1];
    c += card_in_range(b.words, s, e + 1);
  }
  return c;
}
static int R_and_card_R(const Ctr& t, const Ctr& x) {  // :502-571 (same walk as R_and_R)
  int c = 0, rp = 0, xp = 0;
  const int tn = t.nruns(), xn = x.nruns();
  int start = t.vals[0], end = start + t.vals[1] + 1;
  int xstart = x.vals[0], xend = xstart + x.vals[1] + 1;
  while (rp < tn && xp < xn) {
    if (end <= xstart) {
      ++rp;
      if (rp < tn) { start = t.vals[2 * rp]; end = start + t.vals[2 * rp + 1] + 1; }
    } else if (xend <= start) {
      ++xp;
      if (xp < xn) { xstart = x.vals[2 * xp]; xend = xstart + x.vals[2 * xp + 1] + 1; }
    } else {
      int latest = std::max(start, xstart), earliest;
      if (end == xend) {
        earliest = end;
        rp++;
        xp++;
        if (rp < tn) { start = t.vals[2 * rp]; end = start + t.vals[2 * rp + 1] + 1; }
        if (xp < xn) { xstart = x.vals[2 * xp]; xend = xstart + x.vals[2 * xp + 1] + 1; }
      } else if (end < xend) {
        earliest = end;
        rp++;
        if (rp < tn) { start = t.vals[2 * rp]; end = start + t.vals[2 * rp + 1] + 1; }
      } else {
        earliest = xend;
        xp++;
        if (xp < xn) { xstart = x.vals[2 * xp]; xend = xstart + x.vals[2 * xp + 1] + 1; }
      }
      c += earliest - latest;
    }
  }
  return c;
}
static Ctr R_lazy_andnot_A(const Ctr& t, const Ctr& x) {  // :1707-1763
  if (x.card == 0) return t;
  RunBuf ans(t.nruns() + x.card);
  int rp = 0, xp = 0;
  const int tn = t.nruns();
  int start = t.vals[0], end = start + t.vals[1] + 1;
  int xstart = x.vals[0];
  while (rp < tn && xp < x.card) {
    if (end <= xstart) {
      ans.push(start, end - start - 1);
      rp++;
      if (rp < tn) { start = t.vals[2 * rp]; end = start + t.vals[2 * rp + 1] + 1; }
    } else if (xstart + 1 <= start) {
      xp++;
      if (xp < x.card) xstart = x.vals[xp];
    } else {
      if (start < xstart) ans.push(start, xstart - start - 1);
      if (xstart + 1 < end) {
        start = xstart + 1;
      } else {
        rp++;
        if (rp < tn) { start = t.vals[2 * rp]; end = start + t.vals[2 * rp + 1] + 1; }
      }
    }
  }
  if (rp < tn) {
    ans.push(start, end - start - 1);
    rp++;
    for (; rp < tn; rp++) ans.push(t.vals[2 * rp], t.vals[2 * rp + 1]);
  }
  return ans.build();
}
static Ctr R_andnot_A(const Ctr& r, const Ctr& a) {  // :574-591
  if (a.card < kRunVsArrayThreshold) return to_efficient(R_lazy_andnot_A(r, a));
  int card = r.cardinality();
  if (card <= kArrayMax) return make_array(v_diff(run_values(r), a.vals));  // Util.unsignedDifference(it,it)
  return B_iandnot_A(to_bitmap_or_array(r, card), a);
}
static Ctr R_andnot_B(const Ctr& r, const Ctr& b) {  // :594-634
  int card = r.cardinality();
  if (card <= kArrayMax) {
    std::vector<uint16_t> o;
    for (int k = 0; k < r.nruns(); k++) {
      int s = r.vals[2 * k], e = s + r.vals[2 * k + 1];
      for (int x = s; x <= e; x++) if (!bit_value(b, x)) o.push_back((uint16_t)x);
    }
    return make_array(std::move(o));
  }
  Ctr ans = b;
  int last = 0;
  for (int k = 0; k < r.nruns(); k++) {
    int s = r.vals[2 * k], e = s + r.vals[2 * k + 1] + 1;
    int prev = card_in_range(ans.words, last, s);
    int flipped = card_in_range(ans.words, s, e);
    reset_range(ans.words, last, s);
    flip_range(ans.words, s, e);
    ans.card += (e - s - flipped) - (prev + flipped);
    last = e;
  }
  int ones = card_in_range(ans.words, last, kMaxCapacity);
  reset_range(ans.words, last, kMaxCapacity);
  ans.card -= ones;
  if (ans.card > kArrayMax) return ans;
  return bitmap_to_array(ans);
}
// The run difference of RB/RunContainer.java:637-692 before its toEfficientContainer; the buffer
// package's MappeableRunContainer.andNot(MappeableRunContainer) (RB/buffer/MappeableRunContainer.java:600-663)
// returns exactly this.
static Ctr R_andnot_R_runs(const Ctr& t, const Ctr& x) {
  RunBuf ans(t.nruns() + x.nruns());
  int rp = 0, xp = 0;
  const int tn = t.nruns(), xn = x.nruns();
  int start = t.vals[0], end = start + t.vals[1] + 1;
  int xstart = x.vals[0], xend = xstart + x.vals[1] + 1;
  while (rp < tn && xp < xn) {
    if (end <= xstart) {
      ans.push(start, end - start - 1);
      rp++;
      if (rp < tn) { start = t.vals[2 * rp]; end = start + t.vals[2 * rp + 1] + 1; }
    } else if (xend <= start) {
      xp++;
      if (xp < xn) { xstart = x.vals[2 * xp]; xend = xstart + x.vals[2 * xp + 1] + 1; }
    } else {
      if (start < xstart) ans.push(start, xstart - start - 1);
      if (xend < end) {
        start = xend;
      } else {
        rp++;
        if (rp < tn) { start = t.vals[2 * rp]; end = start + t.vals[2 * rp + 1] + 1; }
      }
    }
  }
  if (rp < tn) {
    ans.push(start, end - start - 1);
    rp++;
    for (; rp < tn; rp++) ans.push(t.vals[2 * rp], t.vals[2 * rp + 1]);
  }
  return ans.build();
}
static Ctr R_andnot_R(const Ctr& t, const Ctr& x) { return to_efficient(R_andnot_R_runs(t, x)); }  // :637-692
// lazyorToRun + convertToLazyBitmapIfNeeded, RB/RunContainer.java:1769-1813, 861-875
static Ctr R_lazyor_A(const Ctr& r, const Ctr& a) {
  if (r.full()) return run_full();
  RunBuf ans(r.nruns() + a.card);
  int rp = 0, i = 0;
  const int rn = r.nruns();
  while (i < a.card && rp < rn) {
    if (r.vals[2 * rp] - (int)a.vals[i] <= 0) {
      ans.smart_append(r.vals[2 * rp], r.vals[2 * rp + 1]);
      rp++;
    } else {
      ans.smart_append(a.vals[i++]);
    }
  }
  if (i < a.card) {
    while (i < a.card) ans.smart_append(a.vals[i++]);
  } else {
    while (rp < rn) { ans.smart_append(r.vals[2 * rp], r.vals[2 * rp + 1]); rp++; }
  }
  Ctr out = ans.build();
  if (out.full()) return run_full();
  if (out.nruns() > kArrayMax) {  // convertToLazyBitmapIfNeeded
    Ctr b = make_bitmap_zero();
    for (int k = 0; k < out.nruns(); k++) {
      int s = out.vals[2 * k], e = s + out.vals[2 * k + 1] + 1;
      set_range(b.words, s, e);
    }
    b.card = -1;
    return b;
  }
  return out;
}
static Ctr R_or_A(const Ctr& r, const Ctr& a) { return repair_after_lazy(R_lazyor_A(r, a)); }  // :1926-1929
static Ctr R_or_B(const Ctr& r, const Ctr& b) {  // :1932-1949
  if (r.full()) return run_full();
  Ctr ans = b;
  for (int k = 0; k < r.nruns(); k++) {
    int s = r.vals[2 * k], e = s + r.vals[2 * k + 1] + 1;
    int prev = card_in_range(ans.words, s, e);
    set_range(ans.words, s, e);
    ans.card += (e - s) - prev;
  }
  if (ans.full()) return run_full();
  return ans;
}
static Ctr R_or_R(const Ctr& t, const Ctr& x) {  // :1952-1986
  if (t.full()) return run_full();
  if (x.full()) return run_full();
  RunBuf ans(t.nruns() + x.nruns());
  int rp = 0, xp = 0;
  const int tn = t.nruns(), xn = x.nruns();
  while (xp < xn && rp < tn) {
    if (t.vals[2 * rp] - (int)x.vals[2 * xp] <= 0) {
      ans.smart_append(t.vals[2 * rp], t.vals[2 * rp + 1]);
      rp++;
    } else {
      ans.smart_append(x.vals[2 * xp], x.vals[2 * xp + 1]);
      xp++;
    }
  }
  while (xp < xn) { ans.smart_append(x.vals[2 * xp], x.vals[2 * xp + 1]); xp++; }
  while (rp < tn) { ans.smart_append(t.vals[2 * rp], t.vals[2 * rp + 1]); rp++; }
  Ctr out = ans.build();
  if (out.full()) return run_full();
  return to_efficient(out);
}
static Ctr R_lazyxor_A(const Ctr& t, const Ctr& x) {  // :1815-1853
  if (x.card == 0) return t;
  if (t.nruns() == 0) return x;
  RunBuf ans(t.nruns() + x.card);
  int rp = 0, i = 0;
  const int tn = t.nruns();
  int cv = x.vals[i++];
  while (true) {
    if (t.vals[2 * rp] < cv) {
      ans.smart_append_excl(t.vals[2 * rp], t.vals[2 * rp + 1]);
      rp++;
      if (rp == tn) {
        ans.smart_append_excl(cv);
        while (i < x.card) ans.smart_append_excl(x.vals[i++]);
        break;
      }
    } else {
      ans.smart_append_excl(cv);
      if (i >= x.card) {
        while (rp < tn) { ans.smart_append_excl(t.vals[2 * rp], t.vals[2 * rp + 1]); rp++; }
        break;
      } else {
        cv = x.vals[i++];
      }
    }
  }
  return ans.build();
}
static Ctr A_or_iter_excl(const Ctr& a, const std::vector<uint16_t>& it) {
  // ArrayContainer.or(CharIterator, exclusive=true), RB/ArrayContainer.java:983-1022
  std::vector<uint16_t> o = v_xor(a.vals, it);
  Ctr ac = make_array(std::move(o));
  if (ac.card > kArrayMax) return to_bitmap(ac);
  return ac;
}
static Ctr R_xor_A(const Ctr& r, const Ctr& a) {  // :2410-2424
  if (a.card < kRunVsArrayThreshold) return repair_after_lazy(R_lazyxor_A(r, a));
  int card = r.cardinality();
  if (card <= kArrayMax) return A_or_iter_excl(a, run_values(r));
  return B_xor_A(to_bitmap_or_array(r, card), a);  // BitmapContainer.ixor(ArrayContainer)
}
static Ctr R_xor_B(const Ctr& r, const Ctr& b) {  // :2427-2442
  Ctr ans = b;
  for (int k = 0; k < r.nruns(); k++) {
    int s = r.vals[2 * k], e = s + r.vals[2 * k + 1] + 1;
    int prev = card_in_range(ans.words, s, e);
    flip_range(ans.words, s, e);
    ans.card += (e - s - prev) - prev;
  }
  if (ans.card > kArrayMax) return ans;
  return bitmap_to_array(ans);
}
static Ctr R_xor_R(const Ctr& t, const Ctr& x) {  // :2445-2482
  if (x.nruns() == 0) return t;
  if (t.nruns() == 0) return x;
  RunBuf ans(t.nruns() + x.nruns());
  int rp = 0, xp = 0;
  const int tn = t.nruns(), xn = x.nruns();
  while (true) {
    if (t.vals[2 * rp] < x.vals[2 * xp]) {
      ans.smart_append_excl(t.vals[2 * rp], t.vals[2 * rp + 1]);
      rp++;
      if (rp == tn) {
        while (xp < xn) { ans.smart_append_excl(x.vals[2 * xp], x.vals[2 * xp + 1]); xp++; }
        break;
      }
    } else {
      ans.smart_append_excl(x.vals[2 * xp], x.vals[2 * xp + 1]);
      xp++;
      if (xp == xn) {
        while (rp < tn) { ans.smart_append_excl(t.vals[2 * rp], t.vals[2 * rp + 1]); rp++; }
        break;
      }
    }
  }
  return to_efficient(ans.build());
}

// ============================================================================
// ArrayContainer ops
// ============================================================================
static Ctr A_or_A(const Ctr& x, const Ctr& y) {  // RB/ArrayContainer.java:949-963
  int total = x.card + y.card;
  if (total > kArrayMax) {
    // toBitmapContainer().lazyIOR(value2).repairAfterLazy()
    return repair_after_lazy(b_ilazyor(to_bitmap(x), y));
  }
  return make_array(v_union(x.vals, y.vals));
}
static Ctr A_xor_A(const Ctr& x, const Ctr& y) {  // :1311-1321
  int total = x.card + y.card;
  if (total > kArrayMax) return B_xor_A(to_bitmap(x), y);  // toBitmapContainer().ixor(value2)
  return make_array(v_xor(x.vals, y.vals));
}
static Ctr A_andnot_R(const Ctr& a, const Ctr& r) {  // :245-271
  if (r.nruns() == 0) return a;
  if (r.full()) return make_array({});
  std::vector<uint16_t> o;
  // keep the values of `a` that fall in no run
  int k = 0;
  for (uint16_t v : a.vals) {
    while (k < r.nruns() && r.vals[2 * k] + r.vals[2 * k + 1] < v) k++;
    bool in = k < r.nruns() && r.vals[2 * k] <= v;
    if (!in) o.push_back(v);
  }
  return make_array(std::move(o));
}

// ============================================================================
// dispatch (RB/Container.java)
// ============================================================================
Ctr c_and(const Ctr& a, const Ctr& b) {
  switch (a.kind) {
    case ARRAY:
      if (b.kind == ARRAY) return make_array(v_inter(a.vals, b.vals));  // :184-191
      if (b.kind == BITMAP) return B_and_A(b, a);                      // :194-196
      return R_and_A(b, a);                                            // :199-202
    case BITMAP:
      if (b.kind == ARRAY) return B_and_A(a, b);
      if (b.kind == BITMAP) return B_and_B(a, b);
      return R_and_B(b, a);  // RB/BitmapContainer.java:191-193
    default:
      if (b.kind == ARRAY) return R_and_A(a, b);
      if (b.kind == BITMAP) return R_and_B(a, b);
      return R_and_R(a, b);
  }
}

int c_and_card(const Ctr& a, const Ctr& b) {  // RB/Container.java:113-126
  if (a.empty()) return 0;
  if (b.empty()) return 0;
  switch (a.kind) {
    case ARRAY:
      if (b.kind == ARRAY) return (int)v_inter(a.vals, b.vals).size();
      if (b.kind == BITMAP) { int c = 0; for (uint16_t v : a.vals) c += bit_value(b, v); return c; }
      return R_and_card_A(b, a);
    case BITMAP:
      if (b.kind == ARRAY) { int c = 0; for (uint16_t v : b.vals) c += bit_value(a, v); return c; }
      if (b.kind == BITMAP) { int c = 0; for (int k = 0; k < kWords; k++) c += popc(a.words[k] & b.words[k]); return c; }
      return R_and_card_B(b, a);
    default:
      if (b.kind == ARRAY) return R_and_card_A(a, b);
      if (b.kind == BITMAP) return R_and_card_B(a, b);
      return R_and_card_R(a, b);
  }
}

bool c_intersects(const Ctr& a, const Ctr& b) {
  // set-level predicate; every reference implementation returns |a & b| > 0
  if (a.kind == RUN && a.nruns() == 0) return false;
  if (b.kind == RUN && b.nruns() == 0) return false;
  return c_and_card(a, b) > 0;
}

Ctr c_andnot(const Ctr& a, const Ctr& b) {
  switch (a.kind) {
    case ARRAY:
      if (b.kind == ARRAY) return make_array(v_diff(a.vals, b.vals));  // :222-229
      if (b.kind == BITMAP) {  // :232-242
        std::vector<uint16_t> o;
        for (uint16_t v : a.vals) if (!bit_value(b, v)) o.push_back(v);
        return make_array(std::move(o));
      }
      return A_andnot_R(a, b);
    case BITMAP:
      if (b.kind == ARRAY) return B_andnot_A(a, b);
      if (b.kind == BITMAP) return B_andnot_B(a, b);
      return B_andnot_R(a, b);
    default:
      if (b.kind == ARRAY) return R_andnot_A(a, b);
      if (b.kind == BITMAP) return R_andnot_B(a, b);
      return R_andnot_R(a, b);
  }
}

// In-place OR of RoaringBitmap.or(RoaringBitmap) (RB/RoaringBitmap.java:2481-2523): Container.ior.  Its
// result types are the static or's (A.ior(A) :726-746 = A.or(A); A.ior(B|R) = x.or(this) :748-756;
// B.ior(B|R) :760-785 and R.ior(A|B|R) :1462-1550 end in the same types as or) except
// BitmapContainer.ior(ArrayContainer), which keeps a full bitmap (B_ior_A).
Ctr c_ior(const Ctr& a, const Ctr& b) {
  if (a.kind == BITMAP && b.kind == ARRAY) return B_ior_A(a, b);
  return c_or(a, b);
}

// Buffer package (RB/buffer/): MappeableContainer.and / andNot dispatch like the heap containers and
// type their results alike (MappeableArrayContainer.java:287-384, MappeableBitmapContainer.java:152-348,
// MappeableRunContainer.java:398-663) -- except run AND run and run ANDNOT run, which return the
// merged run container without toEfficientContainer (MappeableRunContainer.java:474-536, 600-663).
Ctr c_and_buf(const Ctr& a, const Ctr& b) {
  if (a.kind == RUN && b.kind == RUN) return R_and_R_runs(a, b);
  return c_and(a, b);
}
Ctr c_andnot_buf(const Ctr& a, const Ctr& b) {
  if (a.kind == RUN && b.kind == RUN) return R_andnot_R_runs(a, b);
  return c_andnot(a, b);
}

Ctr c_or(const Ctr& a, const Ctr& b) {
  switch (a.kind) {
    case ARRAY:
      if (b.kind == ARRAY) return A_or_A(a, b);
      if (b.kind == BITMAP) return B_or_A(b, a);  // :966-968 x.or(this)
      return R_or_A(b, a);                        // :971-973
    case BITMAP:
      if (b.kind == ARRAY) return B_or_A(a, b);
      if (b.kind == BITMAP) return B_ior_B(a, b);  // :1093-1096 clone().ior()
      return R_or_B(b, a);                         // :1099-1101
    default:
      if (b.kind == ARRAY) return R_or_A(a, b);
      if (b.kind == BITMAP) return R_or_B(a, b);
      return R_or_R(a, b);
  }
}

Ctr c_xor(const Ctr& a, const Ctr& b) {
  switch (a.kind) {
    case ARRAY:
      if (b.kind == ARRAY) return A_xor_A(a, b);
      if (b.kind == BITMAP) return B_xor_A(b, a);  // :1324-1326
      return R_xor_A(b, a);                        // :1329-1331
    case BITMAP:
      if (b.kind == ARRAY) return B_xor_A(a, b);
      if (b.kind == BITMAP) return B_xor_B(a, b);
      return R_xor_B(b, a);  // RB/BitmapContainer.java:1411-1413
    default:
      if (b.kind == ARRAY) return R_xor_A(a, b);
      if (b.kind == BITMAP) return R_xor_B(a, b);
      return R_xor_R(a, b);
  }
}

// In-place AND (non-lazy), used by RoaringBitmap.and(RoaringBitmap) :1272-1296
Ctr c_iand(const Ctr& a, const Ctr& b) {
  switch (a.kind) {
    case ARRAY:  // RB/ArrayContainer.java:538-571 -- filters in place, stays an array
      if (b.kind == ARRAY) return make_array(v_inter(a.vals, b.vals));
      if (b.kind == BITMAP) return B_and_A(b, a);
      return R_and_A(b, a);
    case BITMAP:
      if (b.kind == ARRAY) return B_and_A(a, b);  // RB/BitmapContainer.java:523-531 -> b2.and(this)
      if (b.kind == BITMAP) return B_and_B(a, b); // :534-555 (same typing as and)
      {  // :558-599 non-lazy
        int card = b.cardinality();
        if (card <= kArrayMax) return R_and_B(b, a);  // array of run values present in a
        Ctr r = a;
        int start = 0;
        for (int k = 0; k < b.nruns(); k++) {
          int end = b.vals[2 * k];
          int prev = card_in_range(r.words, start, end);
          reset_range(r.words, start, end);
          r.card -= prev;
          start = end + b.vals[2 * k + 1] + 1;
        }
        int ones = card_in_range(r.words, start, kMaxCapacity);
        reset_range(r.words, start, kMaxCapacity);
        r.card -= ones;
        if (r.card <= kArrayMax) return bitmap_to_array(r);
        return r;
      }
    default:
      return c_and(a, b);  // RB/RunContainer.java:1166-1180 iand = and
  }
}

// In-place XOR, used by RoaringBitmap.xor(RoaringBitmap) :3296-3348
Ctr c_ixor(const Ctr& a, const Ctr& b) {
  switch (a.kind) {
    case ARRAY:  // RB/ArrayContainer.java:807-821
      return c_xor(a, b);
    case BITMAP:  // RB/BitmapContainer.java:828-876
      if (b.kind == ARRAY) return B_xor_A(a, b);
      if (b.kind == BITMAP) return B_xor_B(a, b);
      return B_ixor_R(a, b);
    default:  // RB/RunContainer.java:1691-1705 ixor = xor
      return c_xor(a, b);
  }
}

// BitmapContainer.ilazyor(A|B|R): result is a lazy bitmap (card = -1)
Ctr b_ilazyor(const Ctr& lb, const Ctr& x) {
  Ctr r = lb;
  r.card = -1;
  if (x.kind == ARRAY) {
    for (uint16_t v : x.vals) r.words[v >> 6] |= 1ULL << (v & 63);
  } else if (x.kind == BITMAP) {
    for (int k = 0; k < kWords; k++) r.words[k] |= x.words[k];
  } else {
    for (int k = 0; k < x.nruns(); k++) {
      int s = x.vals[2 * k], e = s + x.vals[2 * k + 1] + 1;
      set_range(r.words, s, e);
    }
  }
  return r;
}

// Lazy-mode BitmapContainer.iand branches used by workShyAnd (card stays -1)
Ctr b_lazy_iand(const Ctr& lb, const Ctr& x) {
  Ctr r = lb;
  if (x.kind == ARRAY) {  // Util.intersectArrayIntoBitmap
    std::vector<uint64_t> m(kWords, 0);
    for (uint16_t v : x.vals) m[v >> 6] |= 1ULL << (v & 63);
    for (int k = 0; k < kWords; k++) r.words[k] &= m[k];
  } else if (x.kind == BITMAP) {
    for (int k = 0; k < kWords; k++) r.words[k] &= x.words[k];
  } else {
    int start = 0;
    for (int k = 0; k < x.nruns(); k++) {
      int end = x.vals[2 * k];
      reset_range(r.words, start, end);
      start = end + x.vals[2 * k + 1] + 1;
    }
    reset_range(r.words, start, kMaxCapacity);
  }
  r.card = -1;
  return r;
}

// ============================================================================
// Bitmap level
// ============================================================================
int64_t Bitmap::long_card() const {  // RB/RoaringBitmap.java:1957-1963
  int64_t s = 0;
  for (const Ctr& c : ctrs) s += c.cardinality();
  return s;
}

Bitmap bitmap_of(const uint32_t* vals, size_t n) {
  std::vector<uint32_t> v(vals, vals + n);
  std::sort(v.begin(), v.end());
  v.erase(std::unique(v.begin(), v.end()), v.end());
  Bitmap b;
  size_t i = 0;
  while (i < v.size()) {
    uint16_t key = (uint16_t)(v[i] >> 16);
    std::vector<uint16_t> low;
    while (i < v.size() && (uint16_t)(v[i] >> 16) == key) low.push_back((uint16_t)(v[i++] & 0xFFFF));
    Ctr c = make_array(std::move(low));
    if (c.card > kArrayMax) c = to_bitmap(c);  // ArrayContainer.add converts past 4096
    b.keys.push_back(key);
    b.ctrs.push_back(std::move(c));
  }
  return b;
}

void bitmap_run_optimize(Bitmap& b) {
  for (Ctr& c : b.ctrs) c = run_optimize(c);
}

std::vector<uint32_t> bitmap_values(const Bitmap& b) {
  std::vector<uint32_t> out;
  for (size_t i = 0; i < b.size(); i++) {
    const Ctr& c = b.ctrs[i];
    uint32_t hi = (uint32_t)b.keys[i] << 16;
    if (c.kind == ARRAY) {
      for (uint16_t v : c.vals) out.push_back(hi | v);
    } else if (c.kind == BITMAP) {
      Ctr a = bitmap_to_array(c);
      for (uint16_t v : a.vals) out.push_back(hi | v);
    } else {
      for (uint16_t v : run_values(c)) out.push_back(hi | v);
    }
  }
  return out;
}

// key loop of RoaringBitmap.and (RB/RoaringBitmap.java:377-401); ImmutableRoaringBitmap.and
// (RB/buffer/ImmutableRoaringBitmap.java:299-325) is the same loop over Mappeable containers
template <class F>
static Bitmap and_like(const Bitmap& x1, const Bitmap& x2, F op) {
  Bitmap ans;
  size_t p1 = 0, p2 = 0;
  while (p1 < x1.size() && p2 < x2.size()) {
    uint16_t s1 = x1.keys[p1], s2 = x2.keys[p2];
    if (s1 == s2) {
      Ctr c = op(x1.ctrs[p1], x2.ctrs[p2]);
      if (!c.empty()) { ans.keys.push_back(s1); ans.ctrs.push_back(std::move(c)); }
      p1++;
      p2++;
    } else if (s1 < s2) {
      p1++;
    } else {
      p2++;
    }
  }
  return ans;
}
Bitmap op_and(const Bitmap& x1, const Bitmap& x2) { return and_like(x1, x2, c_and); }
Bitmap op_and_buf(const Bitmap& x1, const Bitmap& x2) { return and_like(x1, x2, c_and_buf); }

int32_t op_and_card(const Bitmap& x1, const Bitmap& x2) {
  uint32_t ans = 0;  // Java int accumulation wraps mod 2^32
  size_t p1 = 0, p2 = 0;
  while (p1 < x1.size() && p2 < x2.size()) {
    uint16_t s1 = x1.keys[p1], s2 = x2.keys[p2];
    if (s1 == s2) {
      ans += (uint32_t)c_and_card(x1.ctrs[p1], x2.ctrs[p2]);
      p1++;
      p2++;
    } else if (s1 < s2) {
      p1++;
    } else {
      p2++;
    }
  }
  return (int32_t)ans;
}

bool op_intersects(const Bitmap& x1, const Bitmap& x2) {
  size_t p1 = 0, p2 = 0;
  while (p1 < x1.size() && p2 < x2.size()) {
    uint16_t s1 = x1.keys[p1], s2 = x2.keys[p2];
    if (s1 == s2) {
      if (c_intersects(x1.ctrs[p1], x2.ctrs[p2])) return true;
      p1++;
      p2++;
    } else if (s1 < s2) {
      p1++;
    } else {
      p2++;
    }
  }
  return false;
}

// key loop of RoaringBitmap.andNot (RB/RoaringBitmap.java:444-473); ImmutableRoaringBitmap.andNot
// (RB/buffer/ImmutableRoaringBitmap.java:441-471) is the same loop over Mappeable containers
template <class F>
static Bitmap andnot_like(const Bitmap& x1, const Bitmap& x2, F op) {
  Bitmap ans;
  size_t p1 = 0, p2 = 0;
  while (p1 < x1.size() && p2 < x2.size()) {
    uint16_t s1 = x1.keys[p1], s2 = x2.keys[p2];
    if (s1 == s2) {
      Ctr c = op(x1.ctrs[p1], x2.ctrs[p2]);
      if (!c.empty()) { ans.keys.push_back(s1); ans.ctrs.push_back(std::move(c)); }
      p1++;
      p2++;
    } else if (s1 < s2) {
      ans.keys.push_back(s1);  // appendCopy (clone)
      ans.ctrs.push_back(x1.ctrs[p1]);
      p1++;
    } else {
      p2++;
    }
  }
  if (p2 == x2.size()) {
    for (; p1 < x1.size(); p1++) { ans.keys.push_back(x1.keys[p1]); ans.ctrs.push_back(x1.ctrs[p1]); }
  }
  return ans;
}
Bitmap op_andnot(const Bitmap& x1, const Bitmap& x2) { return andnot_like(x1, x2, c_andnot); }
Bitmap op_andnot_buf(const Bitmap& x1, const Bitmap& x2) { return andnot_like(x1, x2, c_andnot_buf); }

template <class F>
static Bitmap union_like(const Bitmap& x1, const Bitmap& x2, F op, bool drop_empty) {
  Bitmap ans;
  size_t p1 = 0, p2 = 0;
  while (p1 < x1.size() && p2 < x2.size()) {
    uint16_t s1 = x1.keys[p1], s2 = x2.keys[p2];
    if (s1 == s2) {
      Ctr c = op(x1.ctrs[p1], x2.ctrs[p2]);
      if (!drop_empty || !c.empty()) { ans.keys.push_back(s1); ans.ctrs.push_back(std::move(c)); }
      p1++;
      p2++;
    } else if (s1 < s2) {
      ans.keys.push_back(s1);
      ans.ctrs.push_back(x1.ctrs[p1]);
      p1++;
    } else {
      ans.keys.push_back(s2);
      ans.ctrs.push_back(x2.ctrs[p2]);
      p2++;
    }
  }
  for (; p1 < x1.size(); p1++) { ans.keys.push_back(x1.keys[p1]); ans.ctrs.push_back(x1.ctrs[p1]); }
  for (; p2 < x2.size(); p2++) { ans.keys.push_back(x2.keys[p2]); ans.ctrs.push_back(x2.ctrs[p2]); }
  return ans;
}

Bitmap op_or(const Bitmap& x1, const Bitmap& x2) { return union_like(x1, x2, c_or, false); }
// x1.or(x2) in place (RB/RoaringBitmap.java:2481-2523): the same key loop (x2-only containers
// cloned in, x1-only kept), Container.ior per matched key
Bitmap op_ior(const Bitmap& x1, const Bitmap& x2) { return union_like(x1, x2, c_ior, false); }
Bitmap op_xor(const Bitmap& x1, const Bitmap& x2) { return union_like(x1, x2, c_xor, true); }

int32_t op_or_card(const Bitmap& x1, const Bitmap& x2) {  // :916-920 (int arithmetic)
  return (int32_t)((uint32_t)x1.card() + (uint32_t)x2.card() - (uint32_t)op_and_card(x1, x2));
}
int32_t op_xor_card(const Bitmap& x1, const Bitmap& x2) {  // :931-933
  return (int32_t)((uint32_t)x1.card() + (uint32_t)x2.card() - 2u * (uint32_t)op_and_card(x1, x2));
}
int32_t op_andnot_card(const Bitmap& x1, const Bitmap& x2) {  // :944-985
  if (x2.size() > 4 * x1.size()) return (int32_t)((uint32_t)x1.card() - (uint32_t)op_and_card(x1, x2));
  int64_t card = 0;
  size_t p1 = 0, p2 = 0;
  while (p1 < x1.size() && p2 < x2.size()) {
    uint16_t s1 = x1.keys[p1], s2 = x2.keys[p2];
    if (s1 == s2) {
      card += x1.ctrs[p1].cardinality() - c_and_card(x1.ctrs[p1], x2.ctrs[p2]);
      p1++;
      p2++;
    } else if (s1 < s2) {
      while (s1 < s2 && p1 < x1.size()) {
        card += x1.ctrs[p1].cardinality();
        ++p1;
        if (p1 == x1.size()) break;
        s1 = x1.keys[p1];
      }
    } else {
      p2++;
    }
  }
  if (p2 == x2.size()) {
    while (p1 < x1.size()) card += x1.ctrs[p1++].cardinality();
  }
  return (int32_t)(uint32_t)(uint64_t)card;
}

// ---------------------------------------------------------------------------
// In-place bitmap ops used by the FastAggregation chains
// ---------------------------------------------------------------------------
// RB/RoaringBitmap.java:1272-1296 (heap: Container.iand); the buffer package's
// MutableRoaringBitmap.and(ImmutableRoaringBitmap) (RB/buffer/MutableRoaringBitmap.java:886-910) is the
// same key loop over MappeableContainer.iand
template <class F>
static void ip_and_with(Bitmap& a, const Bitmap& x2, F iand) {
  size_t p1 = 0, p2 = 0, isz = 0;
  const size_t l1 = a.size(), l2 = x2.size();
  while (p1 < l1 && p2 < l2) {
    uint16_t s1 = a.keys[p1], s2 = x2.keys[p2];
    if (s1 == s2) {
      Ctr c = iand(a.ctrs[p1], x2.ctrs[p2]);
      if (!c.empty()) { a.keys[isz] = s1; a.ctrs[isz] = std::move(c); isz++; }
      p1++;
      p2++;
    } else if (s1 < s2) {
      p1++;
    } else {
      p2++;
    }
  }
  a.keys.resize(isz);
  a.ctrs.resize(isz);
}

static void ip_and(Bitmap& a, const Bitmap& x2) { ip_and_with(a, x2, c_iand); }

// MappeableContainer.iand: MappeableRunContainer.iand(R) = and(R) keeps the merged run container
// (RB/buffer/MappeableRunContainer.java:1106-1108 -> :474-536, no toEfficientContainer); every other
// pair types as the heap's c_iand (MappeableArrayContainer.iand :674-700 filters in place,
// MappeableBitmapContainer.iand :572-677 as BitmapContainer.iand, MappeableRunContainer.iand(A|B)
// :1095-1102 = and(A|B) :398-471 as RunContainer.and)
static Ctr c_iand_buf(const Ctr& a, const Ctr& b) {
  if (a.kind == RUN && b.kind == RUN) return R_and_R_runs(a, b);
  return c_iand(a, b);
}
static void ip_and_buf(Bitmap& a, const Bitmap& x2) { ip_and_with(a, x2, c_iand_buf); }

static void ip_xor(Bitmap& a, const Bitmap& x2) {  // RB/RoaringBitmap.java:3296-3348
  size_t p1 = 0, p2 = 0;
  while (p1 < a.size() && p2 < x2.size()) {
    uint16_t s1 = a.keys[p1], s2 = x2.keys[p2];
    if (s1 == s2) {
      Ctr c = c_ixor(a.ctrs[p1], x2.ctrs[p2]);
      if (!c.empty()) {
        a.ctrs[p1] = std::move(c);
        p1++;
      } else {
        a.keys.erase(a.keys.begin() + p1);
        a.ctrs.erase(a.ctrs.begin() + p1);
      }
      p2++;
    } else if (s1 < s2) {
      p1++;
    } else {
      a.keys.insert(a.keys.begin() + p1, s2);
      a.ctrs.insert(a.ctrs.begin() + p1, x2.ctrs[p2]);
      p1++;
      p2++;
    }
  }
  for (; p2 < x2.size(); p2++) { a.keys.push_back(x2.keys[p2]); a.ctrs.push_back(x2.ctrs[p2]); }
}

static void naive_lazy_or(Bitmap& a, const Bitmap& x2) {  // RB/RoaringBitmap.java:2405-2448
  size_t p1 = 0, p2 = 0;
  while (p1 < a.size() && p2 < x2.size()) {
    uint16_t s1 = a.keys[p1], s2 = x2.keys[p2];
    if (s1 == s2) {
      a.ctrs[p1] = b_ilazyor(to_bitmap(a.ctrs[p1]), x2.ctrs[p2]);
      p1++;
      p2++;
    } else if (s1 < s2) {
      p1++;
    } else {
      a.keys.insert(a.keys.begin() + p1, s2);
      a.ctrs.insert(a.ctrs.begin() + p1, x2.ctrs[p2]);
      p1++;
      p2++;
    }
  }
  for (; p2 < x2.size(); p2++) { a.keys.push_back(x2.keys[p2]); a.ctrs.push_back(x2.ctrs[p2]); }
}

static bool all_empty(const Bitmap& b) { return b.size() == 0; }

Bitmap fa_or(const std::vector<const Bitmap*>& bms) {  // naive_or, RB/FastAggregation.java:603-610
  Bitmap ans;
  for (const Bitmap* b : bms) naive_lazy_or(ans, *b);
  for (Ctr& c : ans.ctrs) c = repair_after_lazy(c);  // RB/RoaringBitmap.java:2752-2757
  return ans;
}

Bitmap fa_xor(const std::vector<const Bitmap*>& bms) {  // naive_xor :637-644
  Bitmap ans;
  for (const Bitmap* b : bms) ip_xor(ans, *b);
  return ans;
}

Bitmap fa_naive_and(const std::vector<const Bitmap*>& bms, const int* ids) {  // :328-346
  if (bms.empty()) return Bitmap();
  size_t smallest = 0;
  for (size_t i = 1; i < bms.size(); i++)
    if (bms[i]->size() < bms[smallest]->size()) smallest = i;
  Bitmap ans = *bms[smallest];
  for (size_t k = 0; k < bms.size() && !all_empty(ans); k++) {
    bool same = ids ? (ids[k] == ids[smallest]) : (k == smallest);
    if (!same) ip_and(ans, *bms[k]);
  }
  return ans;
}

Bitmap fa_and_iter(const std::vector<const Bitmap*>& bms) {  // naive_and(Iterator) :304-313
  if (bms.empty()) return Bitmap();
  Bitmap ans = *bms[0];
  for (size_t k = 1; k < bms.size() && !all_empty(ans); k++) ip_and(ans, *bms[k]);
  return ans;
}

// BufferFastAggregation.naive_and(ImmutableRoaringBitmap...) (RB/buffer/BufferFastAggregation.java:347-369):
// smallest.toMutableRoaringBitmap(), then answer.and(bitmap) for every bitmap != smallest, with no
// early exit on an empty answer (an empty answer stays empty: same bytes)
Bitmap buf_naive_and(const std::vector<const Bitmap*>& bms, const int* ids) {
  if (bms.empty()) return Bitmap();
  size_t smallest = 0;
  for (size_t i = 1; i < bms.size(); i++)
    if (bms[i]->size() < bms[smallest]->size()) smallest = i;
  Bitmap ans = *bms[smallest];
  for (size_t k = 0; k < bms.size(); k++) {
    bool same = ids ? (ids[k] == ids[smallest]) : (k == smallest);
    if (!same) ip_and_buf(ans, *bms[k]);
  }
  return ans;
}

// naive_and(Iterator) :383-396 (first.toMutableRoaringBitmap()) and naive_and(MutableRoaringBitmap...)
// :407-416 (bitmaps[0].clone()): the buffer in-place and chain from the first input
Bitmap buf_and_iter(const std::vector<const Bitmap*>& bms) {
  if (bms.empty()) return Bitmap();
  Bitmap ans = *bms[0];
  for (size_t k = 1; k < bms.size(); k++) ip_and_buf(ans, *bms[k]);
  return ans;
}

// and(ImmutableRoaringBitmap...) / and(long[], ImmutableRoaringBitmap...) :28-56: workShyAnd above
// 10 inputs (buffer workShyAnd :426-494 types as the heap's), else the buffer naive_and
Bitmap buf_and(const std::vector<const Bitmap*>& bms, const int* ids) {
  if (bms.size() > 10) return fa_workshy_and(bms);
  return buf_naive_and(bms, ids);
}

// ---------------------------------------------------------------------------
// Range-restricted aggregations (RB/RoaringBitmap.java:1308-1336 and, 1396-1423 andNot, 2536-2557 or,
// 3359-3379 xor): every input through the private static selectRangeWithoutCopy (:3160-3214), then the
// unrestricted op.
// ---------------------------------------------------------------------------
// Container.remove(begin, end): the values of [begin, end) removed.  ArrayContainer.remove / iremove
// (RB/ArrayContainer.java:1039-1061, 759-780) stay arrays; BitmapContainer.remove / iremove
// (RB/BitmapContainer.java:1166-1181, 788-802) become arrays at <= 4096 values; RunContainer.remove
// = clone().iremove (RB/RunContainer.java:2032-2035, 1553-...) stays a run container, its runs clipped.
// end == begin: unchanged (remove returns a clone, iremove this).  buf: the buffer package's
// MappeableBitmapContainer.remove / iremove, an array only below 4096 values
// (RB/buffer/MappeableBitmapContainer.java:1597-1612, 1003-1017); its array and run forms cut alike.
static Ctr c_remove_range(const Ctr& c, int begin, int end, bool buf = false) {
  if (end == begin) return c;
  if (c.kind == ARRAY) {
    std::vector<uint16_t> v;
    for (uint16_t x : c.vals)
      if ((int)x < begin || (int)x >= end) v.push_back(x);
    return make_array(std::move(v));
  }
  if (c.kind == BITMAP) {
    Ctr b = c;
    b.card -= card_in_range(b.words, begin, end);
    reset_range(b.words, begin, end);
    if (buf ? b.card < kArrayMax : b.card <= kArrayMax) return bitmap_to_array(b);
    return b;
  }
  std::vector<uint16_t> pairs;
  for (int r = 0; r < c.nruns(); r++) {
    const int s = c.vals[2 * r], e = s + c.vals[2 * r + 1];  // inclusive
    if (s < begin) {
      const int e1 = std::min(e, begin - 1);
      pairs.push_back((uint16_t)s);
      pairs.push_back((uint16_t)(e1 - s));
    }
    if (e >= end) {
      const int s1 = std::max(s, end);
      pairs.push_back((uint16_t)s1);
      pairs.push_back((uint16_t)(e - s1));
    }
  }
  const int n = (int)pairs.size() / 2;
  return make_run(std::move(pairs), n);
}

// selectRangeWithoutCopy(RoaringBitmap, rangeStart, rangeEnd): the containers of the keys inside the
// range as they are, the first key's container through remove(0, lbStart), the last key's through
// remove(lbLast + 1, 65536) (one key: both), empty ones dropped.  buf: the buffer package's
// ImmutableRoaringBitmap.selectRangeWithoutCopy (RB/buffer/ImmutableRoaringBitmap.java:768-820), the
// same cuts with MappeableContainer.remove
Bitmap select_range(const Bitmap& b, uint64_t start, uint64_t end, bool buf) {
  Bitmap ans;
  if (end <= start) return ans;
  const int hbs = (int)(start >> 16), lbs = (int)(start & 0xFFFF);
  const int hbl = (int)((end - 1) >> 16), lbl = (int)((end - 1) & 0xFFFF);
  for (size_t i = 0; i < b.size(); i++) {
    const int k = b.keys[i];
    if (k < hbs || k > hbl) continue;
    Ctr c = b.ctrs[i];
    if (k == hbs) c = c_remove_range(c, 0, lbs, buf);
    if (k == hbl) c = c_remove_range(c, lbl + 1, 65536, buf);
    if (!c.empty()) {
      ans.keys.push_back((uint16_t)k);
      ans.ctrs.push_back(std::move(c));
    }
  }
  return ans;
}

// op 0: and(Iterator, start, end) -> FastAggregation.and(Iterator) = naive_and(Iterator) (:304-313);
// 1: or -> FastAggregation.or(Iterator) = naive_or; 2: xor -> FastAggregation.xor(Iterator) = naive_xor
Bitmap range_aggregate(int op, const std::vector<const Bitmap*>& bms, uint64_t start, uint64_t end) {
  std::vector<Bitmap> sel;
  sel.reserve(bms.size());
  for (const Bitmap* b : bms) sel.push_back(select_range(*b, start, end));
  std::vector<const Bitmap*> ptrs;
  for (const Bitmap& b : sel) ptrs.push_back(&b);
  if (op == 0) return fa_and_iter(ptrs);
  if (op == 1) return fa_or(ptrs);
  return fa_xor(ptrs);
}

Bitmap op_andnot_range(const Bitmap& x1, const Bitmap& x2, uint64_t start, uint64_t end) {
  return op_andnot(select_range(x1, start, end), select_range(x2, start, end));
}

// The buffer package's range forms, RB/buffer/ImmutableRoaringBitmap.java: every input through its
// selectRangeWithoutCopy, then and(Iterator, start, end) :261-267 -> BufferFastAggregation.and(Iterator)
// = workShyAnd for any count (RB/buffer/BufferFastAggregation.java:66-89, 505-576; no input: empty);
// or :992-998 -> naive_or (:886-888, 791-798); xor :1048-1053 -> naive_xor (:1072-1074, 843-849);
// andNot(x1, x2, start, end) :402-408 -> ImmutableRoaringBitmap.andNot (the buffer run types)
Bitmap range_aggregate_buf(int op, const std::vector<const Bitmap*>& bms, uint64_t start, uint64_t end) {
  std::vector<Bitmap> sel;
  sel.reserve(bms.size());
  for (const Bitmap* b : bms) sel.push_back(select_range(*b, start, end, true));
  std::vector<const Bitmap*> ptrs;
  for (const Bitmap& b : sel) ptrs.push_back(&b);
  if (op == 0) return ptrs.empty() ? Bitmap() : fa_workshy_and(ptrs);
  if (op == 1) return fa_or(ptrs);
  if (op == 2) return fa_xor(ptrs);
  return op_andnot_buf(sel[0], sel[1]);
}

// ---------------------------------------------------------------------------
// orNot (RB/RoaringBitmap.java:1431-1506 in place, :1521-1603 static)
// ---------------------------------------------------------------------------
// Container.not(0, end), end in [1, 65536]:
//  ArrayContainer.not (RB/ArrayContainer.java:876-925): the new cardinality is card - m + (end - m)
//    (m values below end); above 4096 it is toBitmapContainer().not, else an array of the complement
//    in [0, end) followed by the values >= end;
//  BitmapContainer.not = clone().inot (RB/BitmapContainer.java:994-997, 679-687): the range flipped,
//    toArrayContainer at <= 4096 values;
//  RunContainer.not (RB/RunContainer.java:1900-1918): no run starts below 0, so the answer is the run
//    [0, end) followed by every run through smartAppendExclusive, then toEfficientContainer.
Ctr c_not_prefix(const Ctr& c, int end) {
  if (end <= 0) return c;
  if (c.kind == ARRAY) {
    const int m = (int)(std::lower_bound(c.vals.begin(), c.vals.end(), end) - c.vals.begin());
    const int newcard = c.card - m + (end - m);
    if (newcard > kArrayMax) return c_not_prefix(to_bitmap(c), end);
    std::vector<uint16_t> v;
    v.reserve(newcard);
    int i = 0;
    for (int x = 0; x < end; x++) {
      if (i < m && (int)c.vals[i] == x) i++;
      else v.push_back((uint16_t)x);
    }
    for (int j = m; j < c.card; j++) v.push_back(c.vals[j]);
    return make_array(std::move(v));
  }
  if (c.kind == BITMAP) {
    Ctr b = c;
    const int prev = card_in_range(b.words, 0, end);
    flip_range(b.words, 0, end);
    b.card += (end - prev) - prev;
    if (b.card <= kArrayMax) return bitmap_to_array(b);
    return b;
  }
  RunBuf ans(c.nruns() + 1);
  ans.smart_append_excl(0, end - 1);
  for (int k = 0; k < c.nruns(); k++) ans.smart_append_excl(c.vals[2 * k], c.vals[2 * k + 1]);
  return to_efficient(ans.build());
}

// Container.not(start, end) for any range (the static RoaringBitmap.flip's per-key step): as
// c_not_prefix, with the values below `start` kept -- ArrayContainer.not copies them, RunContainer.not
// copies the runs that start below `start` and XOR-appends the range and the rest (RB/RunContainer.java
// :1900-1918)
static Ctr c_not_range(const Ctr& c, int start, int end) {
  if (end <= start) return c;
  if (c.kind == ARRAY) {
    const int i0 = (int)(std::lower_bound(c.vals.begin(), c.vals.end(), start) - c.vals.begin());
    const int i1 = (int)(std::lower_bound(c.vals.begin(), c.vals.end(), end) - c.vals.begin());
    const int m = i1 - i0;
    const int newcard = c.card - m + (end - start - m);
    if (newcard > kArrayMax) return c_not_range(to_bitmap(c), start, end);
    std::vector<uint16_t> v(c.vals.begin(), c.vals.begin() + i0);
    int i = i0;
    for (int x = start; x < end; x++) {
      if (i < i1 && (int)c.vals[i] == x) i++;
      else v.push_back((uint16_t)x);
    }
    v.insert(v.end(), c.vals.begin() + i1, c.vals.end());
    return make_array(std::move(v));
  }
  if (c.kind == BITMAP) {
    Ctr b = c;
    const int prev = card_in_range(b.words, start, end);
    flip_range(b.words, start, end);
    b.card += (end - start - prev) - prev;
    if (b.card <= kArrayMax) return bitmap_to_array(b);
    return b;
  }
  RunBuf ans(c.nruns() + 1);
  int k = 0;
  for (; k < c.nruns() && (int)c.vals[2 * k] < start; k++) ans.push(c.vals[2 * k], c.vals[2 * k + 1]);
  ans.smart_append_excl(start, end - start - 1);
  for (; k < c.nruns(); k++) ans.smart_append_excl(c.vals[2 * k], c.vals[2 * k + 1]);
  return to_efficient(ans.build());
}

// Container.add(begin, end): ArrayContainer.add (RB/ArrayContainer.java:103-135) an array, or above 4096
// values toBitmapContainer().iadd, a bitmap; BitmapContainer.add (RB/BitmapContainer.java:131-143) a
// bitmap, a full one included; RunContainer.add = clone().iadd (RB/RunContainer.java:242-245, 1068-...)
// a run container whatever its size (its runs merged with the range, adjacent ones joined)
static Ctr c_add_range(const Ctr& c, int begin, int end) {
  if (end == begin) return c;
  Ctr b = to_bitmap(c);
  set_range(b.words, begin, end);
  compute_card_inplace(b);
  if (c.kind == BITMAP) return b;
  if (c.kind == ARRAY) return b.card > kArrayMax ? b : bitmap_to_array(b);
  std::vector<uint16_t> v;
  v.reserve(b.card);
  for (int w = 0; w < kWords; w++)
    for (uint64_t x = b.words[w]; x; x &= x - 1) v.push_back((uint16_t)(64 * w + __builtin_ctzll(x)));
  return runs_from_values(v);
}

// Container.rangeOfOnes(0, last) (RB/Container.java:29-37): an array up to 2 values, else a run
static Ctr range_of_ones_at(int start, int last) {
  if (last - start <= 2) {
    std::vector<uint16_t> v;
    for (int x = start; x < last; x++) v.push_back((uint16_t)x);
    return make_array(std::move(v));
  }
  return make_run({(uint16_t)start, (uint16_t)(last - start - 1)}, 1);
}
static Ctr range_of_ones(int last) { return range_of_ones_at(0, last); }

// Container.orNot / iorNot (RB/Container.java:191-196, 536-541): or / ior with
// x.not(0, end).iremove(end, 0x10000) (end < 0x10000) or x.not(0, 0x10000).  buf: the buffer package's
// MappeableContainer.orNot / iorNot (RB/buffer/MappeableContainer.java:214-236), whose containers type
// like the heap's except MappeableBitmapContainer.iremove, which becomes an array below 4096 values,
// not at 4096 (RB/buffer/MappeableBitmapContainer.java:1003-1017)
static Ctr c_ornot(const Ctr& c1, const Ctr& c2, int end, bool inplace, bool buf) {
  Ctr x = c_not_prefix(c2, end);
  if (end < 0x10000) {
    if (buf && x.kind == BITMAP) {
      x.card -= card_in_range(x.words, end, 0x10000);
      reset_range(x.words, end, 0x10000);
      if (x.card < kArrayMax) x = bitmap_to_array(x);
    } else {
      x = c_remove_range(x, end, 0x10000);
    }
  }
  return inplace ? c_ior(c1, x) : c_or(c1, x);
}

Bitmap op_ornot(const Bitmap& x1, const Bitmap& x2, uint64_t range_end, bool inplace, bool* neg, bool buf) {
  *neg = false;
  // (int)((rangeEnd - 1) >>> 16): -1 for rangeEnd == 0
  const int max_key = range_end == 0 ? -1 : (int)((range_end - 1) >> 16);
  const int last_run = (range_end & 0xFFFF) == 0 ? 0x10000 : (int)(range_end & 0xFFFF);
  const int n1 = (int)x1.size(), n2 = (int)x2.size();
  int remainder = 0;
  for (int i = n1 - 1; i >= 0 && (int)x1.keys[i] > max_key; --i) ++remainder;
  int correction = 0;
  for (int i = 0; i < n2 - remainder; ++i) {
    correction += x2.ctrs[i].full() ? 1 : 0;
    if ((int)x2.keys[i] >= max_key) break;
  }
  // the reference's "conservative overestimate", which bounds the key loop below
  const int max_size = std::min(max_key + 1 + remainder - correction + n1, 0x10000);
  if (max_size < 0) {
    *neg = true;
    return Bitmap();
  }
  if (max_size == 0) return inplace ? x1 : Bitmap();
  Bitmap ans;
  int p1 = 0, p2 = 0;
  int s1 = n1 > 0 ? x1.keys[0] : max_key + 1;
  int s2 = n2 > 0 ? x2.keys[0] : max_key + 1;
  int size = 0;
  for (int key = 0; key <= max_key && size < max_size; ++key) {
    const int e = key == max_key ? last_run : 0x10000;
    Ctr v;
    if (key == s1 && key == s2) {
      v = c_ornot(x1.ctrs[p1], x2.ctrs[p2], e, inplace, buf);
      ++p1;
      ++p2;
      s1 = p1 < n1 ? x1.keys[p1] : max_key + 1;
      s2 = p2 < n2 ? x2.keys[p2] : max_key + 1;
    } else if (key == s1) {  // x1.ior(rangeOfOnes) at maxKey (also in the static form), else full
      v = key == max_key ? c_ior(x1.ctrs[p1], range_of_ones(last_run)) : run_full();
      ++p1;
      s1 = p1 < n1 ? x1.keys[p1] : max_key + 1;
    } else if (key == s2) {  // the complement, not clipped at rangeEnd
      v = c_not_prefix(x2.ctrs[p2], e);
      ++p2;
      s2 = p2 < n2 ? x2.keys[p2] : max_key + 1;
    } else {
      v = key == max_key ? range_of_ones(last_run) : run_full();
    }
    if (!v.empty()) {
      ans.keys.push_back((uint16_t)key);
      ans.ctrs.push_back(std::move(v));
      ++size;
    }
  }
  for (int i = n1 - remainder; i < n1; i++) {
    ans.keys.push_back(x1.keys[i]);
    ans.ctrs.push_back(x1.ctrs[i]);
  }
  return ans;
}

// The static range mutations, RB/RoaringBitmap.java: add(rb, rangeStart, rangeEnd) :298-345 (first / last
// key through Container.add, the keys between replaced by full run containers, a missing key by
// rangeOfOnes), remove(rb, ...) :995-1040 (first / last key through Container.remove unless the cut
// covers the whole key, the keys between dropped, emptied containers dropped), flip(rb, ...) :626-668
// (every key of the range through Container.not, a missing key rangeOfOnes, emptied containers dropped);
// the keys outside the range cloned.  buf: MutableRoaringBitmap's (RB/buffer/MutableRoaringBitmap.java
// :152-205, 455-505, 649-700), whose MappeableBitmapContainer.remove keeps a 4096-value bitmap.
// op 0 add, 1 remove, 2 flip, 3 x.add(rangeStart, rangeEnd) in place (:1181-1206: Container.iadd on every
// key of the range, the keys between included -- an array there becomes a full bitmap, not a full run
// container; the in-place remove :2656-2710 and flip :1893-1925 end in the static forms' containers).
// rangeEnd <= rangeStart: a clone.
Bitmap op_range_mut(int op, const Bitmap& b, uint64_t start, uint64_t end, bool buf) {
  if (end <= start) return b;
  const int hbs = (int)(start >> 16), lbs = (int)(start & 0xFFFF);
  const int hbl = (int)((end - 1) >> 16), lbl = (int)((end - 1) & 0xFFFF);
  Bitmap ans;
  auto put = [&](int k, Ctr c) {
    if (!c.empty()) {
      ans.keys.push_back((uint16_t)k);
      ans.ctrs.push_back(std::move(c));
    }
  };
  const Ctr* cur = nullptr;
  size_t i = 0;
  for (; i < b.size() && (int)b.keys[i] < hbs; i++) put(b.keys[i], b.ctrs[i]);
  for (int k = hbs; k <= hbl; k++) {
    cur = (i < b.size() && (int)b.keys[i] == k) ? &b.ctrs[i] : nullptr;
    if (cur) i++;
    const int lo = k == hbs ? lbs : 0, hi = k == hbl ? lbl : 65535;
    if (op == 0 || op == 3) {
      if (op == 0 && k != hbs && k != hbl) put(k, run_full());  // rangeOfOnes(0, 65536)
      else put(k, cur ? c_add_range(*cur, lo, hi + 1) : range_of_ones_at(lo, hi + 1));
    } else if (op == 1) {
      if (!cur) continue;
      if (hbs == hbl) put(k, c_remove_range(*cur, lo, hi + 1, buf));
      else if (k == hbs && lbs != 0) put(k, c_remove_range(*cur, lbs, 65536, buf));
      else if (k == hbl && lbl != 65535) put(k, c_remove_range(*cur, 0, lbl + 1, buf));
    } else {
      put(k, cur ? c_not_range(*cur, lo, hi + 1) : range_of_ones_at(lo, hi + 1));
    }
  }
  for (; i < b.size(); i++) put(b.keys[i], b.ctrs[i]);
  return ans;
}

// Util.addOffset(Container, char offsets) (RB/Util.java:32-126; the buffer package's BufferUtil.addOffset,
// RB/buffer/BufferUtil.java:33-135, is the same): the container's values plus `off`, split at 65536 into
// the part that stays in the key (lo) and the part that moves to key + 1 (hi), not converted except a
// bitmap's, through repairAfterLazy.
static void add_offset_parts(const Ctr& c, int off, Ctr* lo, Ctr* hi) {
  if (c.kind == ARRAY) {  // addOffsetArray :43-79
    std::vector<uint16_t> l, h;
    for (int k = 0; k < c.card; k++) {
      const int v = c.vals[k] + off;
      if (v <= 0xFFFF) l.push_back((uint16_t)v);
      else h.push_back((uint16_t)v);
    }
    *lo = make_array(std::move(l));
    *hi = make_array(std::move(h));
  } else if (c.kind == BITMAP) {  // addOffsetBitmap :81-105
    Ctr l = make_bitmap_zero(), h = make_bitmap_zero();
    l.card = h.card = -1;
    const int b = off >> 6, i = off % 64;
    if (i == 0) {
      for (int k = 0; k < kWords - b; k++) l.words[b + k] = c.words[k];
      for (int k = kWords - b; k < kWords; k++) h.words[k - (kWords - b)] = c.words[k];
    } else {
      l.words[b] = c.words[0] << i;
      for (int k = 1; k < kWords - b; k++) l.words[b + k] = (c.words[k] << i) | (c.words[k - 1] >> (64 - i));
      for (int k = kWords - b; k < kWords; k++)
        h.words[k - (kWords - b)] = (c.words[k] << i) | (c.words[k - 1] >> (64 - i));
      h.words[b] = c.words[kWords - 1] >> (64 - i);
    }
    *lo = repair_after_lazy(l);
    *hi = repair_after_lazy(h);
  } else {  // addOffsetRun :107-126
    RunBuf l(c.nruns()), h(c.nruns());
    for (int k = 0; k < c.nruns(); k++) {
      const int val = c.vals[2 * k] + off, len = c.vals[2 * k + 1];
      const int finalval = val + len;
      if (val <= 0xFFFF) {
        if (finalval <= 0xFFFF) {
          l.smart_append(val, len);
        } else {
          l.smart_append(val, 0xFFFF - val);
          h.smart_append(0, finalval & 0xFFFF);
        }
      } else {
        h.smart_append(val & 0xFFFF, len);
      }
    }
    *lo = l.build();
    *hi = h.build();
  }
}

// RoaringBitmap.addOffset(x, offset) (RB/RoaringBitmap.java:230-288; MutableRoaringBitmap.addOffset,
// RB/buffer/MutableRoaringBitmap.java:84-142, types alike).  A container offset outside [-65536, 65535]:
// empty.  A whole-key offset clones the containers under the shifted keys; keys that leave [0, 65535]
// are dropped here, where the reference's (char) cast wraps them into an unsorted key list (an invalid
// bitmap).  Otherwise each container's two parts go to key and key + 1; a low part whose
// key is the last one appended is OR-ed into it with Container.ior; then repairAfterLazy over the bitmap.
Bitmap op_add_offset(const Bitmap& x, int64_t offset) {
  const int64_t co_l = offset < 0 ? (offset - (1 << 16) + 1) / (1 << 16) : offset / (1 << 16);
  Bitmap ans;
  if (co_l < -(1 << 16) || co_l >= (1 << 16)) return ans;
  const int co = (int)co_l;
  const int off = (int)(offset - co_l * (1LL << 16));
  if (off == 0) {
    for (size_t p = 0; p < x.size(); p++) {
      const int key = x.keys[p] + co;
      if (key < 0 || key > 0xFFFF) continue;
      ans.keys.push_back((uint16_t)key);
      ans.ctrs.push_back(x.ctrs[p]);
    }
    return ans;
  }
  for (size_t p = 0; p < x.size(); p++) {
    const int key = x.keys[p] + co;
    if (key + 1 < 0 || key > 0xFFFF) continue;
    Ctr lo, hi;
    add_offset_parts(x.ctrs[p], off, &lo, &hi);
    if (!lo.empty() && key >= 0) {
      if (!ans.keys.empty() && (int)ans.keys.back() == key) ans.ctrs.back() = c_ior(ans.ctrs.back(), lo);
      else { ans.keys.push_back((uint16_t)key); ans.ctrs.push_back(std::move(lo)); }
    }
    if (!hi.empty() && key + 1 <= 0xFFFF) {
      ans.keys.push_back((uint16_t)(key + 1));
      ans.ctrs.push_back(std::move(hi));
    }
  }
  for (auto& c : ans.ctrs) c = repair_after_lazy(c);  // RB/RoaringBitmap.java:2752-2757
  return ans;
}

// Container.limit(n), n < card: the first n values -- ArrayContainer.limit an array (RB/ArrayContainer.java
// :825-831), BitmapContainer.limit an array at <= 4096 values, else a bitmap (RB/BitmapContainer.java
// :912-938), RunContainer.limit the runs up to the n-th value, a run container (RB/RunContainer.java:1856-1875)
static Ctr c_limit(const Ctr& c, int n) {
  if (c.kind == ARRAY) return make_array(std::vector<uint16_t>(c.vals.begin(), c.vals.begin() + n));
  if (c.kind == BITMAP) {
    std::vector<uint16_t> v;
    for (int w = 0; w < kWords && (int)v.size() < n; w++)
      for (uint64_t x = c.words[w]; x && (int)v.size() < n; x &= x - 1) v.push_back((uint16_t)(64 * w + __builtin_ctzll(x)));
    Ctr a = make_array(std::move(v));
    return n <= kArrayMax ? a : to_bitmap(a);
  }
  std::vector<uint16_t> p;
  int card = 0, r = 0;
  for (; r < c.nruns(); r++) {
    card += c.vals[2 * r + 1] + 1;
    if (n <= card) break;
  }
  p.assign(c.vals.begin(), c.vals.begin() + 2 * (r + 1));
  p[2 * r + 1] = (uint16_t)(p[2 * r + 1] - card + n);
  return make_run(std::move(p), r + 1);
}

// RoaringBitmap.bitmapOfRange(min, max) (RB/RoaringBitmap.java:588-615): RunContainer.rangeOfOnes per key
Bitmap op_bitmap_of_range(uint64_t min, uint64_t max) {
  Bitmap ans;
  if (min >= max) return ans;
  const int hbs = (int)(min >> 16), hbl = (int)((max - 1) >> 16);
  for (int k = hbs; k <= hbl; k++) {
    const int lo = k == hbs ? (int)(min & 0xFFFF) : 0, hi = k == hbl ? (int)((max - 1) & 0xFFFF) : 65535;
    ans.keys.push_back((uint16_t)k);
    ans.ctrs.push_back(make_run(std::vector<uint16_t>{(uint16_t)lo, (uint16_t)(hi - lo)}, 1));
  }
  return ans;
}

// x.limit(maxcardinality) (RB/RoaringBitmap.java:2457-2476): whole containers while they fit, the next
// one through Container.limit(leftover)
Bitmap op_limit(const Bitmap& x, int32_t maxcard) {
  Bitmap ans;
  int32_t cur = 0;
  for (size_t i = 0; cur < maxcard && i < x.size(); i++) {
    const int cc = x.ctrs[i].cardinality();
    if ((int64_t)cc + cur <= maxcard) {
      ans.keys.push_back(x.keys[i]);
      ans.ctrs.push_back(x.ctrs[i]);
      cur += cc;
    } else {
      ans.keys.push_back(x.keys[i]);
      ans.ctrs.push_back(c_limit(x.ctrs[i], maxcard - cur));
      break;
    }
  }
  return ans;
}

// x.removeRunCompression() (RB/RoaringBitmap.java:2738-2749): every run container through
// toBitmapOrArrayContainer(getCardinality()) (RB/RunContainer.java:2300-2323)
Bitmap op_remove_run_compression(const Bitmap& x) {
  Bitmap ans = x;
  for (auto& c : ans.ctrs)
    if (c.kind == RUN) c = to_bitmap_or_array(c, c.cardinality());
  return ans;
}

// key-bitset intersection shared by workShyAnd / workShyAndCardinality
static std::vector<uint16_t> common_keys(const std::vector<const Bitmap*>& bms) {
  std::vector<uint64_t> words(1024, 0);
  const Bitmap& first = *bms[0];
  for (uint16_t k : first.keys) words[k >> 6] |= 1ULL << (k & 63);
  int num = (int)first.size();
  for (size_t i = 1; i < bms.size() && num > 0; i++) {
    // Util.intersectArrayIntoBitmap (RB/Util.java:531-555), returned count only
    std::vector<uint64_t> m(1024, 0);
    for (uint16_t k : bms[i]->keys) m[k >> 6] |= 1ULL << (k & 63);
    num = 0;
    for (int w = 0; w < 1024; w++) { words[w] &= m[w]; num += popc(words[w]); }
  }
  std::vector<uint16_t> keys;
  if (num == 0) return keys;
  for (int w = 0; w < 1024; w++) {
    uint64_t x = words[w];
    while (x) { keys.push_back((uint16_t)(w * 64 + __builtin_ctzll(x))); x &= x - 1; }
  }
  return keys;
}

static const Ctr* find_ctr(const Bitmap& b, uint16_t key) {
  auto it = std::lower_bound(b.keys.begin(), b.keys.end(), key);
  if (it == b.keys.end() || *it != key) return nullptr;
  return &b.ctrs[it - b.keys.begin()];
}

static Ctr lazy_full_bitmap() {
  Ctr b;
  b.kind = BITMAP;
  b.words.assign(kWords, ~0ULL);
  b.card = -1;
  return b;
}

Bitmap fa_workshy_and(const std::vector<const Bitmap*>& bms) {  // :356-414
  Bitmap ans;
  std::vector<uint16_t> keys = common_keys(bms);
  for (uint16_t key : keys) {
    Ctr tmp = lazy_full_bitmap();
    for (const Bitmap* b : bms) tmp = b_lazy_iand(tmp, *find_ctr(*b, key));
    tmp = repair_after_lazy(tmp);
    if (!tmp.empty()) { ans.keys.push_back(key); ans.ctrs.push_back(std::move(tmp)); }
  }
  return ans;
}

Bitmap fa_and(const std::vector<const Bitmap*>& bms, const int* ids) {  // :37-42
  if (bms.size() > 10) return fa_workshy_and(bms);
  return fa_naive_and(bms, ids);
}

int32_t fa_and_card(const std::vector<const Bitmap*>& bms) {  // :71-82, workShyAndCardinality :416-462
  if (bms.empty()) return 0;
  if (bms.size() == 1) return bms[0]->card();
  if (bms.size() == 2) return op_and_card(*bms[0], *bms[1]);
  uint32_t card = 0;
  for (uint16_t key : common_keys(bms)) {
    Ctr tmp = lazy_full_bitmap();
    for (const Bitmap* b : bms) {
      const Ctr* c = find_ctr(*b, key);
      if (c) tmp = b_lazy_iand(tmp, *c);
    }
    card += (uint32_t)repair_after_lazy(tmp).cardinality();
  }
  return (int32_t)card;
}

int32_t fa_or_card(const std::vector<const Bitmap*>& bms) {  // :90-101, horizontalOrCardinality :464-506
  if (bms.empty()) return 0;
  if (bms.size() == 1) return bms[0]->card();
  if (bms.size() == 2) return op_or_card(*bms[0], *bms[1]);
  std::vector<uint64_t> kw(1024, 0);
  for (const Bitmap* b : bms) for (uint16_t k : b->keys) kw[k >> 6] |= 1ULL << (k & 63);
  uint32_t card = 0;
  for (int w = 0; w < 1024; w++) {
    uint64_t x = kw[w];
    while (x) {
      uint16_t key = (uint16_t)(w * 64 + __builtin_ctzll(x));
      x &= x - 1;
      Ctr tmp = make_bitmap_zero();
      tmp.card = -1;
      for (const Bitmap* b : bms) {
        const Ctr* c = find_ctr(*b, key);
        if (c) tmp = b_ilazyor(tmp, *c);
      }
      card += (uint32_t)repair_after_lazy(tmp).cardinality();
    }
  }
  return (int32_t)card;
}

// ============================================================================
// Lazy OR algebra and the alternative aggregations (ParallelAggregation,
// horizontal_*, priorityqueue_*, BufferFastAggregation over Mutable bitmaps)
// ============================================================================
// ArrayContainer.lazyor(ArrayContainer), RB/ArrayContainer.java:1449-1463
static Ctr A_lazyor_A(const Ctr& a, const Ctr& x) {
  if (a.card + x.card > kArrayLazyLowerBound) return b_ilazyor(to_bitmap(a), x);  // toBitmapContainer().lazyIOR
  return make_array(v_union(a.vals, x.vals));
}
// RunContainer.ilazyor(ArrayContainer), RB/RunContainer.java:1198-1240: a full container
// is returned as is; otherwise ilazyorToRun, whose merge equals lazyorToRun's (a full
// merge is the single run (0, 65535) either way) + convertToLazyBitmapIfNeeded
static Ctr R_ilazyor_A(const Ctr& r, const Ctr& a) { return r.full() ? r : R_lazyor_A(r, a); }
// RunContainer.ior(BitmapContainer) :1500-1506 / ior(RunContainer) :1508-1550 (the merge of
// ior(R) then toEfficientContainer; R_or_R's extra full checks give the same container)
static Ctr R_ior_B(const Ctr& r, const Ctr& b) { return r.full() ? r : R_or_B(r, b); }
static Ctr R_ior_R(const Ctr& r, const Ctr& x) { return r.full() ? r : R_or_R(r, x); }

// Container.lazyIOR, RB/Container.java:717-740
Ctr c_lazy_ior(const Ctr& cur, const Ctr& x) {
  switch (cur.kind) {
    case ARRAY:
      if (x.kind == ARRAY) return A_lazyor_A(cur, x);
      if (x.kind == BITMAP) return B_or_A(x, cur);  // ior(BitmapContainer) = x.or(this), :748-750
      return R_lazyor_A(x, cur);                     // x.lazyor(this)
    case RUN:
      if (x.kind == ARRAY) return R_ilazyor_A(cur, x);
      if (x.kind == BITMAP) return R_ior_B(cur, x);
      return R_ior_R(cur, x);
    default:
      return b_ilazyor(cur, x);  // BitmapContainer.ilazyor(A|B|R), RB/BitmapContainer.java:648-676
  }
}

// Container.lazyOR, RB/Container.java:752-774 (not in place)
Ctr c_lazy_or(const Ctr& a, const Ctr& x) {
  switch (a.kind) {
    case ARRAY:
      if (x.kind == ARRAY) return A_lazyor_A(a, x);
      if (x.kind == BITMAP) return b_ilazyor(x, a);  // BitmapContainer.lazyor(A): clone, card -1 (:878-888)
      return R_lazyor_A(x, a);
    case RUN:
      if (x.kind == ARRAY) return R_lazyor_A(a, x);
      if (x.kind == BITMAP) return b_ilazyor(x, a);  // BitmapContainer.lazyor(R) (:900-909)
      return R_or_R(a, x);
    default:
      return b_ilazyor(a, x);  // BitmapContainer.lazyor(A|B|R) :878-909
  }
}

// java.util.PriorityQueue (OpenJDK): array binary heap; add = siftUp, poll = last element
// sifted down from the root.  Ties are resolved by this exact structure, so the poll order
// of equal elements is reproduced.
template <class T, class Cmp>
struct JavaPQ {
  std::vector<T> q;
  Cmp cmp;
  explicit JavaPQ(Cmp c) : cmp(c) {}
  bool empty() const { return q.empty(); }
  size_t size() const { return q.size(); }
  const T& peek() const { return q[0]; }
  void add(T x) {
    size_t k = q.size();
    q.push_back(x);
    while (k > 0) {
      size_t p = (k - 1) >> 1;
      if (cmp(x, q[p]) >= 0) break;
      q[k] = q[p];
      k = p;
    }
    q[k] = x;
  }
  T poll() {
    T r = q[0];
    T x = q.back();
    q.pop_back();
    size_t n = q.size();
    if (n > 0) {
      size_t k = 0, half = n >> 1;
      while (k < half) {
        size_t c = 2 * k + 1, rr = c + 1;
        if (rr < n && cmp(q[c], q[rr]) > 0) c = rr;
        if (cmp(x, q[c]) <= 0) break;
        q[k] = q[c];
        k = c;
      }
      q[k] = x;
    }
    return r;
  }
};

static std::map<uint16_t, std::vector<const Ctr*>> group_by_key(const std::vector<const Bitmap*>& bms) {
  std::map<uint16_t, std::vector<const Ctr*>> g;  // ParallelAggregation.groupByKey :137-153
  for (const Bitmap* b : bms)
    for (size_t i = 0; i < b->size(); i++) g[b->keys[i]].push_back(&b->ctrs[i]);
  return g;
}

// ParallelAggregation.or(List<Container>), RB/ParallelAggregation.java:197-223.  At 512 and
// more containers the reference splits the list over the ForkJoin pool and ORs each part's
// result into a lazy bitmap (OrCollector :103-130); like the 16..511 branch that ends in
// BitmapContainer.repairAfterLazy of the lazy union, so both take the lazy-bitmap branch here.
Ctr pa_or_key(const std::vector<const Ctr*>& cs) {
  if (cs.size() < 16) {
    Ctr r = *cs[0];
    for (size_t i = 1; i < cs.size(); i++) r = c_lazy_ior(r, *cs[i]);
    return repair_after_lazy(r);
  }
  Ctr r = make_bitmap_zero();
  r.card = -1;
  for (const Ctr* c : cs) r = b_ilazyor(r, *c);
  return repair_after_lazy(r);
}

// ParallelAggregation.xor(List<Container>) :189-195: clone + ixor chain, no restart
Ctr pa_xor_key(const std::vector<const Ctr*>& cs) {
  Ctr r = *cs[0];
  for (size_t i = 1; i < cs.size(); i++) r = c_ixor(r, *cs[i]);
  return r;
}

Bitmap pa_or(const std::vector<const Bitmap*>& bms) {  // :161-175 (empty results kept, none occur)
  Bitmap ans;
  for (auto& kv : group_by_key(bms)) {
    ans.keys.push_back(kv.first);
    ans.ctrs.push_back(pa_or_key(kv.second));
  }
  return ans;
}

Bitmap pa_xor(const std::vector<const Bitmap*>& bms) {  // :182-187, ContainerCollector drops empties :71-77
  Bitmap ans;
  for (auto& kv : group_by_key(bms)) {
    Ctr c = pa_xor_key(kv.second);
    if (!c.empty()) {
      ans.keys.push_back(kv.first);
      ans.ctrs.push_back(std::move(c));
    }
  }
  return ans;
}

// RoaringBitmap.lazyor(RoaringBitmap) in place, RB/RoaringBitmap.java:2357-2400
// (MutableRoaringBitmap.lazyor, RB/buffer/MutableRoaringBitmap.java:1309-1351, has the same
// per-key algebra through MappeableContainer.lazyIOR, RB/buffer/MappeableContainer.java:639-662)
static void ip_lazy_or(Bitmap& a, const Bitmap& x2) {
  size_t p1 = 0, p2 = 0;
  while (p1 < a.size() && p2 < x2.size()) {
    uint16_t s1 = a.keys[p1], s2 = x2.keys[p2];
    if (s1 == s2) {
      a.ctrs[p1] = c_lazy_ior(a.ctrs[p1], x2.ctrs[p2]);
      p1++;
      p2++;
    } else if (s1 < s2) {
      p1++;
    } else {
      a.keys.insert(a.keys.begin() + p1, s2);
      a.ctrs.insert(a.ctrs.begin() + p1, x2.ctrs[p2]);
      p1++;
      p2++;
    }
  }
  for (; p2 < x2.size(); p2++) { a.keys.push_back(x2.keys[p2]); a.ctrs.push_back(x2.ctrs[p2]); }
}

static void repair_all(Bitmap& b) {  // RoaringBitmap.repairAfterLazy :2752-2757
  for (Ctr& c : b.ctrs) c = repair_after_lazy(c);
}

// BufferFastAggregation.naive_or(MutableRoaringBitmap...) :810-817 (and or(Mutable...) :896-898)
Bitmap buf_or_mutable(const std::vector<const Bitmap*>& bms) {
  Bitmap ans;
  for (const Bitmap* b : bms) ip_lazy_or(ans, *b);
  repair_all(ans);
  return ans;
}

// ContainerPointer order (RB/RoaringArray.java:708-713): key, then larger cardinality first
namespace {
struct CPtr {
  const Bitmap* b;
  size_t i;
  uint16_t key() const { return b->keys[i]; }
  const Ctr& ctr() const { return b->ctrs[i]; }
};
struct CPtrCmp {
  int operator()(const CPtr& x, const CPtr& y) const {
    if (x.key() != y.key()) return (int)x.key() - (int)y.key();
    return y.ctr().cardinality() - x.ctr().cardinality();
  }
};
}  // namespace

// FastAggregation.horizontal_or(List / RoaringBitmap...), RB/FastAggregation.java:124-231;
// horizontal_xor(RoaringBitmap...) :243-289 (xor = true).  The poll order of the
// container-pointer heap decides each key's chain.
static Bitmap horizontal(const std::vector<const Bitmap*>& bms, bool xor_) {
  Bitmap ans;
  if (bms.empty()) return ans;
  JavaPQ<CPtr, CPtrCmp> pq{CPtrCmp()};
  for (const Bitmap* b : bms)
    if (b->size()) pq.add(CPtr{b, 0});
  auto advance_add = [&](CPtr x) {
    x.i++;
    if (x.i < x.b->size()) pq.add(x);
  };
  while (!pq.empty()) {
    CPtr x1 = pq.poll();
    if (pq.empty() || pq.peek().key() != x1.key()) {
      ans.keys.push_back(x1.key());
      ans.ctrs.push_back(x1.ctr());  // clone, no repair
      advance_add(x1);
      continue;
    }
    CPtr x2 = pq.poll();
    Ctr newc = xor_ ? c_xor(x1.ctr(), x2.ctr()) : c_lazy_or(x1.ctr(), x2.ctr());
    while (!pq.empty() && pq.peek().key() == x1.key()) {
      CPtr x = pq.poll();
      newc = xor_ ? c_ixor(newc, x.ctr()) : c_lazy_ior(newc, x.ctr());
      x.i++;
      if (x.i < x.b->size()) {
        pq.add(x);
      } else if (pq.empty()) {
        break;
      }
    }
    if (!xor_) newc = repair_after_lazy(newc);
    ans.keys.push_back(x1.key());
    ans.ctrs.push_back(std::move(newc));  // appended even when empty (xor)
    advance_add(x1);
    advance_add(x2);
  }
  return ans;
}
Bitmap fa_horizontal_or(const std::vector<const Bitmap*>& bms) { return horizontal(bms, false); }
Bitmap fa_horizontal_xor(const std::vector<const Bitmap*>& bms) { return horizontal(bms, true); }

// RoaringBitmap.getLongSizeInBytes, RB/RoaringBitmap.java:2212-2219 (A :450, B :498, R :1043)
int64_t long_size_in_bytes(const Bitmap& b) {
  int64_t size = 8;
  for (const Ctr& c : b.ctrs)
    size += 2 + (c.kind == ARRAY ? 2 * (int64_t)c.vals.size() + 4 : c.kind == BITMAP ? 8192 : 4 * (int64_t)c.nruns() + 4);
  return size;
}

// FastAggregation.priorityqueue_xor(RoaringBitmap...), RB/FastAggregation.java:790-812
Bitmap fa_priorityqueue_xor(const std::vector<const Bitmap*>& bms) {
  if (bms.empty()) return Bitmap();
  std::vector<Bitmap> pool;
  pool.reserve(2 * bms.size());
  std::vector<int64_t> sizes;
  for (const Bitmap* b : bms) {
    pool.push_back(*b);
    sizes.push_back(long_size_in_bytes(*b));
  }
  auto cmp = [&](int a, int b) { return (int)(int32_t)(uint32_t)(uint64_t)(sizes[a] - sizes[b]); };
  JavaPQ<int, decltype(cmp)> pq(cmp);
  for (int k = 0; k < (int)bms.size(); k++) pq.add(k);
  while (pq.size() > 1) {
    int x1 = pq.poll(), x2 = pq.poll();
    pool.push_back(op_xor(pool[x1], pool[x2]));
    sizes.push_back(long_size_in_bytes(pool.back()));
    pq.add((int)pool.size() - 1);
  }
  return pool[pq.poll()];
}

// RoaringBitmap.lazyor(x1, x2) static, RB/RoaringBitmap.java:723-767
static Bitmap static_lazy_or(const Bitmap& x1, const Bitmap& x2) {
  Bitmap a;
  size_t p1 = 0, p2 = 0;
  while (p1 < x1.size() && p2 < x2.size()) {
    if (x1.keys[p1] == x2.keys[p2]) {
      a.keys.push_back(x1.keys[p1]);
      a.ctrs.push_back(c_lazy_or(x1.ctrs[p1++], x2.ctrs[p2++]));
    } else if (x1.keys[p1] < x2.keys[p2]) {
      a.keys.push_back(x1.keys[p1]);
      a.ctrs.push_back(x1.ctrs[p1++]);
    } else {
      a.keys.push_back(x2.keys[p2]);
      a.ctrs.push_back(x2.ctrs[p2++]);
    }
  }
  for (; p1 < x1.size(); p1++) { a.keys.push_back(x1.keys[p1]); a.ctrs.push_back(x1.ctrs[p1]); }
  for (; p2 < x2.size(); p2++) { a.keys.push_back(x2.keys[p2]); a.ctrs.push_back(x2.ctrs[p2]); }
  return a;
}

// RoaringBitmap.lazyorfromlazyinputs, RB/RoaringBitmap.java:769-818: a bitmap container
// goes first, then lazyIOR
static Bitmap lazy_or_from_lazy(const Bitmap& x1, const Bitmap& x2) {
  Bitmap a;
  size_t p1 = 0, p2 = 0;
  while (p1 < x1.size() && p2 < x2.size()) {
    if (x1.keys[p1] == x2.keys[p2]) {
      const Ctr* c1 = &x1.ctrs[p1];
      const Ctr* c2 = &x2.ctrs[p2];
      if (c2->kind == BITMAP && c1->kind != BITMAP) std::swap(c1, c2);
      a.keys.push_back(x1.keys[p1]);
      a.ctrs.push_back(c_lazy_ior(*c1, *c2));
      p1++;
      p2++;
    } else if (x1.keys[p1] < x2.keys[p2]) {
      a.keys.push_back(x1.keys[p1]);
      a.ctrs.push_back(x1.ctrs[p1++]);
    } else {
      a.keys.push_back(x2.keys[p2]);
      a.ctrs.push_back(x2.ctrs[p2++]);
    }
  }
  for (; p1 < x1.size(); p1++) { a.keys.push_back(x1.keys[p1]); a.ctrs.push_back(x1.ctrs[p1]); }
  for (; p2 < x2.size(); p2++) { a.keys.push_back(x2.keys[p2]); a.ctrs.push_back(x2.ctrs[p2]); }
  return a;
}

// FastAggregation.priorityqueue_or(RoaringBitmap...), RB/FastAggregation.java:733-781
Bitmap fa_priorityqueue_or(const std::vector<const Bitmap*>& bms) {
  if (bms.empty()) return Bitmap();
  const size_t n = bms.size();
  std::vector<Bitmap> buf;
  buf.reserve(n);
  std::vector<int64_t> sizes(n);
  std::vector<char> istmp(n, 0);
  for (size_t k = 0; k < n; k++) {
    buf.push_back(*bms[k]);
    sizes[k] = long_size_in_bytes(buf[k]);
  }
  auto cmp = [&](int a, int b) { return (int)(int32_t)(uint32_t)(uint64_t)(sizes[a] - sizes[b]); };
  JavaPQ<int, decltype(cmp)> pq(cmp);
  for (int k = 0; k < (int)n; k++) pq.add(k);
  while (pq.size() > 1) {
    int x1 = pq.poll(), x2 = pq.poll();
    if (istmp[x2] && istmp[x1]) {
      buf[x1] = lazy_or_from_lazy(buf[x1], buf[x2]);
      sizes[x1] = long_size_in_bytes(buf[x1]);
      istmp[x1] = 1;
      pq.add(x1);
    } else if (istmp[x2]) {
      ip_lazy_or(buf[x2], buf[x1]);
      sizes[x2] = long_size_in_bytes(buf[x2]);
      pq.add(x2);
    } else if (istmp[x1]) {
      ip_lazy_or(buf[x1], buf[x2]);
      sizes[x1] = long_size_in_bytes(buf[x1]);
      pq.add(x1);
    } else {
      buf[x1] = static_lazy_or(buf[x1], buf[x2]);
      sizes[x1] = long_size_in_bytes(buf[x1]);
      istmp[x1] = 1;
      pq.add(x1);
    }
  }
  Bitmap ans = buf[pq.poll()];
  repair_all(ans);
  return ans;
}

// ============================================================================
// portable format, RB/RoaringArray.java
// ============================================================================
static void put16(std::vector<uint8_t>& o, uint16_t v) { o.push_back(v & 0xFF); o.push_back(v >> 8); }
static void put32(std::vector<uint8_t>& o, uint32_t v) { for (int i = 0; i < 4; i++) o.push_back((v >> (8 * i)) & 0xFF); }

std::vector<uint8_t> serialize(const Bitmap& b) {  // :896-940
  std::vector<uint8_t> o;
  const uint32_t size = (uint32_t)b.size();
  bool hasrun = false;
  for (const Ctr& c : b.ctrs) hasrun |= (c.kind == RUN);
  uint32_t start;
  if (hasrun) {
    put32(o, 12347u | ((size - 1) << 16));
    std::vector<uint8_t> flags((size + 7) / 8, 0);
    for (uint32_t i = 0; i < size; i++) if (b.ctrs[i].kind == RUN) flags[i / 8] |= (uint8_t)(1 << (i % 8));
    o.insert(o.end(), flags.begin(), flags.end());
    start = (size < 4) ? 4 + 4 * size + (uint32_t)flags.size() : 4 + 8 * size + (uint32_t)flags.size();
  } else {
    put32(o, 12346u);
    put32(o, size);
    start = 4 + 4 + 4 * size + 4 * size;
  }
  for (uint32_t k = 0; k < size; k++) {
    put16(o, b.keys[k]);
    put16(o, (uint16_t)(b.ctrs[k].cardinality() - 1));
  }
  if (!hasrun || size >= 4) {
    for (uint32_t k = 0; k < size; k++) {
      put32(o, start);
      start += (uint32_t)b.ctrs[k].array_size_bytes();
    }
  }
  for (const Ctr& c : b.ctrs) {
    if (c.kind == ARRAY) {
      for (uint16_t v : c.vals) put16(o, v);
    } else if (c.kind == BITMAP) {
      for (uint64_t w : c.words) { put32(o, (uint32_t)w); put32(o, (uint32_t)(w >> 32)); }
    } else {
      put16(o, (uint16_t)c.nruns());
      for (uint16_t v : c.vals) put16(o, v);
    }
  }
  return o;
}

int deserialize(const uint8_t* p, size_t n, Bitmap* out, size_t* consumed) {  // :547-629 / :276-348
  size_t pos = 0;
  auto need = [&](size_t k) { return pos + k <= n; };
  auto rd16 = [&]() { uint16_t v = (uint16_t)(p[pos] | (p[pos + 1] << 8)); pos += 2; return v; };
  auto rd32 = [&]() { uint32_t v = 0; for (int i = 0; i < 4; i++) v |= (uint32_t)p[pos + i] << (8 * i); pos += 4; return v; };
  if (!need(4)) return ERR_TRUNCATED;
  uint32_t cookie = rd32();
  if ((cookie & 0xFFFF) != 12347u && cookie != 12346u) return ERR_FORMAT;  // "I failed to find a valid cookie"
  bool hasrun = (cookie & 0xFFFF) == 12347u;
  int64_t size;
  if (hasrun) {
    size = (int64_t)(cookie >> 16) + 1;
  } else {
    if (!need(4)) return ERR_TRUNCATED;
    size = (int32_t)rd32();
  }
  if (size > (1 << 16)) return ERR_FORMAT;  // "Size too large"
  if (size < 0) return ERR_FORMAT;          // Java: NegativeArraySizeException
  std::vector<uint8_t> flags;
  if (hasrun) {
    size_t fl = (size_t)(size + 7) / 8;
    if (!need(fl)) return ERR_TRUNCATED;
    flags.assign(p + pos, p + pos + fl);
    pos += fl;
  }
  std::vector<uint16_t> keys(size);
  std::vector<int> cards(size);
  std::vector<uint8_t> kinds(size);
  if (!need(4 * (size_t)size)) return ERR_TRUNCATED;
  for (int64_t k = 0; k < size; k++) {
    keys[k] = rd16();
    cards[k] = 1 + rd16();
    bool is_run = hasrun && (flags[k / 8] & (1 << (k % 8)));
    kinds[k] = is_run ? RUN : (cards[k] > kArrayMax ? BITMAP : ARRAY);
  }
  if (!hasrun || size >= 4) {
    if (!need(4 * (size_t)size)) return ERR_TRUNCATED;
    pos += 4 * (size_t)size;
  }
  Bitmap b;
  b.keys = keys;
  b.ctrs.resize(size);
  for (int64_t k = 0; k < size; k++) {
    Ctr& c = b.ctrs[k];
    if (kinds[k] == BITMAP) {
      if (!need(8192)) return ERR_TRUNCATED;
      c.kind = BITMAP;
      c.words.resize(kWords);
      for (int l = 0; l < kWords; l++) {
        uint64_t lo = rd32();
        uint64_t hi = rd32();
        c.words[l] = lo | (hi << 32);
      }
      c.card = cards[k];  // trusted header cardinality (:606)
    } else if (kinds[k] == RUN) {
      if (!need(2)) return ERR_TRUNCATED;
      int nr = rd16();
      if (!need(4 * (size_t)nr)) return ERR_TRUNCATED;
      c.kind = RUN;
      c.vals.resize(2 * (size_t)nr);
      for (int j = 0; j < 2 * nr; j++) c.vals[j] = rd16();
    } else {
      if (!need(2 * (size_t)cards[k])) return ERR_TRUNCATED;
      c.kind = ARRAY;
      c.vals.resize(cards[k]);
      for (int j = 0; j < cards[k]; j++) c.vals[j] = rd16();
      c.card = cards[k];
    }
  }
  *out = std::move(b);
  if (consumed) *consumed = pos;
  return OK;
}

}  // namespace rbcpu
