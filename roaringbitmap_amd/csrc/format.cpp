// Host-side portable-format layer (see format.hpp).
#include "format.hpp"

#include <algorithm>
#include <cstring>

#include "../../include/roaring_mi355x.h"

namespace rbg {

static inline uint16_t rd16(const uint8_t* p) { return (uint16_t)(p[0] | (p[1] << 8)); }
static inline uint32_t rd32(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

size_t header_size(size_t size, bool has_run) {
  if (has_run) {
    if (size < (size_t)kNoOffsetThreshold) return 4 + (size + 7) / 8 + 4 * size;
    return 4 + (size + 7) / 8 + 8 * size;
  }
  return 4 + 4 + 8 * size;
}

int parse(const uint8_t* p, size_t n, HostBitmap* out, std::string* err) {
  out->ctrs.clear();
  out->card = 0;
  out->has_run = false;
  size_t pos = 0;
  auto trunc = [&](const char* what) {
    if (err) *err = std::string("truncated input: ") + what;
    return RBG_ERR_TRUNCATED;
  };
  if (!p && n) return RBG_ERR_ILLEGAL_ARGUMENT;
  if (n < 4) return trunc("cookie");
  const uint32_t cookie = rd32(p);
  pos = 4;
  // RB/RoaringArray.java:557-559
  if ((cookie & 0xFFFF) != kCookieRun && cookie != kCookieNoRun) {
    if (err) *err = "I failed to find one of the right cookies.";
    return RBG_ERR_INVALID_FORMAT;
  }
  const bool hasrun = (cookie & 0xFFFF) == kCookieRun;
  int64_t size;
  if (hasrun) {
    size = (int64_t)(cookie >> 16) + 1;
  } else {
    if (n < pos + 4) return trunc("size");
    size = (int32_t)rd32(p + pos);
    pos += 4;
  }
  if (size > (1 << 16)) {  // :564-566
    if (err) *err = "Size too large";
    return RBG_ERR_INVALID_FORMAT;
  }
  if (size < 0) {  // Java: NegativeArraySizeException
    if (err) *err = "negative container count";
    return RBG_ERR_INVALID_FORMAT;
  }
  const uint8_t* flags = nullptr;
  if (hasrun) {
    const size_t fl = (size_t)(size + 7) / 8;
    if (n < pos + fl) return trunc("run flags");
    flags = p + pos;
    pos += fl;
  }
  if (n < pos + 4 * (size_t)size) return trunc("descriptors");
  out->ctrs.resize((size_t)size);
  int prev_key = -1;
  for (int64_t k = 0; k < size; k++) {
    HostCtr& c = out->ctrs[k];
    c.key = rd16(p + pos + 4 * k);
    c.card = 1u + rd16(p + pos + 4 * k + 2);
    const bool is_run = hasrun && (flags[k / 8] & (1 << (k % 8)));
    c.kind = is_run ? KR : (c.card > (uint32_t)kArrayMax ? KB : KA);
    c.nruns = 0;
    if ((int)c.key <= prev_key) {
      if (err) *err = "container keys are not strictly increasing";
      return RBG_ERR_INVALID_FORMAT;
    }
    prev_key = c.key;
    out->has_run |= is_run;
  }
  pos += 4 * (size_t)size;
  if (!hasrun || size >= kNoOffsetThreshold) {  // offsets are skipped, as the reference does
    if (n < pos + 4 * (size_t)size) return trunc("offsets");
    pos += 4 * (size_t)size;
  }
  for (int64_t k = 0; k < size; k++) {
    HostCtr& c = out->ctrs[k];
    c.ser_off = pos;
    if (c.kind == KB) {
      c.ser_len = 8192;
    } else if (c.kind == KR) {
      if (n < pos + 2) return trunc("run count");
      c.nruns = rd16(p + pos);
      c.ser_len = 2 + 4 * c.nruns;
    } else {
      c.ser_len = 2 * c.card;
    }
    if (n < pos + c.ser_len) return trunc("container payload");
    if (c.kind == KR) {  // RunContainer cardinality comes from its runs, not the header (RB/RunContainer.java:1003-1009)
      uint32_t rc = 0;
      for (uint32_t j = 0; j < c.nruns; j++) rc += 1u + rd16(p + pos + 2 + 4 * j + 2);
      c.card = rc;
    }
    pos += c.ser_len;
    out->card += c.card;
  }
  out->consumed = pos;
  return RBG_OK;
}

// ---------------------------------------------------------------------------
// construction utilities
// ---------------------------------------------------------------------------
namespace {
struct BuildCtr {
  uint16_t key;
  uint8_t kind;
  uint32_t card;
  std::vector<uint16_t> payload;  // A: values; B: 4096 u16 = 1024 u64 words LE; R: pairs
};

void put16(std::vector<uint8_t>& o, uint16_t v) {
  o.push_back((uint8_t)(v & 0xFF));
  o.push_back((uint8_t)(v >> 8));
}
void put32(std::vector<uint8_t>& o, uint32_t v) {
  for (int i = 0; i < 4; i++) o.push_back((uint8_t)((v >> (8 * i)) & 0xFF));
}

uint32_t ser_len(const BuildCtr& c) {
  if (c.kind == KA) return 2 * c.card;
  if (c.kind == KB) return 8192;
  return 2 + 2 * (uint32_t)c.payload.size();
}

std::vector<uint8_t> serialize(const std::vector<BuildCtr>& cs) {
  const size_t size = cs.size();
  bool hasrun = false;
  for (const BuildCtr& c : cs) hasrun |= c.kind == KR;
  std::vector<uint8_t> o;
  uint32_t start = (uint32_t)header_size(size, hasrun);
  if (hasrun) {
    put32(o, kCookieRun | (uint32_t)((size - 1) << 16));
    std::vector<uint8_t> fl((size + 7) / 8, 0);
    for (size_t i = 0; i < size; i++)
      if (cs[i].kind == KR) fl[i / 8] |= (uint8_t)(1u << (i % 8));
    o.insert(o.end(), fl.begin(), fl.end());
  } else {
    put32(o, kCookieNoRun);
    put32(o, (uint32_t)size);
  }
  for (const BuildCtr& c : cs) {
    put16(o, c.key);
    put16(o, (uint16_t)(c.card - 1));
  }
  if (!hasrun || size >= (size_t)kNoOffsetThreshold) {
    for (const BuildCtr& c : cs) {
      put32(o, start);
      start += ser_len(c);
    }
  }
  for (const BuildCtr& c : cs) {
    if (c.kind == KR) put16(o, (uint16_t)(c.payload.size() / 2));
    for (uint16_t v : c.payload) put16(o, v);
  }
  return o;
}

// maximal runs of a sorted, distinct value list as (start, length-1) pairs
std::vector<uint16_t> runs_of(const std::vector<uint16_t>& vals) {
  std::vector<uint16_t> p;
  size_t i = 0;
  while (i < vals.size()) {
    size_t j = i;
    while (j + 1 < vals.size() && vals[j + 1] == vals[j] + 1) j++;
    p.push_back(vals[i]);
    p.push_back((uint16_t)(vals[j] - vals[i]));
    i = j + 1;
  }
  return p;
}

std::vector<uint16_t> bitmap_words_u16(const std::vector<uint16_t>& vals) {
  std::vector<uint64_t> w(1024, 0);
  for (uint16_t v : vals) w[v >> 6] |= 1ULL << (v & 63);
  std::vector<uint16_t> out(4096);
  std::memcpy(out.data(), w.data(), 8192);
  return out;
}

// Container for a sorted value list: BY_CARD like RoaringBitmap.addN, then the
// runOptimize rule of the resulting type (A: RB/ArrayContainer.java:1085-1099,
// B: RB/BitmapContainer.java:1218-1237).
BuildCtr make_ctr(uint16_t key, const std::vector<uint16_t>& vals, bool run_optimize, int kind_hint) {
  BuildCtr c;
  c.key = key;
  c.card = (uint32_t)vals.size();
  int kind = kind_hint >= 0 ? kind_hint : (c.card > (uint32_t)kArrayMax ? KB : KA);
  if (run_optimize || kind == KR) {
    std::vector<uint16_t> runs = runs_of(vals);
    const uint32_t nr = (uint32_t)(runs.size() / 2);
    bool to_run;
    if (kind == KA) to_run = 2 * c.card > 2 + 4 * nr;
    else if (kind == KB) to_run = 2 + 4 * nr < 8192;
    else to_run = 2 + 4 * nr <= std::min<uint32_t>(8192, 2 + 2 * c.card);  // RB/RunContainer.java:2326-2335
    if (to_run) {
      c.kind = KR;
      c.payload = std::move(runs);
      return c;
    }
    if (kind == KR) kind = c.card > (uint32_t)kArrayMax ? KB : KA;
  }
  c.kind = (uint8_t)kind;
  c.payload = kind == KB ? bitmap_words_u16(vals) : vals;
  return c;
}

int decode(const uint8_t* p, size_t n, std::vector<uint16_t>* keys, std::vector<uint8_t>* kinds,
           std::vector<std::vector<uint16_t>>* vals, std::string* err) {
  HostBitmap hb;
  int st = parse(p, n, &hb, err);
  if (st) return st;
  for (const HostCtr& c : hb.ctrs) {
    keys->push_back(c.key);
    kinds->push_back(c.kind);
    std::vector<uint16_t> v;
    const uint8_t* q = p + c.ser_off;
    if (c.kind == KA) {
      v.resize(c.card);
      for (uint32_t i = 0; i < c.card; i++) v[i] = rd16(q + 2 * i);
    } else if (c.kind == KB) {
      for (int w = 0; w < 1024; w++) {
        uint64_t x = (uint64_t)rd32(q + 8 * w) | ((uint64_t)rd32(q + 8 * w + 4) << 32);
        while (x) {
          v.push_back((uint16_t)(w * 64 + __builtin_ctzll(x)));
          x &= x - 1;
        }
      }
    } else {
      for (uint32_t r = 0; r < c.nruns; r++) {
        uint32_t s = rd16(q + 2 + 4 * r), l = rd16(q + 4 + 4 * r);
        for (uint32_t x = s; x <= s + l; x++) v.push_back((uint16_t)x);
      }
    }
    vals->push_back(std::move(v));
  }
  return RBG_OK;
}
}  // namespace

std::vector<uint8_t> build_from_values(const uint32_t* v, size_t n, bool run_optimize) {
  std::vector<uint32_t> s(v, v + n);
  std::sort(s.begin(), s.end());
  s.erase(std::unique(s.begin(), s.end()), s.end());
  std::vector<BuildCtr> cs;
  size_t i = 0;
  while (i < s.size()) {
    const uint16_t key = (uint16_t)(s[i] >> 16);
    std::vector<uint16_t> low;
    while (i < s.size() && (uint16_t)(s[i] >> 16) == key) low.push_back((uint16_t)(s[i++] & 0xFFFF));
    cs.push_back(make_ctr(key, low, run_optimize, -1));
  }
  return serialize(cs);
}

int run_optimize_serialized(const uint8_t* p, size_t n, std::vector<uint8_t>* out, std::string* err) {
  std::vector<uint16_t> keys;
  std::vector<uint8_t> kinds;
  std::vector<std::vector<uint16_t>> vals;
  int st = decode(p, n, &keys, &kinds, &vals, err);
  if (st) return st;
  std::vector<BuildCtr> cs;
  for (size_t i = 0; i < keys.size(); i++) cs.push_back(make_ctr(keys[i], vals[i], true, kinds[i]));
  *out = serialize(cs);
  return RBG_OK;
}

int values_of_serialized(const uint8_t* p, size_t n, std::vector<uint32_t>* out, std::string* err) {
  std::vector<uint16_t> keys;
  std::vector<uint8_t> kinds;
  std::vector<std::vector<uint16_t>> vals;
  int st = decode(p, n, &keys, &kinds, &vals, err);
  if (st) return st;
  out->clear();
  for (size_t i = 0; i < keys.size(); i++)
    for (uint16_t x : vals[i]) out->push_back(((uint32_t)keys[i] << 16) | x);
  return RBG_OK;
}

}  // namespace rbg
