// Host AddressSanitizer / UBSan driver for the engine's host-side format layer
// (roaringbitmap_amd/csrc/format.cpp: parse, build_from_values, run_optimize_serialized,
// values_of_serialized).  Built and run by tests/test_host_asan.py; sanitizers run on
// host code only.
//
//   format_fuzz FILE...   every input file as is, every truncation of it and seeded
//                         byte mutations; plus seeded random value sets built, parsed,
//                         run-optimized and decoded back (round trips checked)
#include <cstdio>
#include <cstdlib>
#include <fstream>
#include <iterator>
#include <algorithm>
#include <random>
#include <string>
#include <vector>

#include "../../roaringbitmap_amd/csrc/format.hpp"

using rbg::HostBitmap;

static int g_fail = 0;
#define CHECK(c)                                                   \
  do {                                                             \
    if (!(c)) {                                                    \
      std::fprintf(stderr, "%s:%d check failed: %s\n", __FILE__, __LINE__, #c); \
      g_fail++;                                                    \
    }                                                              \
  } while (0)

// every entry point on one buffer: must return a status, never touch memory past n
static void exercise(const std::vector<uint8_t>& b, size_t n) {
  std::vector<uint8_t> copy(b.begin(), b.begin() + (long)n);  // exact-size heap buffer
  const uint8_t* p = copy.empty() ? nullptr : copy.data();
  HostBitmap hb;
  std::string err;
  const int st = rbg::parse(p, n, &hb, &err);
  if (st == 0) {
    CHECK(hb.consumed <= n);
    for (const auto& c : hb.ctrs) CHECK(c.ser_off + c.ser_len <= n);
  }
  std::vector<uint32_t> vals;
  const int sv = rbg::values_of_serialized(p, n, &vals, &err);
  CHECK((sv == 0) == (st == 0));
  std::vector<uint8_t> ro;
  const int sr = rbg::run_optimize_serialized(p, n, &ro, &err);
  CHECK((sr == 0) == (st == 0));
  if (sv == 0 && sr == 0) {
    std::vector<uint32_t> v2;
    CHECK(rbg::values_of_serialized(ro.data(), ro.size(), &v2, &err) == 0);
    CHECK(v2 == vals);
  }
}

int main(int argc, char** argv) {
  std::mt19937_64 rng(0xA5A5);
  size_t cases = 0;
  for (int i = 1; i < argc; i++) {
    std::ifstream f(argv[i], std::ios::binary);
    std::vector<uint8_t> b((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    const size_t step = b.size() > 4096 ? b.size() / 2048 : 1;
    for (size_t n = 0; n <= b.size(); n += step, cases++) exercise(b, n);
    exercise(b, b.size());
    for (int m = 0; m < 60 && !b.empty(); m++, cases++) {  // seeded byte mutations
      std::vector<uint8_t> x = b;
      const int k = 1 + (int)(rng() % 4);
      for (int j = 0; j < k; j++) x[rng() % x.size()] = (uint8_t)rng();
      exercise(x, x.size());
    }
  }
  for (int r = 0; r < 120; r++, cases++) {  // random value sets: every container family
    std::vector<uint32_t> v;
    const int nkeys = 1 + (int)(rng() % 6);
    for (int k = 0; k < nkeys; k++) {
      const uint32_t key = (uint32_t)(rng() % 65536) << 16;
      const int mode = (int)(rng() % 4);
      if (mode == 0) {
        for (int j = 0, c = 1 + (int)(rng() % 5000); j < c; j++) v.push_back(key | (uint32_t)(rng() % 65536));
      } else if (mode == 1) {
        const uint32_t s = (uint32_t)(rng() % 60000), l = 1 + (uint32_t)(rng() % 5000);
        for (uint32_t j = s; j < s + l && j < 65536; j++) v.push_back(key | j);
      } else if (mode == 2) {
        for (uint32_t j = 0; j < 65536; j += 2) v.push_back(key | j);
      } else {
        for (uint32_t j = 0; j < 65536; j++) v.push_back(key | j);
      }
    }
    const bool ro = (r & 1) != 0;
    std::vector<uint8_t> b = rbg::build_from_values(v.data(), v.size(), ro);
    std::sort(v.begin(), v.end());
    v.erase(std::unique(v.begin(), v.end()), v.end());
    std::vector<uint32_t> back;
    std::string err;
    CHECK(rbg::values_of_serialized(b.data(), b.size(), &back, &err) == 0);
    CHECK(back == v);
    exercise(b, b.size());
    exercise(b, b.size() / 2);
  }
  std::printf("format_fuzz: %zu cases, %d failures\n", cases, g_fail);
  return g_fail ? 1 : 0;
}
