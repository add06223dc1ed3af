// Host-side portable-format layer of the engine: header parse/validation and the
// construction utilities behind rbg_from_values / rbg_run_optimize / rbg_to_values.
// Format: RB/RoaringArray.java:896-940 (serialize), :547-629 (deserialize),
// :781-790 (headerSize).  RB/ = RoaringBitmap/src/main/java/org/roaringbitmap/.
#pragma once
#include <cstddef>
#include <cstdint>
#include <string>
#include <vector>

namespace rbg {

enum Kind : uint8_t { KA = 0, KB = 1, KR = 2 };

constexpr uint32_t kCookieNoRun = 12346;  // RB/RoaringArray.java:23
constexpr uint32_t kCookieRun = 12347;    // RB/RoaringArray.java:24
constexpr int kNoOffsetThreshold = 4;     // RB/RoaringArray.java:25
constexpr int kArrayMax = 4096;           // RB/ArrayContainer.java:27

// One container as found in a serialized buffer.
struct HostCtr {
  uint16_t key;
  uint8_t kind;
  uint32_t card;     // 1..65536, from the header (trusted like RB/RoaringArray.java:606)
  uint32_t nruns;    // run containers only
  uint64_t ser_off;  // byte offset of the serialized payload within the buffer
  uint32_t ser_len;  // A: 2*card, B: 8192, R: 2 + 4*nruns
};

struct HostBitmap {
  std::vector<HostCtr> ctrs;
  size_t consumed = 0;   // total serialized bytes
  int64_t card = 0;      // long cardinality (sum of header cards)
  bool has_run = false;
};

// Status codes follow include/roaring_mi355x.h.
int parse(const uint8_t* p, size_t n, HostBitmap* out, std::string* err);

size_t header_size(size_t size, bool has_run);  // RB/RoaringArray.java:781-790

// Construction utilities (host; not the hot path).
std::vector<uint8_t> build_from_values(const uint32_t* v, size_t n, bool run_optimize);
int run_optimize_serialized(const uint8_t* p, size_t n, std::vector<uint8_t>* out, std::string* err);
int values_of_serialized(const uint8_t* p, size_t n, std::vector<uint32_t>* out, std::string* err);

}  // namespace rbg
