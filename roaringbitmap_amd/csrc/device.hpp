// Device-side building blocks shared by every engine kernel (gfx950, wave64).
//
// A workgroup of NT = 256 threads (4 waves) owns one 65536-bit container at a
// time.  Thread t holds four u64 words of it in registers:
//     w0 = word 2t, w1 = word 2t+1        (first half, bytes [16t, 16t+16))
//     w2 = word 512+2t, w3 = word 513+2t  (second half, bytes [4096+16t, ...))
// so a bitmap container streams from HBM as two perfectly coalesced 16-byte
// loads per lane (1 KiB per wave instruction), and LDS copies of it are read
// conflict-free with ds_read_b128.
#pragma once
#include <hip/hip_runtime.h>
#include <cstdint>

namespace rbg {

constexpr int NT = 256;
#ifndef RBG_SLOT_BYTES
#define RBG_SLOT_BYTES 8320
#endif
// max serialized payload (8194) rounded up to 128 B, so every slot (and the B payload
// at its start) is cache-line aligned: C2 AND -1.3 % against 8208 (16 B rounding)
constexpr int kSlotBytes = RBG_SLOT_BYTES;

enum DKind : uint8_t { DK_A = 0, DK_B = 1, DK_R = 2 };

// Input container descriptor (16 B).  Slot layout in the payload arena:
//   A: u16 values at +0 | B: 1024 u64 words at +0 | R: [u16 pad][u16 nruns][u32 pairs]
// The portable-format payload bytes of a container start at slot + (R ? 2 : 0).
struct __align__(16) CDesc {
  uint64_t slot;
  uint32_t card;  // 1..65536 (header cardinality)
  uint16_t key;
  uint8_t kind;
  uint8_t flags;
};

// Output container descriptor (32 B) produced by an op, consumed by the emitter.
struct __align__(16) ODesc {
  uint64_t src;      // device address of the serialized payload bytes
  uint32_t ser_len;  // serialized payload length
  uint32_t card;
  uint16_t key;
  uint8_t kind;
  uint8_t keep;
  uint32_t pad0;
  uint64_t pad1;
};

struct Task {
  uint32_t key;
  int32_t a;  // pairwise: container index in operand A (-1 absent); wide: segment start
  int32_t b;  // pairwise: container index in operand B (-1 absent); wide: segment length
  int32_t aux;
};

// Pairwise task (32 B): the plan kernel resolves both operands' descriptors so
// the compute kernel reads one record per task with scalar loads.
constexpr uint8_t kAbsent = 0xFF;
struct __align__(16) PTask {
  uint64_t slot_a, slot_b;  // payload slot offsets in the operands' arenas
  uint32_t card_a, card_b;
  uint16_t key;
  uint8_t kind_a, kind_b;   // DK_A / DK_B / DK_R, or kAbsent (key not in that operand)
  uint16_t nruns_a, nruns_b;  // run count of R operands (0 otherwise)
};

struct ResultInfo {
  uint32_t n_out;
  uint32_t has_run;
  uint64_t header;    // header bytes
  uint64_t payload;   // payload bytes
  uint64_t total;     // header + payload
  int64_t long_card;  // sum of result cardinalities (64-bit)
  uint32_t card32;    // Java int (mod 2^32)
  uint32_t any;       // nonzero iff some task had a non-empty result
  uint64_t start;     // byte offset of the serialized result inside the result buffer
  uint32_t err;       // nonzero if a look-back spin timed out (result invalid)
  uint32_t pad;
};

// per-task output record, consumed by the header kernels
struct __align__(16) ORec {
  uint64_t off;  // payload offset within the payload region
  uint64_t src;  // scan placement: device address of the serialized payload (scratch or input)
  uint32_t idx;  // output container index (valid if keep)
  uint32_t card;
  uint32_t ser_len;
  uint16_t key;
  uint8_t kind;
  uint8_t keep;
};

// where an op writes its result: payload region at out + payload_base, header in
// front of it; look-back state (ticket, error word, per-task status) and records
// the result's long cardinality is accumulated at ((u64*)OutCtx::err)[kCardWord]
// (inside the zeroed look-back header, 32 B past the error word)
constexpr int kCardWord = 4;
// look-back tile statuses zeroed by every plan kernel (k_place's tiles)
constexpr int kMaxTiles = 128;

struct OutCtx {
  uint8_t* out;
  uint64_t payload_base;
  uint64_t* status;  // per-task look-back words (also the totals word status[n_tasks-1])
  uint32_t* err;
  ORec* recs;
  uint8_t* scratch;  // one kSlotBytes slot per task
  uint64_t* tile_status;  // scan placement: per-tile look-back words
  uint64_t* tile_card;    // scan placement: per-tile result cardinality
  uint8_t* kind_by_out;   // k_place: R / not R per output container (run flags of the serialization)
  // wide OR: a staged bitmap result of task t is written straight to payload offset 8192 t, its place
  // whenever every earlier task kept an 8 KiB container (k_spec_fix moves the others to their slot)
  uint32_t spec;
  // k_place also writes the result's (containers, payload bytes, has_run) here when set: the
  // device layout of a key shard (rbg_ctx_result_layout_device) without a launch of its own
  int64_t* layout_out;
  // pairwise ops (round 6): per tile of kAggTile records, the kept results' (payload bytes, containers,
  // run containers, cardinality) summed by the compute kernel as it writes them (agg_pack), so that the
  // serialization places every tile without a look-back pass (k_serialize_agg); null: not accumulated
  unsigned long long* tile_agg;
};
constexpr int kAggTile = 64;                     // records per aggregate tile
constexpr int kMaxAggTiles = 65536 / kAggTile;  // a result has at most 65,536 records
// a kept result as a tile-aggregate increment: payload bytes [0, 20), containers [20, 27), run
// containers [27, 34), cardinality [34, 57) -- no field of a 64-record tile can overflow
__host__ __device__ __forceinline__ unsigned long long agg_pack(uint32_t len, uint32_t card, uint32_t kind) {
  return (unsigned long long)len | (1ull << 20) | ((unsigned long long)(kind == DK_R ? 1u : 0u) << 27) |
         ((unsigned long long)card << 34);
}
__host__ __device__ __forceinline__ uint32_t agg_bytes(unsigned long long a) { return (uint32_t)(a & 0xFFFFF); }
__host__ __device__ __forceinline__ uint32_t agg_count(unsigned long long a) { return (uint32_t)((a >> 20) & 0x7F); }
__host__ __device__ __forceinline__ uint32_t agg_runs(unsigned long long a) { return (uint32_t)((a >> 27) & 0x7F); }
__host__ __device__ __forceinline__ uint32_t agg_card(unsigned long long a) { return (uint32_t)(a >> 34); }

// Run containers of more than 2047 runs (8 KiB of runs) do not fit a result slot.  Only the buffer
// package's run AND / ANDNOT run make them (no toEfficientContainer); such a result is written to
// this arena (bump allocation; `overflow` set when `cap` is exceeded, `used` then tells the size
// the op needs, and the host reruns it with a larger arena).
struct BigRuns {
  uint8_t* base;
  unsigned long long* used;  // used[0] bytes reserved, used[1] overflow flag
  uint64_t cap;
};
// Portable-format header bytes for `size` containers (RB/RoaringArray.java:781-790)
__host__ __device__ inline uint64_t header_bytes(uint32_t size, uint32_t has_run) {
  if (has_run) return (size < 4) ? 4 + (size + 7) / 8 + 4ull * size : 4 + (size + 7) / 8 + 8ull * size;
  return 8 + 8ull * size;
}

struct OperandView {
  const CDesc* desc;
  const uint8_t* payload;
};

__device__ __forceinline__ int popc64(uint64_t x) { return __popcll(x); }

// splitmix64 finaliser (host and device: the synthetic generators share it)
__host__ __device__ inline uint64_t splitmix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ULL;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
  return x ^ (x >> 31);
}

// Synthetic C3 workloads, shared by the device generators and
// the host-side CSR construction:
//   uniform  : bitmap i holds every key; card(i, k) in [1, 29] (mean 15, ~1M
//              values per bitmap), values stratified over the 65536 range
//   clustered: bitmap i holds keys base(i) .. base(i)+15 as dense bitmap
//              containers (each bit set with p = 0.95)
__host__ __device__ inline uint32_t c3u_card(uint64_t seed, uint32_t i, uint32_t k) {
  return 1 + (uint32_t)(splitmix64(seed ^ ((uint64_t)i << 17) ^ (uint64_t)k) % 29);
}
__host__ __device__ inline uint32_t c3c_base(uint64_t seed, uint32_t i) {
  return (uint32_t)(splitmix64(seed ^ 0xC3100000ULL ^ (uint64_t)i) % (4096 - 16));
}

__device__ __forceinline__ int by_card(int c) { return c <= 4096 ? DK_A : DK_B; }
// RunContainer.toEfficientContainer (RB/RunContainer.java:2326-2335)
__device__ __forceinline__ int eff(int c, int r) {
  const int run_sz = 2 + 4 * r;
  const int arr_sz = 2 + 2 * c;
  return run_sz <= min(8192, arr_sz) ? DK_R : by_card(c);
}

enum PairOp : int { OPR_AND = 0, OPR_OR = 1, OPR_XOR = 2, OPR_ANDNOT = 3 };  // == OpCode (kernels.hpp)

// Result container type of the static pairwise ops as a function of the operand
// kinds and the result's cardinality c and run count r:
//   AND   : R&R -> EFF(c,r) (RB/RunContainer.java:381-456); else BY_CARD(c)
//   OR    : A|R, R|A, R|R -> EFF(c,r) (:1926-1986); A|A -> BY_CARD(c)
//           (RB/ArrayContainer.java:949-963); B|x, x|B -> c==65536 ? R.full : B
//           (RB/BitmapContainer.java:1064-1096, RB/RunContainer.java:1932-1949)
//   XOR   : R^R -> EFF; R^A, A^R with |A| < 32 -> EFF (RB/RunContainer.java:2410-2424);
//           else BY_CARD (RB/BitmapContainer.java:1372-1408)
//   ANDNOT: R\R -> EFF (:637-692); R\A with |A| < 32 -> EFF (:574-591); else BY_CARD
__device__ __forceinline__ bool pairwise_needs_runs(int op, int ka, int ca, int kb, int cb) {
  switch (op) {
    case OPR_AND: return ka == DK_R && kb == DK_R;
    case OPR_OR: return (ka == DK_R && kb != DK_B) || (kb == DK_R && ka != DK_B);
    case OPR_XOR:
      return (ka == DK_R && kb == DK_R) || (ka == DK_R && kb == DK_A && cb < 32) ||
             (kb == DK_R && ka == DK_A && ca < 32);
    default:  // ANDNOT
      return ka == DK_R && (kb == DK_R || (kb == DK_A && cb < 32));
  }
}
__device__ __forceinline__ int pairwise_kind(int op, int ka, int kb, int c) {
  if (op == OPR_OR && (ka == DK_B || kb == DK_B)) return c == 65536 ? DK_R : DK_B;
  return by_card(c);
}

// ---------------------------------------------------------------------------
// wave / block reductions and scans
// ---------------------------------------------------------------------------
// Wave-wide inclusive prefix sum with DPP (row shifts, then row broadcasts):
// six VALU ops, no LDS round trips (ds_bpermute-based shuffles cost ~100
// cycles of latency each and serialise every scan).
__device__ __forceinline__ int dpp_incl_scan(int x) {
  x += __builtin_amdgcn_update_dpp(0, x, 0x111, 0xf, 0xf, false);  // row_shr:1
  x += __builtin_amdgcn_update_dpp(0, x, 0x112, 0xf, 0xf, false);  // row_shr:2
  x += __builtin_amdgcn_update_dpp(0, x, 0x114, 0xf, 0xf, false);  // row_shr:4
  x += __builtin_amdgcn_update_dpp(0, x, 0x118, 0xf, 0xf, false);  // row_shr:8
  x += __builtin_amdgcn_update_dpp(0, x, 0x142, 0xa, 0xf, false);  // row_bcast:15 -> rows 1, 3
  x += __builtin_amdgcn_update_dpp(0, x, 0x143, 0xc, 0xf, false);  // row_bcast:31 -> rows 2, 3
  return x;
}
// value of lane 63 / lane 0 (wave-uniform, SGPR)
__device__ __forceinline__ int lane63(int x) { return __builtin_amdgcn_readlane(x, 63); }
__device__ __forceinline__ uint32_t lane63u(uint32_t x) { return (uint32_t)__builtin_amdgcn_readlane((int)x, 63); }
__device__ __forceinline__ uint32_t lane0u(uint32_t x) { return (uint32_t)__builtin_amdgcn_readlane((int)x, 0); }
// lane l receives lane l-1's / l+1's value; lane 0 / lane 63 receive 0
__device__ __forceinline__ uint32_t from_prev_lane(uint32_t x) {
  return __builtin_amdgcn_update_dpp(0u, x, 0x138, 0xf, 0xf, false);  // wave_shr:1
}
__device__ __forceinline__ uint32_t from_next_lane(uint32_t x) {
  return __builtin_amdgcn_update_dpp(0u, x, 0x130, 0xf, 0xf, false);  // wave_shl:1
}

__device__ __forceinline__ int wave_sum(int v) { return lane63(dpp_incl_scan(v)); }
__device__ __forceinline__ int wave_incl_scan(int v) { return dpp_incl_scan(v); }

// Workgroup barrier that orders LDS only.  __syncthreads() is also a release /
// acquire of global memory, so it waits for every outstanding global load and
// store of the wave; the building blocks below only hand LDS between threads, and
// with this barrier a kernel can keep global loads (e.g. the next task's
// operands) in flight across them.
__device__ __forceinline__ void lds_barrier() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
  __builtin_amdgcn_s_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// Sum of (a, b) over the workgroup; `sh` needs 8 ints.  Ends with a barrier.
__device__ __forceinline__ void block_sum2(int& a, int& b, int* sh) {
  a = wave_sum(a);
  b = wave_sum(b);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    sh[w] = a;
    sh[4 + w] = b;
  }
  lds_barrier();
  a = sh[0] + sh[1] + sh[2] + sh[3];
  b = sh[4] + sh[5] + sh[6] + sh[7];
  lds_barrier();
}

// Exclusive scan in word order (first halves of threads 0..255, then second
// halves).  v0 counts for words {2t, 2t+1}, v1 for {512+2t, 513+2t}.
__device__ __forceinline__ void block_scan_halves(int v0, int v1, int& p0, int& p1, int& total,
                                                  int* sh) {
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int s0 = wave_incl_scan(v0), s1 = wave_incl_scan(v1);
  if (lane == 63) {
    sh[w] = s0;
    sh[4 + w] = s1;
  }
  lds_barrier();
  int o0 = 0, o1 = 0, t0 = 0, t1 = 0;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    const int x = sh[i], y = sh[4 + i];
    if (i < w) {
      o0 += x;
      o1 += y;
    }
    t0 += x;
    t1 += y;
  }
  p0 = o0 + s0 - v0;
  p1 = t0 + o1 + s1 - v1;
  total = t0 + t1;
  lds_barrier();
}

// ---------------------------------------------------------------------------
// 8 KiB LDS bitmaps (u32 words) and register-resident containers
// ---------------------------------------------------------------------------
__device__ __forceinline__ void lds_clear(uint32_t* lds) {
  uint4* p = reinterpret_cast<uint4*>(lds);
  const uint4 z = make_uint4(0, 0, 0, 0);
  p[threadIdx.x] = z;
  p[threadIdx.x + NT] = z;
}

__device__ __forceinline__ void lds_fill_ones(uint32_t* lds) {
  uint4* p = reinterpret_cast<uint4*>(lds);
  const uint4 o = make_uint4(~0u, ~0u, ~0u, ~0u);
  p[threadIdx.x] = o;
  p[threadIdx.x + NT] = o;
}

__device__ __forceinline__ void u4_to_words(const uint4 v, uint64_t& lo, uint64_t& hi) {
  lo = (uint64_t)v.x | ((uint64_t)v.y << 32);
  hi = (uint64_t)v.z | ((uint64_t)v.w << 32);
}
__device__ __forceinline__ uint4 words_to_u4(uint64_t lo, uint64_t hi) {
  return make_uint4((uint32_t)lo, (uint32_t)(lo >> 32), (uint32_t)hi, (uint32_t)(hi >> 32));
}

// owned words from an LDS bitmap
__device__ __forceinline__ void lds_read_owned(const uint32_t* lds, uint64_t r[4]) {
  const uint4* p = reinterpret_cast<const uint4*>(lds);
  u4_to_words(p[threadIdx.x], r[0], r[1]);
  u4_to_words(p[threadIdx.x + NT], r[2], r[3]);
}
__device__ __forceinline__ void lds_write_owned(uint32_t* lds, const uint64_t r[4]) {
  uint4* p = reinterpret_cast<uint4*>(lds);
  p[threadIdx.x] = words_to_u4(r[0], r[1]);
  p[threadIdx.x + NT] = words_to_u4(r[2], r[3]);
}
// owned words of a bitmap container in global memory (two 16 B loads per lane)
__device__ __forceinline__ void load_bitmap_owned(const uint8_t* words, uint64_t r[4]) {
  const uint4* p = reinterpret_cast<const uint4*>(words);
  u4_to_words(p[threadIdx.x], r[0], r[1]);
  u4_to_words(p[threadIdx.x + NT], r[2], r[3]);
}
__device__ __forceinline__ void store_bitmap_owned(uint8_t* words, const uint64_t r[4]) {
  uint4* p = reinterpret_cast<uint4*>(words);
  p[threadIdx.x] = words_to_u4(r[0], r[1]);
  p[threadIdx.x + NT] = words_to_u4(r[2], r[3]);
}

// OR the sorted u16 values of an array container into an LDS bitmap
// (cooperative over the workgroup).  vals is 2 B aligned: 16 B slots, or the packed
// arrays of a C3 synthetic batch; the 16 B vectors covering it are read and the
// values outside [vals, vals + card) are skipped.
template <int MODE = 0>  // 0: or, 1: xor
__device__ __forceinline__ void lds_scatter_array(uint32_t* lds, const uint16_t* vals, int card) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(vals);
  const int lo = (int)((a & 15) >> 1);  // values of the first vector before vals
  const int nvec = (lo + card + 7) >> 3;
  const uint4* v4 = reinterpret_cast<const uint4*>(a & ~(uintptr_t)15);
  for (int i = threadIdx.x; i < nvec; i += NT) {
    const uint4 v = v4[i];
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    const int base = i * 8 - lo;
#pragma unroll
    for (int j = 0; j < 8; j++) {
      if ((unsigned)(base + j) < (unsigned)card) {
        const uint32_t x = (w[j >> 1] >> ((j & 1) * 16)) & 0xFFFF;
        if (MODE == 0) atomicOr(&lds[x >> 5], 1u << (x & 31));
        else atomicXor(&lds[x >> 5], 1u << (x & 31));
      }
    }
  }
}

// The same walk, returning how many of this thread's values hit a set bit (XOR: bits
// turned off) / a clear bit (OR: bits newly set).  An array's values are distinct, so
// the counts over the workgroup are exact: the set's new cardinality follows from the
// old one by arithmetic (XOR: card + n - 2 * off; OR: card + new), with no pass over the
// 8 KiB.
template <int MODE>  // 0: or (counts new bits), 1: xor (counts bits turned off)
__device__ __forceinline__ int lds_apply_array_count(uint32_t* lds, const uint16_t* vals, int card) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(vals);
  const int lo = (int)((a & 15) >> 1);
  const int nvec = (lo + card + 7) >> 3;
  const uint4* v4 = reinterpret_cast<const uint4*>(a & ~(uintptr_t)15);
  int cnt = 0;
  for (int i = threadIdx.x; i < nvec; i += NT) {
    const uint4 v = v4[i];
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
    const int base = i * 8 - lo;
#pragma unroll
    for (int j = 0; j < 8; j++) {
      if ((unsigned)(base + j) < (unsigned)card) {
        const uint32_t x = (w[j >> 1] >> ((j & 1) * 16)) & 0xFFFF;
        const uint32_t m = 1u << (x & 31);
        const uint32_t old = MODE == 0 ? atomicOr(&lds[x >> 5], m) : atomicXor(&lds[x >> 5], m);
        cnt += MODE == 0 ? ((old & m) == 0) : ((old & m) != 0);
      }
    }
  }
  return cnt;
}

// OR one run [s, e] (inclusive) into LDS words, single thread.
__device__ __forceinline__ void lds_or_run_serial(uint32_t* lds, int s, int e) {
  const int ws = s >> 5, we = e >> 5;
  const uint32_t first = ~0u << (s & 31);
  const uint32_t last = ~0u >> (31 - (e & 31));
  if (ws == we) {
    atomicOr(&lds[ws], first & last);
    return;
  }
  atomicOr(&lds[ws], first);
  for (int w = ws + 1; w < we; w++) lds[w] = ~0u;  // no other run of this pass owns w
  atomicOr(&lds[we], last);
}

// OR the runs of a run container into an LDS bitmap.  Short runs are filled by
// one thread each; runs longer than 8 words are queued and filled by the whole
// workgroup so a single long run does not serialise one lane.  `q` needs 257
// ints of LDS.  Must be called by all threads; ends with a barrier.
__device__ __forceinline__ void lds_or_runs(uint32_t* lds, const uint32_t* pairs, int nruns, int* q) {
  if (threadIdx.x == 0) q[256] = 0;
  lds_barrier();
  for (int i = threadIdx.x; i < nruns; i += NT) {
    const uint32_t p = pairs[i];
    const int s = (int)(p & 0xFFFF);
    const int e = s + (int)(p >> 16);
    if ((e >> 5) - (s >> 5) <= 8) {
      lds_or_run_serial(lds, s, e);
    } else {
      const int slot = atomicAdd(&q[256], 1);
      if (slot < 256) q[slot] = i;
      else lds_or_run_serial(lds, s, e);  // queue full: fall back to the serial fill
    }
  }
  lds_barrier();
  const int nq = min(q[256], 256);
  for (int k = 0; k < nq; k++) {
    const uint32_t p = pairs[q[k]];
    const int s = (int)(p & 0xFFFF);
    const int e = s + (int)(p >> 16);
    const int ws = s >> 5, we = e >> 5;
    for (int w = ws + threadIdx.x; w <= we; w += NT) {
      uint32_t m = ~0u;
      if (w == ws) m &= ~0u << (s & 31);
      if (w == we) m &= ~0u >> (31 - (e & 31));
      if (m == ~0u) lds[w] = ~0u;
      else atomicOr(&lds[w], m);
    }
  }
  lds_barrier();
}

// Materialise any container into the caller's owned registers.  `lds` is an
// 8 KiB scratch bitmap, `q` 257 ints.  All threads must call; contains barriers.
__device__ __forceinline__ void materialize(const CDesc& d, const uint8_t* payload, uint32_t* lds,
                                            int* q, uint64_t r[4]) {
  const uint8_t* slot = payload + d.slot;
  if (d.kind == DK_B) {
    load_bitmap_owned(slot, r);
    return;
  }
  lds_barrier();  // previous readers of lds are done
  lds_clear(lds);
  lds_barrier();
  if (d.kind == DK_A) {
    lds_scatter_array(lds, reinterpret_cast<const uint16_t*>(slot), (int)d.card);
    lds_barrier();
  } else {
    const int nr = *reinterpret_cast<const uint16_t*>(slot + 2);
    lds_or_runs(lds, reinterpret_cast<const uint32_t*>(slot + 4), nr, q);
  }
  lds_read_owned(lds, r);
}

// Count runs of the owned words; `lds` receives the words (used to fetch the
// neighbours' edge bits).  Returns per-thread start bits in s[4] and end bits
// in e[4].  Contains barriers.
__device__ __forceinline__ void run_edges(const uint64_t r[4], uint32_t* lds, uint64_t s[4],
                                          uint64_t e[4]) {
  lds_barrier();
  lds_write_owned(lds, r);
  lds_barrier();
  const uint64_t* w = reinterpret_cast<const uint64_t*>(lds);
  const int t = threadIdx.x;
  const uint64_t prev0 = (t == 0) ? 0 : (w[2 * t - 1] >> 63);
  const uint64_t prev2 = w[511 + 2 * t] >> 63;  // t == 0 reads word 511
  const uint64_t next1 = w[2 * t + 2] & 1;      // t == 255 reads word 512
  const uint64_t next3 = (t == NT - 1) ? 0 : (w[514 + 2 * t] & 1);
  s[0] = r[0] & ~((r[0] << 1) | prev0);
  s[1] = r[1] & ~((r[1] << 1) | (r[0] >> 63));
  s[2] = r[2] & ~((r[2] << 1) | prev2);
  s[3] = r[3] & ~((r[3] << 1) | (r[2] >> 63));
  e[0] = r[0] & ~((r[0] >> 1) | ((r[1] & 1) << 63));
  e[1] = r[1] & ~((r[1] >> 1) | (next1 << 63));
  e[2] = r[2] & ~((r[2] >> 1) | ((r[3] & 1) << 63));
  e[3] = r[3] & ~((r[3] >> 1) | (next3 << 63));
}

// ---------------------------------------------------------------------------
// emission of a computed container into a 16 B-aligned slot (slot layout above)
// ---------------------------------------------------------------------------
// Stage the owned container's serialized payload in LDS `stage` (8 KiB):
// A: u16 values; B: 1024 u64 words; R: u16 nruns + (start, length-1) pairs.
// Returns the serialized length.  `lds` is scratch for the run-edge exchange.
__device__ __forceinline__ uint32_t stage_array(const uint64_t r[4], int card, uint32_t* stage, int* sh) {
  const int c0 = popc64(r[0]) + popc64(r[1]);
  const int c1 = popc64(r[2]) + popc64(r[3]);
  int p0, p1, tot;
  block_scan_halves(c0, c1, p0, p1, tot, sh);
  uint16_t* st = reinterpret_cast<uint16_t*>(stage);
  const int t = threadIdx.x;
  const int bases[4] = {(2 * t) * 64, (2 * t + 1) * 64, (512 + 2 * t) * 64, (513 + 2 * t) * 64};
  int pos[4] = {p0, p0 + popc64(r[0]), p1, p1 + popc64(r[2])};
#pragma unroll
  for (int k = 0; k < 4; k++) {
    uint64_t x = r[k];
    int p = pos[k];
    while (x) {
      st[p++] = (uint16_t)(bases[k] + __builtin_ctzll(x));
      x &= x - 1;
    }
  }
  lds_barrier();
  return 2u * (uint32_t)card;
}

__device__ __forceinline__ uint32_t stage_runs(const uint64_t r[4], uint32_t* lds, uint32_t* stage, int* sh) {
  uint64_t s[4], e[4];
  run_edges(r, lds, s, e);
  int ps0, ps1, nr, pe0, pe1, ne;
  block_scan_halves(popc64(s[0]) + popc64(s[1]), popc64(s[2]) + popc64(s[3]), ps0, ps1, nr, sh);
  block_scan_halves(popc64(e[0]) + popc64(e[1]), popc64(e[2]) + popc64(e[3]), pe0, pe1, ne, sh);
  uint16_t* st = reinterpret_cast<uint16_t*>(stage);
  const int t = threadIdx.x;
  const int bases[4] = {(2 * t) * 64, (2 * t + 1) * 64, (512 + 2 * t) * 64, (513 + 2 * t) * 64};
  int sp[4] = {ps0, ps0 + popc64(s[0]), ps1, ps1 + popc64(s[2])};
#pragma unroll
  for (int k = 0; k < 4; k++) {
    uint64_t x = s[k];
    int p = sp[k];
    while (x) {
      if (p < 2047) st[1 + 2 * p] = (uint16_t)(bases[k] + __builtin_ctzll(x));
      p++;
      x &= x - 1;
    }
  }
  lds_barrier();
  int ep[4] = {pe0, pe0 + popc64(e[0]), pe1, pe1 + popc64(e[2])};
#pragma unroll
  for (int k = 0; k < 4; k++) {
    uint64_t x = e[k];
    int p = ep[k];
    while (x) {
      if (p < 2047) st[2 + 2 * p] = (uint16_t)(bases[k] + __builtin_ctzll(x) - st[1 + 2 * p]);
      p++;
      x &= x - 1;
    }
  }
  if (t == 0) st[0] = (uint16_t)nr;
  lds_barrier();
  return 2u + 4u * (uint32_t)nr;
}

// Number of runs of the owned container (block-wide).  Contains barriers.
__device__ __forceinline__ int count_runs(const uint64_t r[4], uint32_t* lds, int* sh) {
  uint64_t s[4], e[4];
  run_edges(r, lds, s, e);
  int a = popc64(s[0]) + popc64(s[1]) + popc64(s[2]) + popc64(s[3]);
  int b = 0;
  block_sum2(a, b, sh);
  return a;
}

__device__ __forceinline__ uint32_t stage_container(int kind, const uint64_t r[4], int card, uint32_t* lds,
                                                    uint32_t* stage, int* sh) {
  if (kind == DK_B) {
    lds_barrier();
    lds_write_owned(stage, r);
    lds_barrier();
    return 8192;
  }
  if (kind == DK_A) return stage_array(r, card, stage, sh);
  return stage_runs(r, lds, stage, sh);
}

// ---------------------------------------------------------------------------
// byte copy with arbitrary source / destination alignment (group-cooperative).
// Reads up to 16 bytes past the end of `src`; every source buffer carries slack.
// ---------------------------------------------------------------------------
template <int G>
__device__ __forceinline__ void group_copy(uint8_t* dst, const uint8_t* src, uint32_t n, int lane) {
  const uintptr_t d = reinterpret_cast<uintptr_t>(dst);
  uint32_t head = (uint32_t)((16 - (d & 15)) & 15);
  if (head > n) head = n;
  for (uint32_t i = lane; i < head; i += G) dst[i] = src[i];
  uint8_t* db = dst + head;
  const uint8_t* sb = src + head;
  const uint32_t rem = n - head;
  const uint32_t nvec = rem >> 4;
  const uintptr_t s = reinterpret_cast<uintptr_t>(sb);
  uint4* dv = reinterpret_cast<uint4*>(db);
  if ((s & 15) == 0) {
    const uint4* sv = reinterpret_cast<const uint4*>(sb);
    for (uint32_t i = lane; i < nvec; i += G) dv[i] = sv[i];
  } else if ((s & 3) == 0) {
    const uint32_t* sw = reinterpret_cast<const uint32_t*>(sb);
    for (uint32_t i = lane; i < nvec; i += G) dv[i] = make_uint4(sw[4 * i], sw[4 * i + 1], sw[4 * i + 2], sw[4 * i + 3]);
  } else {
    const uint32_t sh = (uint32_t)(s & 3);
    const uint32_t* sw = reinterpret_cast<const uint32_t*>(s & ~(uintptr_t)3);
    for (uint32_t i = lane; i < nvec; i += G) {
      const uint32_t* q = sw + 4 * i;
      const uint32_t a0 = q[0], a1 = q[1], a2 = q[2], a3 = q[3], a4 = q[4];
      dv[i] = make_uint4(__builtin_amdgcn_alignbyte(a1, a0, sh), __builtin_amdgcn_alignbyte(a2, a1, sh),
                         __builtin_amdgcn_alignbyte(a3, a2, sh), __builtin_amdgcn_alignbyte(a4, a3, sh));
    }
  }
  const uint32_t done = nvec << 4;
  for (uint32_t i = done + lane; i < rem; i += G) db[i] = sb[i];
}

}  // namespace rbg
