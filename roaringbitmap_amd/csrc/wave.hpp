// Wave-level building blocks: one 64-lane wavefront owns one 65536-bit container.
//
// Lane l holds 16 u64 words of the container in registers: chunk i (0..7),
// word j (0..1) is container word 128*i + 2*l + j, i.e. byte offset 1024*i + 16*l
// + 8*j.  A bitmap container therefore streams from HBM as eight fully coalesced
// 16-byte loads per lane (1 KiB per wave instruction), the wave never needs a
// workgroup barrier, and neighbouring words for run-edge detection come from a
// single lane rotation.
#pragma once
#include "device.hpp"

namespace rbg {

constexpr int WL = 64;  // lanes per wave

__device__ __forceinline__ int lane_id() { return threadIdx.x & 63; }
// wave-uniform copy (value of the first active lane, in an SGPR)
__device__ __forceinline__ uint32_t uni(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }
// (readfirstlane returns int: each half goes through uint32_t, or a low half with bit 31
// set would sign-extend over the high half)
__device__ __forceinline__ uint64_t uni64(uint64_t x) {
  return ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)(x >> 32)) << 32) |
         (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((uint32_t)x);
}

// Operand payload loads (16 B) are nontemporal: every input byte of an op is read once,
// and keeping the inputs out of the caches leaves the Infinity Cache to the result
// slots that the serializer reads back (C2 AND: compute -7 %, andCardinality -10 %).
__device__ __forceinline__ uint4 ld_in(const uint4* p) {
  typedef unsigned int v4u __attribute__((ext_vector_type(4)));
  const v4u v = __builtin_nontemporal_load(reinterpret_cast<const v4u*>(p));
  return make_uint4(v.x, v.y, v.z, v.w);
}

// Bit-field helpers for map probes.  Written as v_bfe_u32 directly: the compiler
// otherwise turns a field extract into shift + mask (2 VALU instead of 1), and a
// variable bit test into shift + shift + and.  The hardware reads only the low
// 5 bits of a bfe offset, so no masking of `bit` is needed.
// map word index of the low / high u16 value packed in a u32 (bits 5..15 / 21..31)
__device__ __forceinline__ uint32_t bfe_lo_word(uint32_t w) {
  uint32_t r;
  asm("v_bfe_u32 %0, %1, 5, 11" : "=v"(r) : "v"(w));
  return r;
}
__device__ __forceinline__ uint32_t bfe_hi_word(uint32_t w) {
  uint32_t r;
  asm("v_bfe_u32 %0, %1, 21, 11" : "=v"(r) : "v"(w));
  return r;
}
// bit (bit & 31) of word, as 0 / 1
__device__ __forceinline__ uint32_t bit_at(uint32_t word, uint32_t bit) {
  uint32_t r;
  asm("v_bfe_u32 %0, %1, %2, 1" : "=v"(r) : "v"(word), "v"(bit));
  return r;
}

// Orders this wave's LDS accesses (LDS ops of one wave complete in issue order;
// this keeps the compiler from reordering across the point).
__device__ __forceinline__ void wsync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ int wave_sum_i(int v) { return lane63(dpp_incl_scan(v)); }
// exclusive prefix over lanes; returns the wave total in *tot (wave-uniform)
__device__ __forceinline__ int wave_excl(int v, int* tot) {
  const int s = dpp_incl_scan(v);
  *tot = lane63(s);
  return s - v;
}

struct WCtr {
  uint64_t w[16];  // w[2*i + j] = container word 128*i + 2*lane + j
};

__device__ __forceinline__ void w_zero(WCtr& x) {
#pragma unroll
  for (int k = 0; k < 16; k++) x.w[k] = 0;
}
__device__ __forceinline__ void w_ones(WCtr& x) {
#pragma unroll
  for (int k = 0; k < 16; k++) x.w[k] = ~0ULL;
}

// bitmap payload (global, 16 B aligned) -> registers
__device__ __forceinline__ void w_load_bitmap(const uint8_t* p, WCtr& x) {
  const uint4* q = reinterpret_cast<const uint4*>(p) + lane_id();
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint4 v = ld_in(q + 64 * i);
    x.w[2 * i] = (uint64_t)v.x | ((uint64_t)v.y << 32);
    x.w[2 * i + 1] = (uint64_t)v.z | ((uint64_t)v.w << 32);
  }
}
// bits [lo, hi] of register k of the wave layout (WCtr: w[2 i + j] = word 128 i + 2 lane + j)
__device__ __forceinline__ uint64_t wrange(int k, int lo, int hi) {
  const int w = 128 * (k >> 1) + 2 * lane_id() + (k & 1);
  const int b0 = 64 * w, b1 = b0 + 63;
  if (b1 < lo || b0 > hi) return 0ull;
  uint64_t m = ~0ull;
  if (lo > b0) m &= ~0ull << (lo - b0);
  if (hi < b1) m &= ~0ull >> (b1 - hi);
  return m;
}

// LDS bitmap (u32[2048]) <-> registers
__device__ __forceinline__ void w_read_lds(const uint32_t* lds, WCtr& x) {
  const uint4* q = reinterpret_cast<const uint4*>(lds) + lane_id();
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint4 v = q[64 * i];
    x.w[2 * i] = (uint64_t)v.x | ((uint64_t)v.y << 32);
    x.w[2 * i + 1] = (uint64_t)v.z | ((uint64_t)v.w << 32);
  }
}
__device__ __forceinline__ void w_write_lds(uint32_t* lds, const WCtr& x) {
  uint4* q = reinterpret_cast<uint4*>(lds) + lane_id();
#pragma unroll
  for (int i = 0; i < 8; i++)
    q[64 * i] = make_uint4((uint32_t)x.w[2 * i], (uint32_t)(x.w[2 * i] >> 32), (uint32_t)x.w[2 * i + 1],
                           (uint32_t)(x.w[2 * i + 1] >> 32));
}
__device__ __forceinline__ void w_clear_lds(uint32_t* lds) {
  uint4* q = reinterpret_cast<uint4*>(lds) + lane_id();
#pragma unroll
  for (int i = 0; i < 8; i++) q[64 * i] = make_uint4(0, 0, 0, 0);
}

// OR/XOR the values of an array container (<= 4096 values, 16 B aligned slot)
// into the wave's LDS bitmap.  All of a lane's 16 B vectors are loaded before
// the first LDS atomic so the loads overlap (one memory latency per container).
constexpr int kVecRound = 4;  // 16 B vectors per lane loaded per round

// OR/XOR the 8 values of one 16 B vector (values base..base+7, those < card).
// Branch-free: one LDS atomic per value, 4 VALU (word index, address, valid bit,
// bit mask).  Values whose bit in `vm` is clear get a zero mask (the valid bits are
// formed once per vector).  An average array has about one value per map word, so
// merging same-word neighbours saved few atomics but cost divergent branches.
template <int MODE>  // MODE 0 or, 1 xor
__device__ __forceinline__ void scatter_vec_mask(uint32_t* lds, const uint4 v, uint32_t vm) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint32_t wi = w[i >> 1];
    uint32_t* p = lds + ((i & 1) ? bfe_hi_word(wi) : bfe_lo_word(wi));
    const uint32_t m = ((vm >> i) & 1u) << (((i & 1) ? (wi >> 16) : wi) & 31u);
    if (MODE == 0) atomicOr(p, m);
    else atomicXor(p, m);
  }
}

template <int MODE>  // MODE 0 or, 1 xor
__device__ __forceinline__ void scatter_vec(uint32_t* lds, const uint4 v, int base, int card) {
  const int rem = card - base;
  scatter_vec_mask<MODE>(lds, v, rem >= 8 ? 0xFFu : (1u << max(rem, 0)) - 1u);
}

// Same-word merging variant: the bits of consecutive values that share a 32-bit map
// word go out in one atomic (branches on the word change).  The batched
// andCardinality's small arrays keep it (C4 0.156 ms against 0.181 branch-free).
template <int MODE>  // MODE 0 or, 1 xor
__device__ __forceinline__ void scatter_vec_merged(uint32_t* lds, const uint4 v, int base, int card) {
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
  uint32_t cur = 0xFFFFFFFFu, mask = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    if (base + i < card) {
      const uint32_t x = (w[i >> 1] >> ((i & 1) * 16)) & 0xFFFF;
      if ((x >> 5) != cur) {
        if (mask) {
          if (MODE == 0) atomicOr(&lds[cur], mask);
          else atomicXor(&lds[cur], mask);
        }
        cur = x >> 5;
        mask = 0;
      }
      mask |= 1u << (x & 31);
    }
  }
  if (mask) {
    if (MODE == 0) atomicOr(&lds[cur], mask);
    else atomicXor(&lds[cur], mask);
  }
}

template <int MODE>  // 0 or, 1 xor
__device__ __forceinline__ void w_scatter_array(uint32_t* lds, const uint16_t* vals, int card) {
  const int nvec = (card + 7) >> 3;  // <= 512 = 8 per lane, in rounds of 4
  const uint4* v4 = reinterpret_cast<const uint4*>(vals);
  const int l = lane_id();
#pragma unroll 1
  for (int j0 = 0; 64 * j0 < nvec; j0 += kVecRound) {
    uint4 v[kVecRound];
#pragma unroll
    for (int j = 0; j < kVecRound; j++) {
      const int k = 64 * (j0 + j) + l;
      v[j] = k < nvec ? ld_in(v4 + k) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < kVecRound; j++) {
      const int base = 8 * (64 * (j0 + j) + l);
      if (base >= card) break;
      scatter_vec<MODE>(lds, v[j], base, card);
    }
  }
}

// Run containers are materialised without per-word fills: every run toggles its
// first bit and the bit after its last one in a cleared LDS bitmap (2 LDS
// atomics per run, no divergence on run length), and an inclusive prefix-XOR
// over the 65536 bits then turns the toggles into the filled runs.  Valid run
// containers have disjoint runs, so toggles of adjacent runs cancel correctly.
// Toggles of the runs held in one 16 B vector of a run slot (runs r0..r0+3).
__device__ __forceinline__ void toggle_vec(uint32_t* lds, const uint4 v, int r0, int nruns) {
  const uint32_t u[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int c = 0; c < 4; c++) {
    const int r = r0 + c;
    if (r >= 0 && r < nruns) {
      const uint32_t s = u[c] & 0xFFFF, e1 = s + (u[c] >> 16) + 1;
      atomicXor(&lds[s >> 5], 1u << (s & 31));
      if (e1 < 65536) atomicXor(&lds[e1 >> 5], 1u << (e1 & 31));
    }
  }
}

// slot = [u16 pad][u16 nruns][u32 (start, len-1) pairs]: u32 k of the slot is
// run k-1, so the slot streams as aligned 16 B vectors (input run containers
// may hold up to 32768 runs; results hold at most 2047).  Vectors from j0 on.
__device__ __forceinline__ void w_toggle_runs(uint32_t* lds, const uint8_t* slot, int nruns, int j_first = 0) {
  const int nvec = (nruns + 4) >> 2;
  const uint4* v4 = reinterpret_cast<const uint4*>(slot);
  const int l = lane_id();
#pragma unroll 1
  for (int j0 = j_first; 64 * j0 < nvec; j0 += kVecRound) {
    uint4 v[kVecRound];
#pragma unroll
    for (int j = 0; j < kVecRound; j++) {
      const int k = 64 * (j0 + j) + l;
      v[j] = k < nvec ? ld_in(v4 + k) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < kVecRound; j++) {
      const int r0 = 4 * (64 * (j0 + j) + l) - 1;
      if (r0 >= nruns) break;
      toggle_vec(lds, v[j], r0, nruns);
    }
  }
}

__device__ __forceinline__ uint64_t prefix_xor64(uint64_t x) {
  x ^= x << 1;
  x ^= x << 2;
  x ^= x << 4;
  x ^= x << 8;
  x ^= x << 16;
  x ^= x << 32;
  return x;
}

// Chunk i (words 128i + 2l + {0,1}) of the filled run bitmap from the toggle
// bitmap in LDS.  `carry` (wave-uniform) is the parity of all earlier chunks.
__device__ __forceinline__ void w_run_chunk(const uint32_t* lds, int i, uint32_t& carry, uint64_t& w0, uint64_t& w1) {
  const int l = lane_id();
  const uint4 v = reinterpret_cast<const uint4*>(lds)[64 * i + l];
  uint64_t a = prefix_xor64((uint64_t)v.x | ((uint64_t)v.y << 32));
  uint64_t b = prefix_xor64((uint64_t)v.z | ((uint64_t)v.w << 32));
  if (a >> 63) b = ~b;
  const uint64_t m = __ballot((b >> 63) != 0);  // per-lane parity of its two words
  const uint32_t pre = ((uint32_t)__popcll(m & ((1ULL << l) - 1)) & 1u) ^ carry;
  if (pre) {
    a = ~a;
    b = ~b;
  }
  carry ^= (uint32_t)__popcll(m) & 1u;
  w0 = a;
  w1 = b;
}

// Materialise any container into registers.  `lds` is the wave's 8 KiB bitmap.
__device__ __forceinline__ void w_materialize(const CDesc& d, const uint8_t* payload, uint32_t* lds, WCtr& x) {
  const uint8_t* slot = payload + d.slot;
  if (d.kind == DK_B) {
    w_load_bitmap(slot, x);
    return;
  }
  wsync();
  w_clear_lds(lds);
  wsync();
  if (d.kind == DK_A) {
    w_scatter_array<0>(lds, reinterpret_cast<const uint16_t*>(slot), (int)d.card);
    wsync();
    w_read_lds(lds, x);
  } else {
    const int nr = *reinterpret_cast<const uint16_t*>(slot + 2);
    w_toggle_runs(lds, slot, nr);
    wsync();
    uint32_t carry = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) w_run_chunk(lds, i, carry, x.w[2 * i], x.w[2 * i + 1]);
  }
}

// x = x OP (container d), materialising d chunk by chunk (no second register copy).
template <int OP>  // 0 and, 1 or, 2 xor, 3 andnot
__device__ __forceinline__ uint64_t w_op(uint64_t a, uint64_t b) {
  if (OP == 0) return a & b;
  if (OP == 1) return a | b;
  if (OP == 2) return a ^ b;
  return a & ~b;
}
template <int OP>
__device__ __forceinline__ void w_combine(const CDesc& d, const uint8_t* payload, uint32_t* lds, WCtr& x) {
  const uint8_t* slot = payload + d.slot;
  if (d.kind == DK_R) {
    wsync();
    w_clear_lds(lds);
    wsync();
    const int nr = *reinterpret_cast<const uint16_t*>(slot + 2);
    w_toggle_runs(lds, slot, nr);
    wsync();
    uint32_t carry = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      uint64_t a, b;
      w_run_chunk(lds, i, carry, a, b);
      x.w[2 * i] = w_op<OP>(x.w[2 * i], a);
      x.w[2 * i + 1] = w_op<OP>(x.w[2 * i + 1], b);
    }
    return;
  }
  // B from global memory and A from the LDS map take separate loops: one loop
  // over a pointer that may be either compiles to flat loads, which wait on both
  // the vector-memory and the LDS counters
  if (d.kind == DK_B) {
    const uint4* g = reinterpret_cast<const uint4*>(slot) + lane_id();
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const uint4 v = ld_in(g + 64 * i);
      x.w[2 * i] = w_op<OP>(x.w[2 * i], (uint64_t)v.x | ((uint64_t)v.y << 32));
      x.w[2 * i + 1] = w_op<OP>(x.w[2 * i + 1], (uint64_t)v.z | ((uint64_t)v.w << 32));
    }
    return;
  }
  wsync();
  w_clear_lds(lds);
  wsync();
  w_scatter_array<0>(lds, reinterpret_cast<const uint16_t*>(slot), (int)d.card);
  wsync();
  const uint4* q = reinterpret_cast<const uint4*>(lds) + lane_id();
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint4 v = q[64 * i];
    x.w[2 * i] = w_op<OP>(x.w[2 * i], (uint64_t)v.x | ((uint64_t)v.y << 32));
    x.w[2 * i + 1] = w_op<OP>(x.w[2 * i + 1], (uint64_t)v.z | ((uint64_t)v.w << 32));
  }
}

__device__ __forceinline__ int w_card(const WCtr& x) {
  int c = 0;
#pragma unroll
  for (int k = 0; k < 16; k++) c += __popcll(x.w[k]);
  return (int)__builtin_amdgcn_readfirstlane((uint32_t)wave_sum_i(c));
}

// Run start / end bit masks of chunk I of the owned container (computed on the
// fly so no full start/end copies are kept in registers).
template <int I>
__device__ __forceinline__ void w_chunk_edges(const WCtr& x, uint64_t& s0, uint64_t& s1, uint64_t& e0, uint64_t& e1) {
  const int l = lane_id();
  const uint64_t w0 = x.w[2 * I], w1 = x.w[2 * I + 1];
  const uint32_t top1 = from_prev_lane((uint32_t)(w1 >> 63));  // lane l-1's word 1 top bit
  const uint32_t pchunk = I > 0 ? lane63u((uint32_t)(x.w[2 * (I > 0 ? I - 1 : 0) + 1] >> 63)) : 0u;
  const uint64_t prev0 = (l == 0) ? pchunk : top1;
  const uint32_t bot0 = from_next_lane((uint32_t)(w0 & 1));  // lane l+1's word 0 bit 0
  const uint32_t nchunk = I < 7 ? lane0u((uint32_t)(x.w[2 * (I < 7 ? I + 1 : 7)] & 1)) : 0u;
  const uint64_t next1 = (l == 63) ? nchunk : bot0;
  s0 = w0 & ~((w0 << 1) | prev0);
  s1 = w1 & ~((w1 << 1) | (w0 >> 63));
  e0 = w0 & ~((w0 >> 1) | ((w1 & 1) << 63));
  e1 = w1 & ~((w1 >> 1) | (next1 << 63));
}

template <int I>
__device__ __forceinline__ int w_runs_acc(const WCtr& x) {
  uint64_t s0, s1, e0, e1;
  w_chunk_edges<I>(x, s0, s1, e0, e1);
  return __popcll(s0) + __popcll(s1) + (I < 7 ? w_runs_acc<(I < 7 ? I + 1 : 7)>(x) : 0);
}

__device__ __forceinline__ int w_runs(const WCtr& x) {
  const int c = w_runs_acc<0>(x);
  return (int)__builtin_amdgcn_readfirstlane((uint32_t)wave_sum_i(c));
}

__device__ __forceinline__ int w_stage_runs(const WCtr& x, uint32_t* lds);

// Serialized payload of the owned container, staged in the wave's LDS
// (A: u16 values; B: 1024 u64 words; R: u16 nruns + (start, len-1) pairs).
// Returns the serialized length.
__device__ __forceinline__ uint32_t w_stage(int kind, const WCtr& x, int card, uint32_t* lds) {
  const int l = lane_id();
  if (kind == DK_B) {
    wsync();
    w_write_lds(lds, x);
    wsync();
    return 8192;
  }
  uint16_t* st = reinterpret_cast<uint16_t*>(lds);
  if (kind == DK_A) {
    wsync();
    int base = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      uint64_t v0 = x.w[2 * i], v1 = x.w[2 * i + 1];
      const int c0 = __popcll(v0);
      int tot;
      int p0 = base + wave_excl(c0 + __popcll(v1), &tot);
      int p1 = p0 + c0;
      const int wb = (128 * i + 2 * l) * 64;
      // both words drained together: iterations = max(popc) instead of the sum
      while (v0 | v1) {
        if (v0) {
          st[p0++] = (uint16_t)(wb + __builtin_ctzll(v0));
          v0 &= v0 - 1;
        }
        if (v1) {
          st[p1++] = (uint16_t)(wb + 64 + __builtin_ctzll(v1));
          v1 &= v1 - 1;
        }
      }
      base += tot;
    }
    wsync();
    return 2u * (uint32_t)card;
  }
  return 2u + 4u * (uint32_t)w_stage_runs(x, lds);
}

// ---------------------------------------------------------------------------
// key planning helpers (one thread per key)
// ---------------------------------------------------------------------------
__device__ __forceinline__ int lower_bound_u16(const uint16_t* keys, int n, uint32_t k) {
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (keys[mid] < k) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// Zeroes the output look-back state of the op about to run (block 0 of a plan
// kernel; saves two memset launches per op).  Either pointer may be null.
// The tile aggregates of a pairwise op (OutCtx::tile_agg) follow the tile statuses and cardinalities in the
// look-back buffer: tile_status + 2 kMaxTiles (engine.cpp: prepare_output), zeroed here too.
__device__ __forceinline__ void plan_zero(uint64_t* lb_header, uint64_t* tile_status) {
  if (blockIdx.x != 0) return;
  if (lb_header && threadIdx.x < 32) lb_header[threadIdx.x] = 0;
  if (tile_status) {
    for (uint32_t i = threadIdx.x; i < (uint32_t)kMaxTiles; i += blockDim.x) tile_status[i] = 0;
    for (uint32_t i = threadIdx.x; i < (uint32_t)kMaxAggTiles; i += blockDim.x) tile_status[2 * kMaxTiles + i] = 0;
  }
}

// Descriptor of key k in a single-bitmap batch through its key CSR (O(1), no search)
__device__ __forceinline__ void resolve(const uint32_t* key_off, const CDesc* desc, const uint8_t* payload, uint32_t k,
                                        uint64_t& slot, uint32_t& card, uint8_t& kind, uint16_t& nruns) {
  const uint32_t p = key_off[k];
  if (key_off[k + 1] > p) {
    const CDesc d = desc[p];
    slot = d.slot;
    card = d.card;
    kind = d.kind;
    nruns = d.kind == DK_R ? *reinterpret_cast<const uint16_t*>(payload + d.slot + 2) : 0;
  } else {
    slot = 0;
    card = 0;
    kind = kAbsent;
    nruns = 0;
  }
}

// a task record through the scalar cache (wave-uniform; loads only)
__device__ __forceinline__ PTask load_task(const PTask* tasks, uint32_t t) {
  typedef const __attribute__((address_space(4))) uint64_t* CU64;
  const CU64 q = reinterpret_cast<CU64>(reinterpret_cast<uintptr_t>(tasks + t));
  union {
    uint64_t u[4];
    PTask p;
  } r;
#pragma unroll
  for (int i = 0; i < 4; i++) r.u[i] = q[i];
  return r.p;
}

// Plan compaction (one thread per key, 256 workgroups of 256 keys, all resident): each workgroup
// publishes its task count tagged with the op's epoch, sums the counts of the workgroups before it
// (one per thread, waiting for the epoch), and writes its flagged tasks straight into the dense task
// list in key order.  The last workgroup writes the task count.
__device__ __forceinline__ void plan_emit(int f, const PTask& t, uint64_t* wg_epoch, uint32_t epoch, PTask* tasks,
                                          uint32_t* n_tasks, uint32_t* err) {
  __shared__ int wt[4];
  __shared__ int wb[4];
  int tot;
  const int lane_pre = wave_excl(f, &tot);
  if ((threadIdx.x & 63) == 0) wt[threadIdx.x >> 6] = tot;
  __syncthreads();
  const int cnt = wt[0] + wt[1] + wt[2] + wt[3];
  if (threadIdx.x == 0)
    __hip_atomic_store(wg_epoch + blockIdx.x, ((uint64_t)epoch << 32) | (uint32_t)cnt, __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  // counts of the workgroups before this one
  uint32_t c = 0;
  if (threadIdx.x < blockIdx.x) {
    uint64_t v;
    uint32_t spins = 0;
    while (((v = __hip_atomic_load(wg_epoch + threadIdx.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)) >> 32) !=
           epoch) {
      if (++spins > (1u << 22)) {
        atomicOr(err, 1u);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    c = (uint32_t)v;
  }
  const int sw = wave_sum_i((int)c);
  if ((threadIdx.x & 63) == 0) wb[threadIdx.x >> 6] = sw;
  __syncthreads();
  const uint32_t base = (uint32_t)(wb[0] + wb[1] + wb[2] + wb[3]);
  int wpre = 0;
  for (int i = 0; i < (int)(threadIdx.x >> 6); i++) wpre += wt[i];
  if (f) tasks[base + wpre + lane_pre] = t;
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) *n_tasks = base + cnt;
}

__device__ __forceinline__ void plan_count(int f, uint32_t* wg_count) {
  __shared__ int wc[4];
  const uint64_t m = __ballot(f);
  if ((threadIdx.x & 63) == 0) wc[threadIdx.x >> 6] = __popcll(m);
  lds_barrier();
  if (threadIdx.x == 0) wg_count[blockIdx.x] = (uint32_t)(wc[0] + wc[1] + wc[2] + wc[3]);
}

// Bitmap from registers straight to a 16 B-aligned global slot (8 coalesced
// 16 B stores per lane; no LDS round trip).
__device__ __forceinline__ void w_store_bitmap(uint8_t* p, const WCtr& x) {
  uint4* q = reinterpret_cast<uint4*>(p) + lane_id();
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint4 v = make_uint4((uint32_t)x.w[2 * i], (uint32_t)(x.w[2 * i] >> 32), (uint32_t)x.w[2 * i + 1],
                               (uint32_t)(x.w[2 * i + 1] >> 32));
    // plain stores: the slot is read back by the serializer right after the op, and plain
    // stores leave it in the Infinity Cache (with the serializer's nontemporal output
    // stores: C2 AND step 0.362 -> 0.351 ms; nontemporal slot stores 0.38)
    *reinterpret_cast<uint4*>(q + 64 * i) = v;
  }
}

// ---------------------------------------------------------------------------
// prefetched operands: both operands' payloads are requested up front (one
// memory latency per task instead of one per operand), then consumed from
// registers.  Lane l holds vectors 64*j + l (j < kPre) of the slot: all of an
// A or B payload, and R payloads of up to 2043 runs (longer inputs stream the
// rest from memory).
// ---------------------------------------------------------------------------
constexpr int kPre = 8;
struct WPre {
  uint4 v[kPre];
};

// 16 B vectors of a slot that hold payload (A: 2c bytes; B: 8192; R: 4 + 4 nruns)
__device__ __forceinline__ int slot_nvec(int kind, int card, int nruns) {
  return kind == DK_A ? (2 * card + 15) >> 4 : kind == DK_B ? 512 : (nruns + 4) >> 2;
}

__device__ __forceinline__ void w_prefetch(const uint8_t* slot, int nvec, WPre& p) {
  const uint4* q = reinterpret_cast<const uint4*>(slot) + lane_id();
  const int l = lane_id();
#pragma unroll
  for (int j = 0; j < kPre; j++) p.v[j] = (64 * j + l < nvec) ? q[64 * j] : make_uint4(0, 0, 0, 0);
}

template <int MODE>
__device__ __forceinline__ void w_scatter_pre(uint32_t* lds, const WPre& p, int card) {
  const int l = lane_id();
#pragma unroll
  for (int j = 0; j < kPre; j++) {
    if (512 * j >= card) break;  // wave-uniform
    scatter_vec<MODE>(lds, p.v[j], 8 * (64 * j + l), card);
    __builtin_amdgcn_sched_barrier(0);  // one vector at a time: keeps register pressure flat
  }
}

__device__ __forceinline__ void w_toggle_pre(uint32_t* lds, const WPre& p, const uint8_t* slot, int nruns) {
  const int l = lane_id();
  const int nvec = (nruns + 4) >> 2;
#pragma unroll
  for (int j = 0; j < kPre; j++) {
    if (64 * j >= nvec) break;  // wave-uniform
    toggle_vec(lds, p.v[j], 4 * (64 * j + l) - 1, nruns);
    __builtin_amdgcn_sched_barrier(0);
  }
  if (nvec > 64 * kPre) w_toggle_runs(lds, slot, nruns, kPre);
}

__device__ __forceinline__ void pre_to_words(const WPre& p, WCtr& x) {
#pragma unroll
  for (int i = 0; i < 8; i++) {
    x.w[2 * i] = (uint64_t)p.v[i].x | ((uint64_t)p.v[i].y << 32);
    x.w[2 * i + 1] = (uint64_t)p.v[i].z | ((uint64_t)p.v[i].w << 32);
  }
}

// operand (kind, card, nruns) of a prefetched slot -> owned registers
__device__ __forceinline__ void w_materialize_pre(int kind, int card, int nruns, const WPre& p, const uint8_t* slot,
                                                  uint32_t* lds, WCtr& x) {
  if (kind == DK_B) {
    pre_to_words(p, x);
    return;
  }
  wsync();
  w_clear_lds(lds);
  wsync();
  if (kind == DK_A) {
    w_scatter_pre<0>(lds, p, card);
    wsync();
    w_read_lds(lds, x);
    return;
  }
  w_toggle_pre(lds, p, slot, nruns);
  wsync();
  uint32_t carry = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) w_run_chunk(lds, i, carry, x.w[2 * i], x.w[2 * i + 1]);
}

template <int OP>  // 0 and, 1 or, 2 xor, 3 andnot
__device__ __forceinline__ void w_combine_pre(int kind, int card, int nruns, const WPre& p, const uint8_t* slot,
                                              uint32_t* lds, WCtr& x) {
  if (kind == DK_B) {
#pragma unroll
    for (int i = 0; i < 8; i++) {
      x.w[2 * i] = w_op<OP>(x.w[2 * i], (uint64_t)p.v[i].x | ((uint64_t)p.v[i].y << 32));
      x.w[2 * i + 1] = w_op<OP>(x.w[2 * i + 1], (uint64_t)p.v[i].z | ((uint64_t)p.v[i].w << 32));
    }
    return;
  }
  wsync();
  w_clear_lds(lds);
  wsync();
  if (kind == DK_A) {
    w_scatter_pre<0>(lds, p, card);
    wsync();
    const uint4* q = reinterpret_cast<const uint4*>(lds) + lane_id();
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const uint4 v = q[64 * i];
      x.w[2 * i] = w_op<OP>(x.w[2 * i], (uint64_t)v.x | ((uint64_t)v.y << 32));
      x.w[2 * i + 1] = w_op<OP>(x.w[2 * i + 1], (uint64_t)v.z | ((uint64_t)v.w << 32));
    }
    return;
  }
  w_toggle_pre(lds, p, slot, nruns);
  wsync();
  uint32_t carry = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint64_t a, b;
    w_run_chunk(lds, i, carry, a, b);
    x.w[2 * i] = w_op<OP>(x.w[2 * i], a);
    x.w[2 * i + 1] = w_op<OP>(x.w[2 * i + 1], b);
  }
}

// Any container as a 65536-bit membership map in the wave's LDS (u32[2048]),
// for probing: B is written from registers, A scattered, R toggled and
// prefix-XOR filled in place.
__device__ __forceinline__ void w_map_pre(int kind, int card, int nruns, const WPre& p, const uint8_t* slot,
                                          uint32_t* lds) {
  const int l = lane_id();
  uint4* q = reinterpret_cast<uint4*>(lds) + l;
  wsync();
  if (kind == DK_B) {
#pragma unroll
    for (int i = 0; i < 8; i++) q[64 * i] = p.v[i];
    wsync();
    return;
  }
  w_clear_lds(lds);
  wsync();
  if (kind == DK_A) {
    w_scatter_pre<0>(lds, p, card);
    wsync();
    return;
  }
  w_toggle_pre(lds, p, slot, nruns);
  wsync();
  uint32_t carry = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint64_t a, b;
    w_run_chunk(lds, i, carry, a, b);  // reads this lane's vector of chunk i, then overwrites it
    q[64 * i] = make_uint4((uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32));
  }
  wsync();
}

// A bitmap payload (8 KiB, 16 B aligned) copied into the wave's LDS map by LDS-DMA:
// eight global_load_lds_dwordx4, 1 KiB each (lane l's 16 B land at base + 16 l, the
// map's own layout), all in flight at once and no VGPRs.  (Loaded through registers,
// the copy was serialised by the register allocator in the pairwise kernels -- one
// 4-VGPR buffer, a full memory round trip per 1 KiB -- whenever the kernel ran at its
// 128-VGPR cap.)  Earlier LDS reads of the map are drained first; the DMA is waited
// for with vmcnt(0) (it also retires any older global load or store of the wave).
typedef __attribute__((address_space(3))) void* lds_void_ptr;
typedef __attribute__((address_space(1))) void* global_void_ptr;
__device__ __forceinline__ void w_bitmap_to_lds_dma(const uint8_t* slot, uint32_t* lds) {
  const uint4* g = reinterpret_cast<const uint4*>(slot) + lane_id();
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
  for (int i = 0; i < 8; i++)
    __builtin_amdgcn_global_load_lds((global_void_ptr)(g + 64 * i), (lds_void_ptr)(lds + 256 * i), 16, 0,
                                     2 /* nt */);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

// The same map built from a container streamed from memory.
__device__ __forceinline__ void w_map_lds(int kind, int card, const uint8_t* slot, uint32_t* lds) {
  wsync();
  if (kind == DK_B) {
    w_bitmap_to_lds_dma(slot, lds);
    wsync();
    return;
  }
  const int l = lane_id();
  uint4* q = reinterpret_cast<uint4*>(lds) + l;
  w_clear_lds(lds);
  wsync();
  if (kind == DK_A) {
    w_scatter_array<0>(lds, reinterpret_cast<const uint16_t*>(slot), card);
    wsync();
    return;
  }
  w_toggle_runs(lds, slot, *reinterpret_cast<const uint16_t*>(slot + 2));
  wsync();
  uint32_t carry = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    uint64_t a, b;
    w_run_chunk(lds, i, carry, a, b);  // reads this lane's vector of chunk i, then overwrites it
    q[64 * i] = make_uint4((uint32_t)a, (uint32_t)(a >> 32), (uint32_t)b, (uint32_t)(b >> 32));
  }
  wsync();
}

// Filter the sorted values of an array container (streamed from memory) by
// membership in the wave's LDS map; see w_probe_pre.
constexpr int kProbeRound = 2;  // 16 B vectors per lane per probe round
template <bool INV, bool WRITE>
__device__ __forceinline__ int w_probe_array(const uint32_t* lds, const uint16_t* vals, int n, uint16_t* out) {
  const int l = lane_id();
  const uint4* v4 = reinterpret_cast<const uint4*>(vals);
  const int nvec = (n + 7) >> 3;  // <= 512 = 8 per lane
  int base = 0;
#pragma unroll 1
  for (int j0 = 0; 64 * j0 < nvec; j0 += kProbeRound) {
    uint4 v[kProbeRound];
#pragma unroll
    for (int j = 0; j < kProbeRound; j++) {
      const int k = 64 * (j0 + j) + l;
      v[j] = k < nvec ? v4[k] : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < kProbeRound; j++) {
      if (64 * (j0 + j) >= nvec) break;  // wave-uniform
      const int first = 8 * (64 * (j0 + j) + l);
      const uint32_t w[4] = {v[j].x, v[j].y, v[j].z, v[j].w};
      uint32_t hit = 0;
#pragma unroll
      for (int i = 0; i < 8; i++) {
        const uint32_t x = (w[i >> 1] >> ((i & 1) * 16)) & 0xFFFF;
        const uint32_t m = (lds[x >> 5] >> (x & 31)) & 1u;
        hit |= ((INV ? (m ^ 1u) : m) & (first + i < n ? 1u : 0u)) << i;
      }
      int tot;
      int q = base + wave_excl(__popc(hit), &tot);
      if (WRITE) {
#pragma unroll
        for (int i = 0; i < 8; i++)
          if ((hit >> i) & 1u) out[q++] = (uint16_t)((w[i >> 1] >> ((i & 1) * 16)) & 0xFFFF);
      }
      base += tot;
    }
  }
  return (int)uni((uint32_t)base);
}

// Filter the sorted values of a prefetched array container by membership in
// the wave's LDS map: keep members (INV = false, A AND x) or non-members
// (INV = true, A ANDNOT x).  The kept values stay sorted; with WRITE they are
// stored to `out` (u16, in order).  Returns the kept count (wave-uniform).
// This is the result of RB/ArrayContainer.java:184-271 (and / andNot with any
// container), RB/BitmapContainer.java:162-171 and RB/RunContainer.java:305-334
// without materialising a result bitmap.
template <bool INV, bool WRITE>
__device__ __forceinline__ int w_probe_pre(const uint32_t* lds, const WPre& p, int n, uint16_t* out) {
  const int l = lane_id();
  int base = 0;
#pragma unroll
  for (int j = 0; j < kPre; j++) {
    if (512 * j >= n) break;  // wave-uniform
    const int first = 8 * (64 * j + l);
    const uint32_t w[4] = {p.v[j].x, p.v[j].y, p.v[j].z, p.v[j].w};
    uint32_t hit = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const uint32_t x = (w[i >> 1] >> ((i & 1) * 16)) & 0xFFFF;
      const uint32_t m = (lds[x >> 5] >> (x & 31)) & 1u;
      hit |= ((INV ? (m ^ 1u) : m) & (first + i < n ? 1u : 0u)) << i;
    }
    int tot;
    int q = base + wave_excl(__popc(hit), &tot);
    if (WRITE) {
#pragma unroll
      for (int i = 0; i < 8; i++)
        if ((hit >> i) & 1u) out[q++] = (uint16_t)((w[i >> 1] >> ((i & 1) * 16)) & 0xFFFF);
    }
    base += tot;
  }
  return (int)uni((uint32_t)base);
}

// Runs of the owned container staged in one pass: per chunk the start and end
// masks are computed once, one packed (starts | ends << 16) scan places both,
// and the four bit streams (starts / ends of the lane's two words) are drained
// together.  Ends are written as absolute positions; a final pass turns them
// into lengths.  The k-th end closes the k-th run.  Stages (u16 nruns,
// (start, len-1) pairs) in LDS when the result has <= 2047 runs (the most a run
// result can have: EFF keeps R only if 2 + 4 * nruns <= 8192).  Returns the
// run count.
// CAP: runs written at most (2047 for an 8 KiB LDS stage; unbounded for a big-run arena slot)
template <int I, int CAP = 2047>
__device__ __forceinline__ int w_stage_runs_chunk(const WCtr& x, uint16_t* st, int base, int base_e) {
  const int l = lane_id();
  uint64_t s0, s1, e0, e1;
  w_chunk_edges<I>(x, s0, s1, e0, e1);
  const int cs0 = __popcll(s0), ce0 = __popcll(e0);
  const int cs = cs0 + __popcll(s1), ce = ce0 + __popcll(e1);
  int tot;
  const int packed = wave_excl(cs | (ce << 16), &tot);
  const int wb = (128 * I + 2 * l) * 64;
  int ps0 = base + (packed & 0xFFFF), ps1 = ps0 + cs0;
  int pe0 = base_e + (packed >> 16), pe1 = pe0 + ce0;
  while (s0 | s1 | e0 | e1) {
    if (s0) {
      if (ps0 < CAP) st[1 + 2 * ps0] = (uint16_t)(wb + __builtin_ctzll(s0));
      ps0++;
      s0 &= s0 - 1;
    }
    if (s1) {
      if (ps1 < CAP) st[1 + 2 * ps1] = (uint16_t)(wb + 64 + __builtin_ctzll(s1));
      ps1++;
      s1 &= s1 - 1;
    }
    if (e0) {
      if (pe0 < CAP) st[2 + 2 * pe0] = (uint16_t)(wb + __builtin_ctzll(e0));
      pe0++;
      e0 &= e0 - 1;
    }
    if (e1) {
      if (pe1 < CAP) st[2 + 2 * pe1] = (uint16_t)(wb + 64 + __builtin_ctzll(e1));
      pe1++;
      e1 &= e1 - 1;
    }
  }
  const int nb = base + (tot & 0xFFFF), nbe = base_e + (tot >> 16);
  if (I < 7) return w_stage_runs_chunk<(I < 7 ? I + 1 : 7), CAP>(x, st, nb, nbe);
  return nb;
}

__device__ __forceinline__ int w_stage_runs(const WCtr& x, uint32_t* lds) {
  uint16_t* st = reinterpret_cast<uint16_t*>(lds);
  wsync();
  const int nr = (int)uni((uint32_t)w_stage_runs_chunk<0>(x, st, 0, 0));
  const int ns = nr < 2047 ? nr : 2047;
  wsync();
  for (int k = lane_id(); k < ns; k += 64) st[2 + 2 * k] = (uint16_t)(st[2 + 2 * k] - st[1 + 2 * k]);
  if (lane_id() == 0) st[0] = (uint16_t)ns;
  wsync();
  return nr;
}

// Copy n bytes (n even) from 16 B-aligned LDS to an even global address.
template <int G>
__device__ __forceinline__ void copy_lds_to_global(uint8_t* dst, const uint32_t* lds, uint32_t n, int lane) {
  const uintptr_t d = reinterpret_cast<uintptr_t>(dst);
  uint32_t head = (uint32_t)((16 - (d & 15)) & 15);
  if (head > n) head = n;
  const uint16_t* l16 = reinterpret_cast<const uint16_t*>(lds);
  uint16_t* d16 = reinterpret_cast<uint16_t*>(dst);
  for (uint32_t i = lane; i < head / 2; i += G) d16[i] = l16[i];
  const uint32_t body = (n - head) & ~15u;
  uint4* dv = reinterpret_cast<uint4*>(dst + head);
  const uint32_t sh = head & 3;  // 0 or 2
  const uint32_t w0 = head >> 2;
  for (uint32_t c = lane; c < body / 16; c += G) {
    const uint32_t* q = lds + w0 + 4 * c;
    if (sh == 0) {
      dv[c] = make_uint4(q[0], q[1], q[2], q[3]);
    } else {
      const uint32_t a0 = q[0], a1 = q[1], a2 = q[2], a3 = q[3], a4 = q[4];
      dv[c] = make_uint4(__builtin_amdgcn_alignbyte(a1, a0, 2), __builtin_amdgcn_alignbyte(a2, a1, 2),
                         __builtin_amdgcn_alignbyte(a3, a2, 2), __builtin_amdgcn_alignbyte(a4, a3, 2));
    }
  }
  const uint32_t done = head + body;
  for (uint32_t i = done / 2 + lane; i < n / 2; i += G) d16[i] = l16[i];
}

// ---------------------------------------------------------------------------
// single-pass output placement: decoupled look-back over task order
// status word: [63:62] state (0 none, 1 aggregate, 2 inclusive) | [61] has_run |
//              [60:44] container count | [43:0] payload bytes
// ---------------------------------------------------------------------------
struct Prefix {
  uint32_t idx;
  uint64_t off;
};

__device__ __forceinline__ uint64_t lb_pack(uint64_t st, uint64_t run, uint64_t cnt, uint64_t bytes) {
  return (st << 62) | (run << 61) | (cnt << 44) | bytes;
}


// n bytes from src to dst (any addresses), one wave.  The destination body is
// written as aligned 16 B vectors; each is the 16 bytes at `shift` (the source's offset
// from 16 B alignment at that point) inside two consecutive aligned source vectors: lane l
// loads aligned source vector i, takes vector i + 1 from lane l + 1 (a DPP lane shift;
// lane 63 from the next group's lane 0) and funnel-shifts the pair (alignbyte).  So every
// load and store is a coalesced 16 B access, 8 per lane in flight.  The unaligned head and
// tail (< 16 bytes each) go as u16, or as bytes when an address is odd: a key shard's payload
// lands at an odd offset of the global bitmap whenever the header size is odd.  Reads up to 16 bytes past the end of src
// (slots and payload arenas carry
// slack).  The pointers come from memory (records, the state header), so they are generic
// to the compiler: the accesses go through global-address-space types (flat instructions
// would also count against lgkmcnt).
typedef __attribute__((address_space(1))) uint8_t g_u8;
typedef __attribute__((address_space(1))) uint16_t g_u16;
typedef __attribute__((address_space(1))) uint32_t g_u32;
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(1))) u32x4 g_u32x4;

__device__ __forceinline__ u32x4 next_lane_vec(u32x4 v) {
  u32x4 r;
  r.x = from_next_lane(v.x);
  r.y = from_next_lane(v.y);
  r.z = from_next_lane(v.z);
  r.w = from_next_lane(v.w);
  return r;
}
__device__ __forceinline__ u32x4 lane0_vec(u32x4 v) {
  u32x4 r;
  r.x = lane0u(v.x);
  r.y = lane0u(v.y);
  r.z = lane0u(v.z);
  r.w = lane0u(v.w);
  return r;
}
// the 16 bytes at byte offset 4q + r (q, r wave-uniform, r < 4) of the 32-byte pair (a, b)
__device__ __forceinline__ u32x4 funnel16(u32x4 a, u32x4 b, uint32_t q, uint32_t r) {
  u32x4 o;
  if (q == 0) {
    o.x = __builtin_amdgcn_alignbyte(a.y, a.x, r);
    o.y = __builtin_amdgcn_alignbyte(a.z, a.y, r);
    o.z = __builtin_amdgcn_alignbyte(a.w, a.z, r);
    o.w = __builtin_amdgcn_alignbyte(b.x, a.w, r);
  } else if (q == 1) {
    o.x = __builtin_amdgcn_alignbyte(a.z, a.y, r);
    o.y = __builtin_amdgcn_alignbyte(a.w, a.z, r);
    o.z = __builtin_amdgcn_alignbyte(b.x, a.w, r);
    o.w = __builtin_amdgcn_alignbyte(b.y, b.x, r);
  } else if (q == 2) {
    o.x = __builtin_amdgcn_alignbyte(a.w, a.z, r);
    o.y = __builtin_amdgcn_alignbyte(b.x, a.w, r);
    o.z = __builtin_amdgcn_alignbyte(b.y, b.x, r);
    o.w = __builtin_amdgcn_alignbyte(b.z, b.y, r);
  } else {
    o.x = __builtin_amdgcn_alignbyte(b.x, a.w, r);
    o.y = __builtin_amdgcn_alignbyte(b.y, b.x, r);
    o.z = __builtin_amdgcn_alignbyte(b.z, b.y, r);
    o.w = __builtin_amdgcn_alignbyte(b.w, b.z, r);
  }
  return o;
}

// serialized-output stores are nontemporal: the op does not read its output again, and
// the result slots it is still copying stay in the Infinity Cache (see w_store_bitmap)
__device__ __forceinline__ void st_out(g_u32x4* p, const u32x4& v) { __builtin_nontemporal_store(v, p); }

struct CopyJob {
  const g_u8* s8;
  g_u8* d8;
  const g_u32x4* sv;  // aligned source vectors
  g_u32x4* dv;        // aligned destination body
  uint32_t n, head, nvec, shift;
};
// the unaligned head (bytes, by the first lanes) and the body's geometry
__device__ __forceinline__ CopyJob copy_begin(uint8_t* dst, const uint8_t* src, uint32_t n) {
  const int l = lane_id();
  CopyJob j;
  const uintptr_t d = reinterpret_cast<uintptr_t>(dst);
  j.head = (uint32_t)((16 - (d & 15)) & 15);
  if (j.head > n) j.head = n;
  j.n = n;
  j.s8 = (const g_u8*)src;
  j.d8 = (g_u8*)dst;
  if (((d | reinterpret_cast<uintptr_t>(src)) & 1) == 0) {  // even addresses (every slot): u16
    if (l < (int)(j.head >> 1)) ((g_u16*)j.d8)[l] = ((const g_u16*)j.s8)[l];
  } else if (l < (int)j.head) {
    j.d8[l] = j.s8[l];
  }
  const uintptr_t s = reinterpret_cast<uintptr_t>(src + j.head);
  j.shift = (uint32_t)(s & 15);
  j.sv = (const g_u32x4*)(s - j.shift);
  j.dv = (g_u32x4*)(dst + j.head);
  j.nvec = (n - j.head) >> 4;
  return j;
}
// pass i0 (512 body vectors): every source vector the pass needs, requested at once
// (nontemporal: each result byte is read once; serialize -10 % against default loads; one
// past the body too: the partner of the last one; lane 63 of the last group also needs
// aligned vector i0 + 512 -- the one past the body when this is the last pass: it still
// holds tail bytes or slack)
__device__ __forceinline__ void copy_load(const CopyJob& j, uint32_t i0, u32x4 a[8], u32x4& last) {
  const int l = lane_id();
#pragma unroll
  for (int k = 0; k < 8; k++) {
    const uint32_t i = i0 + 64 * k + l;
    if (i <= j.nvec && (j.shift != 0 || i < j.nvec)) a[k] = __builtin_nontemporal_load(j.sv + i);
    else a[k] = u32x4{0, 0, 0, 0};
  }
  last = u32x4{0, 0, 0, 0};
  if (j.shift != 0 && l == 63 && i0 + 511 < j.nvec) last = j.sv[i0 + 512];
}
__device__ __forceinline__ void copy_store(const CopyJob& j, uint32_t i0, const u32x4 a[8], const u32x4& last) {
  const int l = lane_id();
  if (j.shift == 0) {
#pragma unroll
    for (int k = 0; k < 8; k++) {
      const uint32_t i = i0 + 64 * k + l;
      if (i < j.nvec) st_out(j.dv + i, a[k]);
    }
    return;
  }
  const uint32_t q = j.shift >> 2, r = j.shift & 3;
#pragma unroll
  for (int k = 0; k < 8; k++) {
    const uint32_t i = i0 + 64 * k + l;
    u32x4 b = next_lane_vec(a[k]);
    if (k < 7) {
      const u32x4 nx = lane0_vec(a[k < 7 ? k + 1 : 7]);
      if (l == 63) b = nx;
    } else if (l == 63) {
      b = last;
    }
    const u32x4 o = funnel16(a[k], b, q, r);
    if (i < j.nvec) st_out(j.dv + i, o);
  }
}
__device__ __forceinline__ void copy_tail(const CopyJob& j) {
  const uint32_t done = j.head + (j.nvec << 4);  // fewer than 16 bytes remain
  if (((reinterpret_cast<uintptr_t>(j.d8) | reinterpret_cast<uintptr_t>(j.s8) | j.n) & 1) == 0) {
    const uint32_t i = (done >> 1) + (uint32_t)lane_id();
    if (i < (j.n >> 1)) ((g_u16*)j.d8)[i] = ((const g_u16*)j.s8)[i];
  } else {
    const uint32_t i = done + (uint32_t)lane_id();
    if (i < j.n) j.d8[i] = j.s8[i];
  }
}
__device__ __forceinline__ void w_copy(uint8_t* dst, const uint8_t* src, uint32_t n) {
  const CopyJob j = copy_begin(dst, src, n);
  for (uint32_t i0 = 0; i0 < j.nvec; i0 += 512) {
    u32x4 a[8], last;
    copy_load(j, i0, a, last);
    copy_store(j, i0, a, last);
  }
  copy_tail(j);
}
// ---------------------------------------------------------------------------
// workgroup-per-task result records (wide / BSI kernels)
// ---------------------------------------------------------------------------
// Workgroup-level output record: staged results go to the task's scratch slot.
__device__ __forceinline__ void wg_place(uint32_t t, bool keep, const uint8_t* src, bool staged,
                                         const uint32_t* stage, uint32_t len, uint32_t card, uint32_t key, int kind,
                                         const OutCtx& oc, Prefix* shp) {
  (void)shp;
  uint64_t srcaddr = reinterpret_cast<uint64_t>(src);
  if (keep && staged) {
    uint8_t* slot = oc.spec && kind == DK_B ? oc.out + oc.payload_base + 8192ull * t
                                            : oc.scratch + (size_t)t * kSlotBytes + (kind == DK_R ? 2 : 0);
    copy_lds_to_global<NT>(slot, stage, len, threadIdx.x);
    srcaddr = reinterpret_cast<uint64_t>(slot);
  }
  if (threadIdx.x == 0) {
    ORec r;
    r.off = 0;
    r.src = srcaddr;
    r.idx = 0;
    r.card = card;
    r.ser_len = len;
    r.key = (uint16_t)key;
    r.kind = (uint8_t)kind;
    r.keep = keep ? 1 : 0;
    oc.recs[t] = r;
  }
  lds_barrier();
}

// A run container of more than 2047 runs (only the buffer package's raw run AND / ANDNOT make
// them: the buffer BSI, BufferFastAggregation's and chains) into the big-run arena:
// [u16 nruns][(start, length - 1) pairs], written from the bits.
__device__ __forceinline__ void place_big_runs(uint32_t t, uint32_t key, const uint64_t r[4], int card, int nr, const OutCtx& oc,
                                               const BigRuns& big, uint32_t* lds, int* sh,
                                               unsigned long long* sh64) {
  const uint32_t len = 2u + 4u * (uint32_t)nr;
  if (threadIdx.x == 0) {
    unsigned long long off = atomicAdd(&big.used[0], (unsigned long long)((len + 15u) & ~15u));
    if (off + len > big.cap) {
      atomicOr(&big.used[1], 1ull);  // the host reruns the op with a larger arena
      off = ~0ull;
    }
    *sh64 = off;
  }
  __syncthreads();
  const unsigned long long off = *sh64;
  __syncthreads();
  if (off == ~0ull) {
    wg_place(t, false, nullptr, true, nullptr, 0, 0, key, DK_A, oc, nullptr);
    return;
  }
  uint16_t* dst = reinterpret_cast<uint16_t*>(big.base + off);
  uint64_t s[4], e[4];
  run_edges(r, lds, s, e);
  int ps0, ps1, ns, pe0, pe1, ne;
  block_scan_halves(popc64(s[0]) + popc64(s[1]), popc64(s[2]) + popc64(s[3]), ps0, ps1, ns, sh);
  block_scan_halves(popc64(e[0]) + popc64(e[1]), popc64(e[2]) + popc64(e[3]), pe0, pe1, ne, sh);
  const int th = threadIdx.x;
  const int bases[4] = {(2 * th) * 64, (2 * th + 1) * 64, (512 + 2 * th) * 64, (513 + 2 * th) * 64};
  const int sp[4] = {ps0, ps0 + popc64(s[0]), ps1, ps1 + popc64(s[2])};
  const int ep[4] = {pe0, pe0 + popc64(e[0]), pe1, pe1 + popc64(e[2])};
#pragma unroll
  for (int k = 0; k < 4; k++) {
    uint64_t x = s[k];
    for (int p = sp[k]; x; p++, x &= x - 1) dst[1 + 2 * p] = (uint16_t)(bases[k] + __builtin_ctzll(x));
    x = e[k];
    for (int p = ep[k]; x; p++, x &= x - 1) dst[2 + 2 * p] = (uint16_t)(bases[k] + __builtin_ctzll(x));
  }
  if (th == 0) dst[0] = (uint16_t)nr;
  __syncthreads();
  for (int p = th; p < nr; p += NT) dst[2 + 2 * p] = (uint16_t)(dst[2 + 2 * p] - dst[1 + 2 * p]);  // end -> length - 1
  __syncthreads();
  wg_place(t, true, big.base + off, false, nullptr, len, (uint32_t)card, key, DK_R, oc, nullptr);
}

// Records one task's output (wave per task: pairwise, workShyAnd).  Staged results (LDS) are copied to the task's
// scratch slot (arena slot layout); results already in the slot or pass-through
// containers are referenced in place.  k_place and the serializer follow.
__device__ __forceinline__ void w_place(uint32_t t, bool keep, const uint8_t* src, bool staged, const uint32_t* lds,
                                        uint32_t len, uint32_t card, uint32_t key, int kind, const OutCtx& oc) {
  const int l = lane_id();
  uint64_t srcaddr = reinterpret_cast<uint64_t>(src);
  if (keep && staged) {
    uint8_t* slot = oc.scratch + (size_t)t * kSlotBytes + (kind == DK_R ? 2 : 0);
    copy_lds_to_global<64>(slot, lds, len, l);
    srcaddr = reinterpret_cast<uint64_t>(slot);
  }
  if (l == 0) {
    ORec r;
    r.off = 0;
    r.src = srcaddr;
    r.idx = 0;
    r.card = card;
    r.ser_len = len;
    r.key = (uint16_t)key;
    r.kind = (uint8_t)kind;
    r.keep = keep ? 1 : 0;
    oc.recs[t] = r;
    if (oc.tile_agg && keep)  // the tile's totals for k_serialize_agg (a non-returning atomic)
      __hip_atomic_fetch_add(oc.tile_agg + t / kAggTile, agg_pack(len, card, (uint32_t)kind), __ATOMIC_RELAXED,
                             __HIP_MEMORY_SCOPE_AGENT);
  }
}

// A run result of more than 2047 runs (results that stay run containers whatever their size: the buffer
// package's run AND / ANDNOT run, add / remove of an input run container that large) into the big-run arena: [u16 nruns][(start, length - 1) pairs], straight from the
// registers (w_stage_runs_chunk without the LDS cap), then the ends turned into lengths.
__device__ __forceinline__ void w_place_big_runs(uint32_t t, uint32_t key, const WCtr& x, int card, int nr,
                                                 const OutCtx& oc, const BigRuns& big, uint32_t* lds) {
  const uint32_t len = 2u + 4u * (uint32_t)nr;
  unsigned long long off = 0;
  if (lane_id() == 0) {
    off = atomicAdd(&big.used[0], (unsigned long long)((len + 15u) & ~15u));
    if (off + len > big.cap) {
      atomicOr(&big.used[1], 1ull);  // the host reruns the op with a larger arena
      off = ~0ull;
    }
  }
  off = __shfl(off, 0);
  if (off == ~0ull) {
    w_place(t, false, nullptr, true, lds, 0, 0, key, DK_A, oc);
    return;
  }
  uint16_t* dst = reinterpret_cast<uint16_t*>(big.base + off);
  w_stage_runs_chunk<0, (1 << 30)>(x, dst, 0, 0);
  __threadfence_block();
  wsync();
  for (int p = lane_id(); p < nr; p += 64) dst[2 + 2 * p] = (uint16_t)(dst[2 + 2 * p] - dst[1 + 2 * p]);
  if (lane_id() == 0) dst[0] = (uint16_t)nr;
  w_place(t, true, big.base + off, false, lds, len, (uint32_t)card, key, DK_R, oc);
}

__device__ __forceinline__ void wg_passthrough(uint32_t t, const CDesc& d, const uint8_t* payload, const OutCtx& oc,
                                               Prefix* shp) {
  uint32_t len;
  if (d.kind == DK_A) len = 2 * d.card;
  else if (d.kind == DK_B) len = 8192;
  else len = 2 + 4 * (uint32_t)(*reinterpret_cast<const uint16_t*>(payload + d.slot + 2));
  wg_place(t, true, payload + d.slot + (d.kind == DK_R ? 2 : 0), false, nullptr, len, d.card, d.key, d.kind, oc, shp);
}

}  // namespace rbg
