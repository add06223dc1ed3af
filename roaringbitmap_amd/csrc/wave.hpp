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

// Orders this wave's LDS accesses (LDS ops of one wave complete in issue order;
// this keeps the compiler from reordering across the point).
__device__ __forceinline__ void wsync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ int wave_sum_i(int v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
// exclusive prefix over lanes; returns the wave total in *tot
__device__ __forceinline__ int wave_excl(int v, int* tot) {
  const int l = lane_id();
  int s = v;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int u = __shfl_up(s, o, 64);
    if (l >= o) s += u;
  }
  *tot = __shfl(s, 63, 64);
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
    const uint4 v = q[64 * i];
    x.w[2 * i] = (uint64_t)v.x | ((uint64_t)v.y << 32);
    x.w[2 * i + 1] = (uint64_t)v.z | ((uint64_t)v.w << 32);
  }
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
// the first LDS atomic so the loads overlap (one memory latency per container),
// and bits of consecutive sorted values that share a 32-bit word are merged
// into one atomic.
constexpr int kVecRound = 4;  // 16 B vectors per lane loaded per round

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
      v[j] = k < nvec ? v4[k] : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
  for (int j = 0; j < kVecRound; j++) {
    const int base = 8 * (64 * (j0 + j) + l);
    if (base >= card) break;
    const uint32_t w[4] = {v[j].x, v[j].y, v[j].z, v[j].w};
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
  }
}

// Run containers are materialised without per-word fills: every run toggles its
// first bit and the bit after its last one in a cleared LDS bitmap (2 LDS
// atomics per run, no divergence on run length), and an inclusive prefix-XOR
// over the 65536 bits then turns the toggles into the filled runs.  Valid run
// containers have disjoint runs, so toggles of adjacent runs cancel correctly.
__device__ __forceinline__ void w_toggle_runs(uint32_t* lds, const uint8_t* slot, int nruns) {
  // slot = [u16 pad][u16 nruns][u32 (start, len-1) pairs]: u32 k of the slot is
  // run k-1, so the slot streams as aligned 16 B vectors (input run containers
  // may hold up to 32768 runs; results hold at most 2047)
  const int nvec = (nruns + 4) >> 2;
  const uint4* v4 = reinterpret_cast<const uint4*>(slot);
  const int l = lane_id();
#pragma unroll 1
  for (int j0 = 0; 64 * j0 < nvec; j0 += kVecRound) {
    uint4 v[kVecRound];
#pragma unroll
    for (int j = 0; j < kVecRound; j++) {
      const int k = 64 * (j0 + j) + l;
      v[j] = k < nvec ? v4[k] : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
  for (int j = 0; j < kVecRound; j++) {
    const int r0 = 4 * (64 * (j0 + j) + l) - 1;
    if (r0 >= nruns) break;
    const uint32_t u[4] = {v[j].x, v[j].y, v[j].z, v[j].w};
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
  const uint4* src;
  if (d.kind == DK_B) {
    src = reinterpret_cast<const uint4*>(slot) + lane_id();
  } else {
    wsync();
    w_clear_lds(lds);
    wsync();
    w_scatter_array<0>(lds, reinterpret_cast<const uint16_t*>(slot), (int)d.card);
    wsync();
    src = reinterpret_cast<const uint4*>(lds) + lane_id();
  }
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint4 v = src[64 * i];
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
  const int up = (l + 63) & 63, dn = (l + 1) & 63;
  const uint64_t w0 = x.w[2 * I], w1 = x.w[2 * I + 1];
  const uint64_t top1 = __shfl(w1 >> 63, up, 64);  // lane l-1's word 1 top bit
  const uint64_t pchunk = I > 0 ? __shfl(x.w[2 * (I > 0 ? I - 1 : 0) + 1] >> 63, 63, 64) : 0;
  const uint64_t prev0 = (l == 0) ? pchunk : top1;
  const uint64_t bot0 = __shfl(w0 & 1, dn, 64);  // lane l+1's word 0 bit 0
  const uint64_t nchunk = I < 7 ? __shfl(x.w[2 * (I < 7 ? I + 1 : 7)] & 1, 0, 64) : 0;
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

template <int I>
__device__ __forceinline__ int w_stage_starts(const WCtr& x, uint16_t* st, int base) {
  const int l = lane_id();
  uint64_t s0, s1, e0, e1;
  w_chunk_edges<I>(x, s0, s1, e0, e1);
  int tot;
  int p = base + wave_excl(__popcll(s0) + __popcll(s1), &tot);
  const int wb = (128 * I + 2 * l) * 64;
  uint64_t v = s0;
  while (v) {
    if (p < 2047) st[1 + 2 * p] = (uint16_t)(wb + __builtin_ctzll(v));
    p++;
    v &= v - 1;
  }
  v = s1;
  while (v) {
    if (p < 2047) st[1 + 2 * p] = (uint16_t)(wb + 64 + __builtin_ctzll(v));
    p++;
    v &= v - 1;
  }
  if (I < 7) return w_stage_starts<(I < 7 ? I + 1 : 7)>(x, st, base + tot);
  return base + tot;
}

template <int I>
__device__ __forceinline__ void w_stage_ends(const WCtr& x, uint16_t* st, int base) {
  const int l = lane_id();
  uint64_t s0, s1, e0, e1;
  w_chunk_edges<I>(x, s0, s1, e0, e1);
  int tot;
  int p = base + wave_excl(__popcll(e0) + __popcll(e1), &tot);
  const int wb = (128 * I + 2 * l) * 64;
  uint64_t v = e0;
  while (v) {
    if (p < 2047) st[2 + 2 * p] = (uint16_t)(wb + __builtin_ctzll(v) - st[1 + 2 * p]);
    p++;
    v &= v - 1;
  }
  v = e1;
  while (v) {
    if (p < 2047) st[2 + 2 * p] = (uint16_t)(wb + 64 + __builtin_ctzll(v) - st[1 + 2 * p]);
    p++;
    v &= v - 1;
  }
  if (I < 7) w_stage_ends<(I < 7 ? I + 1 : 7)>(x, st, base + tot);
}

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
      const int c0 = __popcll(x.w[2 * i]);
      const int c = c0 + __popcll(x.w[2 * i + 1]);
      int tot;
      int p = base + wave_excl(c, &tot);
      const int wb = (128 * i + 2 * l) * 64;
      uint64_t v = x.w[2 * i];
      while (v) {
        st[p++] = (uint16_t)(wb + __builtin_ctzll(v));
        v &= v - 1;
      }
      v = x.w[2 * i + 1];
      while (v) {
        st[p++] = (uint16_t)(wb + 64 + __builtin_ctzll(v));
        v &= v - 1;
      }
      base += tot;
    }
    wsync();
    return 2u * (uint32_t)card;
  }
  // run container: starts first (writes st[1 + 2k]), then ends (st[2 + 2k] = end - start)
  wsync();
  int sb = w_stage_starts<0>(x, st, 0);
  wsync();
  w_stage_ends<0>(x, st, 0);
  if (l == 0) st[0] = (uint16_t)sb;
  wsync();
  return 2u + 4u * (uint32_t)sb;
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

__device__ __forceinline__ uint32_t uni(uint32_t x) { return __builtin_amdgcn_readfirstlane(x); }
__device__ __forceinline__ uint64_t uni64(uint64_t x) {
  return ((uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)(x >> 32)) << 32) |
         (uint64_t)__builtin_amdgcn_readfirstlane((uint32_t)x);
}

// Called by ALL lanes of ONE wave with identical (wave-uniform) arguments; the
// spin loop is wave-uniform and single-exit.  Publishes this task's aggregate,
// walks back to an inclusive predecessor, publishes the inclusive value and
// returns the exclusive prefix.  The spin is bounded; on timeout *err is set
// (the result is then invalid, nothing hangs).
__device__ __forceinline__ Prefix lookback(uint64_t* status, uint32_t t, uint32_t cnt, uint64_t bytes, uint32_t run,
                                           uint32_t* err) {
  const bool leader = (threadIdx.x & 63) == 0;
  t = uni(t);
  uint64_t acc_cnt = 0, acc_bytes = 0, acc_run = 0;
  if (leader)
    __hip_atomic_store(status + t, lb_pack(t == 0 ? 2 : 1, run, cnt, bytes), __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  if (t != 0) {
    uint32_t j = t - 1;
    uint32_t spins = 0;
    bool done = false, timed_out = false;
    while (!done) {
      const uint64_t s = uni64(__hip_atomic_load(status + j, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
      const uint32_t st = (uint32_t)(s >> 62);
      if (st == 0) {
        spins++;
        if (spins > (1u << 22)) {
          timed_out = true;
          done = true;
        } else {
          __builtin_amdgcn_s_sleep(1);
        }
      } else {
        acc_run |= (s >> 61) & 1;
        acc_cnt += (s >> 44) & 0x1FFFF;
        acc_bytes += s & ((1ULL << 44) - 1);
        if (st == 2 || j == 0) done = true;
        else j--;
      }
    }
    if (leader) {
      if (timed_out) atomicOr(err, 1u);
      __hip_atomic_store(status + t, lb_pack(2, run | acc_run, cnt + acc_cnt, bytes + acc_bytes), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  return Prefix{(uint32_t)acc_cnt, acc_bytes};
}

}  // namespace rbg
