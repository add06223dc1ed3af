// Wide (FastAggregation) kernels, batched andCardinality and synthetic
// generators.  RB/ = reference RoaringBitmap/src/main/java/org/roaringbitmap/.
//
// Wide ops read a key-major batch: the containers of key k from every input sit
// contiguously (ascending input index) in [key_off[k], key_off[k+1]), and so do
// their payload slots, so one workgroup streams one key's whole fan-in.
#include <algorithm>

#include "kernels.hpp"
#include "wave.hpp"

namespace rbg {

// Thread-serial OR/XOR of a small array container into LDS (16 B vector loads).
// vals is 2 B aligned (see lds_scatter_array).
template <int MODE>
__device__ __forceinline__ void thread_scatter_array(uint32_t* lds, const uint16_t* vals, int card) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(vals);
  const int lo = (int)((a & 15) >> 1);
  const uint4* v4 = reinterpret_cast<const uint4*>(a & ~(uintptr_t)15);
  for (int base = -lo; base < card; base += 8) {
    const uint4 v = v4[(base + lo) >> 3];
    const uint32_t w[4] = {v.x, v.y, v.z, v.w};
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

constexpr int kSmallArray = 64;  // arrays up to this size are scattered by one lane

// Accumulate (OR or XOR, no run containers for XOR) every container of a key
// segment: small arrays lane-serial, large arrays / runs cooperatively into LDS,
// bitmaps into registers.
constexpr int kBGroup = 2;  // bitmaps loaded together (4 costs the all-array path registers: C3 uniform -8 %)

template <int MODE>
__device__ __forceinline__ void accumulate_segment(const CDesc* desc, const uint8_t* payload, uint32_t s, uint32_t n,
                                                   uint32_t* acc, int* q, int* big, int* nbig, uint32_t* bslot,
                                                   bool slot32, uint64_t r[4]) {
  for (uint32_t base = 0; base < n; base += NT) {
    __syncthreads();
    if (threadIdx.x == 0) nbig[0] = nbig[1] = 0;
    __syncthreads();
    const uint32_t j = base + threadIdx.x;
    if (j < n) {
      const CDesc d = desc[s + j];
      if (d.kind == DK_A && d.card <= (uint32_t)kSmallArray) {
        thread_scatter_array<MODE>(acc, reinterpret_cast<const uint16_t*>(payload + d.slot), (int)d.card);
      } else if (d.kind == DK_B && slot32) {
        bslot[atomicAdd(&nbig[1], 1)] = (uint32_t)(d.slot >> 4);  // bitmaps: loaded in groups below
      } else {
        big[atomicAdd(&nbig[0], 1)] = (int)(s + j);
      }
    }
    __syncthreads();
    // bitmap containers: the loads of up to kBGroup are in flight together
    const int nb = nbig[1];
    for (int k = 0; k < nb; k += kBGroup) {
      uint64_t x[kBGroup][4];
#pragma unroll
      for (int u = 0; u < kBGroup; u++)
        if (k + u < nb) {  // nontemporal: each input byte is read once (C3 clustered 0.70 -> 0.78 of peak)
          const uint4* p = reinterpret_cast<const uint4*>(payload + ((uint64_t)bslot[k + u] << 4));
          u4_to_words(ld_in(p + threadIdx.x), x[u][0], x[u][1]);
          u4_to_words(ld_in(p + threadIdx.x + NT), x[u][2], x[u][3]);
        }
#pragma unroll
      for (int u = 0; u < kBGroup; u++)
        if (k + u < nb) {
#pragma unroll
          for (int i = 0; i < 4; i++) r[i] = MODE == 0 ? (r[i] | x[u][i]) : (r[i] ^ x[u][i]);
        }
    }
    const int no = nbig[0];
    for (int k = 0; k < no; k++) {
      const CDesc d = desc[big[k]];
      const uint8_t* slot = payload + d.slot;
      if (d.kind == DK_B) {  // (payloads of 64 GiB and more)
        uint64_t x[4];
        load_bitmap_owned(slot, x);
#pragma unroll
        for (int i = 0; i < 4; i++) r[i] = MODE == 0 ? (r[i] | x[i]) : (r[i] ^ x[i]);
      } else if (d.kind == DK_A) {
        lds_scatter_array<MODE>(acc, reinterpret_cast<const uint16_t*>(slot), (int)d.card);
      } else {
        const int nr = *reinterpret_cast<const uint16_t*>(slot + 2);
        lds_or_runs(acc, reinterpret_cast<const uint32_t*>(slot + 4), nr, q);
      }
    }
  }
  __syncthreads();
  uint64_t x[4];
  lds_read_owned(acc, x);
#pragma unroll
  for (int i = 0; i < 4; i++) r[i] = MODE == 0 ? (r[i] | x[i]) : (r[i] ^ x[i]);
}

// OR the u16 value stream [b0, b1) (2 B aligned byte addresses) into the LDS bitmap:
// the 16 B vectors covering it, four per thread in flight per round.  Only the first
// and the last vector hold values outside the stream (masked).
__device__ __forceinline__ void stream_or_values(uint32_t* acc, const uint8_t* b0, const uint8_t* b1) {
  constexpr int U = 4;
  const uintptr_t a0 = reinterpret_cast<uintptr_t>(b0);
  const uint4* v4 = reinterpret_cast<const uint4*>(a0 & ~(uintptr_t)15);
  const uint32_t lo = (uint32_t)((a0 & 15) >> 1);
  const uint32_t hi = lo + (uint32_t)((b1 - b0) >> 1);  // values [lo, hi) of the vectors are the stream
  const uint32_t nvec = (hi + 7) >> 3;
  const uint32_t first_m = (0xFFu << lo) & 0xFFu;
  const uint32_t last_m = (hi & 7) ? (1u << (hi & 7)) - 1u : 0xFFu;
  for (uint32_t j0 = 0; j0 < nvec; j0 += U * NT) {
    uint4 v[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint32_t k = j0 + u * NT + threadIdx.x;
      v[u] = k < nvec ? ld_in(v4 + k) : make_uint4(0, 0, 0, 0);  // nontemporal: read once
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      const uint32_t k = j0 + u * NT + threadIdx.x;
      if (k < nvec) scatter_vec_mask<0>(acc, v[u], (k == 0 ? first_m : 0xFFu) & (k == nvec - 1 ? last_m : 0xFFu));
    }
  }
}

__device__ __forceinline__ int block_card(const uint64_t r[4], int* sh) {
  int c = popc64(r[0]) + popc64(r[1]) + popc64(r[2]) + popc64(r[3]);
  int u = 0;
  block_sum2(c, u, sh);
  return (int)uni((uint32_t)c);
}

// FastAggregation result types (DESIGN.md §Type contract):
//   naive_or  (RB/FastAggregation.java:603-610): n == 1 -> clone + repairAfterLazy
//             (A, B unchanged; R -> toEfficientContainer); n >= 2 -> lazy bitmap
//             repaired: BY_CARD, 65536 -> R.full (RB/BitmapContainer.java:1205-1215)
//   workShyAnd (:356-414, k_shy_wave): 0 dropped, <= 4096 A, 65536 R.full, else B
//   naive_and (:328-346): iand chain from the smallest input (RB/RoaringBitmap.java:1272-1296)
//   naive_xor (:637-644): ixor chain with restart after an empty result
//             (RB/RoaringBitmap.java:3296-3348)
template <int MODE>
__global__ __launch_bounds__(256, 4) void k_wide(const Task* __restrict__ tasks, const uint32_t* __restrict__ n_tasks,
                                              WideArgs A, OutCtx oc, uint32_t* __restrict__ task_card) {
  __shared__ __align__(16) uint32_t acc[2048];
  __shared__ __align__(16) uint32_t tmp[2048];
  __shared__ int q[257];
  __shared__ int big[NT];
  __shared__ int nbig[2];
  __shared__ uint32_t bslot[NT];
  __shared__ int sh[8];
  __shared__ Prefix shp;
  __shared__ unsigned long long sh64;
  const uint32_t nt = *n_tasks;
  // static stride over a resident grid (no contended counter)
  uint32_t t = blockIdx.x - gridDim.x;
  while (true) {
    __syncthreads();  // LDS of the previous task is free
    t += gridDim.x;
    if (t >= nt) break;
    const Task tk = tasks[t];
    const uint32_t s = uni((uint32_t)tk.a), n = uni((uint32_t)tk.b);
    uint64_t r[4];
    int kind = DK_A, c = 0;

    if (MODE == WIDE_OR || MODE == WIDE_OR_CARD) {
      if (n == 1) {
        const CDesc d = A.desc[s];
        if (MODE == WIDE_OR_CARD) {
          if (threadIdx.x == 0) task_card[t] = d.card;
          continue;
        }
        if (d.kind != DK_R) {
          wg_passthrough(t, d, A.payload, oc, &shp);
          continue;
        }
        const int nr = *reinterpret_cast<const uint16_t*>(A.payload + d.slot + 2);
        if (eff((int)d.card, nr) == DK_R) {
          wg_passthrough(t, d, A.payload, oc, &shp);
          continue;
        }
        materialize(d, A.payload, tmp, q, r);  // toBitmapOrArrayContainer
        c = (int)d.card;
        kind = by_card(c);
      } else if (A.all_array) {
        // every slot of the segment is an array and the slots are contiguous (16 B
        // slots padded with their last value, or the packed arrays of a C3 synthetic
        // batch): the segment is one u16 value stream
        __syncthreads();
        lds_clear(acc);
#pragma unroll
        for (int i = 0; i < 4; i++) r[i] = 0;
        const CDesc d0 = A.desc[s], d1 = A.desc[s + n - 1];
        __syncthreads();
        stream_or_values(acc, A.payload + d0.slot, A.payload + d1.slot + 2 * (uint64_t)d1.card);
        __syncthreads();
        lds_read_owned(acc, r);
        c = block_card(r, sh);
        if (MODE == WIDE_OR_CARD) {
          if (threadIdx.x == 0) task_card[t] = (uint32_t)c;
          continue;
        }
        kind = c == 65536 ? DK_R : by_card(c);
      } else {
        __syncthreads();
        lds_clear(acc);
#pragma unroll
        for (int i = 0; i < 4; i++) r[i] = 0;
        accumulate_segment<0>(A.desc, A.payload, s, n, acc, q, big, nbig, bslot, A.slot32 != 0, r);
        c = block_card(r, sh);
        if (MODE == WIDE_OR_CARD) {
          if (threadIdx.x == 0) task_card[t] = (uint32_t)c;
          continue;
        }
        kind = c == 65536 ? DK_R : by_card(c);
      }
    } else if (MODE == WIDE_XOR) {
      if (n == 1) {  // one input holds the key: the chain's xor clones it, type and all (a 4096-value
                     // bitmap of the buffer package's range selection included)
        wg_passthrough(t, A.desc[s], A.payload, oc, &shp);
        continue;
      }
      // does a run container take part in this key's chain?
      int has_r = 0;
      for (uint32_t j = threadIdx.x; j < n; j += NT) has_r |= A.desc[s + j].kind == DK_R;
      has_r = __syncthreads_or(has_r);
      if (!has_r) {
        // Without run containers every chain step is BY_CARD, so the type is
        // BY_CARD of the final set and the empty-restart does not change the set.
        __syncthreads();
        lds_clear(acc);
#pragma unroll
        for (int i = 0; i < 4; i++) r[i] = 0;
        accumulate_segment<1>(A.desc, A.payload, s, n, acc, q, big, nbig, bslot, A.slot32 != 0, r);
        c = block_card(r, sh);
        if (c == 0) {
          wg_place(t, false, nullptr, true, tmp, 0, 0, tk.key, DK_A, oc, &shp);
          continue;
        }
        kind = by_card(c);
      } else {
        // exact replay of the in-place xor chain
        bool present = false;
        int clone = -1, st_kind = DK_A, st_card = 0;
        for (uint32_t j = 0; j < n; j++) {
          const CDesc d = A.desc[s + j];
          uint64_t x[4];
          materialize(d, A.payload, tmp, q, x);
          if (!present) {
#pragma unroll
            for (int i = 0; i < 4; i++) r[i] = x[i];
            present = true;
            clone = (int)(s + j);
            st_kind = d.kind;
            st_card = (int)d.card;
            continue;
          }
#pragma unroll
          for (int i = 0; i < 4; i++) r[i] ^= x[i];
          const int cc = block_card(r, sh);
          if (cc == 0) {
            present = false;
            continue;
          }
          const bool need_r = (st_kind == DK_R && d.kind == DK_R) ||
                              (st_kind == DK_R && d.kind == DK_A && d.card < 32) ||
                              (st_kind == DK_A && d.kind == DK_R && st_card < 32);
          st_kind = need_r ? eff(cc, count_runs(r, acc, sh)) : by_card(cc);
          st_card = cc;
          clone = -1;
        }
        if (!present) {
          wg_place(t, false, nullptr, true, tmp, 0, 0, tk.key, DK_A, oc, &shp);
          continue;
        }
        if (clone >= 0) {
          wg_passthrough(t, A.desc[clone], A.payload, oc, &shp);
          continue;
        }
        c = st_card;
        kind = st_kind;
      }
    } else if (MODE == WIDE_LAZY_CHAIN) {
      // Container.lazyIOR chain from a clone of the first container, then repairAfterLazy
      // (RB/Container.java:717-740; ParallelAggregation.or :197-206, RoaringBitmap.lazyor
      // :2357-2400 for BufferFastAggregation.or(Mutable...), horizontal_or :124-231, whose
      // lazyOR first step types alike).  The state is the container class of the running
      // result; its set is the running union r:
      //   A + A: ArrayContainer.lazyor, a lazy bitmap above 1024 values (:1449-1463)
      //   A + B, R + B, B + any: a bitmap (full bitmaps end as R.full either way)
      //   A + R, R + A: lazyorToRun / ilazyorToRun, a lazy bitmap above 4096 runs (:1765-1813)
      //   R + R: RunContainer.ior -> toEfficientContainer (:1508-1550)
      // Once a bitmap, always a bitmap: the rest of the segment is OR-ed in bulk.
      const CDesc d0 = A.desc[A.order ? A.order[s] : s];
      if (n == 1) {
        if ((A.chain & kChainN1Clone) || d0.kind != DK_R) {
          wg_passthrough(t, d0, A.payload, oc, &shp);
          continue;
        }
        const int nr = *reinterpret_cast<const uint16_t*>(A.payload + d0.slot + 2);
        if (eff((int)d0.card, nr) == DK_R) {
          wg_passthrough(t, d0, A.payload, oc, &shp);
          continue;
        }
        materialize(d0, A.payload, tmp, q, r);  // toBitmapOrArrayContainer
        c = (int)d0.card;
        kind = by_card(c);
      } else {
        int st = d0.kind, cur = (int)d0.card;
        bool bulk = (A.chain & kChainLimit16) && n >= 16;  // ParallelAggregation.or :208-214
        if (!bulk) {
          // Without run containers the chain's type is that of the final union: a bitmap
          // operand makes the state a (lazy) bitmap, repaired to BY_CARD; arrays alone stay
          // an array while the union plus the next array holds at most 1024 values
          // (ArrayContainer.lazyor), so an array end state has at most 1024 values and a
          // bitmap end state is repaired to BY_CARD -- an array again below 4097.  Either
          // way BY_CARD of the union (RunContainer.full at 65536), whatever the order.
          int has_r = 0;
          for (uint32_t j = threadIdx.x; j < n; j += NT) has_r |= A.desc[s + j].kind == DK_R;
          if (!__syncthreads_or(has_r)) bulk = true;
        }
        if (bulk) {  // a lazy bitmap of the whole segment
          st = DK_B;
#pragma unroll
          for (int i = 0; i < 4; i++) r[i] = 0;
          __syncthreads();
          lds_clear(acc);
          accumulate_segment<0>(A.desc, A.payload, s, n, acc, q, big, nbig, bslot, A.slot32 != 0, r);
        }
        if (!bulk) {
          materialize(d0, A.payload, tmp, q, r);
          bool in_lds = false;  // the running union lives in acc (array steps), not in r
          for (uint32_t j = 1; j < n; j++) {
            if (st == DK_B) {
              bulk = true;
              break;
            }
            const CDesc d = A.desc[A.order ? A.order[s + j] : s + j];
            if (st == DK_A && d.kind == DK_A) {
              // ArrayContainer.lazyor: the values OR-ed into the LDS set, the new ones
              // counted (cur = |union|), no materialisation or popcount pass
              if (!in_lds) {
                lds_barrier();
                lds_write_owned(acc, r);
                lds_barrier();
                in_lds = true;
              }
              int fresh = lds_apply_array_count<0>(acc, reinterpret_cast<const uint16_t*>(A.payload + d.slot),
                                                   (int)d.card);
              int unused = 0;
              block_sum2(fresh, unused, sh);  // its barriers order this step's atomics before the next
              if (cur + (int)d.card > 1024) st = DK_B;
              else cur += fresh;
              continue;
            }
            if (in_lds) {
              lds_read_owned(acc, r);
              lds_barrier();  // acc is scratch again (count_runs)
              in_lds = false;
            }
            uint64_t x[4];
            materialize(d, A.payload, tmp, q, x);
#pragma unroll
            for (int i = 0; i < 4; i++) r[i] |= x[i];
            if (st == DK_A && d.kind == DK_A) {
              if (cur + (int)d.card > 1024) st = DK_B;
              else cur = block_card(r, sh);
            } else if (d.kind == DK_B) {
              st = DK_B;
            } else if (st == DK_R && d.kind == DK_R) {
              const int cc = block_card(r, sh);
              st = eff(cc, count_runs(r, acc, sh));
              cur = cc;
            } else {  // A + R, R + A
              st = count_runs(r, acc, sh) > 4096 ? DK_B : DK_R;
            }
          }
          if (in_lds) {
            lds_read_owned(acc, r);
            lds_barrier();
          }
          if (bulk) {
            __syncthreads();
            lds_clear(acc);
            accumulate_segment<0>(A.desc, A.payload, s, n, acc, q, big, nbig, bslot, A.slot32 != 0, r);
          }
        }
        c = block_card(r, sh);
        if (st == DK_B) kind = c == 65536 ? DK_R : by_card(c);  // BitmapContainer.repairAfterLazy
        else if (st == DK_R) kind = eff(c, count_runs(r, acc, sh));  // RunContainer.repairAfterLazy
        else kind = DK_A;
      }
    } else if (MODE == WIDE_XOR_CHAIN) {
      // clone + ixor chain with no restart after an empty result (ParallelAggregation.xor
      // :189-195; horizontal_xor :243-289, whose first xor types like ixor).  An empty run
      // container XOR a run container is a clone of the latter (RB/RunContainer.java:2445-2452).
      int clone = (int)(A.order ? A.order[s] : s);
      const CDesc d0 = A.desc[clone];
      if (n == 1) {
        wg_passthrough(t, d0, A.payload, oc, &shp);
        continue;
      }
      // without run containers every step is BY_CARD (A / B ixor), so the type is BY_CARD of
      // the final set, which the chain's order does not change (as naive_xor's fast path)
      int has_r = 0;
      for (uint32_t j = threadIdx.x; j < n; j += NT) has_r |= A.desc[s + j].kind == DK_R;
      if (!__syncthreads_or(has_r)) {
        __syncthreads();
        lds_clear(acc);
#pragma unroll
        for (int i = 0; i < 4; i++) r[i] = 0;
        accumulate_segment<1>(A.desc, A.payload, s, n, acc, q, big, nbig, bslot, A.slot32 != 0, r);
        c = block_card(r, sh);
        if (c == 0 && !(A.chain & kChainKeepEmpty)) {
          wg_place(t, false, nullptr, true, tmp, 0, 0, tk.key, DK_A, oc, &shp);
          continue;
        }
        kind = by_card(c);
      } else {
      materialize(d0, A.payload, tmp, q, r);
      int st_kind = d0.kind, st_card = (int)d0.card;
      bool in_lds = false;  // the running set lives in acc (array steps), not in r
      for (uint32_t j = 1; j < n; j++) {
        const int idx = (int)(A.order ? A.order[s + j] : s + j);
        const CDesc d = A.desc[idx];
        if (d.kind == DK_A && st_kind != DK_R) {
          // A into A / B: BY_CARD, no run count.  The values are toggled in the LDS set
          // and the ones that were present counted: |r ^ a| = |r| + |a| - 2 |r & a|
          if (!in_lds) {
            lds_barrier();
            lds_write_owned(acc, r);
            lds_barrier();
            in_lds = true;
          }
          int off = lds_apply_array_count<1>(acc, reinterpret_cast<const uint16_t*>(A.payload + d.slot), (int)d.card);
          int unused = 0;
          block_sum2(off, unused, sh);  // its barriers order this step's atomics before the next
          st_card += (int)d.card - 2 * off;
          st_kind = by_card(st_card);
          clone = -1;
          continue;
        }
        if (in_lds) {
          lds_read_owned(acc, r);
          lds_barrier();  // acc is scratch again (count_runs)
          in_lds = false;
        }
        if (st_kind == DK_R && d.kind == DK_R && d.card == 0) continue;  // x empty: this.clone()
        uint64_t x[4];
        materialize(d, A.payload, tmp, q, x);
        if (st_kind == DK_R && st_card == 0 && d.kind == DK_R) {  // this empty: x.clone()
#pragma unroll
          for (int i = 0; i < 4; i++) r[i] = x[i];
          st_card = (int)d.card;
          clone = idx;
          continue;
        }
#pragma unroll
        for (int i = 0; i < 4; i++) r[i] ^= x[i];
        const int cc = block_card(r, sh);
        const bool need_r = (st_kind == DK_R && d.kind == DK_R) ||
                            (st_kind == DK_R && d.kind == DK_A && d.card < 32) ||
                            (st_kind == DK_A && d.kind == DK_R && st_card < 32);
        st_kind = need_r ? eff(cc, count_runs(r, acc, sh)) : by_card(cc);
        st_card = cc;
        clone = -1;
      }
      if (in_lds) {
        lds_read_owned(acc, r);
        lds_barrier();
      }
      if (st_card == 0 && !(A.chain & kChainKeepEmpty)) {
        wg_place(t, false, nullptr, true, tmp, 0, 0, tk.key, DK_A, oc, &shp);
        continue;
      }
      if (clone >= 0) {
        wg_passthrough(t, A.desc[clone], A.payload, oc, &shp);
        continue;
      }
      c = st_card;
      kind = st_kind;
      }
    } else {  // WIDE_AND_NAIVE
      // start container: the one from input start_bm (segments are sorted by input index)
      int start = -1;
      for (uint32_t j = threadIdx.x; j < n; j += NT)
        if (A.bm[s + j] == A.start_bm) start = (int)(s + j);
      // reduce: at most one lane found it
      int st = start;
      for (int o = 32; o > 0; o >>= 1) st = max(st, __shfl_xor(st, o, 64));
      if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = st;
      __syncthreads();
      start = max(max(sh[0], sh[1]), max(sh[2], sh[3]));
      __syncthreads();
      const CDesc d0 = A.desc[start];
      materialize(d0, A.payload, tmp, q, r);
      int st_kind = d0.kind, steps = 0;
      bool empty = false;
      for (uint32_t j = 0; j < n; j++) {
        const uint32_t b = A.bm[s + j];
        if (A.skip[b]) continue;
        const CDesc d = A.desc[s + j];
        uint64_t x[4];
        materialize(d, A.payload, tmp, q, x);
#pragma unroll
        for (int i = 0; i < 4; i++) r[i] &= x[i];
        const int cc = block_card(r, sh);
        steps++;
        if (cc == 0) {
          empty = true;
          break;
        }
        // R.iand(R) = R.and(R): toEfficientContainer on the heap (RB/RunContainer.java:381-456); the
        // buffer package keeps the merged run container (RB/buffer/MappeableRunContainer.java:474-536)
        const bool need_r = st_kind == DK_R && d.kind == DK_R;
        st_kind = !need_r ? by_card(cc) : A.buffer ? DK_R : eff(cc, count_runs(r, acc, sh));
        c = cc;
      }
      if (empty) {
        wg_place(t, false, nullptr, true, tmp, 0, 0, tk.key, DK_A, oc, &shp);
        continue;
      }
      if (steps == 0) {  // the clone of the smallest input is the answer
        wg_passthrough(t, d0, A.payload, oc, &shp);
        continue;
      }
      kind = st_kind;
      if (A.buffer && kind == DK_R) {
        const int nr = count_runs(r, acc, sh);
        if (nr > 2047) {  // more than a result slot holds
          place_big_runs(t, tk.key, r, c, nr, oc, A.big, acc, sh, &sh64);
          continue;
        }
      }
    }

    const uint32_t len = stage_container(kind, r, c, acc, tmp, sh);
    wg_place(t, true, nullptr, true, tmp, len, (uint32_t)c, tk.key, kind, oc, &shp);
  }
}

// ===========================================================================
// FastAggregation.workShyAnd / workShyAndCardinality (RB/FastAggregation.java:356-414, :416-462):
// one wave per common key.  The reference ANDs every container of the key into a lazy bitmap
// (BitmapContainer.iand with cardinality -1) and repairs it at the end, so the result is typed by
// its cardinality alone (BY_CARD, 65536 -> RunContainer.full) whatever the chain's order or
// intermediate forms.  Here the running intersection is a sorted array, one value per lane, while
// it holds at most 64 values (a uniform C3 key: ~15 values per input), and a register bitmap
// (16 words per lane) otherwise; it is tested for emptiness after every input, and an empty one
// ends the key's chain (an empty intersection stays empty).
// ===========================================================================
constexpr int kShyArr = 64;

// values [0, card) of an array container at any 2 B alignment (packed batches), from the 16 B
// vectors covering it: OR-scattered into the wave's LDS bitmap (MAP) or written to u16 st[idx]
template <bool MAP>
__device__ __forceinline__ void w_array_any(uint32_t* lds, const uint16_t* vals, int card) {
  const uintptr_t a = reinterpret_cast<uintptr_t>(vals);
  const int lo = (int)((a & 15) >> 1);
  const uint4* v4 = reinterpret_cast<const uint4*>(a & ~(uintptr_t)15);
  const int nvec = (card + lo + 7) >> 3;
  const int l = lane_id();
  uint16_t* st = reinterpret_cast<uint16_t*>(lds);
#pragma unroll 1
  for (int j0 = 0; 64 * j0 < nvec; j0 += kVecRound) {
    uint4 v[kVecRound];
#pragma unroll
    for (int j = 0; j < kVecRound; j++) {
      const int q = 64 * (j0 + j) + l;
      v[j] = q < nvec ? ld_in(v4 + q) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < kVecRound; j++) {
      const int base = 8 * (64 * (j0 + j) + l) - lo;  // value index of the vector's first element
      uint32_t vm = 0;
#pragma unroll
      for (int i = 0; i < 8; i++) vm |= (uint32_t)((unsigned)(base + i) < (unsigned)card) << i;
      if (MAP) {
        scatter_vec_mask<0>(lds, v[j], vm);
      } else {
        const uint32_t w[4] = {v[j].x, v[j].y, v[j].z, v[j].w};
#pragma unroll
        for (int i = 0; i < 8; i++)
          if ((vm >> i) & 1u) st[base + i] = (uint16_t)((w[i >> 1] >> ((i & 1) * 16)) & 0xFFFF);
      }
    }
  }
}

// x &= the wave's LDS bitmap
__device__ __forceinline__ void w_and_lds(const uint32_t* lds, WCtr& x) {
  const uint4* q = reinterpret_cast<const uint4*>(lds) + lane_id();
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint4 v = q[64 * i];
    x.w[2 * i] &= (uint64_t)v.x | ((uint64_t)v.y << 32);
    x.w[2 * i + 1] &= (uint64_t)v.z | ((uint64_t)v.w << 32);
  }
}

__device__ __forceinline__ bool w_any(const WCtr& x) {
  uint64_t o = 0;
#pragma unroll
  for (int k = 0; k < 16; k++) o |= x.w[k];
  return __any(o != 0);
}

// lane l < m holds value `val` of a sorted array: -> register bitmap
__device__ __forceinline__ void w_array_regs_to_bitmap(uint32_t* lds, uint32_t val, int m, WCtr& x) {
  wsync();
  w_clear_lds(lds);
  wsync();
  if (lane_id() < m) atomicOr(&lds[val >> 5], 1u << (val & 31));
  wsync();
  w_read_lds(lds, x);
}

// sorted u16 st[0, m): is v one of them (lower bound)
__device__ __forceinline__ uint32_t lds_contains(const uint16_t* st, int m, uint32_t v) {
  int lo = 0, hi = m;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if ((uint32_t)st[mid] < v) lo = mid + 1;
    else hi = mid;
  }
  return (lo < m && (uint32_t)st[lo] == v) ? 1u : 0u;
}

// keep the lanes of `m` (ballot of the kept lanes): their values, still sorted, to lanes 0..popc - 1
__device__ __forceinline__ uint32_t compact_lanes(uint16_t* st, uint64_t m, bool keep, uint32_t val, int cnt) {
  wsync();
  if (keep) st[__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0))] = (uint16_t)val;
  wsync();
  return lane_id() < cnt ? (uint32_t)st[lane_id()] : 0u;
}

// 16 B descriptor through the scalar cache (wave-uniform address)
__device__ __forceinline__ CDesc load_desc(const CDesc* desc, uint32_t i) {
  typedef const __attribute__((address_space(4))) uint64_t* CU64;
  const CU64 q = reinterpret_cast<CU64>(reinterpret_cast<uintptr_t>(desc + i));
  union {
    uint64_t u[2];
    CDesc d;
  } r;
  r.u[0] = q[0];
  r.u[1] = q[1];
  return r.d;
}

template <int MODE>  // WIDE_AND_SHY or WIDE_AND_SHY_CARD
__global__ __launch_bounds__(256, 4) void k_shy_wave(const Task* __restrict__ tasks, const uint32_t* __restrict__ n_tasks,
                                                  WideArgs A, OutCtx oc, uint32_t* __restrict__ task_card) {
  __shared__ __align__(16) uint32_t lds_all[4][2048];
  const int w = threadIdx.x >> 6, l = lane_id();
  uint32_t* lds = lds_all[w];
  uint16_t* st = reinterpret_cast<uint16_t*>(lds);
  const uint32_t nt = uni(*n_tasks);
  const uint32_t nw = gridDim.x * 4;
  unsigned long long rd_total = 0;  // bytes read (A.rd_bytes): payload + 4 B per container consumed
  for (uint32_t t = uni(blockIdx.x * 4 + (uint32_t)w); t < nt; t += nw) {
    const uint32_t s = uni((uint32_t)tasks[t].a), n = uni((uint32_t)tasks[t].b), key = uni(tasks[t].key);
    bool arr = false, empty = false;
    int cnt = 0;
    uint32_t val = 0;
    WCtr x;
    CDesc d = load_desc(A.desc, s);
    for (uint32_t j = 0; j < n; j++) {
      const CDesc dn = j + 1 < n ? load_desc(A.desc, s + j + 1) : d;  // in flight while d is used
      const uint8_t* slot = A.payload + d.slot;
      const uint16_t* v16 = reinterpret_cast<const uint16_t*>(slot);
      if (A.rd_bytes)
        rd_total += 4 + (d.kind == DK_A   ? 2ull * d.card
                         : d.kind == DK_B ? 8192ull
                                          : 2ull + 4ull * *reinterpret_cast<const uint16_t*>(slot + 2));
      if (j == 0) {
        if (d.kind == DK_A && d.card <= (uint32_t)kShyArr) {
          arr = true;
          cnt = (int)d.card;
          val = l < cnt ? (uint32_t)v16[l] : 0u;
        } else if (d.kind == DK_A) {
          wsync();
          w_clear_lds(lds);
          wsync();
          w_array_any<true>(lds, v16, (int)d.card);
          wsync();
          w_read_lds(lds, x);
        } else {
          w_materialize(d, A.payload, lds, x);
        }
      } else if (arr && d.kind != DK_R) {
        uint32_t keep = 0;
        if (d.kind == DK_B) {  // a bit test per value: one gathered word per lane
          if (l < cnt) keep = (uint32_t)(reinterpret_cast<const uint64_t*>(slot)[val >> 6] >> (val & 63)) & 1u;
        } else {  // the array staged in LDS, a binary search per value
          const int m = (int)d.card;
          wsync();
          if (m <= kShyArr) {
            if (l < m) st[l] = v16[l];
          } else {
            w_array_any<false>(lds, v16, m);
          }
          wsync();
          if (l < cnt) keep = lds_contains(st, m, val);
        }
        const uint64_t km = __ballot(keep);
        cnt = __popcll(km);
        if (cnt == 0) {
          empty = true;
          break;
        }
        val = compact_lanes(st, km, keep != 0, val, cnt);
      } else if (!arr && d.kind == DK_A && d.card <= (uint32_t)kShyArr) {
        // bitmap AND a small array: a subset of the array, back to the array form
        wsync();
        w_write_lds(lds, x);
        wsync();
        const uint32_t v = l < (int)d.card ? (uint32_t)v16[l] : 0u;
        const uint32_t keep = l < (int)d.card ? (lds[v >> 5] >> (v & 31)) & 1u : 0u;
        const uint64_t km = __ballot(keep);
        cnt = __popcll(km);
        arr = true;
        if (cnt == 0) {
          empty = true;
          break;
        }
        val = compact_lanes(st, km, keep != 0, v, cnt);
      } else {
        if (arr) {  // a run container: the running array as a bitmap first
          w_array_regs_to_bitmap(lds, val, cnt, x);
          arr = false;
        }
        if (d.kind == DK_A) {
          wsync();
          w_clear_lds(lds);
          wsync();
          w_array_any<true>(lds, v16, (int)d.card);
          wsync();
          w_and_lds(lds, x);
        } else {
          w_combine<0>(d, A.payload, lds, x);
        }
        if (!w_any(x)) {
          empty = true;
          break;
        }
      }
      d = dn;
    }
    const int c = empty ? 0 : arr ? cnt : w_card(x);
    if (MODE == WIDE_AND_SHY_CARD) {
      if (l == 0) task_card[t] = (uint32_t)c;
      continue;
    }
    if (c == 0) {  // dropped (:408)
      w_place(t, false, nullptr, true, lds, 0, 0, key, DK_A, oc);
      continue;
    }
    if (arr) {
      wsync();
      if (l < cnt) st[l] = (uint16_t)val;
      wsync();
      w_place(t, true, nullptr, true, lds, 2u * (uint32_t)c, (uint32_t)c, key, DK_A, oc);
      continue;
    }
    const int kind = c == 65536 ? DK_R : by_card(c);  // BitmapContainer.repairAfterLazy
    if (kind == DK_B) {
      uint8_t* slot = oc.scratch + (size_t)t * kSlotBytes;
      w_store_bitmap(slot, x);
      w_place(t, true, slot, false, lds, 8192, (uint32_t)c, key, DK_B, oc);
      continue;
    }
    const uint32_t len = w_stage(kind, x, c, lds);
    w_place(t, true, nullptr, true, lds, len, (uint32_t)c, key, kind, oc);
  }
  if (A.rd_bytes && l == 0 && rd_total) atomicAdd(A.rd_bytes, rd_total);
}

template <int MODE>
static void launch_k_wide(hipStream_t s, int grid, const Task* tasks, const uint32_t* nt, WideArgs args, OutCtx oc,
                          uint32_t* task_card) {
  const int g = std::max(1, std::min(grid, resident_grid((const void*)&k_wide<MODE>)));
  hipLaunchKernelGGL((k_wide<MODE>), dim3(g), dim3(256), 0, s, tasks, nt, args, oc, task_card);
}
template <int MODE>
static void launch_k_shy(hipStream_t s, int grid, const Task* tasks, const uint32_t* nt, WideArgs args, OutCtx oc,
                         uint32_t* task_card) {
  // a wave per key: 4 keys per workgroup
  const int g = std::max(1, std::min((grid + 3) / 4, resident_grid((const void*)&k_shy_wave<MODE>)));
  hipLaunchKernelGGL((k_shy_wave<MODE>), dim3(g), dim3(256), 0, s, tasks, nt, args, oc, task_card);
}

void launch_wide(hipStream_t s, int mode, int grid, const Task* tasks, const uint32_t* nt, WideArgs args, OutCtx oc,
                 uint32_t* task_card) {
  switch (mode) {
    case WIDE_OR: launch_k_wide<WIDE_OR>(s, grid, tasks, nt, args, oc, task_card); break;
    case WIDE_OR_CARD: launch_k_wide<WIDE_OR_CARD>(s, grid, tasks, nt, args, oc, task_card); break;
    case WIDE_XOR: launch_k_wide<WIDE_XOR>(s, grid, tasks, nt, args, oc, task_card); break;
    case WIDE_AND_SHY: launch_k_shy<WIDE_AND_SHY>(s, grid, tasks, nt, args, oc, task_card); break;
    case WIDE_AND_SHY_CARD: launch_k_shy<WIDE_AND_SHY_CARD>(s, grid, tasks, nt, args, oc, task_card); break;
    case WIDE_LAZY_CHAIN: launch_k_wide<WIDE_LAZY_CHAIN>(s, grid, tasks, nt, args, oc, task_card); break;
    case WIDE_XOR_CHAIN: launch_k_wide<WIDE_XOR_CHAIN>(s, grid, tasks, nt, args, oc, task_card); break;
    default: launch_k_wide<WIDE_AND_NAIVE>(s, grid, tasks, nt, args, oc, task_card); break;
  }
}

// ===========================================================================
// batched andCardinality (config C4): one wave per pair
// ===========================================================================
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ uint32_t lds_range_card(const uint32_t* lds, int s, int e) {  // [s, e] inclusive
  const int ws = s >> 5, we = e >> 5;
  uint32_t c = 0;
  for (int w = ws; w <= we; w++) {
    uint32_t m = ~0u;
    if (w == ws) m &= ~0u << (s & 31);
    if (w == we) m &= ~0u >> (31 - (e & 31));
    c += __popc(lds[w] & m);
  }
  return c;
}

// |x & y| for one matched key, computed by one wave (RB/Container.java:113-126).
__device__ __forceinline__ uint32_t wave_and_card(const CDesc& x, const CDesc& y, const uint8_t* payload,
                                                  uint32_t* lds, int lane) {
  const uint8_t* px = payload + x.slot;
  const uint8_t* py = payload + y.slot;
  uint32_t c = 0;
  if (x.kind == DK_B && y.kind == DK_B) {
    const uint4* a = reinterpret_cast<const uint4*>(px);
    const uint4* b = reinterpret_cast<const uint4*>(py);
    for (int i = lane; i < 512; i += 64) {
      const uint4 u = a[i], v = b[i];
      c += __popc(u.x & v.x) + __popc(u.y & v.y) + __popc(u.z & v.z) + __popc(u.w & v.w);
    }
  } else {
    // map = a bitmap operand if any, else the larger one; probe with the other
    const bool x_is_map = (x.kind == DK_B) || (y.kind != DK_B && x.card >= y.card);
    const CDesc& m = x_is_map ? x : y;
    const CDesc& p = x_is_map ? y : x;
    const uint8_t* pm = x_is_map ? px : py;
    const uint8_t* pp = x_is_map ? py : px;
    uint4* l4 = reinterpret_cast<uint4*>(lds);
    if (m.kind == DK_B) {
      const uint4* b = reinterpret_cast<const uint4*>(pm);
      for (int i = lane; i < 512; i += 64) l4[i] = b[i];
    } else {
      for (int i = lane; i < 512; i += 64) l4[i] = make_uint4(0, 0, 0, 0);
      wave_sync();
      if (m.kind == DK_A) {
        const uint16_t* v = reinterpret_cast<const uint16_t*>(pm);
        for (uint32_t i = lane; i < m.card; i += 64) atomicOr(&lds[v[i] >> 5], 1u << (v[i] & 31));
      } else {
        const int nr = *reinterpret_cast<const uint16_t*>(pm + 2);
        const uint32_t* pr = reinterpret_cast<const uint32_t*>(pm + 4);
        for (int i = lane; i < nr; i += 64) {
          const uint32_t pq = pr[i];
          lds_or_run_serial(lds, (int)(pq & 0xFFFF), (int)(pq & 0xFFFF) + (int)(pq >> 16));
        }
      }
    }
    wave_sync();
    if (p.kind == DK_A) {
      const uint16_t* v = reinterpret_cast<const uint16_t*>(pp);
      for (uint32_t i = lane; i < p.card; i += 64) c += (lds[v[i] >> 5] >> (v[i] & 31)) & 1;
    } else if (p.kind == DK_R) {
      const int nr = *reinterpret_cast<const uint16_t*>(pp + 2);
      const uint32_t* pr = reinterpret_cast<const uint32_t*>(pp + 4);
      for (int i = lane; i < nr; i += 64) {
        const uint32_t pq = pr[i];
        c += lds_range_card(lds, (int)(pq & 0xFFFF), (int)(pq & 0xFFFF) + (int)(pq >> 16));
      }
    } else {  // p is a bitmap and m is not (cannot happen: a bitmap is always the map)
      const uint4* b = reinterpret_cast<const uint4*>(pp);
      for (int i = lane; i < 512; i += 64) {
        const uint4 u = l4[i], v = b[i];
        c += __popc(u.x & v.x) + __popc(u.y & v.y) + __popc(u.z & v.z) + __popc(u.w & v.w);
      }
    }
    wave_sync();
  }
  return (uint32_t)wave_sum_i((int)c);  // DPP reduction (no LDS permutes)
}

// Batched andCardinality, planned: one thread per pair aligns the (few) keys of
// small pairs (RoaringBitmap.andCardinality, RB/RoaringBitmap.java:402-420) and
// emits one item per matched key; items then take one wave each.  Pairs with
// more than kSmallPairKeys keys keep the wave-per-pair merge.
constexpr uint32_t kSmallPairKeys = 64;

// count (emit = false) or write (emit = true) the matched keys of pair p
// off (EMIT): this pair's exclusive offsets, items | large pairs << 32
template <bool EMIT>
__device__ __forceinline__ uint64_t pair_matches(uint64_t p, const uint32_t* bm_off, const uint16_t* keys,
                                                 const CDesc* desc, uint64_t off, PairItem* items,
                                                 uint32_t* large) {
  const uint32_t a0 = bm_off[2 * p], a1 = bm_off[2 * p + 1], b1 = bm_off[2 * p + 2];
  if ((a1 - a0) + (b1 - a1) > kSmallPairKeys) {
    if (EMIT) large[off >> 32] = (uint32_t)p;
    return 1ull << 32;
  }
  uint64_t q = EMIT ? (off & 0xFFFFFFFFull) : 0;
  uint32_t ia = a0, ib = a1, m = 0;
  uint32_t ka = ia < a1 ? keys[ia] : 0, kb = ib < b1 ? keys[ib] : 0;
  while (ia < a1 && ib < b1) {
    if (ka == kb) {
      if (EMIT) {
        const CDesc da = desc[ia], db = desc[ib];
        items[q++] = PairItem{da.slot, db.slot, da.card, db.card, (uint32_t)p, da.kind, db.kind, 0, 0};
      }
      m++;
      ia++;
      ib++;
      if (ia < a1) ka = keys[ia];
      if (ib < b1) kb = keys[ib];
    } else if (ka < kb) {
      if (++ia < a1) ka = keys[ia];
    } else {
      if (++ib < b1) kb = keys[ib];
    }
  }
  return m;
}

// Plan of the items, per workgroup of 256 pairs: k_pairs_count writes each
// workgroup's total (items | large pairs << 32: at most 16,384 | 256), one small
// scan turns the totals into workgroup offsets, and k_pairs_emit aligns its pairs
// again, scans their counts inside the workgroup and writes the items in pair order.
// (A scan over the 1 M per-pair counts cost three launches over 8 MB.)
__device__ __forceinline__ uint64_t block_sum_packed(uint64_t v, uint64_t* sh4, uint64_t* excl) {
  // v = items | large << 32 with small parts: two DPP int scans
  const int li = (int)(uint32_t)v, ll = (int)(v >> 32);
  const int si = dpp_incl_scan(li), sl = dpp_incl_scan(ll);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 63) sh4[w] = (uint32_t)si | ((uint64_t)(uint32_t)sl << 32);
  __syncthreads();
  uint64_t pre = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < 4; i++) {
    pre += i < w ? sh4[i] : 0;
    tot += sh4[i];
  }
  *excl = pre + ((uint64_t)(uint32_t)(si - li) | ((uint64_t)(uint32_t)(sl - ll) << 32));
  return tot;
}

// pc[p]: the pair's matched keys (<= 32 for a small pair), 0xFF for a large pair
__device__ __forceinline__ uint64_t unpack_pc(uint8_t c) { return c == 0xFF ? 1ull << 32 : (uint64_t)c; }

__global__ __launch_bounds__(256) void k_pairs_count(uint64_t n_pairs, const uint32_t* __restrict__ bm_off,
                                                     const uint16_t* __restrict__ keys, uint64_t* __restrict__ blk,
                                                     uint8_t* __restrict__ pc) {
  __shared__ uint64_t sh4[4];
  const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const uint64_t v = p < n_pairs ? pair_matches<false>(p, bm_off, keys, nullptr, 0, nullptr, nullptr) : 0;
  if (p < n_pairs) pc[p] = (v >> 32) ? (uint8_t)0xFF : (uint8_t)v;
  uint64_t ex;
  const uint64_t tot = block_sum_packed(v, sh4, &ex);
  if (threadIdx.x == 0) blk[blockIdx.x] = tot;
}

// exclusive scan of the workgroup totals in place (one workgroup of 1024 threads,
// four per thread per round); *tot = items | large << 32
__global__ __launch_bounds__(1024) void k_pairs_scan(uint64_t* __restrict__ blk, uint64_t nblk,
                                                    uint64_t* __restrict__ tot) {
  __shared__ uint64_t sw[16];
  uint64_t carry = 0;
  for (uint64_t b0 = 0; b0 < nblk; b0 += 4 * 1024) {
    const uint64_t i0 = b0 + 4 * (uint64_t)threadIdx.x;
    uint64_t v[4], s = 0;
#pragma unroll
    for (int j = 0; j < 4; j++) {
      v[j] = i0 + j < nblk ? blk[i0 + j] : 0;
      s += v[j];
    }
    const int li = (int)(uint32_t)s, ll = (int)(s >> 32);
    const int si = dpp_incl_scan(li), sl = dpp_incl_scan(ll);
    const int w = threadIdx.x >> 6;
    __syncthreads();
    if ((threadIdx.x & 63) == 63) sw[w] = (uint32_t)si | ((uint64_t)(uint32_t)sl << 32);
    __syncthreads();
    uint64_t pre = 0, all = 0;
#pragma unroll
    for (int i = 0; i < 16; i++) {
      pre += i < w ? sw[i] : 0;
      all += sw[i];
    }
    uint64_t run = carry + pre + ((uint64_t)(uint32_t)(si - li) | ((uint64_t)(uint32_t)(sl - ll) << 32));
#pragma unroll
    for (int j = 0; j < 4; j++) {
      if (i0 + j < nblk) blk[i0 + j] = run;
      run += v[j];
    }
    carry += all;
  }
  if (threadIdx.x == 0) *tot = carry;
}

__global__ __launch_bounds__(256) void k_pairs_emit(uint64_t n_pairs, const uint32_t* __restrict__ bm_off,
                                                    const uint16_t* __restrict__ keys, const CDesc* __restrict__ desc,
                                                    const uint64_t* __restrict__ blk, const uint8_t* __restrict__ pc,
                                                    PairItem* __restrict__ items, uint32_t* __restrict__ large,
                                                    int32_t* __restrict__ out) {
  __shared__ uint64_t sh4[4];
  const uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  const bool ok = p < n_pairs;
  const uint64_t v = ok ? unpack_pc(pc[p]) : 0;  // only pairs with matches are aligned again
  uint64_t ex;
  block_sum_packed(v, sh4, &ex);
  if (!ok) return;
  out[p] = 0;
  if (v) pair_matches<true>(p, bm_off, keys, desc, blk[blockIdx.x] + ex, items, large);
}

__device__ __forceinline__ PairItem load_item(const PairItem* items, uint64_t i) {
  typedef const __attribute__((address_space(4))) uint64_t* CU64;
  const CU64 q = reinterpret_cast<CU64>(reinterpret_cast<uintptr_t>(items + i));
  union {
    uint64_t u[4];
    PairItem p;
  } r;
#pragma unroll
  for (int k = 0; k < 4; k++) r.u[k] = q[k];
  return r.p;
}

// |a & b| of two arrays of <= 512 values (RB/ArrayContainer.java:232-240
// andCardinality): one 16 B vector per lane of each, the larger scattered into the
// wave's LDS map, the smaller probed
__device__ __forceinline__ bool small_pair(const PairItem& it) {
  return it.kind_a == DK_A && it.kind_b == DK_A && it.card_a <= 512 && it.card_b <= 512;
}
__device__ __forceinline__ void small_pair_load(const PairItem& it, const uint8_t* payload, int lane, uint4& va,
                                                uint4& vb) {
  const uint32_t na = (it.card_a + 7) >> 3, nb = (it.card_b + 7) >> 3;
  va = (uint32_t)lane < na ? reinterpret_cast<const uint4*>(payload + it.slot_a)[lane] : make_uint4(0, 0, 0, 0);
  vb = (uint32_t)lane < nb ? reinterpret_cast<const uint4*>(payload + it.slot_b)[lane] : make_uint4(0, 0, 0, 0);
}
__device__ __forceinline__ uint32_t small_arrays_and_card(const uint4 va, uint32_t ca, const uint4 vb, uint32_t cb,
                                                         uint32_t* lds, int lane) {
  // the map is all zero on entry and is left all zero: the words the scatter touched
  // are cleared after the probe (at most 8 stores per lane instead of an 8 KiB clear)
  const bool a_map = ca >= cb;
  const uint4 mv = a_map ? va : vb;
  const int mcard = (int)(a_map ? ca : cb);
  scatter_vec_merged<0>(lds, mv, 8 * lane, mcard);
  wave_sync();
  const uint4 v = a_map ? vb : va;
  const int card = (int)(a_map ? cb : ca);
  const uint32_t w[4] = {v.x, v.y, v.z, v.w};
  uint32_t c = 0;
#pragma unroll
  for (int i = 0; i < 8; i++) {
    const uint32_t x = (w[i >> 1] >> ((i & 1) * 16)) & 0xFFFF;
    c += (8 * lane + i < card) ? ((lds[x >> 5] >> (x & 31)) & 1u) : 0u;
  }
  wave_sync();
  const uint32_t mw[4] = {mv.x, mv.y, mv.z, mv.w};
#pragma unroll
  for (int i = 0; i < 8; i++)
    if (8 * lane + i < mcard) lds[((mw[i >> 1] >> ((i & 1) * 16)) & 0xFFFF) >> 5] = 0;
  return (uint32_t)wave_sum_i((int)c);  // DPP reduction (no LDS permutes)
}
// the whole 8 KiB map cleared (k_pair_items: at the start, and after a key that took
// the general path, which leaves the map dirty)
__device__ __forceinline__ void clear_map(uint32_t* lds, int lane) {
  uint4* l4 = reinterpret_cast<uint4*>(lds);
#pragma unroll
  for (int i = 0; i < 8; i++) l4[64 * i + lane] = make_uint4(0, 0, 0, 0);
  wave_sync();
}

// one wave per matched key (resident grid), software-pipelined: while an item is
// counted, the next item's payload vectors (small arrays) are already in flight and
// the record after that is loaded through the scalar cache; sums wrap like Java ints.
// Then the pairs of more than kSmallPairKeys keys, one wave each merging the two key
// arrays itself (in the same launch: a separate one cost ~5 us even with none).
__global__ __launch_bounds__(256) void k_pair_items(const PairItem* __restrict__ items, const uint64_t* __restrict__ tot,
                                                    const uint8_t* __restrict__ payload, int32_t* __restrict__ out,
                                                    const uint32_t* __restrict__ large,
                                                    const uint32_t* __restrict__ bm_off,
                                                    const CDesc* __restrict__ desc) {
  __shared__ __align__(16) uint32_t lds[4][2048];
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint64_t n = *tot & 0xFFFFFFFFull, n_large = *tot >> 32;
  const uint64_t stride = (uint64_t)gridDim.x * 4;
  const uint64_t wid = (uint64_t)blockIdx.x * 4 + w;
  uint64_t i = wid;
  if (i < n) {
    PairItem cur = load_item(items, i), nxt;
    if (i + stride < n) nxt = load_item(items, i + stride);
    uint4 va, vb;
    bool pre = small_pair(cur);
    if (pre) small_pair_load(cur, payload, lane, va, vb);
    clear_map(lds[w], lane);
    for (;;) {
      const uint64_t in = i + stride, in2 = in + stride;
      PairItem nxt2;
      if (in2 < n) nxt2 = load_item(items, in2);
      uint4 na, nb;
      const bool npre = in < n && small_pair(nxt);
      if (npre) small_pair_load(nxt, payload, lane, na, nb);  // in flight while this item is counted
      uint32_t c;
      if (pre) {
        c = small_arrays_and_card(va, cur.card_a, vb, cur.card_b, lds[w], lane);
      } else {
        const CDesc da{cur.slot_a, cur.card_a, 0, cur.kind_a, 0}, db{cur.slot_b, cur.card_b, 0, cur.kind_b, 0};
        c = wave_and_card(da, db, payload, lds[w], lane);
        clear_map(lds[w], lane);
      }
      if (lane == 0 && c) atomicAdd(reinterpret_cast<uint32_t*>(out) + cur.pair, c);
      if (in >= n) break;
      i = in;
      cur = nxt;
      nxt = nxt2;
      pre = npre;
      va = na;
      vb = nb;
    }
  }
  for (uint64_t j = wid; j < n_large; j += stride) {
    const uint32_t p = large[j];
    uint32_t ia = bm_off[2 * p], a1 = bm_off[2 * p + 1];
    uint32_t ib = a1, b1 = bm_off[2 * p + 2];
    uint32_t sum = 0;
    while (ia < a1 && ib < b1) {
      const CDesc da = desc[ia], db = desc[ib];
      if (da.key == db.key) {
        sum += wave_and_card(da, db, payload, lds[w], lane);
        ia++;
        ib++;
      } else if (da.key < db.key) {
        ia++;
      } else {
        ib++;
      }
    }
    if (lane == 0) out[p] = (int32_t)sum;
  }
}

void launch_batch_and_card(hipStream_t s, uint64_t n_pairs, const uint32_t* bm_off, const uint16_t* keys,
                           const CDesc* desc, const uint8_t* payload, int32_t* out, uint64_t* cnt, uint64_t* part,
                           uint64_t* tot, PairItem* items, uint32_t* large) {
  if (n_pairs == 0) return;
  const unsigned g = (unsigned)((n_pairs + 255) / 256);
  // cnt holds the workgroup totals (g u64), then one count byte per pair
  uint8_t* pc = reinterpret_cast<uint8_t*>(cnt + g);
  (void)part;
  hipLaunchKernelGGL(k_pairs_count, dim3(g), dim3(256), 0, s, n_pairs, bm_off, keys, cnt, pc);
  hipLaunchKernelGGL(k_pairs_scan, dim3(1), dim3(1024), 0, s, cnt, (uint64_t)g, tot);
  hipLaunchKernelGGL(k_pairs_emit, dim3(g), dim3(256), 0, s, n_pairs, bm_off, keys, desc, (const uint64_t*)cnt,
                     (const uint8_t*)pc, items, large, out);
  hipLaunchKernelGGL(k_pair_items, dim3(resident_grid((const void*)&k_pair_items)), dim3(256), 0, s,
                     (const PairItem*)items, (const uint64_t*)tot, payload, out, (const uint32_t*)large, bm_off, desc);
}

// upper bound of the items of a batch: sum over small pairs of min(keys of a, keys of b)
uint64_t batch_pair_items_cap(const uint32_t* h_bm_nctr, uint64_t n_pairs) {
  uint64_t cap = 0;
  for (uint64_t p = 0; p < n_pairs; p++) {
    const uint32_t na = h_bm_nctr[2 * p], nb = h_bm_nctr[2 * p + 1];
    if (na + nb <= kSmallPairKeys) cap += std::min(na, nb);
  }
  return cap;
}

}  // namespace rbg
