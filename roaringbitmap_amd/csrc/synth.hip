// Synthetic workloads generated straight into device-resident batches
// (DESIGN.md §8): C2 operands, C3 uniform / clustered key slices.
#include <algorithm>

#include "kernels.hpp"
#include "wave.hpp"

namespace rbg {

// 64 Bernoulli(p = thr / 2^32) bits
__device__ __forceinline__ uint64_t bernoulli_word(uint64_t seed, uint32_t thr) {
  uint64_t w = 0;
#pragma unroll 8
  for (int i = 0; i < 64; i += 2) {
    const uint64_t h = splitmix64(seed + (uint64_t)i);
    w |= (uint64_t)((uint32_t)h < thr) << i;
    w |= (uint64_t)((uint32_t)(h >> 32) < thr) << (i + 1);
  }
  return w;
}

// ===========================================================================
// C3 uniform: one workgroup per key, n containers (one per bitmap) per key
// ===========================================================================
// C3 uniform arrays are packed back to back (2 B granularity, as in the portable
// format): no slot padding, so a key segment streams exactly its payload bytes
__device__ __forceinline__ uint32_t c3u_slot_bytes(uint32_t card) { return 2 * card; }

__global__ __launch_bounds__(256) void k_synth_c3u_sizes(uint64_t seed, uint32_t n, int key_lo,
                                                         unsigned long long* __restrict__ key_bytes) {
  __shared__ int sh[8];
  const uint32_t k = key_lo + blockIdx.x;
  int sum = 0;
  for (uint32_t i = threadIdx.x; i < n; i += NT) sum += (int)c3u_slot_bytes(c3u_card(seed, i, k));
  int u = 0;
  block_sum2(sum, u, sh);
  if (threadIdx.x == 0) key_bytes[blockIdx.x] = (unsigned long long)sum;
}

__global__ __launch_bounds__(256) void k_synth_c3u_fill(uint64_t seed, uint32_t n, int key_lo,
                                                        const unsigned long long* __restrict__ key_base,
                                                        CDesc* __restrict__ desc, uint16_t* __restrict__ keys,
                                                        uint32_t* __restrict__ bm, uint8_t* __restrict__ payload) {
  __shared__ int sh[8];
  const uint32_t k = key_lo + blockIdx.x;
  const uint64_t seg = (uint64_t)blockIdx.x * n;
  uint64_t running = key_base[blockIdx.x];
  for (uint32_t i0 = 0; i0 < n; i0 += NT) {
    const uint32_t i = i0 + threadIdx.x;
    const uint32_t card = i < n ? c3u_card(seed, i, k) : 0;
    const int sz = (int)c3u_slot_bytes(card);
    // workgroup exclusive scan of the slot sizes
    const int incl = wave_incl_scan(sz);
    if ((threadIdx.x & 63) == 63) sh[threadIdx.x >> 6] = incl;
    __syncthreads();
    int pre = incl - sz, tot = 0;
    for (int w = 0; w < 4; w++) {
      if (w < (int)(threadIdx.x >> 6)) pre += sh[w];
      tot += sh[w];
    }
    __syncthreads();
    if (i < n) {
      const uint64_t p = seg + i, off = running + (uint64_t)pre;
      desc[p] = CDesc{off, card, (uint16_t)k, DK_A, 0};
      keys[p] = (uint16_t)k;
      bm[p] = i;
      // stratified sorted distinct values: one per stride of 65536 / card
      uint16_t* v = reinterpret_cast<uint16_t*>(payload + off);
      const uint32_t step = 65536u / card;
      const uint64_t h = splitmix64(seed ^ 0x5EEDULL ^ ((uint64_t)i << 20) ^ ((uint64_t)k << 40));
      uint16_t x = 0;
      for (uint32_t j = 0; j < card; j++) v[j] = x = (uint16_t)(j * step + (uint32_t)(splitmix64(h + j) % step));
    }
    running += (uint64_t)tot;
  }
}

// ===========================================================================
// C3 clustered: one workgroup per container, all bitmap containers (8192 B slots)
// ===========================================================================
__global__ __launch_bounds__(256) void k_synth_c3c_fill(uint64_t seed, uint64_t n_ctr,
                                                        const uint16_t* __restrict__ keys,
                                                        const uint32_t* __restrict__ bm, CDesc* __restrict__ desc,
                                                        uint8_t* __restrict__ payload) {
  __shared__ int sh[8];
  const uint32_t thr = (uint32_t)(0.95 * 4294967296.0);
  for (uint64_t p = blockIdx.x; p < n_ctr; p += gridDim.x) {
    const uint32_t k = keys[p], i = bm[p];
    const uint64_t h = splitmix64(seed ^ ((uint64_t)i << 24) ^ ((uint64_t)k << 48) ^ 0xC3C0ULL);
    const uint32_t t = threadIdx.x;
    const uint32_t widx[4] = {2 * t, 2 * t + 1, 512 + 2 * t, 513 + 2 * t};
    uint64_t r[4];
#pragma unroll
    for (int q = 0; q < 4; q++) r[q] = bernoulli_word(splitmix64(h ^ ((uint64_t)widx[q] * 0x100000001B3ULL)), thr);
    store_bitmap_owned(payload + p * 8192, r);
    int c = popc64(r[0]) + popc64(r[1]) + popc64(r[2]) + popc64(r[3]);
    int u = 0;
    block_sum2(c, u, sh);
    if (t == 0) desc[p] = CDesc{p * 8192, (uint32_t)c, (uint16_t)k, DK_B, 0};
  }
}

// Array payloads of given descriptors (one thread per container): stratified
// sorted distinct values, slot padded with the last value.
__global__ __launch_bounds__(256) void k_synth_arrays(uint64_t seed, const CDesc* __restrict__ desc, uint64_t n,
                                                      uint8_t* __restrict__ payload) {
  for (uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n; p += (uint64_t)gridDim.x * blockDim.x) {
    const CDesc d = desc[p];
    uint16_t* v = reinterpret_cast<uint16_t*>(payload + d.slot);
    const uint32_t step = 65536u / d.card;
    const uint64_t h = splitmix64(seed ^ 0xA77AULL ^ (p << 8));
    uint16_t x = 0;
    for (uint32_t j = 0; j < d.card; j++) v[j] = x = (uint16_t)(j * step + (uint32_t)(splitmix64(h + j) % step));
    for (uint32_t j = d.card; j < ((2 * d.card + 15) & ~15u) / 2; j++) v[j] = x;
  }
}

void launch_synth_arrays(hipStream_t s, uint64_t seed, const CDesc* desc, uint64_t n, uint8_t* payload) {
  if (n == 0) return;
  const unsigned g = (unsigned)std::min<uint64_t>((n + 255) / 256, 16384);
  hipLaunchKernelGGL(k_synth_arrays, dim3(g), dim3(256), 0, s, seed, desc, n, payload);
}

// ===========================================================================
// C5 bit-sliced index over rows 0..rows-1: value(row) = hash & 0x7FFFFFFF, 31
// slices; container (key, input) with input 0 = ebM, 1 + i = slice i.  Typed as
// the reference's BSI after runOptimize (BSI/:141-150): ebM runs, slices by
// RB/BitmapContainer.java:1218-1237 / RB/ArrayContainer.java:1085-1099.
// pass 0: cardinality per (key, input) + value min / max; pass 1: payload + desc.
// ===========================================================================
__device__ __forceinline__ uint32_t c5_value(uint64_t seed, uint64_t row) {
  return (uint32_t)(splitmix64(seed ^ (row * 0x9E3779B97F4A7C15ULL)) & 0x7FFFFFFFu);
}

__device__ __forceinline__ void c5_words(uint64_t seed, uint64_t rows, uint32_t key, int input, uint64_t r[4],
                                         uint32_t* vmin, uint32_t* vmax) {
  const uint32_t t = threadIdx.x;
  const uint32_t widx[4] = {2 * t, 2 * t + 1, 512 + 2 * t, 513 + 2 * t};
  uint32_t mn = 0xFFFFFFFFu, mx = 0;
#pragma unroll
  for (int q = 0; q < 4; q++) {
    uint64_t w = 0;
    const uint64_t base = (uint64_t)key * 65536 + 64ull * widx[q];
    for (int b = 0; b < 64; b++) {
      const uint64_t row = base + b;
      if (row >= rows) break;
      if (input == 0) {
        w |= 1ull << b;
        if (vmin) {
          const uint32_t v = c5_value(seed, row);
          mn = min(mn, v);
          mx = max(mx, v);
        }
      } else {
        w |= (uint64_t)((c5_value(seed, row) >> (input - 1)) & 1u) << b;
      }
    }
    r[q] = w;
  }
  if (vmin) {
    *vmin = mn;
    *vmax = mx;
  }
}

__device__ __forceinline__ int c5_kind(int input, int card, int nruns) {
  (void)input;  // ebM and slices alike: built by add(), then runOptimize
  if (card <= 4096) return 2 * card > 2 + 4 * nruns ? DK_R : DK_A;  // ArrayContainer.runOptimize (strict >)
  return 2 + 4 * nruns < 8192 ? DK_R : DK_B;                         // BitmapContainer.runOptimize
}

__global__ __launch_bounds__(256) void k_synth_c5(uint64_t seed, uint64_t rows, int key_lo, int nbits, int pass,
                                                  uint32_t* __restrict__ cards, const uint32_t* __restrict__ pos,
                                                  unsigned int* __restrict__ minmax, CDesc* __restrict__ desc,
                                                  uint16_t* __restrict__ keys, uint32_t* __restrict__ bm,
                                                  uint8_t* __restrict__ payload) {
  __shared__ __align__(16) uint32_t acc[2048];
  __shared__ __align__(16) uint32_t tmp[2048];
  __shared__ int sh[8];
  const int nin = nbits + 1;
  const uint32_t key = key_lo + blockIdx.x / nin;
  const int input = (int)(blockIdx.x % nin);
  uint64_t r[4];
  uint32_t mn, mx;
  const bool mm = pass == 0 && input == 0;
  c5_words(seed, rows, key, input, r, mm ? &mn : nullptr, &mx);
  int c = popc64(r[0]) + popc64(r[1]) + popc64(r[2]) + popc64(r[3]);
  int u = 0;
  block_sum2(c, u, sh);
  if (pass == 0) {
    if (threadIdx.x == 0) cards[blockIdx.x] = (uint32_t)c;
    if (mm) {
      // workgroup min / max, one atomic each
      for (int o = 32; o > 0; o >>= 1) {
        mn = min(mn, (uint32_t)__shfl_xor((int)mn, o, 64));
        mx = max(mx, (uint32_t)__shfl_xor((int)mx, o, 64));
      }
      if ((threadIdx.x & 63) == 0) {
        atomicMin(&minmax[0], mn);
        atomicMax(&minmax[1], mx);
      }
    }
    return;
  }
  if (c == 0) return;  // empty containers are not stored
  const int kind = c5_kind(input, c, count_runs(r, acc, sh));
  const uint32_t p = pos[blockIdx.x];
  uint8_t* slot = payload + (uint64_t)p * kSlotBytes;
  const uint32_t len = stage_container(kind, r, c, acc, tmp, sh);
  copy_lds_to_global<NT>(slot + (kind == DK_R ? 2 : 0), tmp, len, threadIdx.x);
  if (threadIdx.x == 0) {
    desc[p] = CDesc{(uint64_t)p * kSlotBytes, (uint32_t)c, (uint16_t)key, (uint8_t)kind, 0};
    keys[p] = (uint16_t)key;
    bm[p] = (uint32_t)input;
  }
}

void launch_synth_c5(hipStream_t s, uint64_t seed, uint64_t rows, int key_lo, int nbits, int nkeys, int pass,
                     uint32_t* cards,
                     const uint32_t* pos, unsigned int* minmax, CDesc* desc, uint16_t* keys, uint32_t* bm,
                     uint8_t* payload) {
  const unsigned g = (unsigned)(nkeys * (nbits + 1));
  if (g == 0) return;
  hipLaunchKernelGGL(k_synth_c5, dim3(g), dim3(256), 0, s, seed, rows, key_lo, nbits, pass, cards, pos, minmax, desc,
                     keys, bm, payload);
}

// total cardinality of a batch (64-bit)
__global__ __launch_bounds__(256) void k_sum_cards(const CDesc* __restrict__ desc, uint64_t n,
                                                   unsigned long long* __restrict__ out) {
  unsigned long long s = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    s += desc[i].card;
  const int lo = wave_sum_i((int)(uint32_t)(s & 0xFFFFFF));
  const int hi = wave_sum_i((int)(uint32_t)(s >> 24));
  if ((threadIdx.x & 63) == 0) atomicAdd(out, (unsigned long long)(uint32_t)lo + ((unsigned long long)(uint32_t)hi << 24));
}

void launch_synth_c3u(hipStream_t s, uint64_t seed, uint32_t n, int key_lo, int nkeys, unsigned long long* key_bytes,
                      const unsigned long long* key_base, CDesc* desc, uint16_t* keys, uint32_t* bm,
                      uint8_t* payload, int pass) {
  if (nkeys <= 0) return;
  if (pass == 0)
    hipLaunchKernelGGL(k_synth_c3u_sizes, dim3(nkeys), dim3(256), 0, s, seed, n, key_lo, key_bytes);
  else
    hipLaunchKernelGGL(k_synth_c3u_fill, dim3(nkeys), dim3(256), 0, s, seed, n, key_lo, key_base, desc, keys, bm,
                       payload);
}
void launch_synth_c3c(hipStream_t s, uint64_t seed, uint64_t n_ctr, const uint16_t* keys, const uint32_t* bm,
                      CDesc* desc, uint8_t* payload) {
  if (n_ctr == 0) return;
  const unsigned g = (unsigned)std::min<uint64_t>(n_ctr, 16384);
  hipLaunchKernelGGL(k_synth_c3c_fill, dim3(g), dim3(256), 0, s, seed, n_ctr, keys, bm, desc, payload);
}
void launch_sum_cards(hipStream_t s, const CDesc* desc, uint64_t n, unsigned long long* out) {
  if (n == 0) return;
  const unsigned g = (unsigned)std::min<uint64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(k_sum_cards, dim3(g), dim3(256), 0, s, desc, n, out);
}

// ===========================================================================
// synthetic C2 operand: one workgroup per key, written straight into kSlotBytes slots
// ===========================================================================

__global__ __launch_bounds__(256) void k_synth_c2(uint64_t seed, int force, CDesc* __restrict__ desc,
                                                  uint16_t* __restrict__ keys, uint8_t* __restrict__ payload) {
  __shared__ __align__(16) uint32_t acc[2048];
  __shared__ __align__(16) uint32_t tmp[2048];
  __shared__ int q[257];
  __shared__ int sh[8];
  for (uint32_t k = blockIdx.x; k < 65536; k += gridDim.x) {
    const uint64_t hk = splitmix64(seed ^ ((uint64_t)k << 20));
    const int kind_pick = force >= 0 ? force : (int)(hk % 3);
    uint64_t r[4];
    const uint32_t t = threadIdx.x;
    const uint32_t widx[4] = {2 * t, 2 * t + 1, 512 + 2 * t, 513 + 2 * t};
    if (kind_pick != DK_R) {
      // A: target card U[1,4096]; B: U[4097,65535]; realised by Bernoulli bits
      const uint32_t target = kind_pick == DK_A ? 1 + (uint32_t)((hk >> 8) % 4096) : 4097 + (uint32_t)((hk >> 8) % 61439);
      const uint32_t thr = (uint32_t)(((uint64_t)target << 32) / 65536);
#pragma unroll
      for (int i = 0; i < 4; i++) r[i] = bernoulli_word(splitmix64(hk ^ ((uint64_t)widx[i] * 0x100000001B3ULL)), thr);
    } else {
      // R: nr in U[1,2047] runs, one per equal segment, each followed by a gap
      const int nr = 1 + (int)((hk >> 8) % 2047);
      const int seg = 65536 / nr;
      __syncthreads();
      lds_clear(acc);
      __syncthreads();
      for (int i = t; i < nr; i += NT) {
        const uint64_t h = splitmix64(hk + 0x51ULL * (uint64_t)(i + 1));
        const int half = max(seg / 2, 1);
        const int start = i * seg + (int)(h % (uint64_t)half);
        const int maxlen = (i + 1) * seg - 1 - start;  // keeps a gap before the next segment
        const int len = maxlen > 0 ? 1 + (int)((h >> 32) % (uint64_t)maxlen) : 1;
        lds_or_run_serial(acc, start, start + len - 1);
      }
      __syncthreads();
      lds_read_owned(acc, r);
    }
    int c = popc64(r[0]) + popc64(r[1]) + popc64(r[2]) + popc64(r[3]);
    int u = 0;
    block_sum2(c, u, sh);
    if (c == 0) {  // never emit an empty container
      if (t == 0) r[0] |= 1ULL << (k & 63);
      c = 1;
    }
    int kind;
    if (kind_pick == DK_R) kind = eff(c, count_runs(r, acc, sh));  // runOptimize of a run container
    else kind = by_card(c);
    uint8_t* slot = payload + (size_t)k * kSlotBytes;
    const uint32_t len = stage_container(kind, r, c, acc, tmp, sh);
    copy_lds_to_global<NT>(slot + (kind == DK_R ? 2 : 0), tmp, len, t);
    __syncthreads();
    if (t == 0) {
      CDesc d;
      d.slot = (uint64_t)k * kSlotBytes;
      d.card = (uint32_t)c;
      d.key = (uint16_t)k;
      d.kind = (uint8_t)kind;
      d.flags = 0;
      desc[k] = d;
      keys[k] = (uint16_t)k;
    }
  }
}

void launch_synth_c2(hipStream_t s, uint64_t seed, int force, CDesc* desc, uint16_t* keys, uint8_t* payload) {
  hipLaunchKernelGGL(k_synth_c2, dim3(4096), dim3(256), 0, s, seed, force, desc, keys, payload);
}

}  // namespace rbg
