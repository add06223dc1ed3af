// RoaringBitmap.runOptimize over every container of a device-resident batch
// (RB/RoaringBitmap.java:2764-2774), and the device-wide exclusive scan it (and
// the header decode) places slots with.
//
//   k_runopt_plan  : one wave per container decides the container's new type
//                    and slot size, without materialising it:
//                      A -> R iff 2 card > 2 + 4 nruns  (RB/ArrayContainer.java:1085-1099),
//                           nruns counted on the sorted values themselves;
//                      B -> R iff 2 + 4 nruns < 8192    (RB/BitmapContainer.java:1218-1237);
//                      R -> toEfficientContainer        (RB/RunContainer.java:2083-2085, 2326-2335)
//                           on the stored run count, as the reference does.
//   scan           : exclusive scan of the new slot sizes -> slot offsets
//   k_runopt_write : one wave per container: an unchanged container's slot is
//                    copied verbatim (R kept as R is the reference's `return this`);
//                    a converted one is materialised in registers and staged
//                    through the wave's LDS into its new slot.
#include <algorithm>

#include "kernels.hpp"
#include "wave.hpp"

namespace rbg {

// ---------------------------------------------------------------------------
// exclusive scan of u64 (tiles of 256 threads x 16 elements)
// ---------------------------------------------------------------------------
constexpr int kScanPer = 16;
constexpr int kScanTile = NT * kScanPer;

__device__ __forceinline__ uint64_t wave_incl_u64(uint64_t v) {
  const int l = lane_id();
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const uint64_t u = __shfl_up(v, o, 64);
    if (l >= o) v += u;
  }
  return v;
}

// exclusive block scan of one value per thread; *total = block sum
__device__ __forceinline__ uint64_t block_excl_u64(uint64_t v, uint64_t* sh4, uint64_t* total) {
  const uint64_t inc = wave_incl_u64(v);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if (lane_id() == 63) sh4[w] = inc;
  __syncthreads();
  uint64_t pre = 0, tot = 0;
#pragma unroll
  for (int i = 0; i < NT / 64; i++) {
    pre += i < w ? sh4[i] : 0;
    tot += sh4[i];
  }
  *total = tot;
  return pre + inc - v;
}

__global__ __launch_bounds__(256) void k_scan_reduce(const uint64_t* __restrict__ in, uint64_t n,
                                                     uint64_t* __restrict__ part) {
  __shared__ uint64_t sh4[4];
  const uint64_t base = (uint64_t)blockIdx.x * kScanTile + (uint64_t)threadIdx.x * kScanPer;
  uint64_t s = 0;
#pragma unroll
  for (int j = 0; j < kScanPer; j++) s += base + j < n ? in[base + j] : 0;
  uint64_t tot;
  block_excl_u64(s, sh4, &tot);
  if (threadIdx.x == 0) part[blockIdx.x] = tot;
}

__global__ __launch_bounds__(256) void k_scan_partials(uint64_t* __restrict__ part, uint64_t np,
                                                       uint64_t* __restrict__ total) {
  __shared__ uint64_t sh4[4];
  uint64_t carry = 0;
  for (uint64_t b0 = 0; b0 < np; b0 += NT) {
    const uint64_t i = b0 + threadIdx.x;
    const uint64_t v = i < np ? part[i] : 0;
    uint64_t tot;
    const uint64_t ex = block_excl_u64(v, sh4, &tot);
    if (i < np) part[i] = carry + ex;
    carry += tot;
  }
  if (threadIdx.x == 0) *total = carry;
}

__global__ __launch_bounds__(256) void k_scan_apply(const uint64_t* in, uint64_t n, const uint64_t* __restrict__ part,
                                                    uint64_t* out) {
  __shared__ uint64_t sh4[4];
  const uint64_t base = (uint64_t)blockIdx.x * kScanTile + (uint64_t)threadIdx.x * kScanPer;
  uint64_t v[kScanPer];
  uint64_t s = 0;
#pragma unroll
  for (int j = 0; j < kScanPer; j++) {
    v[j] = base + j < n ? in[base + j] : 0;
    s += v[j];
  }
  uint64_t tot;
  uint64_t run = part[blockIdx.x] + block_excl_u64(s, sh4, &tot);
#pragma unroll
  for (int j = 0; j < kScanPer; j++) {
    if (base + j < n) out[base + j] = run;
    run += v[j];
  }
}

uint64_t scan_parts(uint64_t n) { return (n + kScanTile - 1) / kScanTile; }

void launch_exclusive_scan(hipStream_t s, const uint64_t* in, uint64_t* out, uint64_t n, uint64_t* part,
                           uint64_t* total) {
  const uint64_t np = scan_parts(n);
  if (np) hipLaunchKernelGGL(k_scan_reduce, dim3((unsigned)np), dim3(NT), 0, s, in, n, part);
  hipLaunchKernelGGL(k_scan_partials, dim3(1), dim3(NT), 0, s, part, np, total);
  if (np) hipLaunchKernelGGL(k_scan_apply, dim3((unsigned)np), dim3(NT), 0, s, in, n, (const uint64_t*)part, out);
}

// ---------------------------------------------------------------------------
// runOptimize
// ---------------------------------------------------------------------------
__device__ __forceinline__ uint64_t slot_size_of(int kind, uint32_t ser_len) {
  return kind == DK_R ? (uint64_t)((ser_len + 2 + 15) & ~15u) : (uint64_t)((ser_len + 15) & ~15u);
}

// number of runs of a sorted array (<= 4096 values): 16 B vectors, all requested
// at once; a value starts a run unless it follows its predecessor (the predecessor
// of a vector's first value is the last value of the previous vector: the previous
// lane's, or lane 63's of the previous round)
__device__ __forceinline__ int array_runs(const uint8_t* slot, int card) {
  const int l = lane_id();
  const int nvec = (card + 7) >> 3;  // <= 512
  const uint4* v4 = reinterpret_cast<const uint4*>(slot);
  uint4 v[8];
#pragma unroll
  for (int j = 0; j < 8; j++) v[j] = 64 * j + l < nvec ? v4[64 * j + l] : make_uint4(0, 0, 0, 0);
  int c = 0;
  uint32_t carry = 0;  // last value of the previous round (lane 63)
#pragma unroll
  for (int j = 0; j < 8; j++) {
    if (64 * j >= nvec) break;  // wave-uniform
    const uint32_t w[4] = {v[j].x, v[j].y, v[j].z, v[j].w};
    const uint32_t prev_last = from_prev_lane(w[3] >> 16);
    uint32_t prev = l == 0 ? carry : prev_last;
    const int first = 8 * (64 * j + l);
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const uint32_t x = (w[i >> 1] >> ((i & 1) * 16)) & 0xFFFF;
      const int idx = first + i;
      if (idx < card) c += (idx == 0 || x != prev + 1) ? 1 : 0;
      prev = x;
    }
    carry = lane63u(w[3] >> 16);
  }
  return (int)uni((uint32_t)wave_sum_i(c));
}

// info word: kind | changed << 2 | nruns << 3
__global__ __launch_bounds__(256) void k_runopt_plan(const CDesc* __restrict__ desc, const uint32_t* __restrict__ bm,
                                                     const uint8_t* __restrict__ payload, uint64_t n,
                                                     uint32_t* __restrict__ info, uint64_t* __restrict__ size,
                                                     uint32_t* __restrict__ bm_has_run,
                                                     unsigned long long* __restrict__ totals) {
  const uint64_t nw = (uint64_t)gridDim.x * 4;
  uint64_t cnt[3] = {0, 0, 0}, ser = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6); i < n; i += nw) {
    const CDesc d = desc[i];
    const uint8_t* slot = payload + d.slot;
    const int card = (int)d.card;
    int nruns, kind;
    if (d.kind == DK_A) {
      nruns = array_runs(slot, card);
      kind = 2 * card > 2 + 4 * nruns ? DK_R : DK_A;
    } else if (d.kind == DK_B) {
      WCtr x;
      w_load_bitmap(slot, x);
      nruns = w_runs(x);
      kind = 2 + 4 * nruns < 8192 ? DK_R : DK_B;
    } else {
      nruns = *reinterpret_cast<const uint16_t*>(slot + 2);
      kind = eff(card, nruns);
    }
    const uint32_t len = kind == DK_A ? 2u * card : kind == DK_B ? 8192u : 2u + 4u * nruns;
    if (lane_id() == 0) {
      info[i] = (uint32_t)kind | ((kind != d.kind) ? 4u : 0u) | ((uint32_t)nruns << 3);
      size[i] = slot_size_of(kind, len);
      // one bitmap can own every container: read before writing, so the flag's line
      // takes a few stores rather than one per run container
      if (kind == DK_R) {
        uint32_t* f = bm_has_run + bm[i];
        if (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) *f = 1;
      }
    }
    cnt[kind]++;
    ser += len;
  }
  // workgroup totals, one atomic per counter per workgroup
  __shared__ unsigned long long wsum[4][4];
  if (lane_id() == 0) {
    for (int k = 0; k < 3; k++) wsum[threadIdx.x >> 6][k] = cnt[k];
    wsum[threadIdx.x >> 6][3] = ser;
  }
  __syncthreads();
  if (threadIdx.x < 4) {
    const unsigned long long v =
        wsum[0][threadIdx.x] + wsum[1][threadIdx.x] + wsum[2][threadIdx.x] + wsum[3][threadIdx.x];
    if (v) atomicAdd(&totals[threadIdx.x], v);
  }
}

__global__ __launch_bounds__(256) void k_runopt_write(const CDesc* __restrict__ desc,
                                                         const uint8_t* __restrict__ payload, uint64_t n,
                                                         const uint32_t* __restrict__ info,
                                                         const uint64_t* __restrict__ off, CDesc* __restrict__ out_desc,
                                                         uint8_t* __restrict__ out_payload) {
  __shared__ __align__(16) uint32_t lds_all[4][2048];
  uint32_t* lds = lds_all[threadIdx.x >> 6];
  const int lane = lane_id();
  const uint64_t nw = (uint64_t)gridDim.x * 4;
  for (uint64_t i = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6); i < n; i += nw) {
    const CDesc d = desc[i];
    const uint32_t inf = info[i];
    const int kind = (int)(inf & 3);
    const uint64_t o = off[i];
    uint8_t* dst = out_payload + o;
    if (!(inf & 4)) {  // unchanged: the slot as it is (A padding included)
      const uint32_t nr = inf >> 3;
      const uint32_t len = kind == DK_A ? 2u * d.card : kind == DK_B ? 8192u : 2u + 4u * nr;
      const uint32_t nvec = (uint32_t)(slot_size_of(kind, len) >> 4);
      const uint4* sv = reinterpret_cast<const uint4*>(payload + d.slot);
      uint4* dv = reinterpret_cast<uint4*>(dst);
      for (uint32_t j = lane; j < nvec; j += 64) dv[j] = sv[j];
    } else {
      WCtr x;
      w_materialize(d, payload, lds, x);
      if (kind == DK_B) {
        w_store_bitmap(dst, x);
      } else {
        uint32_t copy = w_stage(kind, x, (int)d.card, lds);
        if (kind == DK_A) {  // pad the slot to 16 B with the last value (batch layout)
          uint16_t* st = reinterpret_cast<uint16_t*>(lds);
          const uint32_t c = d.card, padded = (2u * c + 15) & ~15u;
          const uint16_t last = st[c - 1];
          for (uint32_t j = c + lane; j < padded / 2; j += 64) st[j] = last;
          wsync();
          copy = padded;
        }
        copy_lds_to_global<64>(dst + (kind == DK_R ? 2 : 0), lds, copy, lane);
      }
      wsync();
    }
    if (lane == 0) out_desc[i] = CDesc{o, d.card, d.key, (uint8_t)kind, d.flags};
  }
}

void launch_runopt_plan(hipStream_t s, const CDesc* desc, const uint32_t* bm, const uint8_t* payload, uint64_t n,
                        uint32_t* info, uint64_t* size, uint32_t* bm_has_run, unsigned long long* totals) {
  if (!n) return;
  const uint64_t g = std::min<uint64_t>((n + 3) / 4, 2048);
  hipLaunchKernelGGL(k_runopt_plan, dim3((unsigned)g), dim3(256), 0, s, desc, bm, payload, n, info, size, bm_has_run,
                     totals);
}

void launch_runopt_write(hipStream_t s, const CDesc* desc, const uint8_t* payload, uint64_t n, const uint32_t* info,
                         const uint64_t* off, CDesc* out_desc, uint8_t* out_payload) {
  if (!n) return;
  const uint64_t g = std::min<uint64_t>((n + 3) / 4, 8192);
  hipLaunchKernelGGL(k_runopt_write, dim3((unsigned)g), dim3(256), 0, s, desc, payload, n, info, off, out_desc,
                     out_payload);
}

}  // namespace rbg
