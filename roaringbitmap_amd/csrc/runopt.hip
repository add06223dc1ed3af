// RoaringBitmap.runOptimize over every container of a device-resident batch
// (RB/RoaringBitmap.java:2764-2774), and the device-wide exclusive scan it (and
// the header decode) places slots with.
//
//   k_runopt : one wave per container decides the container's new type
//                A -> R iff 2 card > 2 + 4 nruns  (RB/ArrayContainer.java:1085-1099),
//                     nruns counted on the sorted values themselves;
//                B -> R iff 2 + 4 nruns < 8192    (RB/BitmapContainer.java:1218-1237);
//                R -> toEfficientContainer        (RB/RunContainer.java:2083-2085, 2326-2335)
//                     on the stored run count, as the reference does;
//              and writes it at its own slot offset in the new batch: an unchanged
//              container's slot is copied verbatim (R kept as R is the reference's
//              `return this`), a converted one is materialised in registers and
//              staged through the wave's LDS.
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

// k_scan_apply with the tile prefix summed by the tile itself (up to kScanDirect tiles: at most 16 loads
// per thread), so no k_scan_partials launch; the last tile writes the total
constexpr uint64_t kScanDirect = 16 * NT;
__global__ __launch_bounds__(256) void k_scan_apply_direct(const uint64_t* in, uint64_t n,
                                                           const uint64_t* __restrict__ part, uint64_t* out,
                                                           uint64_t* __restrict__ total) {
  __shared__ uint64_t sh4[4];
  uint64_t pre = 0;
  for (uint64_t j = threadIdx.x; j < blockIdx.x; j += NT) pre += part[j];
  uint64_t pre_sum;
  block_excl_u64(pre, sh4, &pre_sum);  // the sum over the block: the tile's prefix
  pre = pre_sum;
  const uint64_t base = (uint64_t)blockIdx.x * kScanTile + (uint64_t)threadIdx.x * kScanPer;
  uint64_t v[kScanPer];
  uint64_t sum = 0;
#pragma unroll
  for (int j = 0; j < kScanPer; j++) {
    v[j] = base + j < n ? in[base + j] : 0;
    sum += v[j];
  }
  uint64_t tot;
  uint64_t run = pre + block_excl_u64(sum, sh4, &tot);
#pragma unroll
  for (int j = 0; j < kScanPer; j++) {
    if (base + j < n) out[base + j] = run;
    run += v[j];
  }
  if (blockIdx.x == gridDim.x - 1 && threadIdx.x == 0) *total = pre + tot;
}

uint64_t scan_parts(uint64_t n) { return (n + kScanTile - 1) / kScanTile; }

void launch_exclusive_scan(hipStream_t s, const uint64_t* in, uint64_t* out, uint64_t n, uint64_t* part,
                           uint64_t* total) {
  const uint64_t np = scan_parts(n);
  if (np && np <= kScanDirect) {  // two launches: tile totals, then each tile sums its predecessors itself
    hipLaunchKernelGGL(k_scan_reduce, dim3((unsigned)np), dim3(NT), 0, s, in, n, part);
    hipLaunchKernelGGL(k_scan_apply_direct, dim3((unsigned)np), dim3(NT), 0, s, in, n, (const uint64_t*)part, out,
                       total);
    return;
  }
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

// runOptimize in one pass (one wave per container).  Every container keeps its slot offset: a
// conversion only happens when the new form is smaller, and its 16 B-rounded slot is then no larger
// than the old one (A -> R iff 2 card > 2 + 4 nruns, so 4 + 4 nruns <= 2 card; B -> R iff
// 2 + 4 nruns < 8192, so 4 + 4 nruns <= 8192; R -> A / B only where EFF finds them smaller), so the
// new batch takes the input's layout, with a hole after each shrunk container, and needs no size scan
// between deciding a type and writing it.  A bitmap is decided from registers and, if it stays a
// bitmap, stored from them (read once).  Per workgroup g, wstat[4 g + k] = its containers of kind k
// (k < 3) and their serialized payload bytes (k = 3): plain stores, nothing to zero first; the batch's
// totals and run flags are derived only when the host asks (k_runopt_flags, ensure_stats).
__global__ __launch_bounds__(256, 4) void k_runopt(const CDesc* __restrict__ desc, const uint8_t* __restrict__ payload,
                                                uint64_t n, CDesc* __restrict__ out_desc,
                                                uint8_t* __restrict__ out_payload, RoCopy cp,
                                                unsigned long long* __restrict__ wstat) {
  __shared__ __align__(16) uint32_t lds_all[4][2048];
  uint32_t* lds = lds_all[threadIdx.x >> 6];
  const int lane = lane_id();
  const uint64_t nw = (uint64_t)gridDim.x * 4;
  // the new batch's keys, input indices and both CSRs are the input's (runOptimize changes no key):
  // copied here by every thread of the grid instead of four device-to-device copies
  {
    const uint64_t g = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, gs = (uint64_t)gridDim.x * blockDim.x;
    for (uint64_t i = g; i < n; i += gs) {
      cp.out_keys[i] = cp.keys[i];
      cp.out_bm[i] = cp.bm[i];
    }
    for (uint64_t i = g; i < cp.n_koff; i += gs) cp.out_koff[i] = cp.koff[i];
    for (uint64_t i = g; i < cp.n_boff; i += gs) cp.out_boff[i] = cp.boff[i];
  }
  uint64_t cnt[3] = {0, 0, 0}, ser = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6); i < n; i += nw) {
    const CDesc d = desc[i];
    const uint8_t* slot = payload + d.slot;
    uint8_t* dst = out_payload + d.slot;
    const int card = (int)d.card;
    int nruns, kind;
    WCtr x;
    if (d.kind == DK_A) {
      nruns = array_runs(slot, card);
      kind = 2 * card > 2 + 4 * nruns ? DK_R : DK_A;
    } else if (d.kind == DK_B) {
      w_load_bitmap(slot, x);
      nruns = w_runs(x);
      kind = 2 + 4 * nruns < 8192 ? DK_R : DK_B;
    } else {
      nruns = *reinterpret_cast<const uint16_t*>(slot + 2);
      kind = eff(card, nruns);
    }
    const uint32_t len = kind == DK_A ? 2u * card : kind == DK_B ? 8192u : 2u + 4u * nruns;
    if (kind == DK_B) {  // B kept, or R -> B
      if (d.kind != DK_B) w_materialize(d, payload, lds, x);
      w_store_bitmap(dst, x);
      wsync();
    } else if (kind == d.kind) {  // A or R kept: the slot as it is (A padding included)
      const uint32_t nvec = (uint32_t)(slot_size_of(kind, len) >> 4);
      const uint4* sv = reinterpret_cast<const uint4*>(slot);
      uint4* dv = reinterpret_cast<uint4*>(dst);
      uint32_t j = lane;
      for (; j + 192 < nvec; j += 256) {  // four vectors per lane requested before any is stored
        const uint4 a0 = sv[j], a1 = sv[j + 64], a2 = sv[j + 128], a3 = sv[j + 192];
        dv[j] = a0;
        dv[j + 64] = a1;
        dv[j + 128] = a2;
        dv[j + 192] = a3;
      }
      for (; j < nvec; j += 64) dv[j] = sv[j];
    } else {  // A -> R, B -> R, R -> A: staged through the wave's LDS
      if (d.kind != DK_B) w_materialize(d, payload, lds, x);
      uint32_t copy = w_stage(kind, x, card, lds);
      if (kind == DK_A) {  // pad the slot to 16 B with the last value (batch layout)
        uint16_t* st = reinterpret_cast<uint16_t*>(lds);
        const uint32_t c = d.card, padded = (2u * c + 15) & ~15u;
        const uint16_t last = st[c - 1];
        for (uint32_t q = c + lane; q < padded / 2; q += 64) st[q] = last;
        wsync();
        copy = padded;
      }
      copy_lds_to_global<64>(dst + (kind == DK_R ? 2 : 0), lds, copy, lane);
      wsync();
    }
    if (lane == 0) out_desc[i] = CDesc{d.slot, d.card, d.key, (uint8_t)kind, d.flags};
    cnt[kind]++;
    ser += len;
  }
  __shared__ unsigned long long wsum[4][4];
  if (lane == 0) {
    for (int k = 0; k < 3; k++) wsum[threadIdx.x >> 6][k] = cnt[k];
    wsum[threadIdx.x >> 6][3] = ser;
  }
  __syncthreads();
  if (threadIdx.x < 4)
    wstat[4 * (uint64_t)blockIdx.x + threadIdx.x] =
        wsum[0][threadIdx.x] + wsum[1][threadIdx.x] + wsum[2][threadIdx.x] + wsum[3][threadIdx.x];
}

// per-bitmap run flags of a runOptimize result (its new descriptors): flag[bm] = 1 if any container
// of the bitmap is a run container (read before write: one bitmap can own every container)
__global__ __launch_bounds__(256) void k_runopt_flags(const CDesc* __restrict__ desc, const uint32_t* __restrict__ bm,
                                                      uint64_t n, uint32_t* __restrict__ flags) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    if (desc[i].kind != DK_R) continue;
    uint32_t* f = flags + bm[i];
    if (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0) *f = 1;
  }
}

uint64_t runopt_groups(uint64_t n) { return std::max<uint64_t>(1, std::min<uint64_t>((n + 3) / 4, 8192)); }

void launch_runopt(hipStream_t s, const CDesc* desc, const uint8_t* payload, uint64_t n, CDesc* out_desc,
                   uint8_t* out_payload, RoCopy cp, unsigned long long* wstat) {
  hipLaunchKernelGGL(k_runopt, dim3((unsigned)runopt_groups(n)), dim3(256), 0, s, desc, payload, n, out_desc,
                     out_payload, cp, wstat);
}

void launch_runopt_flags(hipStream_t s, const CDesc* desc, const uint32_t* bm, uint64_t n, uint32_t* flags) {
  if (!n) return;
  const uint64_t g = std::min<uint64_t>((n + 255) / 256, 1024);
  hipLaunchKernelGGL(k_runopt_flags, dim3((unsigned)g), dim3(256), 0, s, desc, bm, n, flags);
}

// ---------------------------------------------------------------------------
// selectRangeWithoutCopy (RB/RoaringBitmap.java:3160-3214) of every bitmap of a batch, into a new batch:
// the input of the range-restricted aggregations and(Iterator, start, end) :1308-1316, or :2536-2543,
// xor :3359-3365 and andNot(x1, x2, start, end) :1396-1404.  Keys outside [hbs, hbl] go; the first key
// loses [0, lbs), the last (lbl, 65535] through Container.remove (A stays A, B becomes A at <= 4096
// values, R stays R with its runs clipped: RB/ArrayContainer.java:1039-1061, RB/BitmapContainer.java:
// 1166-1181, RB/RunContainer.java:2032-2035); a container left empty goes too.
// ---------------------------------------------------------------------------
// the bits of owned word k (chunk i, word j) inside [lo, hi]
__device__ __forceinline__ uint64_t range_mask_word(int i, int j, int lo, int hi) {
  const int w = 128 * i + 2 * lane_id() + j;
  const int b0 = 64 * w, b1 = b0 + 63;
  if (b1 < lo || b0 > hi) return 0;
  uint64_t m = ~0ull;
  if (lo > b0) m &= ~0ull << (lo - b0);
  if (hi < b1) m &= ~0ull >> (b1 - hi);
  return m;
}

// the cut [lo, hi] of container i (cut = false: the key lies inside the range, unchanged)
__device__ __forceinline__ void rsel_bounds(const CDesc& d, const RselArgs& ra, bool* keep_key, bool* cut, int* lo,
                                            int* hi) {
  const int k = d.key;
  *keep_key = k >= ra.hbs && k <= ra.hbl;
  *lo = k == ra.hbs ? ra.lbs : 0;
  *hi = k == ra.hbl ? ra.lbl : 65535;
  *cut = *keep_key && (*lo > 0 || *hi < 65535);
}

// A: values [first, first + cnt) lie in [lo, hi] (the array is sorted)
__device__ __forceinline__ void array_window(const uint16_t* v, int card, int lo, int hi, int* first, int* cnt) {
  int below = 0, in = 0;
  for (int x = lane_id(); x < card; x += 64) {
    const int y = v[x];
    below += y < lo;
    in += y >= lo && y <= hi;
  }
  *first = (int)uni((uint32_t)wave_sum_i(below));
  *cnt = (int)uni((uint32_t)wave_sum_i(in));
}

// R: runs overlapping [lo, hi] and their clipped cardinality
__device__ __forceinline__ void run_window(const uint8_t* slot, int lo, int hi, int* nr_out, int* card_out) {
  const int nr = *reinterpret_cast<const uint16_t*>(slot + 2);
  const uint32_t* pr = reinterpret_cast<const uint32_t*>(slot + 4);
  int c = 0, n = 0;
  for (int r = lane_id(); r < nr; r += 64) {
    const uint32_t p = pr[r];
    const int s = (int)(p & 0xFFFF), e = s + (int)(p >> 16);
    const int s1 = max(s, lo), e1 = min(e, hi);
    if (s1 <= e1) {
      n++;
      c += e1 - s1 + 1;
    }
  }
  *nr_out = (int)uni((uint32_t)wave_sum_i(n));
  *card_out = (int)uni((uint32_t)wave_sum_i(c));
}

// info[i] = kind | keep << 2 | cut << 3; card[i], size[i] (new slot bytes), keep[i]; per bitmap kept
// containers and cardinality; totals = {#A, #B, #R, serialized bytes of containers above 8194 B}
__global__ __launch_bounds__(256) void k_rsel_plan(const CDesc* __restrict__ desc, const uint32_t* __restrict__ bm,
                                                   const uint8_t* __restrict__ payload, uint64_t n, RselArgs ra,
                                                   uint32_t* __restrict__ info, uint32_t* __restrict__ ncard,
                                                   uint64_t* __restrict__ size, uint64_t* __restrict__ keepv,
                                                   unsigned long long* __restrict__ bm_cnt,
                                                   unsigned long long* __restrict__ bm_card,
                                                   unsigned long long* __restrict__ totals) {
  const uint64_t nw = (uint64_t)gridDim.x * 4;
  unsigned long long cnt[3] = {0, 0, 0}, big = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6); i < n; i += nw) {
    const CDesc d = desc[i];
    const uint8_t* slot = payload + d.slot;
    bool keep_key, cut;
    int lo, hi;
    rsel_bounds(d, ra, &keep_key, &cut, &lo, &hi);
    int kind = d.kind, card = keep_key ? (int)d.card : 0;
    uint32_t len = 0;
    if (keep_key && !cut) {
      len = kind == DK_A ? 2u * card : kind == DK_B ? 8192u : 2u + 4u * *reinterpret_cast<const uint16_t*>(slot + 2);
    } else if (cut && kind == DK_A) {
      int first;
      array_window(reinterpret_cast<const uint16_t*>(slot), card, lo, hi, &first, &card);
      len = 2u * card;
    } else if (cut && kind == DK_B) {
      WCtr x;
      w_load_bitmap(slot, x);
#pragma unroll
      for (int k = 0; k < 16; k++) x.w[k] &= range_mask_word(k >> 1, k & 1, lo, hi);
      card = w_card(x);
      // BitmapContainer.remove: an array at <= 4096 values (RB/BitmapContainer.java:1166-1181); the
      // buffer package's MappeableBitmapContainer.remove below 4096 (RB/buffer/MappeableBitmapContainer.java
      // :1597-1612), so a 4096-value bitmap stays one
      kind = (ra.buf ? card < 4096 : card <= 4096) ? DK_A : DK_B;
      len = kind == DK_A ? 2u * card : 8192u;
    } else if (cut) {  // R
      int nr;
      run_window(slot, lo, hi, &nr, &card);
      len = 2u + 4u * nr;
    }
    const bool keep = keep_key && card > 0;
    if (lane_id() == 0) {
      info[i] = (uint32_t)kind | (keep ? 4u : 0u) | (cut ? 8u : 0u);
      ncard[i] = (uint32_t)card;
      size[i] = keep ? slot_size_of(kind, len) : 0;
      keepv[i] = keep ? 1 : 0;
      if (keep) {
        atomicAdd(&bm_cnt[bm[i]], 1ull);
        atomicAdd(&bm_card[bm[i]], (unsigned long long)card);
      }
    }
    if (keep) {
      cnt[kind]++;
      if (len > 8194) big += len;
    }
  }
  __shared__ unsigned long long wsum[4][4];
  if (lane_id() == 0) {
    wsum[threadIdx.x >> 6][0] = cnt[0];
    wsum[threadIdx.x >> 6][1] = cnt[1];
    wsum[threadIdx.x >> 6][2] = cnt[2];
    wsum[threadIdx.x >> 6][3] = big;
  }
  __syncthreads();
  if (threadIdx.x < 4) {
    const unsigned long long v = wsum[0][threadIdx.x] + wsum[1][threadIdx.x] + wsum[2][threadIdx.x] +
                                 wsum[3][threadIdx.x];
    if (v) atomicAdd(&totals[threadIdx.x], v);
  }
}

// kept container i -> index idx[i], slot at off[i] of the new batch
__global__ __launch_bounds__(256, 4) void k_rsel_write(const CDesc* __restrict__ desc, const uint32_t* __restrict__ bm,
                                                    const uint8_t* __restrict__ payload, uint64_t n, RselArgs ra,
                                                    const uint32_t* __restrict__ info,
                                                    const uint32_t* __restrict__ ncard,
                                                    const uint64_t* __restrict__ off, const uint64_t* __restrict__ idx,
                                                    CDesc* __restrict__ out_desc, uint16_t* __restrict__ out_keys,
                                                    uint32_t* __restrict__ out_bm, uint8_t* __restrict__ out_payload) {
  __shared__ __align__(16) uint32_t lds_all[4][2048];
  uint32_t* lds = lds_all[threadIdx.x >> 6];
  const int lane = lane_id();
  const uint64_t nw = (uint64_t)gridDim.x * 4;
  for (uint64_t i = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6); i < n; i += nw) {
    const uint32_t inf = info[i];
    if (!(inf & 4)) continue;  // wave-uniform
    const CDesc d = desc[i];
    const int kind = (int)(inf & 3);
    const uint32_t card = ncard[i];
    const uint64_t j = idx[i], o = off[i];
    const uint8_t* slot = payload + d.slot;
    uint8_t* dst = out_payload + o;
    if (!(inf & 8)) {  // inside the range: the slot as it is
      const uint32_t len = kind == DK_A   ? 2u * card
                           : kind == DK_B ? 8192u
                                          : 2u + 4u * *reinterpret_cast<const uint16_t*>(slot + 2);
      const uint32_t nvec = (uint32_t)(slot_size_of(kind, len) >> 4);
      const uint4* sv = reinterpret_cast<const uint4*>(slot);
      uint4* dv = reinterpret_cast<uint4*>(dst);
      for (uint32_t q = lane; q < nvec; q += 64) dv[q] = sv[q];
    } else {
      bool keep_key, cut;
      int lo, hi;
      rsel_bounds(d, ra, &keep_key, &cut, &lo, &hi);
      if (d.kind == DK_A) {  // the window of the sorted values, padded to 16 B with the last one
        int first, cnt;
        array_window(reinterpret_cast<const uint16_t*>(slot), (int)d.card, lo, hi, &first, &cnt);
        const uint16_t* v = reinterpret_cast<const uint16_t*>(slot) + first;
        uint16_t* w = reinterpret_cast<uint16_t*>(dst);
        const int padded = (int)((2u * card + 15) & ~15u) / 2;
        for (int x = lane; x < padded; x += 64) w[x] = v[min(x, (int)card - 1)];
      } else if (d.kind == DK_B) {
        WCtr x;
        w_load_bitmap(slot, x);
#pragma unroll
        for (int k = 0; k < 16; k++) x.w[k] &= range_mask_word(k >> 1, k & 1, lo, hi);
        if (kind == DK_B) {
          w_store_bitmap(dst, x);
        } else {
          w_stage(DK_A, x, (int)card, lds);
          uint16_t* st = reinterpret_cast<uint16_t*>(lds);
          const uint32_t padded = (2u * card + 15) & ~15u;
          const uint16_t last = st[card - 1];
          for (uint32_t q = card + lane; q < padded / 2; q += 64) st[q] = last;
          wsync();
          copy_lds_to_global<64>(dst, lds, padded, lane);
          wsync();
        }
      } else {  // R: the overlapping runs, clipped, in order
        const int nr = *reinterpret_cast<const uint16_t*>(slot + 2);
        const uint32_t* pr = reinterpret_cast<const uint32_t*>(slot + 4);
        uint32_t* out = reinterpret_cast<uint32_t*>(dst + 4);
        int base = 0;
        for (int r0 = 0; r0 < nr; r0 += 64) {
          const int r = r0 + lane;
          uint32_t np = 0;
          int ov = 0;
          if (r < nr) {
            const uint32_t p = pr[r];
            const int s = (int)(p & 0xFFFF), e = s + (int)(p >> 16);
            const int s1 = max(s, lo), e1 = min(e, hi);
            ov = s1 <= e1;
            np = (uint32_t)s1 | ((uint32_t)(e1 - s1) << 16);
          }
          int tot;
          const int pos = base + wave_excl(ov, &tot);
          if (ov) out[pos] = np;
          base += tot;
        }
        if (lane == 0) {
          reinterpret_cast<uint16_t*>(dst)[0] = 0;
          reinterpret_cast<uint16_t*>(dst)[1] = (uint16_t)base;
        }
      }
    }
    if (lane == 0) {
      out_desc[j] = CDesc{o, card, d.key, (uint8_t)kind, 0};
      out_keys[j] = d.key;
      out_bm[j] = bm[i];
    }
  }
}

void launch_rsel_plan(hipStream_t s, const CDesc* desc, const uint32_t* bm, const uint8_t* payload, uint64_t n,
                      RselArgs ra, uint32_t* info, uint32_t* card, uint64_t* size, uint64_t* keep,
                      unsigned long long* bm_cnt, unsigned long long* bm_card, unsigned long long* totals) {
  if (!n) return;
  const uint64_t g = std::min<uint64_t>((n + 3) / 4, 8192);
  hipLaunchKernelGGL(k_rsel_plan, dim3((unsigned)g), dim3(256), 0, s, desc, bm, payload, n, ra, info, card, size, keep,
                     bm_cnt, bm_card, totals);
}
void launch_rsel_write(hipStream_t s, const CDesc* desc, const uint32_t* bm, const uint8_t* payload, uint64_t n,
                       RselArgs ra, const uint32_t* info, const uint32_t* card, const uint64_t* off,
                       const uint64_t* idx, CDesc* out_desc, uint16_t* out_keys, uint32_t* out_bm,
                       uint8_t* out_payload) {
  if (!n) return;
  const uint64_t g = std::min<uint64_t>((n + 3) / 4, 8192);
  hipLaunchKernelGGL(k_rsel_write, dim3((unsigned)g), dim3(256), 0, s, desc, bm, payload, n, ra, info, card, off, idx,
                     out_desc, out_keys, out_bm, out_payload);
}

}  // namespace rbg
