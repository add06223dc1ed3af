// HIP kernels of the MI355X Roaring engine (gfx950).  RB/ = reference
// RoaringBitmap/src/main/java/org/roaringbitmap/.
//
// Every op is one pipeline on the context stream with no host sync:
//   plan    : per-key (65536 threads) "does key k produce a task", per-WG counts
//   compact : 256 workgroups place the flagged keys into a dense task list
//   compute : one wavefront per task (static stride over a resident grid)
//             computes the result container in registers and parks its payload
//             in the task's scratch slot (arena slot layout) + a task record
//   place   : tile scan over the task records (container index, payload offset,
//             totals) -- the result is now materialised on the device
//   serialize: payload copies into the portable layout, descriptors, offset
//             table, run flags and cookie in front of it (one launch)

#include <algorithm>
#include <mutex>
#include <unordered_map>

#include "kernels.hpp"
#include <cstdlib>

#include "wave.hpp"

namespace rbg {

// ===========================================================================
// plan / compact
// ===========================================================================
// Wide plan from the key-major CSR: n_k = key_off[k+1] - key_off[k].
// mode 0: n_k > 0 (or / xor / orCardinality); mode 1: n_k == n_req (and).
__global__ __launch_bounds__(256) void k_plan_wide(int mode, const uint32_t* __restrict__ key_off, uint32_t n_req,
                                                   int key_lo, int key_hi, Task* __restrict__ by_key,
                                                   uint8_t* __restrict__ flag, uint32_t* __restrict__ wg_count,
                                                   uint64_t* zlb, uint64_t* ztile) {
  plan_zero(zlb, ztile);
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t s = key_off[k], n = key_off[k + 1] - s;
  int f = (mode == 0) ? (n > 0) : (n == n_req && n > 0);
  if ((int)k < key_lo || (int)k >= key_hi) f = 0;
  flag[k] = (uint8_t)f;
  by_key[k] = Task{k, (int32_t)s, (int32_t)n, 0};
  plan_count(f, wg_count);
}

// 256 workgroups x 256 keys: each sums the counts of the workgroups before it.
template <class T>
__global__ __launch_bounds__(256) void k_compact(const uint8_t* __restrict__ flag, const T* __restrict__ by_key,
                                                 const uint32_t* __restrict__ wg_count, T* __restrict__ tasks,
                                                 uint32_t* __restrict__ n_tasks) {
  __shared__ int wsum[4];
  __shared__ uint32_t base_sh;
  const int t = threadIdx.x;
  // prefix over previous workgroups (256 counts, one per thread)
  uint32_t c = (t < (int)blockIdx.x) ? wg_count[t] : 0;
  int v = wave_sum_i((int)c);
  if ((t & 63) == 0) wsum[t >> 6] = v;
  __syncthreads();
  if (t == 0) base_sh = (uint32_t)(wsum[0] + wsum[1] + wsum[2] + wsum[3]);
  __syncthreads();
  const uint32_t k = blockIdx.x * 256 + t;
  const int f = flag[k];
  int tot;
  const int lane_pre = wave_excl(f, &tot);
  __shared__ int wt[4];
  if ((t & 63) == 0) wt[t >> 6] = tot;
  __syncthreads();
  int wpre = 0;
  for (int i = 0; i < (t >> 6); i++) wpre += wt[i];
  if (f) tasks[base_sh + wpre + lane_pre] = by_key[k];
  if (blockIdx.x == gridDim.x - 1 && t == 0) *n_tasks = base_sh + wt[0] + wt[1] + wt[2] + wt[3];
}

__device__ __forceinline__ uint32_t ser_len_of(const CDesc& d, const uint8_t* payload) {
  if (d.kind == DK_A) return 2 * d.card;
  if (d.kind == DK_B) return 8192;
  return 2 + 4 * (uint32_t)(*reinterpret_cast<const uint16_t*>(payload + d.slot + 2));
}

// Shape of the materialised result (container count, run flag, byte sizes)
__device__ __forceinline__ void write_info(ResultInfo* info, const OutCtx& oc, uint32_t size, uint32_t has_run,
                                           uint64_t payload) {
  const uint64_t H = header_bytes(size, has_run);
  ResultInfo ri;
  ri.n_out = size;
  ri.has_run = has_run;
  ri.header = H;
  ri.payload = payload;
  ri.total = H + payload;
  ri.long_card = 0;
  ri.card32 = 0;
  ri.any = size > 0;
  ri.start = oc.payload_base - H;
  ri.err = *oc.err;
  *info = ri;
}

// ===========================================================================
// serialization (RB/RoaringArray.java:896-940), after k_place: one launch writes the
// whole portable bitmap in front of / into the payload region
// ===========================================================================
__device__ __forceinline__ void totals(const OutCtx& oc, uint32_t nt, uint32_t* n_out, uint32_t* has_run,
                                       uint64_t* payload) {
  if (nt == 0) {
    *n_out = 0;
    *has_run = 0;
    *payload = 0;
    return;
  }
  const uint64_t s = __hip_atomic_load(oc.status + nt - 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  *has_run = (uint32_t)((s >> 61) & 1);
  *n_out = (uint32_t)((s >> 44) & 0x1FFFF);
  *payload = s & ((1ULL << 44) - 1);
}

__device__ __forceinline__ void write_cookie(uint8_t* base, uint32_t size, uint32_t has_run) {
  uint32_t cookie[2];
  int nb;
  if (has_run) {  // RB/RoaringArray.java:900-904
    cookie[0] = 12347u | ((size - 1) << 16);
    nb = 4;
  } else {  // :914-917
    cookie[0] = 12346u;
    cookie[1] = size;
    nb = 8;
  }
  const uint8_t* cb = reinterpret_cast<const uint8_t*>(cookie);
  for (int i = 0; i < nb; i++) base[i] = cb[i];
}

// One wave per task record (grid-stride): a kept result's payload bytes go to their offset
// (w_copy: aligned 16 B loads and stores, the source's misalignment funnel-shifted in
// registers); one thread per record writes its descriptor (key, card - 1) and offset-table
// entry -- both tables are 4 B aligned (they end at payload_base).  Threads below the flag-byte
// count pack the run-flag bitset from k_place's kind-by-output bytes; thread 0 writes the
// cookie.
//   PART bit 0: the header (cookie, run flags, descriptors, offsets) -- needs the placement of every record;
//   PART bit 1: the payload copies of records [t_lo, t_hi) -- need only theirs (a key range of a pipelined op).
template <int PART>
__global__ __launch_bounds__(256) void k_serialize(const uint32_t* __restrict__ n_tasks, OutCtx oc,
                                                   const uint8_t* __restrict__ kind_by_out, uint32_t t_lo,
                                                   uint32_t t_hi) {
  const uint32_t nt = *n_tasks;
  uint32_t size, has_run;
  uint64_t payload;
  totals(oc, nt, &size, &has_run, &payload);
  const uint64_t H = header_bytes(size, has_run);
  uint8_t* base = oc.out + oc.payload_base - H;
  const uint64_t desc_base = has_run ? 4 + (size + 7) / 8 : 8;
  const bool offsets = !has_run || size >= 4;
  const uint64_t off_base = desc_base + 4ull * size;
  const uint32_t gid = blockIdx.x * blockDim.x + threadIdx.x;
  if ((PART & 1) && has_run) {
    for (uint32_t b = gid; b < (size + 7) / 8; b += gridDim.x * blockDim.x) {
      uint8_t v = 0;
      for (int k = 0; k < 8; k++) {
        const uint32_t i = 8 * b + k;
        if (i < size && kind_by_out[i] == DK_R) v |= (uint8_t)(1u << k);
      }
      base[4 + b] = v;
    }
  }
  if (PART & 1) {
    if (gid == 0) write_cookie(base, size, has_run);
    // descriptors and offsets by thread (record i -> its output index): neighbouring threads
    // write neighbouring entries, so the stores coalesce (written by each task's copying wave
    // they were scattered 4 B stores: serialize 0.107 -> 0.105 ms)
    for (uint32_t i = gid; i < nt; i += gridDim.x * blockDim.x) {
      const ORec r = oc.recs[i];
      if (!r.keep) continue;
      *(g_u32*)(base + desc_base + 4ull * r.idx) = (uint32_t)r.key | ((r.card - 1) << 16);
      if (offsets) *(g_u32*)(base + off_base + 4ull * r.idx) = (uint32_t)(H + r.off);
    }
  }
  if (!(PART & 2)) return;
  uint8_t* pay = oc.out + oc.payload_base;
  const uint32_t nw = gridDim.x * (blockDim.x >> 6);
  const uint32_t te = min(nt, t_hi);
  for (uint32_t t = uni(t_lo + blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)); t < te; t += nw) {
    const ORec& r = oc.recs[t];
    if (!uni(r.keep)) continue;
    const uint64_t off = uni64(r.off);
    const uint64_t src = uni64(r.src);
    if (src == reinterpret_cast<uint64_t>(pay + off)) continue;  // written in place by the op (OutCtx::spec)
    w_copy(pay + off, reinterpret_cast<const uint8_t*>(src), uni(r.ser_len));
  }
}

// After k_place, before the serialization of a result written with OutCtx::spec: a bitmap
// result written at 8192 t whose placement differs (an earlier task kept fewer bytes or
// nothing) is moved to its scratch slot, so the serialization's copies into the payload
// region never overwrite a source they have yet to read.  One wave per task (grid-stride).
__global__ __launch_bounds__(256) void k_spec_fix(const uint32_t* __restrict__ n_tasks, OutCtx oc) {
  const uint32_t nt = *n_tasks;
  const uint8_t* pay = oc.out + oc.payload_base;
  const uint32_t nw = gridDim.x * (blockDim.x >> 6);
  for (uint32_t t = uni(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)); t < nt; t += nw) {
    const ORec& r = oc.recs[t];
    const uint64_t at = 8192ull * t;
    if (!uni(r.keep) || uni64(r.src) != reinterpret_cast<uint64_t>(pay + at) || uni64(r.off) == at) continue;
    uint8_t* slot = oc.scratch + (size_t)t * kSlotBytes;
    w_copy(slot, pay + at, 8192);
    if (lane_id() == 0) oc.recs[t].src = reinterpret_cast<uint64_t>(slot);
  }
}

// Java-int sum of task cardinalities (mod 2^32) plus "any nonzero" for intersects.
// `err` is the op's look-back error word: a plan spin that timed out makes the task list
// (and so the sum) invalid, which ctx_info reports as a device error.
__global__ __launch_bounds__(1024) void k_reduce_card(const uint32_t* __restrict__ task_card,
                                                      const uint32_t* __restrict__ n_tasks, ResultInfo* __restrict__ info,
                                                      const uint32_t* __restrict__ err) {
  __shared__ unsigned long long ws[16];
  __shared__ int wa[16];
  const uint32_t nt = *n_tasks;
  unsigned long long s = 0;
  int any = 0;
  // 16 B loads, four rounds in flight per thread (one dependent load round for 65,536
  // tasks instead of 64 serial ones)
  const uint4* v4 = reinterpret_cast<const uint4*>(task_card);
  const uint32_t nv = nt >> 2;
  for (uint32_t i0 = 0; i0 < nv; i0 += 4 * 1024) {
    uint4 v[4];
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const uint32_t i = i0 + u * 1024 + threadIdx.x;
      v[u] = i < nv ? v4[i] : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < 4; u++) {
      s += (unsigned long long)v[u].x + v[u].y + v[u].z + v[u].w;
      any |= (v[u].x | v[u].y | v[u].z | v[u].w) != 0;
    }
  }
  for (uint32_t i = 4 * nv + threadIdx.x; i < nt; i += 1024) {
    const uint32_t c = task_card[i];
    s += c;
    any |= c != 0;
  }
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  const int a = __any(any) ? 1 : 0;
  if ((threadIdx.x & 63) == 0) {
    ws[threadIdx.x >> 6] = s;
    wa[threadIdx.x >> 6] = a;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long tot = 0;
    int an = 0;
    for (int i = 0; i < 16; i++) {
      tot += ws[i];
      an |= wa[i];
    }
    ResultInfo r = {};
    r.long_card = (int64_t)tot;
    r.card32 = (uint32_t)tot;
    r.any = (uint32_t)an;
    r.err = *err;
    *info = r;
  }
}

// ===========================================================================
// batch statistics
// ===========================================================================
// serialized payload bytes of a batch (for statistics)
__global__ __launch_bounds__(256) void k_batch_bytes(const CDesc* __restrict__ desc, uint64_t n,
                                                     const uint8_t* __restrict__ payload,
                                                     unsigned long long* __restrict__ out) {
  unsigned long long s = 0;
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    s += ser_len_of(desc[i], payload);
  for (int o = 32; o > 0; o >>= 1) s += __shfl_xor(s, o, 64);
  if ((threadIdx.x & 63) == 0) atomicAdd(out, s);
}

// ===========================================================================
// scan placement: tile scan of the task records (uniform tiles, so a decoupled
// look-back over tiles never waits on a slow container), then the payload copy
// ===========================================================================
constexpr int kTile = 1024;  // tasks per workgroup tile (4 per thread; 512-record tiles measured slower)

// Look-back of tile t over all earlier tiles at once (t < 64): lane i reads the
// status of tile t - 1 - i; the nearest inclusive status ends the window, and every
// status before it must at least hold its aggregate (else spin).  Lane 0 then
// publishes t's inclusive status.  One wave.
__device__ __forceinline__ Prefix lookback_wave(uint64_t* status, uint32_t t, uint32_t cnt, uint64_t bytes,
                                                uint32_t run, uint32_t* err) {
  const int lane = lane_id();
  if (lane == 0)
    __hip_atomic_store(status + t, lb_pack(t == 0 ? 2 : 1, run, cnt, bytes), __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_AGENT);
  uint64_t acc_cnt = 0, acc_bytes = 0, acc_run = 0;
  if (t != 0) {
    const int j = (int)t - 1 - lane;
    uint32_t spins = 0;
    for (;;) {
      const uint64_t sv = j >= 0 ? __hip_atomic_load(status + j, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT)
                                 : (2ull << 62);  // before tile 0: an empty inclusive prefix
      const uint32_t st = (uint32_t)(sv >> 62);
      const uint64_t incl = __ballot(st == 2);  // lane t-1-0 ... : the nearest inclusive is the lowest lane
      // exists for t <= 64 (lane t, tile -1, is always inclusive); further back, wait for one
      const int k = incl ? __builtin_ctzll(incl) : 64;
      const uint64_t window = k >= 63 ? ~0ull : ((2ull << k) - 1);
      if (incl != 0 && (__ballot(st == 0) & window) == 0) {
        const bool in = lane <= k;
        uint64_t c = in ? (sv >> 44) & 0x1FFFF : 0, by = in ? sv & ((1ULL << 44) - 1) : 0;
        const uint32_t r = in ? (uint32_t)((sv >> 61) & 1) : 0u;
        for (int o = 32; o > 0; o >>= 1) {
          c += __shfl_xor(c, o, 64);
          by += __shfl_xor(by, o, 64);
        }
        acc_cnt = c;
        acc_bytes = by;
        acc_run = __ballot(r != 0) ? 1 : 0;
        break;
      }
      if (++spins > (1u << 22)) {
        if (lane == 0) atomicOr(err, 1u);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    if (lane == 0)
      __hip_atomic_store(status + t, lb_pack(2, run | acc_run, cnt + acc_cnt, bytes + acc_bytes), __ATOMIC_RELEASE,
                         __HIP_MEMORY_SCOPE_AGENT);
  }
  return Prefix{(uint32_t)acc_cnt, acc_bytes};
}

// One workgroup per tile of kTile task records (all tiles resident: <= 64), in
// blockIdx order: counts, payload bytes and run flags scanned in the workgroup and
// across tiles by lookback_wave; each tile's result cardinality goes to tile_card
// before its status is published, and the last tile sums them.
// tile_lo: the launch's first tile (a pipelined op places its key ranges one launch each, in order;
// a tile's look-back reads the statuses the earlier launches published).
__global__ __launch_bounds__(256) void k_place(const uint32_t* __restrict__ n_tasks, OutCtx oc, ResultInfo* __restrict__ info,
                                               uint32_t tile_lo) {
  __shared__ int wsum[3][4];
  __shared__ unsigned long long wbytes[4];
  __shared__ unsigned long long wcard[4];
  __shared__ Prefix shp;
  const uint32_t nt = *n_tasks;
  const uint32_t ntiles = (nt + kTile - 1) / kTile;
  if (nt == 0) {
    if (blockIdx.x == 0 && tile_lo == 0 && threadIdx.x == 0) {
      write_info(info, oc, 0, 0, 0);
      if (oc.layout_out) oc.layout_out[0] = oc.layout_out[1] = oc.layout_out[2] = 0;
    }
    return;
  }
  const uint32_t tile = tile_lo + blockIdx.x;
  if (tile >= ntiles) return;
  constexpr int kPer = kTile / 256;  // records per thread
  const uint32_t t0 = tile * kTile + kPer * threadIdx.x;
  uint32_t keep[kPer], len[kPer], run[kPer];
  uint32_t c = 0, r = 0;
  unsigned long long b = 0;
  uint32_t card = 0;  // <= kPer x 65536 per thread
#pragma unroll
  for (int i = 0; i < kPer; i++) {
    keep[i] = len[i] = run[i] = 0;
    if (t0 + i < nt) {
      const ORec x = oc.recs[t0 + i];
      keep[i] = x.keep;
      len[i] = x.keep ? x.ser_len : 0;
      run[i] = x.keep && x.kind == DK_R;
      card += x.keep ? x.card : 0;
    }
    c += keep[i];
    b += len[i];
    r |= run[i];
  }
  // workgroup exclusive scan of (count, bytes), OR of run, sum of cardinality
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  int tc;
  const int pc = wave_excl((int)c, &tc);
  unsigned long long sb = b;
  for (int o = 1; o < 64; o <<= 1) {
    const unsigned long long u = __shfl_up(sb, o, 64);
    if (lane >= o) sb += u;
  }
  const unsigned long long wb = __shfl(sb, 63, 64);
  unsigned long long cw = card;
  for (int o = 32; o > 0; o >>= 1) cw += __shfl_xor(cw, o, 64);
  const int wr = __any(r) ? 1 : 0;
  if (lane == 0) {
    wsum[0][w] = tc;
    wsum[1][w] = wr;
    wbytes[w] = wb;
    wcard[w] = cw;
  }
  __syncthreads();
  uint32_t oc_c = 0, tot_c = 0, tot_r = 0;
  unsigned long long oc_b = 0, tot_b = 0, tot_card = 0;
  for (int i = 0; i < 4; i++) {  // the workgroup's 4 waves
    if (i < w) {
      oc_c += wsum[0][i];
      oc_b += wbytes[i];
    }
    tot_c += wsum[0][i];
    tot_b += wbytes[i];
    tot_r |= wsum[1][i];
    tot_card += wcard[i];
  }
  if (threadIdx.x < 64) {
    if (threadIdx.x == 0) oc.tile_card[tile] = tot_card;  // published by the release store of the status
    const Prefix pw = lookback_wave(oc.tile_status, tile, tot_c, tot_b, tot_r, oc.err);
    if (threadIdx.x == 0) shp = pw;
  }
  __syncthreads();
  uint32_t idx = shp.idx + oc_c + (uint32_t)pc;
  unsigned long long off = shp.off + oc_b + (sb - b);
#pragma unroll
  for (int i = 0; i < kPer; i++) {
    if (t0 + i < nt) {
      oc.recs[t0 + i].idx = idx;
      oc.recs[t0 + i].off = off;
      if (keep[i] && oc.kind_by_out) oc.kind_by_out[idx] = run[i] ? DK_R : DK_A;  // (the run flags need only R / not R)
    }
    idx += keep[i];
    off += len[i];
  }
  if (tile == ntiles - 1 && threadIdx.x < 64) {
    // every earlier tile is published (its status was read as aggregate or inclusive,
    // with acquire): sum the tile cardinalities
    unsigned long long cs = threadIdx.x == 0 ? tot_card : 0;
    for (uint32_t i = threadIdx.x; i < tile; i += 64)
      cs += __hip_atomic_load(oc.tile_card + i, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    for (int o = 32; o > 0; o >>= 1) cs += __shfl_xor(cs, o, 64);
    if (threadIdx.x == 0) {
      reinterpret_cast<unsigned long long*>(oc.err)[kCardWord] = cs;
      // totals word where the header kernels look for it (status[n_tasks - 1])
      const uint64_t incl = __hip_atomic_load(oc.tile_status + tile, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __hip_atomic_store(oc.status + nt - 1, incl, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      write_info(info, oc, (uint32_t)((incl >> 44) & 0x1FFFF), (uint32_t)((incl >> 61) & 1), incl & ((1ULL << 44) - 1));
      if (oc.layout_out) {
        oc.layout_out[0] = (int64_t)((incl >> 44) & 0x1FFFF);
        oc.layout_out[1] = (int64_t)(incl & ((1ULL << 44) - 1));
        oc.layout_out[2] = (int64_t)((incl >> 61) & 1);
      }
    }
  }
}

// ===========================================================================
// placement + serialization of a pairwise result in one launch (round 6).  The compute kernel
// summed every tile of kAggTile records as it wrote them (OutCtx::tile_agg, agg_pack), so a
// tile's place in the output is a prefix over <= 1024 tile sums that every workgroup reads at
// once: no look-back chain between tiles and no k_place launch.  One workgroup per tile:
//   all threads : exclusive prefix of the tile sums (containers, payload bytes) and the totals;
//   every wave  : the tile's records -> output index and payload offset (wave scans), then the
//                 payload copies of records w, w + 8, ... (w_copy);
//   wave 0      : first the records' placement written back (like k_place), the descriptor and
//                 offset-table entries, and the run-flag bytes whose first container is in the tile
//                 (the last byte's tail from the next tiles' records);
//   workgroup 0 : cookie, ResultInfo, totals word, result cardinality and device layout.
// ===========================================================================
constexpr int kAggThreads = 512;  // 8 waves: 8 payload copies each (4 waves of 16: 9 % slower serialization)
__device__ __forceinline__ uint64_t wave_or64(uint64_t v) {
  for (int o = 32; o > 0; o >>= 1) v |= __shfl_xor(v, o, 64);
  return v;
}

// 64 VGPRs (8 waves per SIMD): all 1024 workgroups of a 65,536-record result resident at once (at the
// compiler's 77 VGPRs, 6 waves per SIMD, a quarter of them ran as a second round: +14 us)
__global__ __launch_bounds__(kAggThreads) __attribute__((amdgpu_waves_per_eu(8))) void k_serialize_agg(const uint32_t* __restrict__ n_tasks, OutCtx oc,
                                                       ResultInfo* __restrict__ info) {
  __shared__ uint8_t tcount[kMaxAggTiles];
  constexpr int kW = kAggThreads / 64;
  __shared__ uint32_t red[5][kW];
  __shared__ unsigned long long red_card[kW];
  __shared__ unsigned long long s_off[kW][kAggTile], s_src[kW][kAggTile];
  __shared__ uint32_t s_len[kW][kAggTile];
  const uint32_t nt = *n_tasks;
  const uint32_t ntiles = (nt + kAggTile - 1) / kAggTile;
  const uint32_t T = blockIdx.x;
  if (T != 0 && T >= ntiles) return;
  const int lane = threadIdx.x & 63, w = (int)uni(threadIdx.x >> 6);  // (w in an SGPR: scalar copy loop)
  // prefix (tiles < T) and totals of the tile sums
  // (payload bytes of a result fit 32 bits: <= 65,536 x 8 KiB; its cardinality does not)
  uint32_t pc = 0, pb = 0, tc = 0, tb = 0, tr = 0;
  unsigned long long tcard = 0;
  for (uint32_t i = threadIdx.x; i < ntiles; i += blockDim.x) {
    const unsigned long long a = oc.tile_agg[i];
    const uint32_t c = agg_count(a), b = agg_bytes(a);
    tcount[i] = (uint8_t)c;
    if (i < T) {
      pc += c;
      pb += b;
    }
    tc += c;
    tb += b;
    tr += agg_runs(a);
    tcard += agg_card(a);
  }
  for (int o = 32; o > 0; o >>= 1) {
    pc += __shfl_xor(pc, o, 64);
    pb += __shfl_xor(pb, o, 64);
    tc += __shfl_xor(tc, o, 64);
    tb += __shfl_xor(tb, o, 64);
    tr += __shfl_xor(tr, o, 64);
    tcard += __shfl_xor(tcard, o, 64);
  }
  if (lane == 0) {
    red[0][w] = pc;
    red[1][w] = pb;
    red[2][w] = tc;
    red[3][w] = tb;
    red[4][w] = tr;
    red_card[w] = tcard;
  }
  __syncthreads();
  uint32_t sum[5] = {0, 0, 0, 0, 0};
#pragma unroll
  for (int j = 0; j < 5; j++)
#pragma unroll
    for (int i = 0; i < kW; i++) sum[j] += red[j][i];
  pc = sum[0];
  pb = sum[1];
  const uint32_t size = (uint32_t)sum[2];
  const uint64_t bytes = sum[3];
  const uint32_t has_run = sum[4] != 0;
  const uint64_t H = header_bytes(size, has_run);
  uint8_t* base = oc.out + oc.payload_base - H;
  if (T == 0 && threadIdx.x == 0) {
    write_cookie(base, size, has_run);
    write_info(info, oc, size, has_run, bytes);
    if (nt > 0) {
      // the result's long cardinality and the totals word, where k_place leaves them
      unsigned long long card = 0;
      for (int i = 0; i < kW; i++) card += red_card[i];
      reinterpret_cast<unsigned long long*>(oc.err)[kCardWord] = card;
      __hip_atomic_store(oc.status + nt - 1, lb_pack(2, has_run, size, bytes), __ATOMIC_RELAXED,
                         __HIP_MEMORY_SCOPE_AGENT);
    }
    if (oc.layout_out) {
      oc.layout_out[0] = (int64_t)size;
      oc.layout_out[1] = (int64_t)bytes;
      oc.layout_out[2] = (int64_t)has_run;
    }
  }
  if (T >= ntiles) return;
  // every wave scans the tile's records itself (lane = record; 2 KiB from L2), so no wave waits for another
  // before its copies
  const uint32_t t = T * kAggTile + lane;
  const bool in = t < nt;
  ORec r{};
  if (in) r = oc.recs[t];
  const int keep = in && r.keep;
  const uint32_t len = keep ? r.ser_len : 0u;
  int tk, tb_;
  const int ek = wave_excl(keep, &tk);
  const int eb = wave_excl((int)len, &tb_);  // <= 64 x 8 KiB
  const uint64_t off = (uint64_t)pb + (uint64_t)eb;
  // the copy list through the wave's own LDS rows (held in registers across w_copy they spilled)
  s_off[w][lane] = off;
  s_src[w][lane] = r.src;
  s_len[w][lane] = len;
  if (w == 0) {
    const uint32_t idx = pc + (uint32_t)ek;
    if (in) {
      oc.recs[t].idx = idx;
      oc.recs[t].off = off;
    }
    if (keep) {
      const uint64_t desc_base = has_run ? 4 + (size + 7) / 8 : 8;
      *(g_u32*)(base + desc_base + 4ull * idx) = (uint32_t)r.key | ((r.card - 1) << 16);
      if (!has_run || size >= 4) *(g_u32*)(base + desc_base + 4ull * size + 4ull * idx) = (uint32_t)(H + off);
    }
    if (has_run && tk > 0) {
      // run flags of this tile's containers [first, e), in output order
      const uint32_t first = pc, e = first + (uint32_t)tk;
      const uint64_t runs = wave_or64(keep && r.kind == DK_R ? 1ull << ek : 0ull);
      const uint32_t b0 = (first + 7) / 8, b1 = (e - 1) / 8;  // the bytes that start in this tile
      uint64_t ahead = 0;  // run flags of the containers after e that share byte b1
      if (b1 >= b0 && (e & 7) != 0 && e < size) {
        const uint32_t need = min(8u - (e & 7), size - e);
        uint32_t got = 0;
        for (uint32_t u = T + 1; got < need && u < ntiles; u++) {
          if (tcount[u] == 0) continue;
          const uint32_t tu = u * kAggTile + lane;
          const bool k2 = tu < nt && oc.recs[tu].keep;
          const bool r2 = k2 && oc.recs[tu].kind == DK_R;
          int t2;
          const int e2 = wave_excl(k2 ? 1 : 0, &t2);
          ahead |= wave_or64(r2 && got + e2 < 8 ? 1ull << (got + e2) : 0ull);
          got += (uint32_t)t2;
        }
      }
      if (b1 >= b0 && (uint32_t)lane <= b1 - b0) {
        const uint32_t b = b0 + lane;
        uint32_t v = 0;
        for (uint32_t k = 0; k < 8; k++) {
          const uint32_t o = 8 * b + k;
          if (o >= size) break;
          const uint32_t rank = o - first;
          const uint32_t bit = rank < (uint32_t)tk ? (uint32_t)(runs >> rank) & 1u
                                                   : (uint32_t)(ahead >> (rank - (uint32_t)tk)) & 1u;
          v |= bit << k;
        }
        base[4 + b] = (uint8_t)v;
      }
    }
  }
  wsync();
  uint8_t* pay = oc.out + oc.payload_base;
  for (int i = w; i < kAggTile; i += kW) {
    const uint32_t n = uni(s_len[w][i]);
    if (n == 0) continue;
    w_copy(pay + uni64(s_off[w][i]), reinterpret_cast<const uint8_t*>(uni64(s_src[w][i])), n);
  }
}

// payload copies of the scan placement (key-shard fetch): one wave per task (grid-stride)
// dst: the payload region (a key shard's place in a global bitmap)
__global__ __launch_bounds__(256) void k_emit(const uint32_t* __restrict__ n_tasks, OutCtx oc, uint8_t* __restrict__ dst) {
  const uint32_t nt = *n_tasks;
  const uint32_t nw = gridDim.x * (blockDim.x >> 6);
  for (uint32_t t = uni(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)); t < nt; t += nw) {
    const ORec& r = oc.recs[t];
    if (!uni(r.keep)) continue;
    w_copy(dst + uni64(r.off), reinterpret_cast<const uint8_t*>(uni64(r.src)), uni(r.ser_len));
  }
}

// Key-shard placement: this shard's descriptors, its entries of the
// global offset table (global header bytes + the shard's payload base + local offset) and
// one run-flag byte per container, written straight into the caller's buffers.
__global__ __launch_bounds__(256) void k_shard_table(const uint32_t* __restrict__ n_tasks, OutCtx oc, uint64_t off0,
                                                     uint8_t* __restrict__ desc, uint8_t* __restrict__ offs,
                                                     uint8_t* __restrict__ runb) {
  const uint32_t nt = *n_tasks;
  for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < nt; t += gridDim.x * blockDim.x) {
    const ORec r = oc.recs[t];
    if (!r.keep) continue;
    const uint32_t idx = r.idx;
    const uint64_t roff = r.off;
    const uint32_t d = (uint32_t)r.key | ((r.card - 1) << 16);
    for (int k = 0; k < 4; k++) desc[4ull * idx + k] = (uint8_t)(d >> (8 * k));
    if (offs) {
      const uint32_t o = (uint32_t)(off0 + roff);
      for (int k = 0; k < 4; k++) offs[4ull * idx + k] = (uint8_t)(o >> (8 * k));
    }
    if (runb) runb[idx] = r.kind == DK_R ? 1 : 0;
  }
}

// The same placement with the global layout read from device memory (an all-gather's output:
// world x {containers, payload bytes, has_run} int64, ranks in key-range order), so a sharded
// op needs no host round trip between its compute and its slice's place in the global bitmap.
// `out` is laid out as the whole global bitmap; this rank writes its descriptors, offset-table
// entries and payload there, one run byte per container into runb, and rank 0 the cookie
// (RB/RoaringArray.java:896-940; the run-flag bitset is packed once every rank's bytes are in).
struct ShardGeo {
  uint64_t total, first, base, header, desc_base, off_base;
  uint32_t has_run, offsets;
};
__device__ __forceinline__ ShardGeo shard_geo(const int64_t* __restrict__ lay, int rank, int world) {
  ShardGeo g{};
  for (int i = 0; i < world; i++) {
    const uint64_t n = (uint64_t)lay[3 * i], p = (uint64_t)lay[3 * i + 1];
    g.total += n;
    g.has_run |= lay[3 * i + 2] != 0;
    if (i < rank) {
      g.first += n;
      g.base += p;
    }
  }
  g.header = header_bytes((uint32_t)g.total, g.has_run);
  g.desc_base = g.has_run ? 4 + (g.total + 7) / 8 : 8;
  g.offsets = !g.has_run || g.total >= 4;
  g.off_base = g.desc_base + 4 * g.total;
  return g;
}
// One launch: one wave per record copies its payload (when `emit`) and its lane 0 writes the
// descriptor, offset-table entry and run byte; rank 0 also the cookie.
__global__ __launch_bounds__(256) void k_shard_dyn(const uint32_t* __restrict__ n_tasks, OutCtx oc,
                                                   const int64_t* __restrict__ lay, int rank, int world,
                                                   uint8_t* __restrict__ out, uint8_t* __restrict__ runb, int emit) {
  const ShardGeo g = shard_geo(lay, rank, world);
  const uint32_t nt = *n_tasks;
  if (rank == 0 && blockIdx.x == 0 && threadIdx.x < 8) {  // the cookie (RB/RoaringArray.java:900-901,918-921)
    const uint32_t c0 = g.has_run ? 12347u | ((uint32_t)(g.total - 1) << 16) : 12346u;
    const uint32_t w = threadIdx.x < 4 ? c0 : (uint32_t)g.total;
    if (threadIdx.x < 4 || !g.has_run) out[threadIdx.x] = (uint8_t)(w >> (8 * (threadIdx.x & 3)));
  }
  uint8_t* dst = out + g.header + g.base;
  const uint32_t nw = gridDim.x * (blockDim.x >> 6);
  for (uint32_t t = uni(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)); t < nt; t += nw) {
    const ORec& r = oc.recs[t];
    if (!uni(r.keep)) continue;
    if (emit) w_copy(dst + uni64(r.off), reinterpret_cast<const uint8_t*>(uni64(r.src)), uni(r.ser_len));
    const int l = lane_id();
    if (l < 4) {
      const uint64_t idx = g.first + r.idx;
      const uint32_t d = (uint32_t)r.key | ((r.card - 1) << 16);
      out[g.desc_base + 4 * idx + l] = (uint8_t)(d >> (8 * l));
      if (g.offsets) {
        const uint32_t o = (uint32_t)(g.header + g.base + r.off);
        out[g.off_base + 4 * idx + l] = (uint8_t)(o >> (8 * l));
      }
      if (runb && l == 0) runb[idx] = r.kind == DK_R ? 1 : 0;
    }
  }
}
// x1.or(x2) in place (RB/RoaringBitmap.java:2481-2523): Container.ior types like the static or,
// except BitmapContainer.ior(ArrayContainer) (RB/BitmapContainer.java:740-757), which keeps a full
// result a bitmap: such keys' R.full records become an 8 KiB bitmap of ones.  Runs after the OR's
// compute kernel, before placement.  koa / kob: the operands' key CSR (one container per key).
__global__ __launch_bounds__(256) void k_ior_fix(const uint32_t* __restrict__ n_tasks, ORec* __restrict__ recs,
                                                 const uint32_t* __restrict__ koa, const CDesc* __restrict__ da,
                                                 const uint32_t* __restrict__ kob, const CDesc* __restrict__ db,
                                                 const uint8_t* __restrict__ ones) {
  const uint32_t nt = *n_tasks;
  for (uint32_t t = blockIdx.x * blockDim.x + threadIdx.x; t < nt; t += gridDim.x * blockDim.x) {
    const ORec r = recs[t];
    if (!r.keep || r.kind != DK_R || r.card != 65536) continue;
    const uint32_t ia = koa[r.key], ib = kob[r.key];
    if (koa[r.key + 1] == ia || kob[r.key + 1] == ib) continue;
    if (da[ia].kind == DK_B && db[ib].kind == DK_A) {
      recs[t].kind = DK_B;
      recs[t].src = reinterpret_cast<uint64_t>(ones);
      recs[t].ser_len = 8192;
    }
  }
}
void launch_ior_fix(hipStream_t s, const uint32_t* nt, ORec* recs, const uint32_t* koa, const CDesc* da,
                    const uint32_t* kob, const CDesc* db, const uint8_t* ones) {
  hipLaunchKernelGGL(k_ior_fix, dim3(256), dim3(256), 0, s, nt, recs, koa, da, kob, db, ones);
}

// the pending result's (containers, payload bytes, has_run) as int64, from k_place's ResultInfo
__global__ void k_layout_out(const ResultInfo* __restrict__ info, int64_t* __restrict__ dst) {
  if (threadIdx.x == 0) {
    dst[0] = (int64_t)info->n_out;
    dst[1] = (int64_t)info->payload;
    dst[2] = (int64_t)info->has_run;
  }
}

// ===========================================================================
// slot gather (batch fetch): one wave per slot, into a contiguous download buffer
// ===========================================================================
__global__ __launch_bounds__(256) void k_gather(const GatherItem* __restrict__ items, uint64_t n,
                                                const uint8_t* __restrict__ src, uint8_t* __restrict__ dst) {
  const uint64_t nw = (uint64_t)gridDim.x * 4;
  for (uint64_t i = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6); i < n; i += nw) {
    const GatherItem it = items[i];
    group_copy<64>(dst + it.dst, src + it.src, (uint32_t)it.len, lane_id());
  }
}

// ===========================================================================
// host launchers
// ===========================================================================

int resident_grid(const void* kernel, int block) {
  static std::mutex mu;
  static std::unordered_map<const void*, int> cache;  // kernels launch with one block size each
  std::lock_guard<std::mutex> g(mu);
  auto it = cache.find(kernel);
  if (it != cache.end()) return it->second;
  int dev = 0, cus = 0, per_cu = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  (void)hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kernel, block, 0);
  const int r = std::max(1, cus) * std::max(1, per_cu);
  cache[kernel] = r;
  return r;
}

static inline int clamp_grid(int grid, const void* kernel) { return std::max(1, std::min(grid, resident_grid(kernel))); }
void launch_plan_wide(hipStream_t s, int mode, const uint32_t* key_off, uint32_t n_req, int key_lo, int key_hi,
                      Task* by_key, uint8_t* flag, uint32_t* wg_count, uint64_t* zlb, uint64_t* ztile) {
  hipLaunchKernelGGL(k_plan_wide, dim3(256), dim3(256), 0, s, mode, key_off, n_req, key_lo, key_hi, by_key, flag,
                     wg_count, zlb, ztile);
}
void launch_compact(hipStream_t s, const uint8_t* flag, const Task* by_key, const uint32_t* wg_count, Task* tasks,
                    uint32_t* n_tasks) {
  hipLaunchKernelGGL(k_compact<Task>, dim3(256), dim3(256), 0, s, flag, by_key, wg_count, tasks, n_tasks);
}

void launch_place(hipStream_t s, const uint32_t* nt, OutCtx oc, ResultInfo* info) {
  hipLaunchKernelGGL(k_place, dim3(65536 / kTile), dim3(256), 0, s, nt, oc, info, 0u);
}
void launch_place_tiles(hipStream_t s, const uint32_t* nt, OutCtx oc, ResultInfo* info, uint32_t t_lo, uint32_t t_hi) {
  const uint32_t tl = t_lo / kTile, th = (t_hi + kTile - 1) / kTile;
  if (th > tl) hipLaunchKernelGGL(k_place, dim3(th - tl), dim3(256), 0, s, nt, oc, info, tl);
}
void launch_serialize_agg(hipStream_t s, const uint32_t* nt, OutCtx oc, ResultInfo* info, size_t max_tasks) {
  const size_t tiles = std::min<size_t>((max_tasks + kAggTile - 1) / kAggTile, kMaxAggTiles);
  hipLaunchKernelGGL(k_serialize_agg, dim3((unsigned)std::max<size_t>(1, tiles)), dim3(kAggThreads), 0, s, nt, oc, info);
}
void launch_spec_fix(hipStream_t s, const uint32_t* nt, OutCtx oc) {
  hipLaunchKernelGGL(k_spec_fix, dim3(std::max(1, resident_grid((const void*)&k_spec_fix))), dim3(256), 0, s, nt, oc);
}
void launch_serialize(hipStream_t s, const uint32_t* nt, OutCtx oc) {
  hipLaunchKernelGGL(k_serialize<3>, dim3(std::max(1, resident_grid((const void*)&k_serialize<3>))), dim3(256), 0, s, nt,
                     oc, (const uint8_t*)oc.kind_by_out, 0u, 0xFFFFFFFFu);
}
void launch_serialize_part(hipStream_t s, const uint32_t* nt, OutCtx oc, int part, uint32_t t_lo, uint32_t t_hi,
                           int grid) {
  if (part == 1) {
    hipLaunchKernelGGL(k_serialize<1>, dim3(std::max(1, std::min(grid, 256))), dim3(256), 0, s, nt, oc,
                       (const uint8_t*)oc.kind_by_out, t_lo, t_hi);
  } else {
    const int g = std::max(1, std::min(grid, resident_grid((const void*)&k_serialize<2>)));
    hipLaunchKernelGGL(k_serialize<2>, dim3(g), dim3(256), 0, s, nt, oc, (const uint8_t*)oc.kind_by_out, t_lo, t_hi);
  }
}
void launch_serialize_shard(hipStream_t s, int grid, const uint32_t* nt, OutCtx oc, uint8_t* payload_dst, uint64_t off0,
                            uint8_t* desc, uint8_t* offs, uint8_t* runb) {
  if (payload_dst)
    hipLaunchKernelGGL(k_emit, dim3(std::max(1, resident_grid((const void*)&k_emit))), dim3(256), 0, s, nt, oc,
                       payload_dst);
  hipLaunchKernelGGL(k_shard_table, dim3(grid), dim3(256), 0, s, nt, oc, off0, desc, offs, runb);
}
void launch_serialize_shard_dyn(hipStream_t s, int grid, const uint32_t* nt, OutCtx oc, const int64_t* lay, int rank,
                                int world, uint8_t* out, uint8_t* runb, bool emit) {
  (void)grid;
  hipLaunchKernelGGL(k_shard_dyn, dim3(std::max(1, resident_grid((const void*)&k_shard_dyn))), dim3(256), 0, s, nt, oc,
                     lay, rank, world, out, runb, emit ? 1 : 0);
}
void launch_layout_out(hipStream_t s, const ResultInfo* info, int64_t* dst) {
  hipLaunchKernelGGL(k_layout_out, dim3(1), dim3(64), 0, s, info, dst);
}
void launch_reduce_card(hipStream_t s, const uint32_t* task_card, const uint32_t* nt, ResultInfo* info,
                        const uint32_t* err) {
  hipLaunchKernelGGL(k_reduce_card, dim3(1), dim3(1024), 0, s, task_card, nt, info, err);
}
void launch_batch_bytes(hipStream_t s, const CDesc* desc, uint64_t n, const uint8_t* payload,
                        unsigned long long* out) {
  uint64_t g = (n + 255) / 256;
  if (g > 4096) g = 4096;
  if (g == 0) return;
  hipLaunchKernelGGL(k_batch_bytes, dim3((unsigned)g), dim3(256), 0, s, desc, n, payload, out);
}

void launch_gather(hipStream_t s, const GatherItem* items, uint64_t n, const uint8_t* src, uint8_t* dst) {
  if (!n) return;
  const unsigned g = (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((n + 3) / 4, 8192));
  hipLaunchKernelGGL(k_gather, dim3(g), dim3(256), 0, s, items, n, src, dst);
}

}  // namespace rbg
