// RoaringBitmap.orNot on the MI355X: the static RoaringBitmap.orNot(x1, x2, rangeEnd)
// (RB/RoaringBitmap.java:1521-1603) and x1.orNot(x2, rangeEnd) in place (:1431-1506).
//
// Per key k <= maxKey = (rangeEnd - 1) >>> 16, with end = lastRun at maxKey, else 65536:
//   x1 and x2 : c1.orNot(c2, end) = c1.or(c2.not(0, end).iremove(end, 0x10000)) (RB/Container.java
//               :191-196; the in-place form iorNot :536-541 ends in ior)
//   x1 only   : full, or c1.ior(rangeOfOnes(0, lastRun)) at maxKey
//   x2 only   : c2.not(0, end) -- not clipped at rangeEnd
//   neither   : full, or rangeOfOnes(0, lastRun) at maxKey
// empty results dropped; then x1's containers above maxKey, as they are.  The reference sizes its
// key array with maxSize = min(maxKey + 1 + remainder - correction + |x1|, 65536) and stops the key
// loop once that many containers are out -- which can cut the result short (correction counts full
// x2 containers, some of which sit under an x1 container); k_ornot_scan computes the same bound.
//
//   k_ornot_scan : one workgroup: remainder, correction, maxSize, and the number of keys the loop
//                  reaches (an exact walk only when maxSize < maxKey + 1)
//   k_plan_ornot : one thread per key (the pairwise plan's compaction): the reached keys [0, k_end)
//                  and x1's keys above maxKey, in key order
//   k_ornot      : one wave per task; the container in registers (wave.hpp), typed as the
//                  reference's chain: not() -> iremove -> or / ior.  Full containers (the bulk of a
//                  dense result) reference one constant run payload; nothing is staged for them.
#include <algorithm>
#include <cstdio>
#include <cstdlib>

#include "kernels.hpp"
#include "wave.hpp"

namespace rbg {

// serialized payload of RunContainer.full() (RB/RunContainer.java:1663-1665): nruns = 1, (0, 65535);
// slack after it for the serializer's 16 B over-read
__device__ uint16_t g_full_run[16] = {1, 0, 0xFFFF};

// 1024-thread block sum / inclusive scan (LDS `red` of 17 ints)
__device__ __forceinline__ int ornot_block_sum(int v, int* red) {
  v = wave_sum_i(v);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  int s = 0;
#pragma unroll
  for (int i = 0; i < 16; i++) s += red[i];
  __syncthreads();
  return s;
}
__device__ __forceinline__ int ornot_block_incl(int v, int* red, int* total) {
  const int incl = dpp_incl_scan(v);
  if ((threadIdx.x & 63) == 63) red[threadIdx.x >> 6] = incl;
  __syncthreads();
  int before = 0, s = 0;
  const int w = threadIdx.x >> 6;
#pragma unroll
  for (int i = 0; i < 16; i++) {
    before += i < w ? red[i] : 0;
    s += red[i];
  }
  __syncthreads();
  *total = s;
  return before + incl;
}

// RB/RoaringBitmap.java:1527-1548 (static) / :1436-1458 (in place): remainder = x1's keys above
// maxKey; correction = full x2 containers among indices [0, |x2| - remainder), up to and including the
// first key >= maxKey; maxSize.  The loop `for key <= maxKey && size < maxSize` reaches key k iff the
// non-empty results before k number fewer than maxSize; a result is empty only for an x2-only full
// container below maxKey (its complement), so that count is k - E(k), E(k) = such keys below k.
__global__ __launch_bounds__(1024) void k_ornot_scan(const uint32_t* __restrict__ koa, int na,
                                                     const uint32_t* __restrict__ kob, const CDesc* __restrict__ db,
                                                     int nb, int max_key, OrNotPlan* __restrict__ plan) {
  __shared__ int red[17];
  const int th = threadIdx.x;
  const int rem = na - (int)koa[max_key + 1];
  const int lim = nb - rem;
  int last = -1;
  if (lim > 0) last = min(max_key < 0 ? 0 : (int)kob[max_key], lim - 1);
  int c = 0;
  for (int i = th; i <= last; i += 1024) c += db[i].card == 65536u;
  const int corr = ornot_block_sum(c, red);
  const int max_size = min(max_key + 1 + rem - corr + na, 65536);
  int k_end = max_key + 1;
  if (max_size < 0) {
    k_end = 0;
  } else if (max_size < max_key + 1) {  // the bound can bind: walk the keys in 1024-key segments
    int e_before = 0, reached = 0;
    for (int s0 = 0; s0 <= max_key; s0 += 1024) {
      const int k = s0 + th;
      int e = 0;
      if (k < max_key) {
        const uint32_t b0 = kob[k];
        e = kob[k + 1] > b0 && koa[k + 1] == koa[k] && db[b0].card == 65536u;
      }
      int tot;
      const int incl = ornot_block_incl(e, red, &tot);
      const int nonempty_before = k - (e_before + incl - e);
      reached += ornot_block_sum(k <= max_key && nonempty_before < max_size, red);
      e_before += tot;
    }
    k_end = reached;
  }
  if (th == 0) {
    plan->k_end = k_end;
    plan->neg = max_size < 0 ? 1 : 0;
    plan->max_size = max_size;
    plan->correction = corr;
  }
}

// one thread per key: tasks for the keys the loop reaches and for x1's keys above maxKey
__global__ __launch_bounds__(256) void k_plan_ornot(const uint32_t* __restrict__ koa, const CDesc* __restrict__ da,
                                                    const uint8_t* __restrict__ pa, const uint32_t* __restrict__ kob,
                                                    const CDesc* __restrict__ db, const uint8_t* __restrict__ pb,
                                                    int max_key, const OrNotPlan* __restrict__ plan,
                                                    uint64_t* __restrict__ wg_epoch, uint32_t epoch,
                                                    PTask* __restrict__ tasks, uint32_t* __restrict__ n_tasks,
                                                    uint64_t* zlb, uint64_t* ztile, uint32_t* err) {
  plan_zero(zlb, ztile);
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  PTask t;
  resolve(koa, da, pa, k, t.slot_a, t.card_a, t.kind_a, t.nruns_a);
  resolve(kob, db, pb, k, t.slot_b, t.card_b, t.kind_b, t.nruns_b);
  t.key = (uint16_t)k;
  const int k_end = plan->k_end;
  int f = (int)k < k_end || ((int)k > max_key && t.kind_a != kAbsent);
  if (plan->neg) f = 0;
  plan_emit(f, t, wg_epoch, epoch, tasks, n_tasks, err);
}

// bits [0, e) of container word w
__device__ __forceinline__ uint64_t prefix_mask(int w, int e) {
  const int lo = 64 * w;
  if (e >= lo + 64) return ~0ull;
  if (e <= lo) return 0ull;
  return (1ull << (e - lo)) - 1;
}
// ... of register k of the wave layout (WCtr: w[2 i + j] = word 128 i + 2 lane + j)
__device__ __forceinline__ uint64_t wprefix(int k, int e) {
  return prefix_mask(128 * (k >> 1) + 2 * lane_id() + (k & 1), e);
}

// One task, one wave (20 waves per CU in flight: the per-task chain is a few dependent memory
// latencies, so the task rate comes from the waves in flight).  Result types:
//  * c2.not(0, e): ArrayContainer.not (RB/ArrayContainer.java:876-925, through toBitmapContainer().not
//    above 4096 values) and BitmapContainer.not = clone().inot (RB/BitmapContainer.java:994-997, 679-687)
//    give an array at <= 4096 values, else a bitmap; RunContainer.not (RB/RunContainer.java:1900-1918)
//    ends in toEfficientContainer;
//  * .iremove(e, 0x10000) (both present, e < 65536): an array stays an array, a bitmap becomes one at
//    <= 4096 values (RB/BitmapContainer.java:788-802), a run container stays one; BUF: the buffer
//    package's MappeableBitmapContainer.iremove converts only below 4096 values
//    (RB/buffer/MappeableBitmapContainer.java:1003-1017), so a 4096-value bitmap keeps its words;
//  * rangeOfOnes(0, e) (RB/Container.java:29-37): an array up to 2 values, else a run container;
//  * c1.or / c1.ior of that: the pairwise OR rule (device.hpp); Container.ior's one difference,
//    BitmapContainer.ior(ArrayContainer) keeping a full bitmap (RB/BitmapContainer.java:740-757),
//    applies to x1-only at maxKey in both forms and to both-present in the in-place form.
template <bool INPLACE, bool BUF>
__device__ __forceinline__ void ornot_task(uint32_t t, const PTask& tk, const uint8_t* pa, const uint8_t* pb,
                                           int max_key, int last_run, const OutCtx& oc, uint32_t* lds) {
  const int key = tk.key;
  const bool ia = tk.kind_a != kAbsent, ib = tk.kind_b != kAbsent;
  if (key > max_key) {  // x1's containers above the range, appended as they are (:1493-1500 / :1588-1596)
    const uint32_t len = tk.kind_a == DK_A ? 2u * tk.card_a : tk.kind_a == DK_B ? 8192u : 2u + 4u * tk.nruns_a;
    w_place(t, true, pa + tk.slot_a + (tk.kind_a == DK_R ? 2 : 0), false, lds, len, tk.card_a, (uint32_t)key,
            tk.kind_a, oc);
    return;
  }
  const int e = key == max_key ? last_run : 65536;
  if (!ib && e == 65536) {
    // RunContainer.full(); at maxKey with lastRun = 0x10000, x1's c1.ior(full run) and the full
    // rangeOfOnes are full run containers as well (RunContainer.or / BitmapContainer.ior(RunContainer) /
    // RunContainer.ior return full() on a full union)
    w_place(t, true, reinterpret_cast<const uint8_t*>(g_full_run), false, lds, 6, 65536, (uint32_t)key, DK_R, oc);
    return;
  }
  if (!ia && !ib) {  // rangeOfOnes(0, lastRun) at maxKey, written by lane 0
    uint8_t* slot = oc.scratch + (size_t)t * kSlotBytes;
    const bool arr = e <= 2;
    uint16_t* p = reinterpret_cast<uint16_t*>(arr ? slot : slot + 2);
    if (lane_id() == 0) {
      if (arr) {
        p[0] = 0;
        p[1] = 1;
      } else {
        p[0] = 1;
        p[1] = 0;
        p[2] = (uint16_t)(e - 1);
      }
    }
    w_place(t, true, reinterpret_cast<const uint8_t*>(p), false, lds, arr ? 2u * e : 6u, (uint32_t)e, (uint32_t)key,
            arr ? DK_A : DK_R, oc);
    return;
  }
  WCtr x, y;
  const int kx = ia ? tk.kind_a : DK_A, cx = ia ? (int)tk.card_a : 0;
  if (ia) w_materialize(CDesc{tk.slot_a, tk.card_a, tk.key, tk.kind_a, 0}, pa, lds, x);
  int ky, cy;
  if (ib) {
    w_materialize(CDesc{tk.slot_b, tk.card_b, tk.key, tk.kind_b, 0}, pb, lds, y);
#pragma unroll
    for (int k = 0; k < 16; k++) y.w[k] ^= wprefix(k, e);
    cy = w_card(y);
    ky = tk.kind_b == DK_R ? eff(cy, w_runs(y)) : by_card(cy);
    if (ia && e < 65536) {
#pragma unroll
      for (int k = 0; k < 16; k++) y.w[k] &= wprefix(k, e);
      cy = w_card(y);
      if (ky == DK_B && (BUF ? cy < 4096 : cy <= 4096)) ky = DK_A;
    }
  } else {  // x1 only, maxKey: c1.ior(rangeOfOnes(0, e))
#pragma unroll
    for (int k = 0; k < 16; k++) y.w[k] = wprefix(k, e);
    cy = e;
    ky = e <= 2 ? DK_A : DK_R;
  }
  int kz, cz;
  if (ia) {
#pragma unroll
    for (int k = 0; k < 16; k++) x.w[k] |= y.w[k];
    cz = w_card(x);
    kz = pairwise_needs_runs(OPR_OR, kx, cx, ky, cy) ? eff(cz, w_runs(x)) : pairwise_kind(OPR_OR, kx, ky, cz);
    if ((INPLACE || !ib) && kx == DK_B && ky == DK_A) kz = DK_B;
  } else {  // x2 only: its complement, dropped when empty
    if (cy == 0) {
      w_place(t, false, nullptr, true, lds, 0, 0, (uint32_t)key, DK_A, oc);
      return;
    }
#pragma unroll
    for (int k = 0; k < 16; k++) x.w[k] = y.w[k];
    cz = cy;
    kz = ky;
  }
  if (kz == DK_B) {  // registers straight to the task's slot
    uint8_t* slot = oc.scratch + (size_t)t * kSlotBytes;
    w_store_bitmap(slot, x);
    w_place(t, true, slot, false, lds, 8192, (uint32_t)cz, (uint32_t)key, DK_B, oc);
    return;
  }
  const uint32_t len = w_stage(kz, x, cz, lds);
  w_place(t, true, nullptr, true, lds, len, (uint32_t)cz, (uint32_t)key, kz, oc);
}

constexpr int kOrnWaves = 4;

// INPLACE: x1.orNot (iorNot, ior); BUF: the buffer package's ImmutableRoaringBitmap.orNot /
// MutableRoaringBitmap.orNot (RB/buffer/ImmutableRoaringBitmap.java:484-548, MutableRoaringBitmap.java
// :962-1030).  Static wave stride over the task list; the next record is fetched while a task runs.
template <bool INPLACE, bool BUF>
__global__ __launch_bounds__(256, 3) void k_ornot(const PTask* __restrict__ tasks, const uint32_t* __restrict__ n_tasks,
                                               const uint8_t* pa, const uint8_t* pb, int max_key, int last_run,
                                               OutCtx oc) {
  __shared__ __align__(16) uint32_t lds_all[kOrnWaves][2048];
  const int w = threadIdx.x >> 6;
  uint32_t* lds = lds_all[w];
  const uint32_t nt = uni(*n_tasks);
  const uint32_t stride = gridDim.x * kOrnWaves;
  uint32_t t = uni(blockIdx.x * kOrnWaves + w);
  if (t >= nt) return;
  PTask cur = load_task(tasks, t);
  for (;;) {
    const uint32_t tn = t + stride;
    PTask nxt;
    if (tn < nt) nxt = load_task(tasks, tn);  // in flight while this task runs
    ornot_task<INPLACE, BUF>(t, cur, pa, pb, max_key, last_run, oc, lds);
    if (tn >= nt) break;
    t = tn;
    cur = nxt;
  }
}

void launch_ornot(hipStream_t s, const uint32_t* koa, const CDesc* da, const uint8_t* pa, int na, const uint32_t* kob,
                  const CDesc* db, const uint8_t* pb, int nb, int max_key, int last_run, int flags, OrNotPlan* plan,
                  uint64_t* wg_epoch, uint32_t epoch, PTask* tasks, uint32_t* n_tasks, OutCtx oc, uint64_t* zlb,
                  uint64_t* ztile, int grid) {
  hipLaunchKernelGGL(k_ornot_scan, dim3(1), dim3(1024), 0, s, koa, na, kob, db, nb, max_key, plan);
  hipLaunchKernelGGL(k_plan_ornot, dim3(256), dim3(256), 0, s, koa, da, pa, kob, db, pb, max_key, plan, wg_epoch,
                     epoch, tasks, n_tasks, zlb, ztile, oc.err);
  const int g0 = std::max(1, (grid + kOrnWaves - 1) / kOrnWaves);
#define RBG_ORNOT_LAUNCH(I, B)                                                                            \
  hipLaunchKernelGGL((k_ornot<I, B>), dim3(std::min(g0, resident_grid((const void*)&k_ornot<I, B>))), dim3(256), 0, \
                     s, tasks, n_tasks, pa, pb, max_key, last_run, oc)
  switch (flags & 3) {
    case 0: RBG_ORNOT_LAUNCH(false, false); break;
    case 1: RBG_ORNOT_LAUNCH(true, false); break;
    case 2: RBG_ORNOT_LAUNCH(false, true); break;
    default: RBG_ORNOT_LAUNCH(true, true); break;
  }
#undef RBG_ORNOT_LAUNCH
}

}  // namespace rbg
