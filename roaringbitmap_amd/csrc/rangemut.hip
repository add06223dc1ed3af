// Static range mutations on the MI355X: RoaringBitmap.add(rb, rangeStart, rangeEnd)
// (RB/RoaringBitmap.java:298-345), remove(rb, ...) (:995-1040), flip(rb, ...) (:626-668), and the
// buffer package's MutableRoaringBitmap.add / remove / flip (RB/buffer/MutableRoaringBitmap.java
// :152-205, 649-700, 455-505; ImmutableRoaringBitmap.flip :592-640).
//
// Keys outside [hbStart, hbLast] are cloned.  Inside, per key with the cut [lo, hi]:
//   add    : Container.add(lo, hi + 1) on the first / last key (a missing key: rangeOfOnes), a full run
//            container on every key between them
//   remove : Container.remove(lo, hi + 1) on the first / last key unless the cut covers the whole key;
//            the keys between (and fully covered ones) dropped, emptied containers dropped
//   flip   : Container.not(lo, hi + 1) on every key (a missing key: rangeOfOnes), emptied dropped
// Result types (the per-key container methods):
//   add    : ArrayContainer.add -> an array, or above 4096 values toBitmapContainer().iadd, a bitmap
//            (RB/ArrayContainer.java:103-135); BitmapContainer.add a bitmap, full included (:131-143);
//            RunContainer.add = clone().iadd, a run container whatever its size (RB/RunContainer.java:242)
//   remove : an array stays one; a bitmap becomes an array at <= 4096 values (RB/BitmapContainer.java
//            :1166-1181), the buffer package's below 4096 (RB/buffer/MappeableBitmapContainer.java
//            :1597-1612); a run container keeps its clipped runs
//   flip   : arrays / bitmaps by cardinality (ArrayContainer.not, BitmapContainer.inot), run containers
//            through toEfficientContainer (RB/RunContainer.java:1900-1918)
//   x.add(rangeStart, rangeEnd) in place (RB/RoaringBitmap.java:1181-1206, RB/buffer/MutableRoaringBitmap.java
//            :831-858): Container.iadd on every key of the range, the keys between included (an array there
//            becomes a full bitmap, a bitmap stays one, a run container a full run); the in-place remove and
//            flip end in the static forms' containers (iremove / inot keep remove / not's thresholds)
// Run results that stay run containers whatever their size (add / remove of an input with more than
// 2047 runs) go to the big-run arena (w_place_big_runs), as the buffer package's run AND results do.
//
//   k_plan_rmut : one thread per key (the pairwise plan's compaction), the keys that give a container
//   k_rmut      : one wave per task, the container in registers (wave.hpp)
#include <algorithm>
#include <cstdio>
#include <cstdlib>

#include "kernels.hpp"
#include "wave.hpp"

namespace rbg {

__device__ uint16_t g_full_run_rm[16] = {1, 0, 0xFFFF};  // RunContainer.full(); slack for the 16 B over-read

__device__ __forceinline__ void rmut_cut(int key, const RmutArgs& ra, int* lo, int* hi) {
  *lo = key == ra.hbs ? ra.lbs : 0;
  *hi = key == ra.hbl ? ra.lbl : 65535;
}

__global__ __launch_bounds__(256) void k_plan_rmut(const uint32_t* __restrict__ koa, const CDesc* __restrict__ da,
                                                   const uint8_t* __restrict__ pa, RmutArgs ra,
                                                   uint64_t* __restrict__ wg_epoch, uint32_t epoch,
                                                   PTask* __restrict__ tasks, uint32_t* __restrict__ n_tasks,
                                                   uint64_t* zlb, uint64_t* ztile, uint32_t* err) {
  plan_zero(zlb, ztile);
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  PTask t;
  resolve(koa, da, pa, k, t.slot_a, t.card_a, t.kind_a, t.nruns_a);
  t.slot_b = 0;
  t.card_b = 0;
  t.kind_b = kAbsent;
  t.nruns_b = 0;
  t.key = (uint16_t)k;
  const bool present = t.kind_a != kAbsent;
  const bool in = (int)k >= ra.hbs && (int)k <= ra.hbl;
  int f;
  if (ra.op == RMUT_LIMIT) {
    f = present && ((int)k < ra.hbs || ((int)k == ra.hbs && ra.lbs > 0));
  } else if (!in || ra.op == RMUT_DERUN) {
    f = present;
  } else if (ra.op == RMUT_REMOVE) {
    int lo, hi;
    rmut_cut((int)k, ra, &lo, &hi);
    f = present && !(lo == 0 && hi == 65535);
  } else {
    f = 1;
  }
  plan_emit(f, t, wg_epoch, epoch, tasks, n_tasks, err);
}

template <int OP, bool BUF>
__device__ __forceinline__ void rmut_task(uint32_t t, const PTask& tk, const uint8_t* pa, const RmutArgs& ra,
                                          const OutCtx& oc, const BigRuns& big, uint32_t* lds) {
  const int key = tk.key;
  const bool present = tk.kind_a != kAbsent;
  if (OP == RMUT_DERUN && tk.kind_a == DK_R) {  // RunContainer.toBitmapOrArrayContainer (RB/RunContainer.java:2300-2323)
    WCtr x;
    w_materialize(CDesc{tk.slot_a, tk.card_a, tk.key, tk.kind_a, 0}, pa, lds, x);
    const int c = (int)tk.card_a;
    if (c > 4096) {
      uint8_t* slot = oc.scratch + (size_t)t * kSlotBytes;
      w_store_bitmap(slot, x);
      w_place(t, true, slot, false, lds, 8192, (uint32_t)c, (uint32_t)key, DK_B, oc);
    } else {
      const uint32_t len = w_stage(DK_A, x, c, lds);
      w_place(t, true, nullptr, true, lds, len, (uint32_t)c, (uint32_t)key, DK_A, oc);
    }
    return;
  }
  if (OP == RMUT_LIMIT && key == ra.hbs) {  // Container.limit(lbs): the first lbs values
    WCtr x;
    w_materialize(CDesc{tk.slot_a, tk.card_a, tk.key, tk.kind_a, 0}, pa, lds, x);
    const int n = ra.lbs;
    int base = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      const int c0 = __popcll(x.w[2 * i]), c1 = __popcll(x.w[2 * i + 1]);
      int tot;
      const int p0 = base + wave_excl(c0 + c1, &tot);
      base += tot;
#pragma unroll
      for (int j = 0; j < 2; j++) {
        const int pre = p0 + (j ? c0 : 0), cw = j ? c1 : c0;
        uint64_t& w = x.w[2 * i + j];
        if (pre >= n) {
          w = 0;
        } else if (pre + cw > n) {  // keep the word's lowest n - pre set bits
          uint64_t rest = w;
          for (int q = 0; q < n - pre; q++) rest &= rest - 1;
          w ^= rest;
        }
      }
    }
    const int kind = tk.kind_a == DK_B ? by_card(n) : tk.kind_a;
    if (kind == DK_B) {
      uint8_t* slot = oc.scratch + (size_t)t * kSlotBytes;
      w_store_bitmap(slot, x);
      w_place(t, true, slot, false, lds, 8192, (uint32_t)n, (uint32_t)key, DK_B, oc);
      return;
    }
    if (kind == DK_R) {
      const int nr = w_runs(x);
      if (nr > 2047) {
        w_place_big_runs(t, (uint32_t)key, x, n, nr, oc, big, lds);
        return;
      }
    }
    const uint32_t len = w_stage(kind, x, n, lds);
    w_place(t, true, nullptr, true, lds, len, (uint32_t)n, (uint32_t)key, kind, oc);
    return;
  }
  if (OP == RMUT_DERUN || OP == RMUT_LIMIT || key < ra.hbs || key > ra.hbl) {  // cloned: outside the range,
                                                                                // not a run container, or kept whole
    const uint32_t len = tk.kind_a == DK_A ? 2u * tk.card_a : tk.kind_a == DK_B ? 8192u : 2u + 4u * tk.nruns_a;
    w_place(t, true, pa + tk.slot_a + (tk.kind_a == DK_R ? 2 : 0), false, lds, len, tk.card_a, (uint32_t)key,
            tk.kind_a, oc);
    return;
  }
  int lo, hi;
  rmut_cut(key, ra, &lo, &hi);
  constexpr bool ADD = OP == RMUT_ADD || OP == RMUT_ADD_INPLACE || OP == RMUT_RANGE;
  if ((OP == RMUT_ADD || OP == RMUT_RANGE) && key != ra.hbs && key != ra.hbl) {  // rangeOfOnes(0, 65536): a full run container
    w_place(t, true, reinterpret_cast<const uint8_t*>(g_full_run_rm), false, lds, 6, 65536, (uint32_t)key, DK_R, oc);
    return;
  }
  if (!present) {  // rangeOfOnes(lo, hi + 1) (add / flip), written by lane 0
    uint8_t* slot = oc.scratch + (size_t)t * kSlotBytes;
    const int n = hi - lo + 1;
    const bool arr = OP != RMUT_RANGE && n <= 2;  // Container.rangeOfOnes; bitmapOfRange: RunContainer's
    uint16_t* p = reinterpret_cast<uint16_t*>(arr ? slot : slot + 2);
    if (lane_id() == 0) {
      if (arr) {
        p[0] = (uint16_t)lo;
        p[1] = (uint16_t)hi;
      } else {
        p[0] = 1;
        p[1] = (uint16_t)lo;
        p[2] = (uint16_t)(hi - lo);
      }
    }
    w_place(t, true, reinterpret_cast<const uint8_t*>(p), false, lds, arr ? 2u * n : 6u, (uint32_t)n, (uint32_t)key,
            arr ? DK_A : DK_R, oc);
    return;
  }
  WCtr x;
  w_materialize(CDesc{tk.slot_a, tk.card_a, tk.key, tk.kind_a, 0}, pa, lds, x);
#pragma unroll
  for (int k = 0; k < 16; k++) {
    const uint64_t m = wrange(k, lo, hi);
    if (ADD) x.w[k] |= m;
    else if (OP == RMUT_REMOVE) x.w[k] &= ~m;
    else x.w[k] ^= m;
  }
  const int c = w_card(x);
  if (c == 0) {  // remove / flip emptied the container: dropped
    w_place(t, false, nullptr, true, lds, 0, 0, (uint32_t)key, DK_A, oc);
    return;
  }
  const int kx = tk.kind_a;
  int kind;
  if (ADD) kind = kx == DK_A ? by_card(c) : kx;
  else if (OP == RMUT_REMOVE) kind = kx == DK_B ? ((BUF ? c < 4096 : c <= 4096) ? DK_A : DK_B) : kx;
  else kind = kx == DK_R ? eff(c, w_runs(x)) : by_card(c);
  if (kind == DK_B) {  // registers straight to the task's slot
    uint8_t* slot = oc.scratch + (size_t)t * kSlotBytes;
    w_store_bitmap(slot, x);
    w_place(t, true, slot, false, lds, 8192, (uint32_t)c, (uint32_t)key, DK_B, oc);
    return;
  }
  if (kind == DK_R && OP != RMUT_FLIP) {
    const int nr = w_runs(x);
    if (nr > 2047) {
      w_place_big_runs(t, (uint32_t)key, x, c, nr, oc, big, lds);
      return;
    }
  }
  const uint32_t len = w_stage(kind, x, c, lds);
  w_place(t, true, nullptr, true, lds, len, (uint32_t)c, (uint32_t)key, kind, oc);
}

constexpr int kRmWaves = 4;

// one wave per task over a static stride, the next record fetched while a task runs
template <int OP, bool BUF>
__global__ __launch_bounds__(256, 4) void k_rmut(const PTask* __restrict__ tasks, const uint32_t* __restrict__ n_tasks,
                                              const uint8_t* pa, RmutArgs ra, OutCtx oc, BigRuns big) {
  __shared__ __align__(16) uint32_t lds_all[kRmWaves][2048];
  const int w = threadIdx.x >> 6;
  uint32_t* lds = lds_all[w];
  const uint32_t nt = uni(*n_tasks);
  const uint32_t stride = gridDim.x * kRmWaves;
  uint32_t t = uni(blockIdx.x * kRmWaves + w);
  if (t >= nt) return;
  PTask cur = load_task(tasks, t);
  for (;;) {
    const uint32_t tn = t + stride;
    PTask nxt;
    if (tn < nt) nxt = load_task(tasks, tn);
    rmut_task<OP, BUF>(t, cur, pa, ra, oc, big, lds);
    if (tn >= nt) break;
    t = tn;
    cur = nxt;
  }
}

void launch_rmut(hipStream_t s, const uint32_t* koa, const CDesc* da, const uint8_t* pa, RmutArgs ra, bool buf,
                 uint64_t* wg_epoch, uint32_t epoch, PTask* tasks, uint32_t* n_tasks, OutCtx oc, uint64_t* zlb,
                 uint64_t* ztile, BigRuns big, int grid) {
  hipLaunchKernelGGL(k_plan_rmut, dim3(256), dim3(256), 0, s, koa, da, pa, ra, wg_epoch, epoch, tasks, n_tasks, zlb,
                     ztile, oc.err);
  const int g0 = std::max(1, (grid + kRmWaves - 1) / kRmWaves);
#define RBG_RMUT_LAUNCH(O, B)                                                                                    \
  hipLaunchKernelGGL((k_rmut<O, B>), dim3(std::min(g0, resident_grid((const void*)&k_rmut<O, B>))), dim3(256), 0, s, \
                     tasks, n_tasks, pa, ra, oc, big)
  if (ra.op == RMUT_ADD) RBG_RMUT_LAUNCH(RMUT_ADD, false);
  else if (ra.op == RMUT_ADD_INPLACE) RBG_RMUT_LAUNCH(RMUT_ADD_INPLACE, false);
  else if (ra.op == RMUT_DERUN) RBG_RMUT_LAUNCH(RMUT_DERUN, false);
  else if (ra.op == RMUT_LIMIT) RBG_RMUT_LAUNCH(RMUT_LIMIT, false);
  else if (ra.op == RMUT_RANGE) RBG_RMUT_LAUNCH(RMUT_RANGE, false);
  else if (ra.op == RMUT_FLIP) RBG_RMUT_LAUNCH(RMUT_FLIP, false);
  else if (buf) RBG_RMUT_LAUNCH(RMUT_REMOVE, true);
  else RBG_RMUT_LAUNCH(RMUT_REMOVE, false);
#undef RBG_RMUT_LAUNCH
}

}  // namespace rbg
