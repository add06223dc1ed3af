// RoaringBitmap.addOffset(x, offset) on the MI355X (RB/RoaringBitmap.java:230-288; the buffer package's
// MutableRoaringBitmap.addOffset, RB/buffer/MutableRoaringBitmap.java:84-142, types alike).
//
// offset = 65536 co + off, off in [0, 65535] (the reference's floor division).  off == 0: every container
// is cloned under key + co (keys outside [0, 65535] dropped).  Otherwise output key k is the union of
//   P: the part of input container k - co - 1 that crosses 65536 (Util.addOffset's high part, values
//      v + off - 65536)
//   Q: the part of input container k - co that stays (the low part, values v + off)
// and its type is what the reference's chain gives (RB/Util.java:32-126, then Container.ior of the low
// part into the previous high part, then RoaringBitmap.repairAfterLazy :2752-2757):
//   parts: an array's are arrays; a bitmap's go through BitmapContainer.repairAfterLazy (<= 4096 values
//          an array; never full, as a part of a shifted container cannot be); a run container's are run
//          containers (toEfficientContainer at the end)
//   one part: its type (a run part through toEfficientContainer)
//   two parts (disjoint: P below off, Q from off up): with a bitmap part, a bitmap, or a full run
//          container when full -- except bitmap P OR array Q (BitmapContainer.ior(ArrayContainer),
//          RB/BitmapContainer.java:740-757), which keeps a full bitmap; else with a run part,
//          toEfficientContainer; else two arrays by cardinality (ArrayContainer.ior :726-745)
//
//   k_plan_aoff : one thread per output key, the keys with an input container at k - co or k - co - 1
//   k_aoff      : one wave per contiguous chunk of tasks: P and Q materialised in registers, the words
//                 of both that reach the output written into an 8 KiB LDS window at a wave-uniform word
//                 offset, the output read from it as a funnel shift of adjacent words; the next key's
//                 P is this key's Q, kept in registers
#include <algorithm>

#include "kernels.hpp"
#include "wave.hpp"

namespace rbg {

__global__ __launch_bounds__(256) void k_plan_aoff(const uint32_t* __restrict__ koa, const CDesc* __restrict__ da,
                                                   const uint8_t* __restrict__ pa, AoffArgs aa,
                                                   uint64_t* __restrict__ wg_epoch, uint32_t epoch,
                                                   PTask* __restrict__ tasks, uint32_t* __restrict__ n_tasks,
                                                   uint64_t* zlb, uint64_t* ztile, uint32_t* err) {
  plan_zero(zlb, ztile);
  const int k = (int)(blockIdx.x * blockDim.x + threadIdx.x);
  PTask t;
  t.key = (uint16_t)k;
  const int q = k - aa.co, p = q - 1;
  if (!aa.none && q >= 0 && q <= 65535) {
    resolve(koa, da, pa, (uint32_t)q, t.slot_a, t.card_a, t.kind_a, t.nruns_a);
  } else {
    t.slot_a = 0;
    t.card_a = 0;
    t.kind_a = kAbsent;
    t.nruns_a = 0;
  }
  if (!aa.none && aa.off != 0 && p >= 0 && p <= 65535) {
    resolve(koa, da, pa, (uint32_t)p, t.slot_b, t.card_b, t.kind_b, t.nruns_b);
  } else {
    t.slot_b = 0;
    t.card_b = 0;
    t.kind_b = kAbsent;
    t.nruns_b = 0;
  }
  plan_emit(t.kind_a != kAbsent || t.kind_b != kAbsent, t, wg_epoch, epoch, tasks, n_tasks, err);
}

// the kind of a nonempty part of an input container of kind `kind` holding `pc` values
__device__ __forceinline__ int part_kind(int kind, int pc) {
  if (kind == DK_B) return by_card(pc);  // BitmapContainer.repairAfterLazy (RB/BitmapContainer.java:1205-1215)
  return kind;
}

// Per-wave state across consecutive tasks: a task whose P is the previous task's Q (output keys k - 1
// and k) takes it from the registers, so each input container is materialised once per chunk.
struct AoffCarry {
  WCtr q;         // the previous task's Q container (all its bits)
  int prev_key;   // key of the previous task (-2: none)
  int prev_q;     // the previous task had a Q container
  int prev_high;  // that container's values in [s, 65535]: the next key's P part
};

__device__ __forceinline__ void aoff_task(uint32_t t, const PTask& tk, const uint8_t* pa, const AoffArgs& aa,
                                          const OutCtx& oc, uint32_t* lds, AoffCarry& cy) {
  const int key = tk.key;
  if (aa.off == 0) {  // a clone under the shifted key
    const uint32_t len = tk.kind_a == DK_A ? 2u * tk.card_a : tk.kind_a == DK_B ? 8192u : 2u + 4u * tk.nruns_a;
    w_place(t, true, pa + tk.slot_a + (tk.kind_a == DK_R ? 2 : 0), false, lds, len, tk.card_a, (uint32_t)key,
            tk.kind_a, oc);
    return;
  }
  const int s = 65536 - aa.off;  // P's part is its bits [s, 65535], Q's its bits [0, s - 1]
  const int sb = s >> 6, r = s & 63;
  WCtr p;
  int cp = 0;
  if (tk.kind_b != kAbsent && cy.prev_key == key - 1 && cy.prev_q) {
    p = cy.q;
    cp = cy.prev_high;
  } else if (tk.kind_b != kAbsent) {
    w_materialize(CDesc{tk.slot_b, tk.card_b, tk.key, tk.kind_b, 0}, pa, lds, p);
#pragma unroll
    for (int k = 0; k < 16; k++) cp += __popcll(p.w[k] & wrange(k, s, 65535));
    cp = wave_sum_i(cp);
  } else {
#pragma unroll
    for (int k = 0; k < 16; k++) p.w[k] = 0;
  }
  int cq = 0, qhigh = 0;
  if (tk.kind_a != kAbsent) {
    w_materialize(CDesc{tk.slot_a, tk.card_a, tk.key, tk.kind_a, 0}, pa, lds, cy.q);
#pragma unroll
    for (int k = 0; k < 16; k++) {
      cq += __popcll(cy.q.w[k] & wrange(k, 0, s - 1));
      qhigh += __popcll(cy.q.w[k] & wrange(k, s, 65535));
    }
    cq = wave_sum_i(cq);
    qhigh = wave_sum_i(qhigh);
  } else {
#pragma unroll
    for (int k = 0; k < 16; k++) cy.q.w[k] = 0;
  }
  cy.prev_key = key;
  cy.prev_q = tk.kind_a != kAbsent;
  cy.prev_high = qhigh;
  // window W[j] = (P || Q) word j + sb, j in [0, 1024]: P's words from sb on, Q's words up to sb
  uint64_t* win = reinterpret_cast<uint64_t*>(lds);
  const int l = lane_id();
  wsync();
#pragma unroll
  for (int k = 0; k < 16; k++) {
    const int w = 128 * (k >> 1) + 2 * l + (k & 1);
    if (w >= sb) win[w - sb] = p.w[k];
    if (w <= sb) win[w + 1024 - sb] = cy.q.w[k];
  }
  wsync();
  // output bit b = window bit b + r
  WCtr& x = p;
#pragma unroll
  for (int k = 0; k < 16; k++) {
    const int w = 128 * (k >> 1) + 2 * l + (k & 1);
    const uint64_t lo = win[w];
    x.w[k] = r ? (lo >> r) | (win[w + 1] << (64 - r)) : lo;
  }
  const int c = w_card(x);
  if (c == 0) {  // both parts empty
    w_place(t, false, nullptr, true, lds, 0, 0, (uint32_t)key, DK_A, oc);
    return;
  }
  int kind;
  if (cp == 0 || cq == 0) {
    const int pk = cp ? part_kind(tk.kind_b, cp) : part_kind(tk.kind_a, cq);
    kind = pk == DK_R ? eff(c, w_runs(x)) : pk;
  } else {
    const int tp = part_kind(tk.kind_b, cp), tq = part_kind(tk.kind_a, cq);
    if (tp == DK_B || tq == DK_B) kind = (c == 65536 && !(tp == DK_B && tq == DK_A)) ? DK_R : DK_B;
    else if (tp == DK_R || tq == DK_R) kind = eff(c, w_runs(x));
    else kind = by_card(c);
  }
  if (kind == DK_B) {  // registers straight to the task's slot
    uint8_t* slot = oc.scratch + (size_t)t * kSlotBytes;
    w_store_bitmap(slot, x);
    w_place(t, true, slot, false, lds, 8192, (uint32_t)c, (uint32_t)key, DK_B, oc);
    return;
  }
  // a run result here holds <= 2047 runs (toEfficientContainer, or the full container)
  const uint32_t len = w_stage(kind, x, c, lds);
  w_place(t, true, nullptr, true, lds, len, (uint32_t)c, (uint32_t)key, kind, oc);
}

constexpr int kAoWaves = 4;
constexpr int kAoLds = 2064;  // u32 per wave: the 8 KiB scratch / staging area and the window's 1025th word

// one wave per contiguous chunk of tasks (consecutive keys share an input container), the next record
// fetched while a task runs
__global__ __launch_bounds__(256) void k_aoff(const PTask* __restrict__ tasks, const uint32_t* __restrict__ n_tasks,
                                              const uint8_t* pa, AoffArgs aa, OutCtx oc) {
  __shared__ __align__(16) uint32_t lds_all[kAoWaves][kAoLds];
  const int w = threadIdx.x >> 6;
  uint32_t* lds = lds_all[w];
  const uint32_t nt = uni(*n_tasks);
  const uint32_t nw = gridDim.x * kAoWaves;
  const uint32_t per = (nt + nw - 1) / nw;
  uint32_t t = uni((blockIdx.x * kAoWaves + w) * per);
  const uint32_t tend = min(nt, t + per);
  if (t >= tend) return;
  AoffCarry cy;
  cy.prev_key = -2;
  cy.prev_q = 0;
  cy.prev_high = 0;
  PTask cur = load_task(tasks, t);
  for (;;) {
    const uint32_t tn = t + 1;
    PTask nxt;
    if (tn < tend) nxt = load_task(tasks, tn);
    aoff_task(t, cur, pa, aa, oc, lds, cy);
    if (tn >= tend) break;
    t = tn;
    cur = nxt;
  }
}

void launch_aoff(hipStream_t s, const uint32_t* koa, const CDesc* da, const uint8_t* pa, AoffArgs aa,
                 uint64_t* wg_epoch, uint32_t epoch, PTask* tasks, uint32_t* n_tasks, OutCtx oc, uint64_t* zlb,
                 uint64_t* ztile, int grid) {
  hipLaunchKernelGGL(k_plan_aoff, dim3(256), dim3(256), 0, s, koa, da, pa, aa, wg_epoch, epoch, tasks, n_tasks, zlb,
                     ztile, oc.err);
  const int g0 = std::max(1, (grid + kAoWaves - 1) / kAoWaves);
  hipLaunchKernelGGL(k_aoff, dim3(std::min(g0, resident_grid((const void*)&k_aoff))), dim3(256), 0, s, tasks,
                     n_tasks, pa, aa, oc);
}

}  // namespace rbg
