// Pairwise static ops (RB/RoaringBitmap.java and :377, or :860, xor :1071,
// andNot :444, andCardinality :413) on the MI355X.  RB/ = reference
// RoaringBitmap/src/main/java/org/roaringbitmap/.
//
//   k_plan_pairwise : one thread per key: key alignment of the two operands
//                     (the advanceUntil walks, here O(1) lookups in each batch's
//                     key CSR), resolution of both operands' descriptors into a
//                     32 B task record, and compaction into the dense task list
//   k_pair_wave     : one wavefront per task over a resident grid; the next
//                     task's record is fetched with scalar loads while the
//                     current one runs, and both operand payloads are requested
//                     before either is consumed
// Placement and serialization follow in kernels.hip (k_place, k_serialize).
#include <algorithm>
#include <cstdio>
#include <cstdlib>

#include "kernels.hpp"
#include "wave.hpp"

namespace rbg {

// Task class: 1 = filter class (pass-through clones, AND with an array, ANDNOT
// of an array: results are subsets of one array), 2 = bitmap class.
__device__ __forceinline__ int pair_class(int op, int ka, int kb) {
  if (ka == kAbsent || kb == kAbsent) return 1;
  if (op == OP_AND && (ka == DK_A || kb == DK_A)) return 1;
  if (op == OP_ANDNOT && ka == DK_A) return 1;
  return 2;
}

// RB/RoaringBitmap.java:382-400 (and), :864-896 (or), :1076-1113 (xor), :449-471 (andNot)
// One thread per key, 256 workgroups of 256 keys, all resident.  Each workgroup
// publishes its task count tagged with this op's epoch, sums the counts of the
// workgroups before it (one per thread, waiting for the epoch), and writes its
// tasks straight into the dense task list -- plan and compaction in one launch.  Keys
// outside [key_lo, key_hi) give no task (a key-range shard of the op: every key's result
// depends on that key's containers only, RB/RoaringBitmap.java:382-399).
__global__ __launch_bounds__(256) void k_plan_pairwise(int op, int key_lo, int key_hi, const uint32_t* __restrict__ koa,
                                                       const CDesc* __restrict__ da, const uint8_t* __restrict__ pa,
                                                       const uint32_t* __restrict__ kob,
                                                       const CDesc* __restrict__ db, const uint8_t* __restrict__ pb,
                                                       uint64_t* __restrict__ wg_epoch, uint32_t epoch,
                                                       PTask* __restrict__ tasks, uint32_t* __restrict__ n_tasks,
                                                       uint64_t* zlb, uint64_t* ztile, uint32_t* err) {
  plan_zero(zlb, ztile);
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  PTask t;
  resolve(koa, da, pa, k, t.slot_a, t.card_a, t.kind_a, t.nruns_a);
  resolve(kob, db, pb, k, t.slot_b, t.card_b, t.kind_b, t.nruns_b);
  t.key = (uint16_t)k;
  const bool ia = t.kind_a != kAbsent, ib = t.kind_b != kAbsent;
  int f;
  switch (op) {
    case OP_OR:
    case OP_XOR: f = ia || ib; break;
    case OP_ANDNOT: f = ia; break;
    default: f = ia && ib; break;  // AND and andCardinality
  }
  if ((int)k < key_lo || (int)k >= key_hi) f = 0;
  plan_emit(f, t, wg_epoch, epoch, tasks, n_tasks, err);
}

// ---------------------------------------------------------------------------
// Balanced task order (dense key ranges).  A wave of the static-stride grid gets one task of every
// block of S = waves tasks of the list; over a list in key order the families fall at random, so the
// waves' work differs by the sum of ~16 random task costs (measured with the per-wave probe build,
// scripts/xcd_probe.py: mean wave life ~165 us against a 227 us launch, equal over the XCDs).  Here
// the plan sorts the tasks into kBalBins bins by an estimated cost (family, array size, run count),
// heaviest first, so each block of S tasks holds similar costs and every wave draws one task of each
// cost band; the kernel then walks its bands in a per-wave rotated order (wave w starts at band
// w mod bands), so at any instant the waves run a mix of families.  Records and scratch slots stay
// at key positions (key - key_lo; the plan writes the records of keys without a task), so placement
// and serialization see key order as before.  The binning is per workgroup of the plan (256 keys, a
// counting sort in LDS, no cross-workgroup step: a global sort's inter-workgroup exchange cost 20 us);
// the workgroups' key ranges hold the same family mix, so per-segment ranks are global cost bands.
// ---------------------------------------------------------------------------
constexpr int kBalBins = 32;

// estimated per-task cost (arbitrary units, ~1 per 0.6 us of one wave) -> bin, heaviest first
template <int OP>
__device__ __forceinline__ int bal_bin(const PTask& t) {
  const int ka = t.kind_a, kb = t.kind_b;
  int c;
  if (ka == kAbsent || kb == kAbsent) {
    c = 2;  // a clone: its record only
  } else if (pair_class(OP, ka, kb) == 1) {  // filter class: the array's values probed in a map of the other
    const bool probe_a = ka == DK_A && (OP == OP_ANDNOT || kb != DK_A || t.card_a <= t.card_b);  // filter_class_task
    const int arr = (int)(probe_a ? t.card_a : t.card_b);
    const int mk = probe_a ? kb : ka;
    const int mn = probe_a ? t.nruns_b : t.nruns_a;
    c = 9 + arr / 800 + (mk == DK_R ? 4 + mn / 400 : mk == DK_B ? 3 : (int)(probe_a ? t.card_b : t.card_a) / 1600);
  } else if (ka == DK_B && kb == DK_B) {
    c = 24;
  } else if (ka == DK_R && kb == DK_R) {
    const int n = t.nruns_a + t.nruns_b;
    c = n + 2 > 2560 ? 30 : 14 + n / 200;
  } else {  // B with R, or any other bitmap-class pair (OR / XOR / ANDNOT of arrays and bitmaps)
    const int n = ka == DK_R ? t.nruns_a : kb == DK_R ? t.nruns_b : 0;
    c = 18 + n / 300;
  }
  return kBalBins - 1 - min(c, kBalBins - 1);
}

template <int OP, int MODE>
__global__ __launch_bounds__(256) void k_plan_balanced(int key_lo, uint32_t nkeys, const uint32_t* __restrict__ koa,
                                                       const CDesc* __restrict__ da, const uint8_t* __restrict__ pa,
                                                       const uint32_t* __restrict__ kob,
                                                       const CDesc* __restrict__ db, const uint8_t* __restrict__ pb,
                                                       PTask* __restrict__ tasks, uint32_t* __restrict__ n_tasks,
                                                       OutCtx oc, uint32_t* __restrict__ task_card, uint64_t* zlb,
                                                       uint64_t* ztile) {
  __shared__ int hist[kBalBins];
  __shared__ int off[kBalBins];
  plan_zero(zlb, ztile);
  if (threadIdx.x < kBalBins) hist[threadIdx.x] = 0;
  __syncthreads();
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;  // key position in the range
  PTask t;
  int bin = kBalBins - 1, rank = 0;
  if (i < nkeys) {
    const uint32_t k = (uint32_t)key_lo + i;
    resolve(koa, da, pa, k, t.slot_a, t.card_a, t.kind_a, t.nruns_a);
    resolve(kob, db, pb, k, t.slot_b, t.card_b, t.kind_b, t.nruns_b);
    t.key = (uint16_t)k;
    const bool ia = t.kind_a != kAbsent, ib = t.kind_b != kAbsent;
    const bool has = (OP == OP_OR || OP == OP_XOR) ? (ia || ib) : OP == OP_ANDNOT ? ia : (ia && ib);
    if (has) {
      bin = bal_bin<OP>(t);
    } else {  // no task: marked (both kinds absent) and skipped by the compute kernel
      t.kind_a = t.kind_b = kAbsent;
      if (MODE == 1) {
        task_card[i] = 0;
      } else {  // no result container for this key (RB/RoaringBitmap.java:382-400): an empty record
        ORec r;
        r.off = 0;
        r.src = 0;
        r.idx = 0;
        r.card = 0;
        r.ser_len = 0;
        r.key = (uint16_t)k;
        r.kind = DK_A;
        r.keep = 0;
        oc.recs[i] = r;
      }
    }
    rank = atomicAdd(&hist[bin], 1);
  }
  __syncthreads();
  if (threadIdx.x == 0) {  // heaviest bin first
    int run = 0;
    for (int b = 0; b < kBalBins; b++) {
      off[b] = run;
      run += hist[b];
    }
  }
  __syncthreads();
  if (i < nkeys) {
    // this workgroup's segment [256 g, 256 g + m) holds its keys' tasks by cost rank r (0 = heaviest) at
    // offset (r + g) mod m: a wave takes one offset of every 16th segment, so its tasks are ranks
    // spaced 16 apart (every cost band of the segments) rather than one rank over and over
    const uint32_t m = min(256u, nkeys - blockIdx.x * 256u);
    const uint32_t r = (uint32_t)(off[bin] + rank);
    tasks[blockIdx.x * 256u + (r + blockIdx.x) % m] = t;
  }
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    n_tasks[0] = nkeys;  // records: one per key of the range
    n_tasks[1] = nkeys;  // list positions (keys without a task are marked)
  }
}

constexpr int kWaves = 4;  // waves per workgroup
// u32 words of LDS per wave: the 8 KiB bitmap map / staging area, plus room for
// the run lists of run-domain R AND R (4 waves x 10 KiB x 4 workgroups = 160 KiB; two words
// short of 10 KiB, so that k_pair_cu's 16 waves and its task counter fit one CU's 160 KiB)
constexpr int kWaveLds = 2558;
static_assert(kWaveLds >= 2048, "the 8 KiB bitmap map / staging area");


// Wave priority: a task runs at priority 3 until its operand loads have been
// consumed, then drops, so waves that are issuing loads win instruction
// arbitration over waves in their compute / output phases and more of the CU's
// memory requests are in flight (C2 AND -1 %, andCardinality -2.5 %).  The per-wave probe
// (round 5, profiles/r05/experiments/xcd_probe_*) showed the workgroups of a CU finishing in
// dispatch order at equal priority (the issue arbitration favours the oldest waves), so the
// compute / output phases run at half the workgroup's dispatch tier, (blockIdx * 4 / grid) / 2:
// with the balanced task order the AND kernel 0.244 -> 0.233 ms (profiles/r05/experiments/c2_prio_tiers.txt).
__device__ __forceinline__ void prio_hi() { __builtin_amdgcn_s_setprio(3); }
__device__ __forceinline__ void prio_lo() {
  const uint32_t tier = __builtin_amdgcn_readfirstlane((blockIdx.x * 4u) / gridDim.x) >> 1;
  if (tier == 0) __builtin_amdgcn_s_setprio(0);
  else __builtin_amdgcn_s_setprio(1);
}

// Filter path: AND with an array operand and ANDNOT of an array c1 always give an
// array that is a subset of that array (App. A.1 / A.3; RB/ArrayContainer.java:
// 184-271, RB/BitmapContainer.java:162-171, RB/RunContainer.java:305-334).  The
// other operand is made an LDS membership map, the array's values are probed
// (kept = member, or non-member for ANDNOT) and the kept values -- still sorted
// -- go straight to the task's scratch slot.
template <int OP, int MODE>
__device__ __forceinline__ void filter_task(uint32_t t, uint32_t key, int pcard, const uint8_t* pslot, int mkind,
                                            int mcard, const uint8_t* mslot, const OutCtx& oc, uint32_t* task_card,
                                            uint32_t* lds) {
  // the array's values are requested first, so their memory latency overlaps the
  // map construction (one round trip per task instead of two)
  const int l = lane_id();
  const int nvec = (pcard + 7) >> 3;  // <= 512: 8 vectors per lane
  const uint4* pv = reinterpret_cast<const uint4*>(pslot) + l;
  uint4 v[8];
#pragma unroll
  for (int j = 0; j < 8; j++) v[j] = (64 * j + l < nvec) ? ld_in(pv + 64 * j) : make_uint4(0, 0, 0, 0);
  w_map_lds(mkind, mcard, mslot, lds);
  prio_lo();
  uint32_t hit[8];
  int cnt = 0;
#pragma unroll
  for (int j = 0; j < 8; j++) {
    hit[j] = 0;
    if (512 * j < pcard) {  // wave-uniform
      const int first = 8 * (64 * j + l);
      const uint32_t w[4] = {v[j].x, v[j].y, v[j].z, v[j].w};
      // 5 VALU per value: bit-field word index + address, shift, place (the
      // hardware shift reads only the low 5 bits, so no masking); the tail of
      // the array is masked once per vector, not per value
      uint32_t h = 0;
#pragma unroll
      for (int i = 0; i < 8; i++) {
        const uint32_t wi = w[i >> 1];
        const uint32_t word = lds[(i & 1) ? bfe_hi_word(wi) : bfe_lo_word(wi)];
        h |= bit_at(word, (i & 1) ? (wi >> 16) : wi) << i;
      }
      if (OP == OP_ANDNOT) h = ~h & 0xFFu;
      const int rem = pcard - first;
      hit[j] = rem >= 8 ? h : h & ((1u << max(rem, 0)) - 1u);
      cnt += __popc(hit[j]);
    }
  }
  if (MODE == 1) {
    const int c = wave_sum_i(cnt);
    if (l == 0) task_card[t] = (uint32_t)c;
    return;
  }
  // the map is dead: compact the kept values over it, then 16 B stores.  Vectors
  // j and j+1 share one scan (16-bit count fields); every value is written, the
  // dropped ones to a per-lane dummy just past the kept ones (u16 index ctot + l),
  // so the writes need no branches.  When fewer than 64 u16 are left past the
  // kept values (ctot > 4032), only kept values are written.
  uint16_t* st = reinterpret_cast<uint16_t*>(lds);
  const uint32_t ctot = uni((uint32_t)wave_sum_i(cnt));
  const bool dummies = ctot <= 4096u - 64u;  // wave-uniform
  const uint32_t dummy = ctot + (uint32_t)l;
  wsync();
  int base = 0;
#pragma unroll
  for (int j = 0; j < 8; j += 2) {
    if (512 * j >= pcard) break;  // wave-uniform
    int tot;
    const int ex = wave_excl(__popc(hit[j]) | (__popc(hit[j + 1]) << 16), &tot);
    int q0 = base + (ex & 0xFFFF);
    int q1 = base + (tot & 0xFFFF) + (ex >> 16);
#pragma unroll
    for (int h = 0; h < 2; h++) {
      const uint32_t hj = hit[j + h];
      int q = h == 0 ? q0 : q1;
      const uint32_t w[4] = {v[j + h].x, v[j + h].y, v[j + h].z, v[j + h].w};
#pragma unroll
      for (int i = 0; i < 8; i++) {
        const uint32_t keep = (hj >> i) & 1u;
        const uint16_t val = (uint16_t)((w[i >> 1] >> ((i & 1) * 16)) & 0xFFFF);
        if (dummies) st[keep ? (uint32_t)q : dummy] = val;
        else if (keep) st[q] = val;
        q += (int)keep;
      }
    }
    base += (tot & 0xFFFF) + (tot >> 16);
  }
  const int c = (int)ctot;
  wsync();
  uint8_t* slot = oc.scratch + (size_t)t * kSlotBytes;
  const uint4* sv = reinterpret_cast<const uint4*>(lds);
  uint4* dv = reinterpret_cast<uint4*>(slot);
  for (int k = l; k < (2 * c + 15) >> 4; k += 64) dv[k] = sv[k];  // the slot has room for the rounded tail
  // empty results are dropped (RB/RoaringBitmap.java:389,456)
  w_place(t, c > 0, slot, false, lds, 2u * (uint32_t)c, (uint32_t)c, key, DK_A, oc);
}

// Filter-class task (pass-through clone, or a filter), one wave, wave-uniform branches.
template <int OP, int MODE>
__device__ __forceinline__ void filter_class_task(uint32_t t, const PTask& tk, const uint8_t* pa, const uint8_t* pb,
                                                  const OutCtx& oc, uint32_t* task_card, uint32_t* lds) {
  const int ka = tk.kind_a, kb = tk.kind_b;
  if (ka == kAbsent || kb == kAbsent) {  // unmatched key: clone (appendCopy), RB/RoaringArray.java:184-205
    if (MODE == 0) {
      const bool from_a = ka != kAbsent;
      const int kind = from_a ? ka : kb;
      const uint32_t card = from_a ? tk.card_a : tk.card_b;
      const uint32_t nr = from_a ? tk.nruns_a : tk.nruns_b;
      const uint8_t* src = (from_a ? pa + tk.slot_a : pb + tk.slot_b) + (kind == DK_R ? 2 : 0);
      const uint32_t len = kind == DK_A ? 2 * card : kind == DK_B ? 8192u : 2 + 4 * nr;
      w_place(t, true, src, false, lds, len, card, tk.key, kind, oc);
    }
    return;
  }
  const int ca = (int)tk.card_a, cb = (int)tk.card_b;
  const uint8_t* sa = pa + tk.slot_a;
  const uint8_t* sb = pb + tk.slot_b;
  // filter the array (A & A: the smaller one; A \ x: c1) through a map of the other operand
  if (ka == DK_A && (OP == OP_ANDNOT || kb != DK_A || ca <= cb))
    filter_task<OP, MODE>(t, tk.key, ca, sa, kb, cb, sb, oc, task_card, lds);
  else
    filter_task<OP, MODE>(t, tk.key, cb, sb, ka, ca, sa, oc, task_card, lds);
}

// R AND R in the run domain (RB/RunContainer.java and(RunContainer)): the
// intersection of two sorted disjoint run lists is the list of overlaps of their
// runs, already canonical.  Both run lists go to the wave's LDS as
// (start | end << 16) -- kWaveLds u32 words hold na + nb runs and two sentinels -- and the lanes
// split the merge path evenly (rr_merge).  Pass 1 counts runs and cardinality; the type is EFF
// (App. A.1); an R result is written by pass 2 straight into the task's scratch
// slot.  Returns false (nothing written) when the result is not a run container or
// the runs do not fit: the bitmap path then runs.
// Merge path over the run ends: step d of the two-pointer intersection advances
// whichever current run ends first (A on ties); every overlapping pair of runs is
// current at exactly one step, and overlaps come out in ascending order.  Lane l
// takes steps [d0, d1) of na + nb, found by a binary search on the diagonal.
// A's run list lives at lds[0, na) followed by a sentinel at lds[na], B's at
// lds[na + 1, na + 1 + nb) followed by a sentinel.  The sentinel is the empty run
// (start 0xFFFF, end 0xFFFE): it overlaps nothing, so a lane may keep stepping
// after either side is exhausted (no further overlap exists then; the index is
// clamped at the sentinel) and every lane runs its d1 - d0 steps without branches:
// each step selects which side advances and issues one LDS read for that side's
// next-but-one run (R AND R card -8 % against the branching two-pointer loop).
constexpr uint32_t kRunSentinel = 0xFFFEFFFFu;
template <bool EMIT>
__device__ __forceinline__ void rr_merge(const uint32_t* lds, int na, int nb, int d0, int d1, int& cnt, int& card,
                                         uint32_t* out) {
  const uint32_t* al = lds;
  const uint32_t* bl = lds + na + 1;
  int lo = max(0, d0 - nb), hi = min(d0, na);
  while (lo < hi) {
    const int m = (lo + hi) >> 1;
    if ((al[m] >> 16) <= (bl[d0 - m - 1] >> 16)) lo = m + 1;
    else hi = m;
  }
  int i = lo, j = d0 - lo;
  // current and next run of each side in registers: the LDS read of a side's
  // next-but-one run is off the step's dependency chain
  uint32_t a = al[i], b = bl[j];
  uint32_t an = al[min(i + 1, na)], bn = bl[min(j + 1, nb)];
  for (int d = d0; d < d1; d++) {
    const uint32_t as = a & 0xFFFF, ae = a >> 16, bs = b & 0xFFFF, be = b >> 16;
    const uint32_t s0 = max(as, bs), e0 = min(ae, be);
    const bool ov = s0 <= e0;
    if (EMIT && ov) out[cnt] = s0 | ((e0 - s0) << 16);
    cnt += ov ? 1 : 0;
    card += ov ? (int)(e0 - s0 + 1) : 0;
    const bool adv = ae <= be;  // A's run ends first (A on ties)
    i = adv ? min(i + 1, na) : i;
    j = adv ? j : min(j + 1, nb);
    const uint32_t nx = adv ? al[min(i + 1, na)] : bl[min(j + 1, nb)];
    b = adv ? b : bn;
    bn = adv ? bn : nx;
    a = adv ? an : a;
    an = adv ? nx : an;
  }
}

// run list of a slot -> LDS as (start | end << 16), from 16 B slot vectors (vector q
// holds runs 4q - 1 .. 4q + 2; run -1 is the pad and count)
__device__ __forceinline__ void run_vec_to_lds(const uint4 v, int q, int n, uint32_t* dst) {
  const uint32_t u[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int c = 0; c < 4; c++) {
    const int r = 4 * q + c - 1;
    if (r >= 0 && r < n) dst[r] = (u[c] & 0xFFFF) | (min((u[c] & 0xFFFF) + (u[c] >> 16), 65535u) << 16);
  }
}

// both operands' run lists, all of a round's vectors requested before any is used
__device__ __forceinline__ void runs_to_lds2(const uint8_t* sa, int na, uint32_t* da, const uint8_t* sb, int nb,
                                             uint32_t* db) {
  constexpr int R = 4;
  const int l = lane_id();
  const int nva = (na + 4) >> 2, nvb = (nb + 4) >> 2;
  const uint4* a4 = reinterpret_cast<const uint4*>(sa);
  const uint4* b4 = reinterpret_cast<const uint4*>(sb);
#pragma unroll 1
  for (int j0 = 0; 64 * j0 < max(nva, nvb); j0 += R) {
    uint4 va[R], vb[R];
#pragma unroll
    for (int j = 0; j < R; j++) {
      const int q = 64 * (j0 + j) + l;
      va[j] = q < nva ? ld_in(a4 + q) : make_uint4(0, 0, 0, 0);
      vb[j] = q < nvb ? ld_in(b4 + q) : make_uint4(0, 0, 0, 0);
    }
#pragma unroll
    for (int j = 0; j < R; j++) {
      const int q = 64 * (j0 + j) + l;
      run_vec_to_lds(va[j], q, na, da);
      run_vec_to_lds(vb[j], q, nb, db);
    }
  }
}

template <int MODE>
__device__ __forceinline__ bool rr_and_task(uint32_t t, const PTask& tk, const uint8_t* pa, const uint8_t* pb,
                                            const OutCtx& oc, uint32_t* task_card, uint32_t* lds) {
  const int na = tk.nruns_a, nb = tk.nruns_b;
  if (na + nb + 2 > kWaveLds) return false;
  const int l = lane_id();
  wsync();
  runs_to_lds2(pa + tk.slot_a, na, lds, pb + tk.slot_b, nb, lds + na + 1);
  if (l == 0) {
    lds[na] = kRunSentinel;
    lds[na + 1 + nb] = kRunSentinel;
  }
  prio_lo();
  wsync();
  const int d0 = (l * (na + nb)) >> 6, d1 = ((l + 1) * (na + nb)) >> 6;
  int cnt = 0, card = 0;
  rr_merge<false>(lds, na, nb, d0, d1, cnt, card, nullptr);
  const int c = (int)uni((uint32_t)wave_sum_i(card));
  if (MODE == 1) {
    if (l == 0) task_card[t] = (uint32_t)c;
    return true;
  }
  if (c == 0) {  // empty results are dropped (RB/RoaringBitmap.java:389)
    w_place(t, false, nullptr, true, lds, 0, 0, tk.key, DK_A, oc);
    return true;
  }
  int nr;
  const int off = wave_excl(cnt, &nr);
  nr = (int)uni((uint32_t)nr);
  if (eff(c, nr) != DK_R) return false;
  uint8_t* slot = oc.scratch + (size_t)t * kSlotBytes;
  int cnt2 = 0, card2 = 0;
  rr_merge<true>(lds, na, nb, d0, d1, cnt2, card2, reinterpret_cast<uint32_t*>(slot + 4) + off);
  if (l == 0) *reinterpret_cast<uint16_t*>(slot + 2) = (uint16_t)nr;
  w_place(t, true, slot + 2, false, lds, 2u + 4u * (uint32_t)nr, (uint32_t)c, tk.key, DK_R, oc);
  return true;
}

// Bitmap-class task: both operands in registers (16 words per lane), combined,
// counted, typed (App. A) and written out (B straight from registers, A and R
// staged in LDS).  One wave, wave-uniform branches.
template <int OP, int MODE>
__device__ __forceinline__ void bitmap_class_task(uint32_t t, const PTask& tk, const uint8_t* pa, const uint8_t* pb,
                                                  const OutCtx& oc, uint32_t* task_card, uint32_t* lds) {
  const int ka = tk.kind_a, kb = tk.kind_b;
  const int ca = (int)tk.card_a, cb = (int)tk.card_b;
  if (OP == OP_AND && ka == DK_R && kb == DK_R && rr_and_task<MODE>(t, tk, pa, pb, oc, task_card, lds)) return;
  WCtr x;
  w_materialize(CDesc{tk.slot_a, tk.card_a, tk.key, (uint8_t)ka, 0}, pa, lds, x);
  w_combine<OP>(CDesc{tk.slot_b, tk.card_b, tk.key, (uint8_t)kb, 0}, pb, lds, x);
  prio_lo();
  const int c = w_card(x);
  if (MODE == 1) {
    if (lane_id() == 0) task_card[t] = (uint32_t)c;
    return;
  }
  if (c == 0) {  // empty results are dropped (RB/RoaringBitmap.java:389,456,1084)
    w_place(t, false, nullptr, true, lds, 0, 0, tk.key, DK_A, oc);
    return;
  }
  const bool use_eff = pairwise_needs_runs(OP, ka, ca, kb, cb);
  const int kind = use_eff ? eff(c, w_runs(x)) : pairwise_kind(OP, ka, kb, c);
  if (kind == DK_B) {
    uint8_t* slot = oc.scratch + (size_t)t * kSlotBytes;
    w_store_bitmap(slot, x);
    w_place(t, true, slot, false, lds, 8192, (uint32_t)c, tk.key, DK_B, oc);
    return;
  }
  uint32_t len;
  if (kind == DK_A) len = w_stage(DK_A, x, c, lds);
  else len = 2u + 4u * (uint32_t)w_stage_runs(x, lds);
  w_place(t, true, nullptr, true, lds, len, (uint32_t)c, tk.key, kind, oc);
}

// 32 B task record through the scalar cache (wave-uniform address)

// ---------------------------------------------------------------------------
// Direct mode: the compute kernel resolves its tasks itself (no plan launch).  Task t is key
// key_lo + t (see k_pair_wave).  A key without a task (by the op's key rule,
// RB/RoaringBitmap.java:382-400 and, :864-896 or, :1076-1113 xor, :449-471 andNot) gives an
// empty record (or a zero count).
// does key k give a task of op OP (the plan kernel's rule)
template <int OP>
__device__ __forceinline__ bool has_task(const PTask& t) {
  const bool ia = t.kind_a != kAbsent, ib = t.kind_b != kAbsent;
  if (OP == OP_OR || OP == OP_XOR) return ia || ib;
  if (OP == OP_ANDNOT) return ia;
  return ia && ib;
}

template <int OP, int MODE>
__device__ __forceinline__ void any_task(uint32_t t, const PTask& tk, const uint8_t* pa, const uint8_t* pb,
                                         const OutCtx& oc, uint32_t* task_card, uint32_t* lds) {
  prio_hi();
  if (pair_class(OP, tk.kind_a, tk.kind_b) == 1)
    filter_class_task<OP, MODE>(t, tk, pa, pb, oc, task_card, lds);
  else
    bitmap_class_task<OP, MODE>(t, tk, pa, pb, oc, task_card, lds);
}

// One wave per task, static stride over a resident grid (a contended ticket
// counter costs ~12 ns per task chip-wide, a workgroup per task pays a dispatch
// each).  The next task's record is loaded while this one runs.  Filter-class
// and bitmap-class tasks share the launch: separate kernels per class were
// measured 15 % slower on the C2 mix (tail + an extra dependent index load).
// MODE 0: materialise results.  MODE 1: andCardinality only (task_card[t]).
// DIRECT false: planned task list (key order, sparse key ranges); true: direct (task t = key key_lo + t; the
// pipelined op's key ranges, and dense ranges with RBG_PW_BALANCE=0)
template <int OP, int MODE, bool DIRECT>
__global__ __launch_bounds__(256, 4) void k_pair_wave(const PTask* __restrict__ tasks,
                                                      const uint32_t* __restrict__ n_tasks, const uint8_t* pa,
                                                      const uint8_t* pb, OutCtx oc, uint32_t* __restrict__ task_card,
                                                      PwDirect dsrc) {
  __shared__ __align__(16) uint32_t lds_all[kWaves][kWaveLds];
  if (DIRECT) {
    // the plan kernel's other duties: the task count and the op's zeroed look-back state
    plan_zero(dsrc.zlb, dsrc.ztile);
    if (blockIdx.x == 0 && threadIdx.x == 0) dsrc.n_tasks_out[0] = dsrc.n_tasks_write;
  }
  const uint32_t nt = DIRECT ? dsrc.nkeys : uni(*n_tasks);
  const int w = threadIdx.x >> 6;
  uint32_t* lds = lds_all[w];
  const uint32_t stride = gridDim.x * kWaves;
  const uint32_t t0 = uni(blockIdx.x * kWaves + w);
  if (t0 >= nt) return;
  uint32_t t = t0;
  if (DIRECT) {
    // The wave first resolves all of its tasks at once (lane k: task t0 + k * stride, vector
    // loads through both key CSRs) into its own region of the task buffer, wave-major, then
    // runs them with the planned form's one scalar record load per task.  (Resolving each
    // task through a chain of scalar loads in the loop made every load's result wait at the
    // loop head: SMEM returns out of order, so any use waits for all of them.)
    // tasks of the first wave (the most), rounded to 4 records (128 B): no scalar-cache line
    // holds records of two waves
    const uint32_t per = (((nt + stride - 1) / stride) + 3) & ~3u;
    PTask* mine = const_cast<PTask*>(tasks) + (size_t)t0 * per;
    const int l = lane_id();
    for (uint32_t k0 = 0; k0 < per; k0 += 64) {
      const uint32_t k = k0 + (uint32_t)l, tk = t0 + k * stride;
      if (k < per && tk < nt) {
        const uint32_t key = (uint32_t)dsrc.key_lo + tk;
        PTask r;
        resolve(dsrc.koa, dsrc.da, pa, key, r.slot_a, r.card_a, r.kind_a, r.nruns_a);
        resolve(dsrc.kob, dsrc.db, pb, key, r.slot_b, r.card_b, r.kind_b, r.nruns_b);
        r.key = (uint16_t)key;
        mine[k] = r;
      }
    }
    // the records are read back through the scalar cache (a fresh line per wave region: no
    // other wave writes it, and the scalar cache holds nothing of it yet)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the stores are in the L2 the scalar loads read
    uint32_t k = 0;
    PTask cur = load_task(mine, 0);
    for (;;) {
      const uint32_t tn = t + stride;
      PTask nxt;
      if (tn < nt) nxt = load_task(mine, k + 1);  // in flight while this task runs
      if (has_task<OP>(cur)) {
        any_task<OP, MODE>(t, cur, pa, pb, oc, task_card, lds);
      } else if (MODE == 1) {
        if (l == 0) task_card[t] = 0;
      } else {
        w_place(t, false, nullptr, true, lds, 0, 0, cur.key, DK_A, oc);
      }
      if (tn >= nt) break;
      t = tn;
      k++;
      cur = nxt;
    }
    return;
  }
  PTask cur = load_task(tasks, t);
  for (;;) {
    const uint32_t tn = t + stride;
    PTask nxt;
    if (tn < nt) nxt = load_task(tasks, tn);  // in flight while this task runs
    any_task<OP, MODE>(t, cur, pa, pb, oc, task_card, lds);
    if (tn >= nt) break;
    t = tn;
    cur = nxt;
  }
}

// ---------------------------------------------------------------------------
// Balanced list, one workgroup of 16 waves per CU (the CU's whole LDS), the CU's tasks claimed
// through an LDS counter.  The per-wave probe showed each CU's waves ending 50-60 us apart with
// equal work: the issue arbiter favours older waves, so the youngest workgroups of a CU form the
// tail.  Here the 16 waves of a CU drain one pool, so a wave that loses arbitration simply runs
// fewer tasks and the CU ends with its last task, not with its slowest wave.  CU b owns positions
// 16 b + w (w < 16) of every band of S = 16 x grid list positions: 16 consecutive cost ranks per
// band, every rank once over the bands (k_plan_balanced's layout).  Claim k takes band
// (k mod nb + b) mod nb, slot k / nb: the CU's waves work on different bands at once.  A claim is one LDS atomic; the next task is claimed and its
// record requested while a task runs.  (Round 5 measured, profiles/r05/experiments/: claim orders
// putting each CU's heaviest ranks first, or each round of claims heavy to light, the same or
// slower, c2_cu_claim_order.txt; pools of the last 1 / 2 / 4 bands shared by ALL CUs through one
// agent-scope counter 0.23 -> 0.34 / 0.44 / 0.60 ms, c2_cu_tail_pools.txt -- one counter saturates
// at ~88 claims per us (MI355X_MICROARCH.md, dequeue row), i.e. 47 us for one band's 4,096 claims.)
// (Round 6, profiles/r06/experiments/cu_tail_pools.txt: the lightest two bands left out of the own pools
// and claimed from 8 shared agent-scope counters once a CU's own pool is dry: +1.6 %, not kept.)
// ---------------------------------------------------------------------------
constexpr int kCuWaves = 16;
static_assert(kCuWaves * kWaveLds * 4 + 16 <= 163840, "16 waves and the counter in one CU's LDS");
template <int OP, int MODE>
__global__ __launch_bounds__(1024, 1) void k_pair_cu(const PTask* __restrict__ tasks, const uint32_t* __restrict__ n_tasks,
                                                     const uint8_t* pa, const uint8_t* pb, OutCtx oc,
                                                     uint32_t* __restrict__ task_card, PwDirect dsrc) {
  __shared__ __align__(16) uint32_t lds_all[kCuWaves][kWaveLds];
  __shared__ uint32_t ctr;
  if (threadIdx.x == 0) ctr = 0;
  __syncthreads();
  const uint32_t nt = uni(n_tasks[1]);
  uint32_t* lds = lds_all[threadIdx.x >> 6];
  const uint32_t S = gridDim.x * kCuWaves;
  const uint32_t nb = (nt + S - 1) / S;
  const uint32_t total = nb * kCuWaves, base = blockIdx.x * kCuWaves;
  auto claim = [&]() -> uint32_t {  // the next list position of this wave, ~0u when none is left
    for (;;) {
      uint32_t v = 0;
      if (lane_id() == 0) v = atomicAdd(&ctr, 1u);
      const uint32_t k = uni(v);
      if (k >= total) return ~0u;
      const uint32_t p = ((k % nb + blockIdx.x) % nb) * S + base + k / nb;  // band (k mod nb + b) mod nb, slot k / nb
      if (p < nt) return p;
    }
  };
  uint32_t p = claim();
  if (p == ~0u) return;
  PTask cur = load_task(tasks, p);
  for (;;) {
    const uint32_t pn = claim();
    PTask nxt;
    if (pn != ~0u) nxt = load_task(tasks, pn);  // in flight while this task runs
    if (cur.kind_a != kAbsent || cur.kind_b != kAbsent)  // marked: no task (the plan wrote its record)
      any_task<OP, MODE>((uint32_t)cur.key - (uint32_t)dsrc.key_lo, cur, pa, pb, oc, task_card, lds);
    if (pn == ~0u) break;
    cur = nxt;
  }
}

template <int OP, int MODE>
static void launch_pw(hipStream_t s, int grid, const PTask* tasks, const uint32_t* nt, const uint8_t* pa,
                      const uint8_t* pb, OutCtx oc, uint32_t* task_card, const PwDirect* direct, bool balanced) {
  if (direct && balanced) {  // one workgroup per CU, all of them resident
    const int g = std::max(1, resident_grid((const void*)&k_pair_cu<OP, MODE>, 1024));
    hipLaunchKernelGGL((k_pair_cu<OP, MODE>), dim3(g), dim3(1024), 0, s, tasks, nt, pa, pb, oc, task_card, *direct);
    return;
  }
  if (direct) {
    // Direct mode lays each wave's tasks out in a region of per = ceil(nt / stride) + 3 (rounded to 4)
    // records, stride = 4 g waves: at most nt + 4 stride records.  The task buffer holds
    // kMaxKeys + 32768 (engine.cpp: ctx_init), so stride <= 8192 waves: g <= 2048 workgroups.
    const int g = std::max(1, std::min({grid, resident_grid((const void*)&k_pair_wave<OP, MODE, true>), 2048}));
    hipLaunchKernelGGL((k_pair_wave<OP, MODE, true>), dim3(g), dim3(256), 0, s, tasks, nt, pa, pb, oc, task_card,
                       *direct);
    return;
  }
  const int g = std::max(1, std::min(grid, resident_grid((const void*)&k_pair_wave<OP, MODE, false>)));
  hipLaunchKernelGGL((k_pair_wave<OP, MODE, false>), dim3(g), dim3(256), 0, s, tasks, nt, pa, pb, oc, task_card,
                     PwDirect{});
}

// the diagnostic per-phase stamps builds were retired in round 6 (their results are in profiles/r02-r05)
void debug_stamps(uint64_t* out20, bool) {
  for (int i = 0; i < 20; i++) out20[i] = 0;
}

template <int OP, int MODE>
static void launch_pb(hipStream_t s, int key_lo, uint32_t nkeys, const uint32_t* koa, const CDesc* da,
                      const uint8_t* pa, const uint32_t* kob, const CDesc* db, const uint8_t* pb, PTask* tasks,
                      uint32_t* n_tasks, OutCtx oc, uint32_t* task_card, uint64_t* zlb, uint64_t* ztile) {
  hipLaunchKernelGGL((k_plan_balanced<OP, MODE>), dim3((nkeys + 255) / 256), dim3(256), 0, s, key_lo, nkeys, koa, da,
                     pa, kob, db, pb, tasks, n_tasks, oc, task_card, zlb, ztile);
}
void launch_plan_balanced(hipStream_t s, int op, int mode, int key_lo, uint32_t nkeys, const uint32_t* koa,
                          const CDesc* da, const uint8_t* pa, const uint32_t* kob, const CDesc* db, const uint8_t* pb,
                          PTask* tasks, uint32_t* n_tasks, OutCtx oc, uint32_t* task_card, uint64_t* zlb,
                          uint64_t* ztile) {
#define RBG_LPB(O)                                                                                                  \
  if (mode == 0)                                                                                                    \
    launch_pb<O, 0>(s, key_lo, nkeys, koa, da, pa, kob, db, pb, tasks, n_tasks, oc, task_card, zlb, ztile); \
  else                                                                                                              \
    launch_pb<O, 1>(s, key_lo, nkeys, koa, da, pa, kob, db, pb, tasks, n_tasks, oc, task_card, zlb, ztile);
  switch (op) {
    case OP_AND: RBG_LPB(OP_AND) break;
    case OP_OR: RBG_LPB(OP_OR) break;
    case OP_XOR: RBG_LPB(OP_XOR) break;
    default: RBG_LPB(OP_ANDNOT) break;
  }
#undef RBG_LPB
}

void launch_plan_pairwise(hipStream_t s, int op, int key_lo, int key_hi, const uint32_t* koa, const CDesc* da,
                          const uint8_t* pa, const uint32_t* kob, const CDesc* db, const uint8_t* pb,
                          uint64_t* wg_epoch, uint32_t epoch, PTask* tasks, uint32_t* n_tasks, uint64_t* zlb,
                          uint64_t* ztile, uint32_t* err) {
  hipLaunchKernelGGL(k_plan_pairwise, dim3(256), dim3(256), 0, s, op, key_lo, key_hi, koa, da, pa, kob, db, pb, wg_epoch,
                     epoch, tasks, n_tasks, zlb, ztile, err);
}

void launch_pairwise(hipStream_t s, int op, int mode, int grid, const PTask* tasks, const uint32_t* nt, const uint8_t* pa,
                     const uint8_t* pb, OutCtx oc, uint32_t* task_card, const PwDirect* direct, bool balanced) {
#define RBG_LPW(O)                                                                             \
  if (mode == 0) launch_pw<O, 0>(s, grid, tasks, nt, pa, pb, oc, task_card, direct, balanced); \
  else launch_pw<O, 1>(s, grid, tasks, nt, pa, pb, oc, task_card, direct, balanced);
  switch (op) {
    case OP_AND: RBG_LPW(OP_AND) break;
    case OP_OR: RBG_LPW(OP_OR) break;
    case OP_XOR: RBG_LPW(OP_XOR) break;
    default: RBG_LPW(OP_ANDNOT) break;
  }
#undef RBG_LPW
}

}  // namespace rbg
