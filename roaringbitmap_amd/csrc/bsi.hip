// Bit-sliced index query on the MI355X: RoaringBitmapSliceIndex.compare + sum
// (bsi/src/main/java/org/roaringbitmap/bsi/RoaringBitmapSliceIndex.java, BSI/
// below).
//
// The reference runs the O'Neil circuit (BSI/:432-468) as a chain of whole-bitmap
// pairwise ops, about 4 per slice. Each op is independent per high-16 key, so a
// workgroup takes one key. The result container types must be the reference's,
// so every step follows the pairwise type rule of the op it stands for (App. A,
// device.hpp): present / absent (an unmatched container is cloned, an empty result
// dropped), kind, cardinality, and the run count where EFF decides.
//
// Two forms:
//  * k_bsi_reg + k_bsi_types (compare ops, <= 32 slices): the slices of a key are
//    held in registers and read once; bits, counts and types are separate passes
//    (see "Register-resident query" below).  sum (BSI/:581-592) comes from the
//    same registers.
//  * bsi_task_streamed (k_bsi: BSI_ALL / sum alone, and k_bsi_defer: keys whose
//    type replay needs a run count): slices streamed step by step, each step's
//    cardinality reduced over the workgroup; sum re-reads the slices.
//
// Batch inputs (key-major): input 0 = ebM, inputs 1..nb = bA[0..nb-1],
// input nb+1 = foundSet (optional).
#include <algorithm>
#include <cstdio>
#include <cstdlib>

#include "kernels.hpp"
#include "vb.hpp"
#include "wave.hpp"

namespace rbg {

__device__ __forceinline__ void vb_load(int p, const WideArgs& A, uint32_t* tmp, int* q, VB& z) {
  if (p < 0) {
    vb_absent(z);
    return;
  }
  const CDesc d = A.desc[p];
  materialize(d, A.payload, tmp, q, z.r);
  z.present = 1;
  z.kind = d.kind;
  z.card = (int)d.card;
  z.src = p;
}

// O'Neil circuit step for one predicate (BSI/:441-452)
__device__ __forceinline__ void oneil_step(int bit, const VB& s, VB& gt, VB& lt, VB& eq, VB& t, uint32_t* lds,
                                           int* sh) {
  if (bit) {
    vb_op<OPR_ANDNOT>(eq, s, t, lds, sh);  // LT = or(LT, andNot(EQ, bA[i]))
    vb_op<OPR_OR>(lt, t, lt, lds, sh);
    vb_op<OPR_AND>(eq, s, eq, lds, sh);  // EQ = and(EQ, bA[i])
  } else {
    vb_op<OPR_AND>(eq, s, t, lds, sh);  // GT = or(GT, and(EQ, bA[i]))
    vb_op<OPR_OR>(gt, t, gt, lds, sh);
    vb_op<OPR_ANDNOT>(eq, s, eq, lds, sh);  // EQ = andNot(EQ, bA[i])
  }
}

// BSI/:453-467: the op's result from the circuit state
__device__ __forceinline__ void oneil_finish(int op, const VB& fixed, const VB& gt, const VB& lt, VB& eq, VB& out,
                                             uint32_t* lds, int* sh) {
  vb_op<OPR_AND>(fixed, eq, eq, lds, sh);  // EQ = and(fixedFoundSet, EQ)
  switch (op) {
    case BSI_EQ: out = eq; break;
    case BSI_NEQ: vb_op<OPR_ANDNOT>(fixed, eq, out, lds, sh); break;
    case BSI_GT: vb_op<OPR_AND>(gt, fixed, out, lds, sh); break;
    case BSI_LT: vb_op<OPR_AND>(lt, fixed, out, lds, sh); break;
    case BSI_LE: vb_op<OPR_OR>(lt, eq, out, lds, sh); break;
    default: vb_op<OPR_OR>(gt, eq, out, lds, sh); break;  // GE
  }
}

// Block 0 also zeroes the op's sum words (zsums, kBsiSumWords u64) and the defer count.
__global__ __launch_bounds__(256) void k_plan_bsi(const uint32_t* __restrict__ key_off, const uint32_t* __restrict__ bm,
                                                  uint32_t need, Task* __restrict__ by_key, uint8_t* __restrict__ flag,
                                                  uint32_t* __restrict__ wg_count, uint64_t* zlb, uint64_t* ztile,
                                                  unsigned long long* zsums, uint32_t* zdefer) {
  plan_zero(zlb, ztile);
  if (blockIdx.x == 0) {
    if (zsums)
      for (int i = threadIdx.x; i < kBsiSumAll; i += blockDim.x) zsums[i] = 0;
    if (zdefer && threadIdx.x == 0) zdefer[0] = 0;
  }
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t s = key_off[k], n = key_off[k + 1] - s;
  // a key yields a result only where input `need` (ebM, or foundSet for sum alone) has a container
  int f = need == 0xFFFFFFFEu && n > 0;  // 0xFFFFFFFE: any input (buffer package: every key of any input)
  for (uint32_t j = 0; j < n; j++) f |= bm[s + j] == need;
  flag[k] = (uint8_t)f;
  by_key[k] = Task{k, (int32_t)s, (int32_t)n, 0};
  plan_count(f, wg_count);
}

// One key of the query, streamed: every slice container is loaded when its
// circuit step runs and every pairwise step reduces its cardinality over the
// workgroup right away (two barriers per step); sum re-reads the slices against
// the result.  Used for BSI_ALL / BSI_SUM_ONLY and, inside k_bsi_reg, for keys
// whose type replay needs a run count.
__device__ __forceinline__ void bsi_task_streamed(uint32_t t, const Task tk, const WideArgs& A, const BsiArgs& P,
                                               const OutCtx& oc, unsigned long long* __restrict__ sums, uint32_t* acc,
                                               uint32_t* tmp, int* q, int* sh, int* pos) {
  const int nb = P.nbits;
  const uint32_t s = uni((uint32_t)tk.a), n = uni((uint32_t)tk.b);
  __syncthreads();
  for (int j = threadIdx.x; j < kBsiMaxInputs; j += NT) pos[j] = -1;
  __syncthreads();
  for (uint32_t j = threadIdx.x; j < n; j += NT) pos[A.bm[s + j]] = (int)(s + j);
  __syncthreads();
  VB res;
  if (P.op == BSI_SUM_ONLY) {
    vb_load(pos[nb + 1], A, tmp, q, res);
  } else if (P.op == BSI_ALL) {
    VB ebm;
    vb_load(pos[0], A, tmp, q, ebm);
    if (P.has_found) {
      VB f;
      vb_load(pos[nb + 1], A, tmp, q, f);
      vb_op<OPR_AND>(ebm, f, res, acc, sh);
    } else {
      res = ebm;  // ebM.clone()
    }
  } else {
    VB ebm, eq0, gt0, lt0, eq1, gt1, lt1, sl, tv;
    vb_load(pos[0], A, tmp, q, ebm);
    eq0 = ebm;
    eq1 = ebm;
    vb_absent(gt0);
    vb_absent(lt0);
    vb_absent(gt1);
    vb_absent(lt1);
    const bool two = P.op == BSI_RANGE;
    for (int i = nb - 1; i >= 0; i--) {
      vb_load(pos[1 + i], A, tmp, q, sl);
      oneil_step((P.pred0 >> i) & 1, sl, gt0, lt0, eq0, tv, acc, sh);
      if (two) oneil_step((P.pred1 >> i) & 1, sl, gt1, lt1, eq1, tv, acc, sh);
    }
    VB fixed;
    if (P.has_found) vb_load(pos[nb + 1], A, tmp, q, fixed);
    else fixed = ebm;
    if (two) {  // RANGE = and(GE(start), LE(end)), BSI/:503-507
      VB left, right;
      oneil_finish(BSI_GE, fixed, gt0, lt0, eq0, left, acc, sh);
      oneil_finish(BSI_LE, fixed, gt1, lt1, eq1, right, acc, sh);
      vb_op<OPR_AND>(left, right, res, acc, sh);
    } else {
      oneil_finish(P.op, fixed, gt0, lt0, eq0, res, acc, sh);
    }
  }
  if (sums) {
    // sum: |bA[x] & found| per slice (Java int per slice, wrapped on the host), count
    if (res.present) {
      for (int x = 0; x < nb; x++) {
        const int p = pos[1 + x];
        if (p < 0) continue;
        uint64_t r[4];
        materialize(A.desc[p], A.payload, tmp, q, r);
        int c = 0;
#pragma unroll
        for (int i = 0; i < 4; i++) c += popc64(r[i] & res.r[i]);
        int u = 0;
        block_sum2(c, u, sh);
        if (threadIdx.x == 0 && c) atomicAdd(&sums[x], (unsigned long long)c);
      }
      if (threadIdx.x == 0) atomicAdd(&sums[kBsiMaxInputs], (unsigned long long)res.card);
    }
  }
  if (P.op == BSI_SUM_ONLY) return;
  if (!res.present) {
    wg_place(t, false, nullptr, true, tmp, 0, 0, tk.key, DK_A, oc, nullptr);
  } else if (res.src >= 0) {
    wg_passthrough(t, A.desc[res.src], A.payload, oc, nullptr);
  } else {
    const uint32_t len = stage_container(res.kind, res.r, res.card, acc, tmp, sh);
    wg_place(t, true, nullptr, true, tmp, len, (uint32_t)res.card, tk.key, res.kind, oc, nullptr);
  }
}

// mode: BSI_* op (compare, + sum of the result when `sums` is set), or BSI_SUM_ONLY
__global__ __launch_bounds__(256) void k_bsi(const Task* __restrict__ tasks, const uint32_t* __restrict__ n_tasks,
                                             WideArgs A, BsiArgs P, OutCtx oc,
                                             unsigned long long* __restrict__ sums) {
  __shared__ __align__(16) uint32_t acc[2048];
  __shared__ __align__(16) uint32_t tmp[2048];
  __shared__ int q[257];
  __shared__ int sh[8];
  __shared__ int pos[kBsiMaxInputs];
  const uint32_t nt = *n_tasks;
  for (uint32_t t = blockIdx.x; t < nt; t += gridDim.x) bsi_task_streamed(t, tasks[t], A, P, oc, sums, acc, tmp, q, sh, pos);
}

// ===========================================================================
// Register-resident query (compare ops, nbits <= 32): k_bsi_reg + k_bsi_types
// ===========================================================================
// The streamed form above is bound by its ~6 workgroup reductions per slice (two
// barriers each, a dependent chain of ~190 per key) and reads every slice twice.
// The bits of the circuit are independent per container word; only the
// cardinalities that decide the result types (App. A) need the whole key.  So:
//  * k_bsi_reg works on units of 256 container words (a quarter key) with one
//    thread per word.  A unit holds all of its slices in registers (one u64 per
//    slice per thread), requests them all at once, runs the circuit on the bits
//    and writes its quarter of the result bits to the task's scratch slot.  Per
//    step only t = EQ & bA[i] (or EQ & ~bA[i]) is counted: t and the new EQ
//    partition the old EQ, and t is disjoint from GT / LT, so |EQ'| = |EQ| - |t|
//    and |GT'| = |GT| + |t| follow by arithmetic.  sum's shares |bA[x] & result|
//    come from the same registers, so the index is read once.  Each unit writes
//    its partial counts; several units per CU are resident, so one unit's loads
//    overlap another's compute.
//  * k_bsi_types, one thread per key, adds the units' partial counts and replays
//    the reference's type rule of every step (see there).
// A key whose replay needs a run count (EFF) is redone by k_bsi_defer with the
// streamed form; array / run results are staged there from the bits.
constexpr int kBsiRegSlices = 32;
// compare without sum: slices [0, kBsiCut) wait for EQ to survive the rest (13 measured
// against 10 and 15, profiles/r04/experiments/bsi_cut_variants.txt)
constexpr int kBsiCut = 13;
constexpr int kBsiUnits = 4;                // units per key
constexpr int kUnitWords = 1024 / kBsiUnits;  // container words per unit = threads per workgroup
static_assert(kUnitWords == NT, "a unit is one 256-thread workgroup");
constexpr int kBsiRows = 69 + kBsiRegSlices;  // |ebM|, circuit steps, finish, sum shares (rows below)
constexpr int kRowB = kUnitWords + 16;  // row stride in bytes (a wave reads a row; the pad spreads banks)
// fixed count rows: |ebM|; one per circuit step (slice i, predicate p); the finish;
// the sum shares.  Fixed (not sequential) so every row offset is a compile-time
// constant in the unrolled circuit; rows of skipped steps are never read.
constexpr int kRowEbm = 0;
__host__ __device__ constexpr int step_row(int i, int p) { return 1 + 2 * (31 - i) + p; }
constexpr int kRowFin = 65;  // single op: fixed & EQ, then NEQ / GT / LT; RANGE: GE's, LE's fixed & EQ, result
constexpr int kRowSum = 69;  // + slice

// Wave-uniform type state of a circuit bitmap (the bits live elsewhere).  card 0
// means absent: a present container is never empty (inputs hold >= 1 value,
// empty results are dropped), so presence needs no field of its own.
struct TB {
  int kind, card;
  int src;  // desc index of the input container it is a clone of, else -1
  int pad;
};
__device__ __forceinline__ TB tb_absent() { return TB{DK_A, 0, -1, 0}; }

// vb_op's type rule with the step's cardinality c already known, without
// branches (scalar selects); `slow` is set when the rule needs the result's run
// count.  AND: absent unless both present and c > 0; OR: a clone of the present
// side when the other is absent; ANDNOT: a clone of x when y is absent.
template <int OP>
__device__ __forceinline__ TB tb_op(const TB& x, const TB& y, int c, int& slow) {
  const bool xp = x.card > 0, yp = y.card > 0;
  int kind = by_card(c);
  if (OP == OPR_OR && (x.kind == DK_B || y.kind == DK_B)) kind = c == 65536 ? DK_R : DK_B;
  const bool need = pairwise_needs_runs(OP, x.kind, x.card, y.kind, y.card);
  const bool both = xp && yp && c > 0;
  TB r;
  if (OP == OPR_OR) {
    r.kind = !xp ? y.kind : !yp ? x.kind : kind;
    r.card = !xp ? y.card : !yp ? x.card : c;
    r.src = !xp ? y.src : !yp ? x.src : -1;
  } else if (OP == OPR_ANDNOT) {
    r.kind = !yp ? x.kind : both ? kind : DK_A;
    r.card = !yp ? x.card : both ? c : 0;
    r.src = !yp ? x.src : -1;
  } else {
    r.kind = both ? kind : DK_A;
    r.card = both ? c : 0;
    r.src = -1;
  }
  r.pad = 0;
  slow |= (both && need) ? 1 : 0;
  return r;
}

// this thread's share of count k (<= 64)
__device__ __forceinline__ void rec1(uint64_t z, int k, uint8_t* rows) {
  rows[k * kRowB + threadIdx.x] = (uint8_t)popc64(z);
}
// row sums of rows [0, nk), one thread per row (16 B reads, v_dot4 over the bytes),
// written as this unit's partial counts: cnt[row], contiguous (one coalesced store per
// wave; a transposed layout made each count a scattered 4 B write).
// Begins and ends with a barrier.
__device__ __forceinline__ void sum_rows_unit(const uint8_t* rows, int nk, int* cnt) {
  lds_barrier();
  const int r = threadIdx.x;
  if (r < nk) {
    const uint4* v = reinterpret_cast<const uint4*>(rows + r * kRowB);
    uint32_t c = 0;
#pragma unroll
    for (int j = 0; j < kUnitWords / 16; j++) {
      const uint4 x = v[j];
      c = __builtin_amdgcn_udot4(x.x, 0x01010101u, c, false);
      c = __builtin_amdgcn_udot4(x.y, 0x01010101u, c, false);
      c = __builtin_amdgcn_udot4(x.z, 0x01010101u, c, false);
      c = __builtin_amdgcn_udot4(x.w, 0x01010101u, c, false);
    }
    cnt[r] = (int)c;
  }
  lds_barrier();
}
// Type replay of a step / finish, in the order of the bits.  c* are the exact
// cardinalities of the bits (0 for an absent bitmap).
struct CircuitT {
  TB gt, lt, eq;
  int cgt, clt, ceq;
};
template <class CNT>
__device__ __forceinline__ void types_step(int bit, const TB& s, CircuitT& z, int row, const CNT& tv, int& slow) {
  const int ct = tv(row);
  if (bit) {
    const TB t = tb_op<OPR_ANDNOT>(z.eq, s, ct, slow);
    z.lt = tb_op<OPR_OR>(z.lt, t, z.clt + ct, slow);
    z.eq = tb_op<OPR_AND>(z.eq, s, z.ceq - ct, slow);
    z.clt += ct;
  } else {
    const TB t = tb_op<OPR_AND>(z.eq, s, ct, slow);
    z.gt = tb_op<OPR_OR>(z.gt, t, z.cgt + ct, slow);
    z.eq = tb_op<OPR_ANDNOT>(z.eq, s, z.ceq - ct, slow);
    z.cgt += ct;
  }
  z.ceq -= ct;
}
// BSI/:453-467 on types: counted are fixed & EQ (row re) and the NEQ / GT / LT
// results (row ro); LE / GE are disjoint unions
template <class CNT>
__device__ __forceinline__ TB types_finish(int op, const TB& fixed, CircuitT& z, int re, int ro, const CNT& tv,
                                           int& slow) {
  const int ce = tv(re);
  z.eq = tb_op<OPR_AND>(fixed, z.eq, ce, slow);
  z.ceq = ce;
  switch (op) {
    case BSI_EQ: return z.eq;
    case BSI_NEQ: return tb_op<OPR_ANDNOT>(fixed, z.eq, tv(ro), slow);
    case BSI_GT: return tb_op<OPR_AND>(z.gt, fixed, tv(ro), slow);
    case BSI_LT: return tb_op<OPR_AND>(z.lt, fixed, tv(ro), slow);
    case BSI_LE: return tb_op<OPR_OR>(z.lt, z.eq, z.clt + ce, slow);
    default: return tb_op<OPR_OR>(z.gt, z.eq, z.cgt + ce, slow);  // GE
  }
}
// the same on bits (this thread's word); counted: fixed & EQ (row re), NEQ / GT / LT (row ro)
__device__ __forceinline__ uint64_t bits_finish1(int op, uint64_t fixed, uint64_t gt, uint64_t lt, uint64_t& eq, int re,
                                                 int ro, uint8_t* rows) {
  eq &= fixed;
  rec1(eq, re, rows);
  uint64_t out;
  switch (op) {
    case BSI_EQ: return eq;
    case BSI_NEQ: out = fixed & ~eq; break;
    case BSI_GT: out = gt & fixed; break;
    case BSI_LT: out = lt & fixed; break;
    case BSI_LE: return lt | eq;
    default: return gt | eq;  // GE
  }
  rec1(out, ro, rows);
  return out;
}

// Word w of a container: a bitmap directly, arrays / runs through the 8 KiB LDS
// scratch (the whole container, 256-thread helpers).  All threads; barriers.
__device__ __forceinline__ uint64_t mat_unit_word(const CDesc& d, const uint8_t* payload, uint32_t* lds, int* q,
                                                  int w) {
  const uint8_t* slot = payload + d.slot;
  if (d.kind == DK_B) return reinterpret_cast<const uint64_t*>(slot)[w];
  lds_barrier();
  lds_clear(lds);
  lds_barrier();
  if (d.kind == DK_A) {
    lds_scatter_array(lds, reinterpret_cast<const uint16_t*>(slot), (int)d.card);
    lds_barrier();
  } else {
    lds_or_runs(lds, reinterpret_cast<const uint32_t*>(slot + 4), *reinterpret_cast<const uint16_t*>(slot + 2), q);
  }
  const uint64_t x = reinterpret_cast<const uint64_t*>(lds)[w];
  lds_barrier();
  return x;
}

// the per-workgroup probe build of k_bsi_reg was retired in round 6 (its results: profiles/r05/experiments)
void debug_bsi_stamps(uint64_t* out20, bool) {
  for (int i = 0; i < 20; i++) out20[i] = 0;
}

// task record of a result written by k_bsi_reg / k_bsi_defer (wg_place's record)
__device__ __forceinline__ void bsi_rec(uint32_t t, const OutCtx& oc, bool keep, const uint8_t* src, uint32_t len,
                                        uint32_t card, uint32_t key, int kind) {
  ORec r;
  r.off = 0;
  r.src = reinterpret_cast<uint64_t>(src);
  r.idx = 0;
  r.card = card;
  r.ser_len = len;
  r.key = (uint16_t)key;
  r.kind = (uint8_t)kind;
  r.keep = keep ? 1 : 0;
  oc.recs[t] = r;
}

constexpr int kBsiCnt = 128;
constexpr int kBsiKin = kBsiRegSlices + 2;
static_assert(kBsiRows <= kBsiCnt, "count rows");

// One input of a key (16 B): its container's slot, cardinality and kind, or absent
// (didx < 0).  k_bsi_table writes a row of kBsiKin per task, indexed by input
// (ebM, bA[0..nb-1], foundSet), so a wave of k_bsi_reg reads a key's inputs with one
// load (lane = input) and needs no search of the key segment.
struct BsiIn {
  uint64_t slot;
  uint32_t card_kind;  // card | kind << 24
  int32_t didx;        // desc index, -1 when the key has no container of this input
};
// One wave per key (4 keys per workgroup): lane j takes the key segment's container
// j, so the segment is read in one round instead of a serial walk per thread.
__global__ __launch_bounds__(256) void k_bsi_table(const Task* __restrict__ tasks, const uint32_t* __restrict__ n_tasks,
                                                   WideArgs A, BsiIn* __restrict__ table) {
  __shared__ unsigned long long present[4];
  const uint32_t nt = *n_tasks;
  const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const uint32_t t = blockIdx.x * 4 + w;
  if (t >= nt) return;  // wave-uniform
  const Task tk = tasks[t];
  BsiIn* row = table + (size_t)t * kBsiKin;
  if (lane == 0) present[w] = 0;
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  for (uint32_t j = (uint32_t)lane; j < (uint32_t)tk.b; j += 64) {
    const uint32_t p = (uint32_t)tk.a + j;
    const uint32_t b = A.bm[p];
    if (b < (uint32_t)kBsiKin) {
      const CDesc d = A.desc[p];
      row[b] = BsiIn{d.slot, d.card | ((uint32_t)d.kind << 24), (int32_t)p};
      atomicOr(&present[w], 1ull << b);
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
  __builtin_amdgcn_wave_barrier();
  if (lane < kBsiKin && !((present[w] >> lane) & 1)) row[lane] = BsiIn{0, 0, -1};  // the key has no container of input lane
}

// Word w of a key's input from its table entry: a full container needs no memory
// access, a bitmap one load, arrays / runs the LDS scratch (all threads; barriers).
__device__ __forceinline__ uint64_t in_word(uint64_t slot, uint32_t card_kind, int32_t didx, const WideArgs& A,
                                           uint32_t* lds, int* q, int w) {
  if (didx < 0) return 0;
  const uint32_t card = card_kind & 0xFFFFFF, kind = card_kind >> 24;
  if (card == 65536) return ~0ull;
  if (kind == DK_B) return reinterpret_cast<const uint64_t*>(A.payload + slot)[w];
  return mat_unit_word(A.desc[didx], A.payload, lds, q, w);
}

// compare ops (BSI_EQ .. BSI_RANGE) with nbits <= kBsiRegSlices.  cnts: per task and unit,
// kBsiCnt partial counts (one per count row); kin: per task, kBsiKin input types (slices,
// ebM, the fixed found set), contiguous.
__global__ __launch_bounds__(256, 4) void k_bsi_reg(const Task* __restrict__ tasks,
                                                                const uint32_t* __restrict__ n_tasks,
                                                 WideArgs A, BsiArgs P, OutCtx oc, bool want_sum,
                                                 const BsiIn* __restrict__ table, int* __restrict__ cnts,
                                                 TB* __restrict__ kin, size_t tstride, BsiScratch z) {
  if (blockIdx.x == 0 && z.table_ready) {  // the per-query zeroing of the (skipped) plan kernel
    plan_zero(z.zlb, z.ztile);
    if (z.zsums)
      for (int i = threadIdx.x; i < kBsiSumAll; i += blockDim.x) z.zsums[i] = 0;
    if (threadIdx.x == 0) {
      if (z.defer) z.defer[0] = 0;
      if (z.nt_dst) *z.nt_dst = *z.nt_src;
    }
  }
  // the 8 KiB scratch for array / run inputs aliases the count rows: inputs are
  // materialised before the circuit writes the rows, and after the last unit's sums
  __shared__ __align__(16) uint8_t rows[kBsiRows * kRowB];
  static_assert(kBsiRows * kRowB >= 8192, "scratch bitmap inside the rows");
  uint32_t* tmp = reinterpret_cast<uint32_t*>(rows);
  __shared__ int q[257];
  const uint64_t nunits = (uint64_t)*n_tasks * kBsiUnits;
  const int nb = P.nbits;
  const bool two = P.op == BSI_RANGE;
  const int tid = threadIdx.x, lane = tid & 63;
  // Units claimed from a pool per group of kBsiGroup workgroups (blockIdx mod G): the per-workgroup
  // probe showed a CU's four workgroups ending 653 / 695 / 736 / 771 us (dispatch order wins issue
  // arbitration) with a fixed 59-60 units each.  Group g owns the units [g U, g U + U); a claim is one
  // agent-scope atomic on the group's counter (zeroed by k_bsi_types after every query), issued a unit
  // ahead so its latency hides behind a unit's work.  Groups of 4 / 8 / 16 / 32 / 64 / 128 / 256
  // workgroups: C5 step 0.843 / 0.836 / 0.826 / 0.822 / 0.815 / 0.806 / 0.807 ms against 0.864 static
  // (profiles/r05/experiments/c5_bsi_pool_groups.txt): 128, i.e. 8 counters for a 1,024-workgroup grid.
  const uint32_t G = min((uint32_t)kBsiMaxGroups, max(1u, gridDim.x / kBsiGroup)), grp = blockIdx.x % G;
  const uint64_t U = (nunits + G - 1) / G, g0 = (uint64_t)grp * U;
  const uint64_t gcnt = g0 < nunits ? min(U, nunits - g0) : 0;
  unsigned int* gctr = z.claims + 16 * grp;
  __shared__ unsigned int claim_sh[2];
  if (tid == 0) {
    const unsigned int c0 = __hip_atomic_fetch_add(gctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned int c1 = __hip_atomic_fetch_add(gctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    claim_sh[0] = c0;
    claim_sh[1] = c1;
  }
  __syncthreads();
  const uint64_t kNone = ~0ull;
  auto unit_of = [&](unsigned int c) -> uint64_t { return (uint64_t)c < gcnt ? g0 + c : kNone; };
  uint64_t wi = unit_of(claim_sh[0]);
  uint64_t wn_claimed = unit_of(claim_sh[1]);
  if (wi == kNone) return;
  uint32_t parity = 0;
  // this unit's key inputs: lane i holds input i (0 = ebM, 1 + x = bA[x], nb + 1 = foundSet);
  // the next unit's row is requested while this unit runs
  BsiIn e = lane < kBsiKin ? table[(wi / kBsiUnits) * kBsiKin + lane] : BsiIn{0, 0, -1};
  // every bitmap slice word of a unit requested at once (slots through readlane); slice
  // x's bit in the returned mask says it was loaded.  The next unit's words are
  // requested as soon as this unit's slice registers are dead (after the circuit and
  // the sum shares), so they are in flight during this unit's result store and count
  // rows.
  uint64_t sl[kBsiRegSlices];
  // Without sum shares the slices below kBsiCut are requested only once EQ survives the ones
  // above (see the circuit): xlo = the lowest slice requested up front.
  const bool split = !want_sum && nb > kBsiCut;
  const int xlo = split ? kBsiCut : 0;
  auto request_slices = [&](const BsiIn& r, uint64_t unit) -> uint64_t {
    const int wq = (int)((unit % kBsiUnits) * kUnitWords) + tid;
    const uint32_t lo = (uint32_t)r.slot, hi = (uint32_t)(r.slot >> 32);
    const bool bmp = r.didx >= 0 && (r.card_kind >> 24) == DK_B && (r.card_kind & 0xFFFFFF) != 65536;
    const uint64_t m = __ballot(bmp && lane >= 1 && lane <= nb) >> 1;  // slice x at bit x
#pragma unroll
    for (int x = 0; x < kBsiRegSlices; x++) {
      const uint64_t slot = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)lo, 1 + x) |
                            ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)hi, 1 + x) << 32);
      // nontemporal: every index word is read once (C5 step -1.8 %, alternating runs on one box)
      sl[x] = ((m >> x) & 1) && x >= xlo
                  ? __builtin_nontemporal_load(reinterpret_cast<const uint64_t*>(A.payload + slot) + wq)
                  : 0;
    }
    return m;
  };
  uint64_t bmask = request_slices(e, wi);
  for (;;) {
    const uint32_t t = (uint32_t)(wi / kBsiUnits), u = (uint32_t)(wi % kBsiUnits);
    const uint64_t wn = wn_claimed == kNone ? nunits : wn_claimed;  // >= nunits: no next unit
    unsigned int pending = 0;
    if (tid == 0 && wn < nunits)  // the claim after the next one, consumed at this unit's end
      pending = __hip_atomic_fetch_add(gctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    BsiIn en{0, 0, -1};
    if (wn < nunits && lane < kBsiKin) en = table[(wn / kBsiUnits) * kBsiKin + lane];
    const int w = (int)(u * kUnitWords) + tid;  // this thread's container word
    const uint32_t lo = (uint32_t)e.slot, hi = (uint32_t)(e.slot >> 32);
    auto input_word = [&](int i) -> uint64_t {
      const uint64_t slot = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)lo, i) |
                            ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)hi, i) << 32);
      return in_word(slot, (uint32_t)__builtin_amdgcn_readlane((int)e.card_kind, i),
                     __builtin_amdgcn_readlane(e.didx, i), A, tmp, q, w);
    };
    const uint64_t ebm = input_word(0);  // a task exists only where ebM has the key
    const uint64_t fixed = P.has_found ? input_word(nb + 1) : ebm;
#pragma unroll
    for (int x = 0; x < kBsiRegSlices; x++) {  // full, array and run slices
      if (x < nb && !((bmask >> x) & 1) && __builtin_amdgcn_readlane(e.didx, 1 + x) >= 0) sl[x] = input_word(1 + x);
    }
    // 2. bits of the whole circuit; each thread's share of every count to LDS.  GT is
    // not tracked: GT, LT and EQ partition ebM, so GT = ebM ^ LT ^ EQ at the end.
    uint64_t eq0 = ebm, lt0 = 0, eq1 = ebm, lt1 = 0, res;
    rec1(ebm, kRowEbm, rows);  // |ebM| of the bits: the start of the derived cardinalities
    // predicate bits i = 31 .. 0 as the top bit of running copies; the asm keeps the
    // compiler from precomputing 64 per-step flags (SGPR spills)
    uint32_t p0 = P.pred0, p1 = P.pred1;
    int live = 32 - nb;  // steps i >= nb are skipped
#pragma unroll
    for (int i = kBsiRegSlices - 1; i >= 0; i--) {
      if (i == kBsiCut - 1 && split) {
        // Where EQ is empty every remaining step counts 0 and changes no bit, so the low
        // slices matter only if EQ survived the high ones somewhere in the unit.  (The
        // reference's and(EQ, bA[i]) skips a key whose EQ holds no container, so it does
        // not read the slice there either.)
        if (__syncthreads_or((two ? (eq0 | eq1) : eq0) != 0)) {
#pragma unroll
          for (int x = 0; x < kBsiCut; x++) {
            const uint64_t slot = (uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)lo, 1 + x) |
                                  ((uint64_t)(uint32_t)__builtin_amdgcn_readlane((int)hi, 1 + x) << 32);
            if ((bmask >> x) & 1)
              sl[x] = __builtin_nontemporal_load(reinterpret_cast<const uint64_t*>(A.payload + slot) + w);
          }
        }
      }
      asm volatile("" : "+s"(p0), "+s"(p1), "+s"(live));
      if (live <= 0) {
        // bit i of the predicate (the top bit of the opaque running copy) picks the
        // step's form with a scalar branch
        if ((int32_t)p0 < 0) {  // LT |= EQ & ~bA[i]; EQ &= bA[i]
          const uint64_t tv = eq0 & ~sl[i];
          rec1(tv, step_row(i, 0), rows);
          lt0 |= tv;
          eq0 ^= tv;
        } else {  // GT |= EQ & bA[i]; EQ &= ~bA[i]
          const uint64_t tv = eq0 & sl[i];
          rec1(tv, step_row(i, 0), rows);
          eq0 ^= tv;
        }
        if (two) {
          if ((int32_t)p1 < 0) {
            const uint64_t tw = eq1 & ~sl[i];
            rec1(tw, step_row(i, 1), rows);
            lt1 |= tw;
            eq1 ^= tw;
          } else {
            const uint64_t tw = eq1 & sl[i];
            rec1(tw, step_row(i, 1), rows);
            eq1 ^= tw;
          }
        }
      }
      p0 <<= 1;
      p1 <<= 1;
      live--;
    }
    if (two) {  // RANGE = and(GE(start), LE(end)), BSI/:503-507
      const uint64_t left = bits_finish1(BSI_GE, fixed, ebm ^ lt0 ^ eq0, lt0, eq0, kRowFin, 0, rows);
      const uint64_t right = bits_finish1(BSI_LE, fixed, ebm ^ lt1 ^ eq1, lt1, eq1, kRowFin + 1, 0, rows);
      res = left & right;
      rec1(res, kRowFin + 2, rows);
    } else {
      res = bits_finish1(P.op, fixed, ebm ^ lt0 ^ eq0, lt0, eq0, kRowFin, kRowFin + 1, rows);
    }
    // sum shares |bA[x] & result| (an absent result has no bits: all zero)
    if (want_sum) {
#pragma unroll
      for (int x = 0; x < kBsiRegSlices; x++)
        if (x < nb) rec1(sl[x] & res, kRowSum + x, rows);
    }
    // the slice registers are dead: the next unit's bitmap slices are requested now
    uint64_t bmask_n = 0;
    if (wn < nunits) bmask_n = request_slices(en, wn);
    // this unit's result words to the task's scratch slot (the container itself when
    // it is a bitmap, else the input k_bsi_defer stages it from)
    reinterpret_cast<uint64_t*>(oc.scratch + (size_t)t * kSlotBytes)[w] = res;
    // (two slots: the slot read after this unit's barriers is written again only after the next
    // unit's first barrier)
    if (tid == 0) claim_sh[parity] = wn < nunits ? pending : 0xFFFFFFFFu;
    sum_rows_unit(rows, want_sum ? kRowSum + nb : kRowSum, cnts + ((size_t)t * kBsiUnits + u) * kBsiCnt);
    const unsigned int cnext = claim_sh[parity];
    parity ^= 1u;
    if (u == 0 && tid < kBsiKin) {  // the key's input types, for k_bsi_types
      const int i = tid == kBsiRegSlices ? 0 : tid == kBsiRegSlices + 1 ? (P.has_found ? nb + 1 : 0) : 1 + tid;
      const BsiIn x = table[(size_t)t * kBsiKin + (i < kBsiKin ? i : 0)];
      const bool present = x.didx >= 0 && (tid >= kBsiRegSlices || tid < nb);
      kin[(size_t)t * kBsiKin + tid] =
          present ? TB{(int)(x.card_kind >> 24), (int)(x.card_kind & 0xFFFFFF), x.didx, 0} : tb_absent();
    }
    if (wn >= nunits) break;
    wi = wn;
    e = en;
    bmask = bmask_n;
    wn_claimed = cnext == 0xFFFFFFFFu ? kNone : unit_of(cnext);
  }
}

// Types of the keys k_bsi_reg computed, one THREAD per key (64 keys per 256-thread
// block): the keys' counts (the units' partials added) and input types are first
// staged in LDS by all four waves -- every load independent -- then the reference's
// type rule of every step is replayed from them with branch-free selects, 16 keys per
// wave (the replay is a serial chain per key: spread over four times the waves it
// ends sooner), and the result record written.  A bitmap result is already in the scratch slot; array / run
// results (staged from it) and keys whose replay needs a run count go to
// k_bsi_defer.  Sums: per slice one wave reduction, one atomic.
struct LdsCounts {
  const int* col;  // this lane's column of the staged counts (row stride 64)
  __device__ __forceinline__ int operator()(int r) const { return col[r * 64]; }
};
__global__ __launch_bounds__(256) void k_bsi_types(const Task* __restrict__ tasks, const uint32_t* __restrict__ n_tasks,
                                                   WideArgs A, BsiArgs P, OutCtx oc,
                                                   unsigned long long* __restrict__ sums, const int* __restrict__ cnts,
                                                   const TB* __restrict__ kin, size_t tstride,
                                                   uint32_t* __restrict__ defer, unsigned int* __restrict__ claims) {
  __shared__ int lc[kBsiRows * 64];
  __shared__ TB lk[kBsiKin * 64];
  if (blockIdx.x == 0 && claims)  // k_bsi_reg's unit pools, for the next query
    for (int i = threadIdx.x; i < kBsiClaimWords; i += blockDim.x) claims[i] = 0;
  const uint32_t nt = *n_tasks;
  const int nb = P.nbits;
  const bool two = P.op == BSI_RANGE;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (uni(blockIdx.x * 64) >= nt) return;
  // the block stages the 64 keys' counts: each key's units wrote their rows contiguously
  // (cnts[(task * kBsiUnits + unit) * kBsiCnt + row]); a thread takes four rows of a key as
  // 16 B, adds the units' partials, and every thread's loads are issued at once (one round
  // trip for the block)
  {
    constexpr int kQuads = (kBsiRows + 3) / 4;
    constexpr int kIt = (64 * kQuads + NT - 1) / NT;
    static_assert(kBsiCnt % 4 == 0 && 4 * kQuads <= kBsiCnt, "row quads");
    int4 acc[kIt];
#pragma unroll
    for (int it = 0; it < kIt; it++) {  // every load first
      const int x = it * NT + (int)threadIdx.x;
      const int j = x / kQuads, q = x - j * kQuads;
      const uint32_t tj = blockIdx.x * 64 + j;
      acc[it] = make_int4(0, 0, 0, 0);
      if (x < 64 * kQuads && tj < nt) {
        const int4* p = reinterpret_cast<const int4*>(cnts + (size_t)tj * kBsiUnits * kBsiCnt) + q;
#pragma unroll
        for (int u = 0; u < kBsiUnits; u++) {
          const int4 v = p[u * (kBsiCnt / 4)];
          acc[it].x += v.x;
          acc[it].y += v.y;
          acc[it].z += v.z;
          acc[it].w += v.w;
        }
      }
    }
#pragma unroll
    for (int it = 0; it < kIt; it++) {
      const int x = it * NT + (int)threadIdx.x;
      const int j = x / kQuads, r = 4 * (x - j * kQuads);
      if (x < 64 * kQuads) {
        lc[r * 64 + j] = acc[it].x;
        if (r + 1 < kBsiRows) lc[(r + 1) * 64 + j] = acc[it].y;
        if (r + 2 < kBsiRows) lc[(r + 2) * 64 + j] = acc[it].z;
        if (r + 3 < kBsiRows) lc[(r + 3) * 64 + j] = acc[it].w;
      }
    }
  }
  // the 64 keys' input types: kBsiKin contiguous entries per key, read coalesced, every load
  // issued before the first LDS store
  {
    constexpr int kIt = (64 * kBsiKin + NT - 1) / NT;
    static_assert(sizeof(TB) == sizeof(int4), "TB as 16 B");
    int4 v[kIt];
#pragma unroll
    for (int it = 0; it < kIt; it++) {
      const int x = it * NT + (int)threadIdx.x;
      const int j = x / kBsiKin;
      const uint32_t tj = blockIdx.x * 64 + j;
      v[it] = make_int4(0, 0, 0, 0);
      if (x < 64 * kBsiKin && tj < nt)
        v[it] = reinterpret_cast<const int4*>(kin)[(size_t)tj * kBsiKin + (x - j * kBsiKin)];
    }
#pragma unroll
    for (int it = 0; it < kIt; it++) {
      const int x = it * NT + (int)threadIdx.x;
      const int j = x / kBsiKin;
      if (x < 64 * kBsiKin && blockIdx.x * 64 + j < nt)
        reinterpret_cast<int4*>(lk)[(x - j * kBsiKin) * 64 + j] = v[it];
    }
  }
  __syncthreads();
  // replay: 16 keys per wave, all four waves (the type chain is serial per key, so
  // four times the waves of a key-per-lane replay finish about four times sooner)
  const int kl = 16 * wv + (lane & 15);
  const uint32_t tk_ = blockIdx.x * 64 + kl;
  const bool live2 = lane < 16 && tk_ < nt;
  const LdsCounts tv{lc + kl};
  const TB ebmT = lk[kBsiRegSlices * 64 + kl];
  const TB fixT = lk[(kBsiRegSlices + 1) * 64 + kl];
  int slow = 0;
  CircuitT z0{tb_absent(), tb_absent(), ebmT, 0, 0, tv(kRowEbm)}, z1 = z0;
#pragma unroll 1
  for (int i = nb - 1; i >= 0; i--) {
    const TB sT = lk[i * 64 + kl];
    types_step((P.pred0 >> i) & 1, sT, z0, step_row(i, 0), tv, slow);
    if (two) types_step((P.pred1 >> i) & 1, sT, z1, step_row(i, 1), tv, slow);
  }
  TB rt;
  if (two) {
    const TB left = types_finish(BSI_GE, fixT, z0, kRowFin, 0, tv, slow);
    const TB right = types_finish(BSI_LE, fixT, z1, kRowFin + 1, 0, tv, slow);
    rt = tb_op<OPR_AND>(left, right, tv(kRowFin + 2), slow);
  } else {
    rt = types_finish(P.op, fixT, z0, kRowFin, kRowFin + 1, tv, slow);
  }
  const bool ok = live2 && !slow;
  if (sums) {  // per slice: a wave sum, the block's four added in LDS, one atomic per block
    __shared__ int bs[kBsiRegSlices + 1][4];
    const bool add = ok && rt.card > 0;
    for (int x = 0; x < nb; x++) {
      const int c = wave_sum(add ? tv(kRowSum + x) : 0);
      if (lane == 0) bs[x][wv] = c;
    }
    const int cc = wave_sum(add ? rt.card : 0);
    if (lane == 0) bs[kBsiRegSlices][wv] = cc;
    __syncthreads();
    if (threadIdx.x <= (unsigned)kBsiRegSlices && ((int)threadIdx.x < nb || threadIdx.x == kBsiRegSlices)) {
      const int x = threadIdx.x;
      const int c = bs[x][0] + bs[x][1] + bs[x][2] + bs[x][3];
      unsigned long long* rep = sums + kBsiSumWords + 64 * (blockIdx.x % kBsiSumReps);
      if (c) atomicAdd(&rep[x == kBsiRegSlices ? kBsiMaxInputs : x], (unsigned long long)(uint32_t)c);
    }
  }
  if (!live2) return;
  const uint32_t t = tk_;
  if (slow) {  // a step's type needs its run count: k_bsi_defer redoes this key
    defer[1 + atomicAdd(defer, 1u)] = t | 0x80000000u;
    return;
  }
  const uint32_t key = tasks[t].key;
  if (rt.card == 0) {
    bsi_rec(t, oc, false, nullptr, 0, 0, key, DK_A);
  } else if (rt.src >= 0) {  // an input container, cloned
    const CDesc d = A.desc[rt.src];
    const uint8_t* src = A.payload + d.slot;
    const uint32_t len = d.kind == DK_A ? 2 * d.card
                         : d.kind == DK_B ? 8192u
                                          : 2u + 4u * *reinterpret_cast<const uint16_t*>(src + 2);
    bsi_rec(t, oc, true, src + (d.kind == DK_R ? 2 : 0), len, d.card, key, d.kind);
  } else if (rt.kind == DK_B) {
    bsi_rec(t, oc, true, oc.scratch + (size_t)t * kSlotBytes, 8192, (uint32_t)rt.card, key, DK_B);
  } else {  // array / run: staged from the bits in the scratch slot by k_bsi_defer
    defer[1 + atomicAdd(defer, 1u)] = t | ((rt.kind == DK_A ? 1u : 2u) << 29);
    bsi_rec(t, oc, true, nullptr, 0, (uint32_t)rt.card, key, rt.kind);  // k_bsi_defer rewrites it
  }
}

// keys k_bsi_types handed over (defer[1..]): bit 31 = redo with the streamed form,
// bits 29-30 = stage the array (1) / run (2) result from the bits in the scratch slot
__global__ __launch_bounds__(256) void k_bsi_defer(const Task* __restrict__ tasks, const uint32_t* __restrict__ defer,
                                                   WideArgs A, BsiArgs P, OutCtx oc,
                                                   unsigned long long* __restrict__ sums) {
  __shared__ __align__(16) uint32_t acc[2048];
  __shared__ __align__(16) uint32_t tmp[2048];
  __shared__ int q[257];
  __shared__ int sh[8];
  __shared__ int pos[kBsiMaxInputs];
  const uint32_t n = defer[0];
  for (uint32_t j = blockIdx.x; j < n; j += gridDim.x) {
    const uint32_t e = defer[1 + j];
    const uint32_t t = e & 0x1FFFFFFFu;
    if (e >> 31) {
      bsi_task_streamed(t, tasks[t], A, P, oc, sums, acc, tmp, q, sh, pos);
      continue;
    }
    const int kind = ((e >> 29) & 3) == 1 ? DK_A : DK_R;
    const uint32_t card = oc.recs[t].card;
    uint64_t r[4];
    load_bitmap_owned(oc.scratch + (size_t)t * kSlotBytes, r);
    lds_barrier();
    const uint32_t len = stage_container(kind, r, (int)card, acc, tmp, sh);
    wg_place(t, true, nullptr, true, tmp, len, card, tasks[t].key, kind, oc, nullptr);
  }
}

// ===========================================================================
// Buffer-package BSI: BitSliceIndexBase.compare
// (bsi/src/main/java/org/roaringbitmap/bsi/buffer/BitSliceIndexBase.java, BBSI/ below)
// ===========================================================================
// ImmutableBitSliceIndex / MutableBitSliceIndex run their own circuit (BBSI/:422-453), and
// every pairwise step is ImmutableRoaringBitmap's (vb_op<OP, true>):
//   EQ    rangeEQ  (BBSI/:351-375): from and(ebM, foundSet), then and / andNot per slice
//   NEQ   rangeNEQ (BBSI/:384-387): andNot(ebM, rangeEQ(...)); rangeEQ's own min / max shortcut
//         (the empty bitmap) is decided on the host and makes the op ebM's clone (BSI_ALL)
//   GT / LT / LE  oNeilCompare (BBSI/:190-234): the heap circuit, tracking GT or LT only
//   GE    owenGreatEqual (BBSI/:243-275): from the top slice down to beGtrThan's least
//         significant zero, the 1 bits of beGtrThan = start - 1 AND their slice into a spine
//         and the 0 bits make orInputs (the slice itself above the first 1 bit, else
//         and(spine, slice)); BufferFastAggregation.horizontal_or unites them
//         (RB/buffer/BufferFastAggregation.java:187-235), then and(result, foundSet)
//   RANGE and(owenGreatEqual(start), oNeilCompare(LE, end)) (BBSI/:444-449)
//   ALL   compareUsingMinMax's "all" (BBSI/:456): ebM.clone() or and(ebM, foundSet)
// One workgroup per key, streamed like bsi_task_streamed.  horizontal_or's chain for a key
// follows the poll order of its container-pointer queue (key, then larger cardinality first,
// ties in heap order, which depends on every earlier key).  With three orInputs or more,
// k_bsi_owen_pre first records every orInput's type per key and the host replays the queue
// (engine.cpp: owen_order); the chain of a key then rebuilds each orInput's bits in that
// order.  With two or fewer the order does not matter (lazyOR is symmetric) and the
// orInputs are chained as the spine makes them.

__device__ __forceinline__ int bsi_card(const uint64_t r[4], int* sh) {
  int c = popc64(r[0]) + popc64(r[1]) + popc64(r[2]) + popc64(r[3]);
  int u = 0;
  block_sum2(c, u, sh);
  return (int)uni((uint32_t)c);
}

// horizontal_or's per-key chain (RB/buffer/BufferFastAggregation.java:200-233): one container
// is cloned; else x1.lazyOR(x2), lazyIOR of the rest, repairAfterLazy.  The state is the
// container class of the running union (the machine of WIDE_LAZY_CHAIN in wide.hip):
//   A + A: lazyor, a lazy bitmap once the cardinalities add past 1024
//          (RB/buffer/MappeableArrayContainer.java:1167-1191)
//   x + B, B + x: a bitmap (MappeableBitmapContainer lazyor / ilazyor)
//   A + R, R + A: lazyorToRun, a lazy bitmap above 4096 runs (RB/buffer/MappeableRunContainer.java:1709-1750, 748-762)
//   R + R: or / ior -> toEfficientContainer (:1911-1944)
// and repairAfterLazy: bitmap -> BY_CARD, full -> R (RB/buffer/MappeableBitmapContainer.java:1639-1649),
// run -> toEfficientContainer (RB/buffer/MappeableRunContainer.java:2037-2039).
struct HChain {
  VB acc;
  int n, st, cur;
};
__device__ __forceinline__ void hchain_add(HChain& h, const VB& x, uint32_t* lds, int* sh) {
  if (!x.present) return;
  if (h.n == 0) {
    h.acc = x;
    h.n = 1;
    h.st = x.kind;
    h.cur = x.card;
    return;
  }
#pragma unroll
  for (int i = 0; i < 4; i++) h.acc.r[i] |= x.r[i];
  if (h.st == DK_B) {
  } else if (h.st == DK_A && x.kind == DK_A) {
    if (h.cur + x.card > 1024) h.st = DK_B;
    else h.cur = bsi_card(h.acc.r, sh);
  } else if (x.kind == DK_B) {
    h.st = DK_B;
  } else if (h.st == DK_R && x.kind == DK_R) {
    const int cc = bsi_card(h.acc.r, sh);
    h.st = eff(cc, count_runs(h.acc.r, lds, sh));
    h.cur = cc;
  } else {
    h.st = count_runs(h.acc.r, lds, sh) > 4096 ? DK_B : DK_R;
  }
  h.n++;
}
__device__ __forceinline__ void hchain_finish(HChain& h, VB& out, uint32_t* lds, int* sh) {
  if (h.n == 0) {
    vb_absent(out);
    return;
  }
  out = h.acc;
  if (h.n == 1) return;  // x1.getContainer().clone()
  const int c = bsi_card(out.r, sh);
  out.kind = h.st == DK_B ? (c == 65536 ? DK_R : by_card(c)) : h.st == DK_R ? eff(c, count_runs(out.r, lds, sh)) : DK_A;
  out.card = c;
  out.src = -1;
}

// pos[input] = desc index of the key's container of each input (-1: none)
__device__ __forceinline__ void bsi_positions(const Task& tk, const WideArgs& A, int* pos) {
  const uint32_t s = uni((uint32_t)tk.a), n = uni((uint32_t)tk.b);
  __syncthreads();
  for (int j = threadIdx.x; j < kBsiMaxInputs; j += NT) pos[j] = -1;
  __syncthreads();
  for (uint32_t j = threadIdx.x; j < n; j += NT) pos[A.bm[s + j]] = (int)(s + j);
  __syncthreads();
}

// owenGreatEqual's orInputs of one key, top down (BBSI/:250-264): rec != null records each
// orInput's type (k_bsi_owen_pre), else each is chained into h as it is made.
__device__ __forceinline__ void owen_walk(const WideArgs& A, const BsiArgs& P, const int* pos, HChain& h, TB* rec,
                                          uint32_t* acc, uint32_t* tmp, int* q, int* sh) {
  VB spine, s, x;
  vb_absent(spine);
  bool spine_null = true;
  int j = 0;
  for (int w = P.nbits - 1; w >= 0; w--) {
    const uint32_t bit = 1u << w;
    const bool zero = (P.owen_zeros & bit) != 0;
    if (!zero && !(P.owen_ones & bit)) continue;  // below leastSignifZero
    if (!spine_null && !spine.present) {          // the spine lacks the key: every later AND does too
      if (zero) {
        if (rec && threadIdx.x == 0) rec[j] = tb_absent();
        j++;
      }
      continue;
    }
    vb_load(pos[1 + w], A, tmp, q, s);
    if (zero) {  // orInputs.add(lastSpineGate == null ? bA[w] : and(lastSpineGate, bA[w]))
      if (spine_null) x = s;
      else vb_op<OPR_AND, true>(spine, s, x, acc, sh);
      if (rec) {
        if (threadIdx.x == 0) rec[j] = x.present ? TB{x.kind, x.card, x.src, 0} : tb_absent();
      } else {
        hchain_add(h, x, acc, sh);
      }
      j++;
    } else if (spine_null) {  // lastSpineGate = bA[w]
      spine = s;
      spine_null = false;
    } else {  // lastSpineGate = and(lastSpineGate, bA[w])
      vb_op<OPR_AND, true>(spine, s, spine, acc, sh);
    }
  }
}

// orInput j (top-down index) of a key, rebuilt for the chain: its bits are the AND of the spine
// slices above it and its own slice (in any order); its type is k_bsi_owen_pre's record.
__device__ __forceinline__ void owen_input(int j, const WideArgs& A, const BsiArgs& P, const int* pos, const TB& tb,
                                           VB& x, uint32_t* tmp, int* q) {
  uint32_t z = P.owen_zeros;
  for (int k = 0; k < j; k++) z &= ~(1u << (31 - __builtin_clz(z)));
  const int w = 31 - __builtin_clz(z);
  const uint32_t above = P.owen_ones & ~((2u << w) - 1u);  // (w = 31: nothing above)
  if (!above) {  // above the first 1 bit: the slice itself
    vb_load(pos[1 + w], A, tmp, q, x);
    return;
  }
#pragma unroll
  for (int i = 0; i < 4; i++) x.r[i] = ~0ull;
  for (uint32_t m = above | (1u << w); m; m &= m - 1) {
    const int v = __builtin_ctz(m);
    uint64_t y[4];
    materialize(A.desc[pos[1 + v]], A.payload, tmp, q, y);
#pragma unroll
    for (int i = 0; i < 4; i++) x.r[i] &= y[i];
  }
  x.present = 1;
  x.kind = tb.kind;
  x.card = tb.card;
  x.src = -1;
}

__device__ __forceinline__ void place_buf(uint32_t t, uint32_t key, const VB& res, const WideArgs& A, const OutCtx& oc,
                                          const BigRuns& big, uint32_t* acc, uint32_t* tmp, int* sh,
                                          unsigned long long* sh64) {
  if (!res.present) {
    wg_place(t, false, nullptr, true, tmp, 0, 0, key, DK_A, oc, nullptr);
    return;
  }
  if (res.src >= 0) {
    wg_passthrough(t, A.desc[res.src], A.payload, oc, nullptr);
    return;
  }
  if (res.kind == DK_R) {
    const int nr = count_runs(res.r, acc, sh);
    if (nr > 2047) {
      place_big_runs(t, key, res.r, res.card, nr, oc, big, acc, sh, sh64);
      return;
    }
  }
  const uint32_t len = stage_container(res.kind, res.r, res.card, acc, tmp, sh);
  wg_place(t, true, nullptr, true, tmp, len, (uint32_t)res.card, key, res.kind, oc, nullptr);
}

__device__ __forceinline__ void bsi_task_buffer(uint32_t t, const Task& tk, const WideArgs& A, const BsiArgs& P,
                                                const OutCtx& oc, uint32_t* acc, uint32_t* tmp, int* q, int* sh,
                                                int* pos, unsigned long long* sh64) {
  const int nb = P.nbits;
  bsi_positions(tk, A, pos);
  VB ebm, fixed, res;
  vb_load(pos[0], A, tmp, q, ebm);
  if (P.has_found) vb_load(pos[P.found_input], A, tmp, q, fixed);
  else fixed = ebm;
  const int op = P.op;
  if (op == BSI_ALL) {  // ebM.clone() / and(ebM, foundSet)
    if (P.has_found) vb_op<OPR_AND, true>(ebm, fixed, res, acc, sh);
    else res = ebm;
  } else if (op == BSI_EQ || op == BSI_NEQ) {  // rangeEQ, BBSI/:351-375
    VB eq, sl;
    if (P.has_found) vb_op<OPR_AND, true>(ebm, fixed, eq, acc, sh);
    else eq = ebm;
    for (int i = nb - 1; i >= 0 && eq.present; i--) {  // an absent EQ stays absent
      vb_load(pos[1 + i], A, tmp, q, sl);
      if ((P.pred0 >> i) & 1) vb_op<OPR_AND, true>(eq, sl, eq, acc, sh);
      else vb_op<OPR_ANDNOT, true>(eq, sl, eq, acc, sh);
    }
    if (op == BSI_EQ) res = eq;
    else vb_op<OPR_ANDNOT, true>(ebm, eq, res, acc, sh);  // rangeNEQ: andNot(ebM, EQ)
  } else {
    const bool two = op == BSI_RANGE;
    VB left;
    if (op == BSI_GE || two) {  // owenGreatEqual, BBSI/:243-275
      HChain h;
      h.n = 0;
      h.st = DK_A;
      h.cur = 0;
      vb_absent(h.acc);
      if (P.owen_order) {
        const uint8_t* ord = P.owen_order + (size_t)t * kOwenOrder;
        const TB* tb = reinterpret_cast<const TB*>(P.owen_tb) + (size_t)t * 32;
        const int cnt = (int)uni(ord[0]);
        for (int k = 0; k < cnt; k++) {
          const int j = (int)uni(ord[1 + k]);
          VB x;
          owen_input(j, A, P, pos, tb[j], x, tmp, q);
          hchain_add(h, x, acc, sh);
        }
      } else {
        owen_walk(A, P, pos, h, nullptr, acc, tmp, q, sh);
      }
      hchain_finish(h, left, acc, sh);
      if (P.has_found) vb_op<OPR_AND, true>(left, fixed, left, acc, sh);  // and(result, foundSet)
    }
    if (op == BSI_GE) {
      res = left;
    } else {  // oNeilCompare (BBSI/:190-234): GT, LT, LE, or RANGE's LE(end)
      const int oop = two ? BSI_LE : op;
      const uint32_t pred = two ? P.pred1 : P.pred0;
      VB gt, lt, eq, sl, tv;
      vb_absent(gt);
      vb_absent(lt);
      eq = ebm;
      for (int i = nb - 1; i >= 0 && eq.present; i--) {  // an absent EQ adds nothing more
        vb_load(pos[1 + i], A, tmp, q, sl);
        if ((pred >> i) & 1) {
          if (oop != BSI_GT) {  // LT = or(LT, andNot(EQ, bA[i]))
            vb_op<OPR_ANDNOT, true>(eq, sl, tv, acc, sh);
            vb_op<OPR_OR>(lt, tv, lt, acc, sh);
          }
          vb_op<OPR_AND, true>(eq, sl, eq, acc, sh);
        } else {
          if (oop == BSI_GT) {  // GT = or(GT, and(EQ, bA[i]))
            vb_op<OPR_AND, true>(eq, sl, tv, acc, sh);
            vb_op<OPR_OR>(gt, tv, gt, acc, sh);
          }
          vb_op<OPR_ANDNOT, true>(eq, sl, eq, acc, sh);
        }
      }
      if (oop == BSI_GT) {
        vb_op<OPR_AND, true>(gt, fixed, res, acc, sh);
      } else if (oop == BSI_LT) {
        vb_op<OPR_AND, true>(lt, fixed, res, acc, sh);
      } else {  // LE: or(LT, and(fixedFoundSet, EQ))
        vb_op<OPR_AND, true>(fixed, eq, eq, acc, sh);
        vb_op<OPR_OR>(lt, eq, res, acc, sh);
      }
      if (two) vb_op<OPR_AND, true>(left, res, res, acc, sh);  // and(left, right)
    }
  }
  place_buf(t, tk.key, res, A, oc, P.big, acc, tmp, sh, sh64);
}

__global__ __launch_bounds__(256) void k_bsi_owen_pre(const Task* __restrict__ tasks, const uint32_t* __restrict__ n_tasks,
                                                      WideArgs A, BsiArgs P) {
  __shared__ __align__(16) uint32_t acc[2048];
  __shared__ __align__(16) uint32_t tmp[2048];
  __shared__ int q[257];
  __shared__ int sh[8];
  __shared__ int pos[kBsiMaxInputs];
  const uint32_t nt = *n_tasks;
  for (uint32_t t = blockIdx.x; t < nt; t += gridDim.x) {
    const Task tk = tasks[t];
    bsi_positions(tk, A, pos);
    HChain h;
    h.n = 0;
    owen_walk(A, P, pos, h, reinterpret_cast<TB*>(P.owen_tb) + (size_t)t * 32, acc, tmp, q, sh);
    if (threadIdx.x == 0) P.task_keys[t] = tk.key;
  }
}

__global__ __launch_bounds__(256) void k_bsi_buf(const Task* __restrict__ tasks, const uint32_t* __restrict__ n_tasks,
                                                 WideArgs A, BsiArgs P, OutCtx oc) {
  __shared__ __align__(16) uint32_t acc[2048];
  __shared__ __align__(16) uint32_t tmp[2048];
  __shared__ int q[257];
  __shared__ int sh[8];
  __shared__ int pos[kBsiMaxInputs];
  __shared__ unsigned long long sh64;
  const uint32_t nt = *n_tasks;
  for (uint32_t t = blockIdx.x; t < nt; t += gridDim.x) bsi_task_buffer(t, tasks[t], A, P, oc, acc, tmp, q, sh, pos, &sh64);
}

void launch_bsi_owen_pre(hipStream_t s, int grid, const Task* tasks, const uint32_t* nt, WideArgs args, BsiArgs p) {
  const int g = std::max(1, std::min(grid, resident_grid((const void*)&k_bsi_owen_pre)));
  hipLaunchKernelGGL(k_bsi_owen_pre, dim3(g), dim3(256), 0, s, tasks, nt, args, p);
}
void launch_bsi_buf(hipStream_t s, int grid, const Task* tasks, const uint32_t* nt, WideArgs args, BsiArgs p, OutCtx oc) {
  const int g = std::max(1, std::min(grid, resident_grid((const void*)&k_bsi_buf)));
  hipLaunchKernelGGL(k_bsi_buf, dim3(g), dim3(256), 0, s, tasks, nt, args, p, oc);
}

// ImmutableRoaringBitmap.and / andNot (RB/buffer/ImmutableRoaringBitmap.java:299-325, 441-471) and
// MutableRoaringBitmap's static and / andNot (RB/buffer/MutableRoaringBitmap.java:235-301): per key
// c1.and(c2) / c1.andNot(c2) with the buffer package's container types -- vb_op<OP, true>, the
// buffer BSI's step: run AND / ANDNOT run keep the merged run container (more than 2047 runs go to
// the big-run arena), every other pair types like the heap's.  Tasks from the
// pairwise plan (k_plan_pairwise: AND = keys of both, ANDNOT = keys of x1); an x1 container with
// no x2 counterpart is appended as is (appendCopy, :460-469).
// one wave per task (20 per CU, the next record in flight): both operands in registers (wave.hpp), the
// buffer package's type rule (vb_op<OP, true>'s), a run result of more than 2047 runs into the arena
template <int OP>
__device__ __forceinline__ void pair_buf_task(uint32_t t, const PTask& tk, const uint8_t* pa, const uint8_t* pb,
                                              const OutCtx& oc, const BigRuns& big, uint32_t* lds) {
  const int ka = tk.kind_a, kb = tk.kind_b;
  if (OP == OPR_ANDNOT && kb == kAbsent) {  // x1's container alone: appendCopy (:460-469)
    const uint32_t len = ka == DK_A ? 2u * tk.card_a : ka == DK_B ? 8192u : 2u + 4u * tk.nruns_a;
    w_place(t, true, pa + tk.slot_a + (ka == DK_R ? 2 : 0), false, lds, len, tk.card_a, tk.key, ka, oc);
    return;
  }
  WCtr x;
  w_materialize(CDesc{tk.slot_a, tk.card_a, tk.key, (uint8_t)ka, 0}, pa, lds, x);
  w_combine<OP>(CDesc{tk.slot_b, tk.card_b, tk.key, (uint8_t)kb, 0}, pb, lds, x);
  const int c = w_card(x);
  if (c == 0) {  // empty results are dropped
    w_place(t, false, nullptr, true, lds, 0, 0, tk.key, DK_A, oc);
    return;
  }
  const bool raw_run = ka == DK_R && kb == DK_R;  // the merged run container, no toEfficientContainer
  int kind;
  if (raw_run) kind = DK_R;
  else if (pairwise_needs_runs(OP, ka, (int)tk.card_a, kb, (int)tk.card_b)) kind = eff(c, w_runs(x));
  else kind = pairwise_kind(OP, ka, kb, c);
  if (kind == DK_B) {
    uint8_t* slot = oc.scratch + (size_t)t * kSlotBytes;
    w_store_bitmap(slot, x);
    w_place(t, true, slot, false, lds, 8192, (uint32_t)c, tk.key, DK_B, oc);
    return;
  }
  if (raw_run) {
    const int nr = w_runs(x);
    if (nr > 2047) {
      w_place_big_runs(t, tk.key, x, c, nr, oc, big, lds);
      return;
    }
  }
  const uint32_t len = w_stage(kind, x, c, lds);
  w_place(t, true, nullptr, true, lds, len, (uint32_t)c, tk.key, kind, oc);
}

constexpr int kPbWaves = 4;

template <int OP>
__global__ __launch_bounds__(256, 4) void k_pair_buf(const PTask* __restrict__ tasks, const uint32_t* __restrict__ n_tasks,
                                                  const uint8_t* pa, const uint8_t* pb, OutCtx oc, BigRuns big) {
  __shared__ __align__(16) uint32_t lds_all[kPbWaves][2048];
  const int w = threadIdx.x >> 6;
  uint32_t* lds = lds_all[w];
  const uint32_t nt = uni(*n_tasks);
  const uint32_t stride = gridDim.x * kPbWaves;
  uint32_t t = uni(blockIdx.x * kPbWaves + w);
  if (t >= nt) return;
  PTask cur = load_task(tasks, t);
  for (;;) {
    const uint32_t tn = t + stride;
    PTask nxt;
    if (tn < nt) nxt = load_task(tasks, tn);
    pair_buf_task<OP>(t, cur, pa, pb, oc, big, lds);
    if (tn >= nt) break;
    t = tn;
    cur = nxt;
  }
}

void launch_pair_buf(hipStream_t s, int op, int grid, const PTask* tasks, const uint32_t* nt, const uint8_t* pa,
                     const uint8_t* pb, OutCtx oc, BigRuns big) {
  const void* k = op == OPR_AND ? (const void*)&k_pair_buf<OPR_AND> : (const void*)&k_pair_buf<OPR_ANDNOT>;
  const int g = std::max(1, std::min((grid + kPbWaves - 1) / kPbWaves, resident_grid(k)));
  if (op == OPR_AND) hipLaunchKernelGGL(k_pair_buf<OPR_AND>, dim3(g), dim3(256), 0, s, tasks, nt, pa, pb, oc, big);
  else hipLaunchKernelGGL(k_pair_buf<OPR_ANDNOT>, dim3(g), dim3(256), 0, s, tasks, nt, pa, pb, oc, big);
}

void launch_plan_bsi(hipStream_t s, const uint32_t* key_off, const uint32_t* bm, uint32_t need, Task* by_key,
                     uint8_t* flag, uint32_t* wg_count, uint64_t* zlb, uint64_t* ztile, unsigned long long* zsums,
                     uint32_t* zdefer) {
  hipLaunchKernelGGL(k_plan_bsi, dim3(256), dim3(256), 0, s, key_off, bm, need, by_key, flag, wg_count, zlb, ztile,
                     zsums, zdefer);
}

// sum(foundSet) as Java longs (BSI/:581-592) from the per-slice counts, on the device:
// sum = sum over x of (long) (1 << x) * andCardinality(bA[x], found), each andCardinality a
// Java int (RB/RoaringBitmap.java:413-434); (0, 0) when the found set is empty.  Lane x
// takes slice x; the result stays on the device (sums[kBsiSumOut], [kBsiSumOut + 1]).
__global__ __launch_bounds__(64) void k_bsi_sum_final(unsigned long long* __restrict__ sums, int nbits,
                                                      unsigned long long* __restrict__ dst) {
  const int x = threadIdx.x;
  // lane x: word x summed over the base words and k_bsi_types' replicas
  unsigned long long wx = x < kBsiSumWords ? sums[x] : 0;
#pragma unroll
  for (int r = 0; r < kBsiSumReps; r++) wx += sums[kBsiSumWords + 64 * r + x];
  const unsigned long long count = __shfl(wx, kBsiMaxInputs, 64);
  unsigned long long v = 0;
  if (x < nbits && count) {
    const int64_t card = (int32_t)(uint32_t)wx;
    const int64_t w = (int64_t)(int32_t)(1u << x);
    v = (unsigned long long)(w * card);
  }
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  if (x == 0) {
    sums[kBsiSumOut] = v;
    sums[kBsiSumOut + 1] = count;
    if (dst) {  // the caller's copy (rbg_ctx_bsi_sums_target), without a launch of its own
      dst[0] = v;
      dst[1] = count;
    }
  }
}

// (sum, count) to caller memory on the stream: one tiny kernel (a D2D hipMemcpyAsync goes
// through a blit kernel at ~12 us)
__global__ __launch_bounds__(64) void k_bsi_sums_out(const unsigned long long* __restrict__ sums,
                                                     unsigned long long* __restrict__ dst) {
  if (threadIdx.x < 2) dst[threadIdx.x] = sums[kBsiSumOut + threadIdx.x];
}
void launch_bsi_sums_out(hipStream_t s, const unsigned long long* sums, void* dst) {
  hipLaunchKernelGGL(k_bsi_sums_out, dim3(1), dim3(64), 0, s, sums, reinterpret_cast<unsigned long long*>(dst));
}

bool bsi_reg_path(int op, int nbits) { return op >= 0 && op <= BSI_RANGE && nbits <= kBsiRegSlices; }
void launch_bsi_table(hipStream_t s, const Task* tasks, const uint32_t* nt, WideArgs args, void* table, size_t stride) {
  hipLaunchKernelGGL(k_bsi_table, dim3((unsigned)((stride + 3) / 4)), dim3(256), 0, s, tasks, nt, args,
                     reinterpret_cast<BsiIn*>(table));
}
void launch_bsi(hipStream_t s, int grid, const Task* tasks, const uint32_t* nt, WideArgs args, BsiArgs p, OutCtx oc,
                unsigned long long* sums, BsiScratch* sc, void* sums_dst) {
  if (p.op <= BSI_RANGE && p.nbits <= kBsiRegSlices && sc) {
    if (!sc->table_ready) launch_bsi_table(s, tasks, nt, args, sc->table, sc->stride);
    const int g = std::max(1, std::min(grid * kBsiUnits, resident_grid((const void*)&k_bsi_reg)));
    hipLaunchKernelGGL(k_bsi_reg, dim3(g), dim3(256), 0, s, tasks, nt, args, p, oc, sums != nullptr,
                       reinterpret_cast<const BsiIn*>(sc->table), sc->cnts,
                       reinterpret_cast<TB*>(sc->kin), sc->stride, *sc);
    const int g2 = (int)((sc->stride + 63) / 64);
    hipLaunchKernelGGL(k_bsi_types, dim3(g2), dim3(256), 0, s, tasks, nt, args, p, oc, sums, sc->cnts,
                       reinterpret_cast<const TB*>(sc->kin), sc->stride, sc->defer, sc->claims);
    const int g3 = std::max(1, std::min(grid, resident_grid((const void*)&k_bsi_defer)));
    hipLaunchKernelGGL(k_bsi_defer, dim3(g3), dim3(256), 0, s, tasks, sc->defer, args, p, oc, sums);
  } else {
    const int g = std::max(1, std::min(grid, resident_grid((const void*)&k_bsi)));
    hipLaunchKernelGGL(k_bsi, dim3(g), dim3(256), 0, s, tasks, nt, args, p, oc, sums);
  }
  if (sums)
    hipLaunchKernelGGL(k_bsi_sum_final, dim3(1), dim3(64), 0, s, sums, p.nbits,
                       reinterpret_cast<unsigned long long*>(sums_dst));
}

}  // namespace rbg
