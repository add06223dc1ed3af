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

#include "kernels.hpp"
#include "wave.hpp"

namespace rbg {

// one bitmap of the circuit, for the current key
struct VB {
  uint64_t r[4];
  int present, kind, card;
  int src;  // desc index of the input container it is an unmodified clone of, else -1
};

__device__ __forceinline__ void vb_absent(VB& z) {
  z.present = 0;
  z.kind = DK_A;
  z.card = 0;
  z.src = -1;
#pragma unroll
  for (int i = 0; i < 4; i++) z.r[i] = 0;
}

// z = x OP y with the reference's result-type rule; x / y may alias z
template <int OP>
__device__ __forceinline__ void vb_op(const VB& x, const VB& y, VB& z, uint32_t* lds, int* sh) {
  if (OP == OPR_AND && (!x.present || !y.present)) {
    vb_absent(z);
    return;
  }
  if (OP == OPR_OR && !x.present) {  // unmatched: appendCopy keeps the container
    z = y;
    return;
  }
  if ((OP == OPR_OR || OP == OPR_ANDNOT) && !y.present) {
    z = x;
    return;
  }
  if (OP == OPR_ANDNOT && !x.present) {
    vb_absent(z);
    return;
  }
  uint64_t r[4];
#pragma unroll
  for (int i = 0; i < 4; i++)
    r[i] = OP == OPR_AND ? (x.r[i] & y.r[i]) : OP == OPR_OR ? (x.r[i] | y.r[i]) : (x.r[i] & ~y.r[i]);
  int c = popc64(r[0]) + popc64(r[1]) + popc64(r[2]) + popc64(r[3]);
  int u = 0;
  block_sum2(c, u, sh);
  c = (int)uni((uint32_t)c);
  if (c == 0) {  // empty results are dropped (RB/RoaringBitmap.java:389,456)
    vb_absent(z);
    return;
  }
  const bool use_eff = pairwise_needs_runs(OP, x.kind, x.card, y.kind, y.card);
  const int kind = use_eff ? eff(c, count_runs(r, lds, sh)) : pairwise_kind(OP, x.kind, y.kind, c);
#pragma unroll
  for (int i = 0; i < 4; i++) z.r[i] = r[i];
  z.present = 1;
  z.kind = kind;
  z.card = c;
  z.src = -1;
}

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

__global__ __launch_bounds__(256) void k_plan_bsi(const uint32_t* __restrict__ key_off, const uint32_t* __restrict__ bm,
                                                  uint32_t need, Task* __restrict__ by_key, uint8_t* __restrict__ flag,
                                                  uint32_t* __restrict__ wg_count, uint64_t* zlb, uint64_t* ztile) {
  plan_zero(zlb, ztile);
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  const uint32_t s = key_off[k], n = key_off[k + 1] - s;
  // a key yields a result only where input `need` (ebM, or foundSet for sum alone) has a container
  int f = 0;
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
// Register-resident query (compare ops, nbits <= 32): k_bsi_reg + k_bsi_defer
// ===========================================================================
// The streamed form above is bound by its ~6 workgroup reductions per slice (two
// barriers each, a dependent chain of ~190 per key) and reads every slice twice.
// k_bsi_reg runs one key per 1,024-thread workgroup, thread t owning container
// word t, and holds ALL slices of the key in registers (one u64 per slice per
// thread):
//   1. every slice of the key is requested at once;
//   2. bits: the whole circuit on registers.  Per step only t = EQ & bA[i] (or
//      EQ & ~bA[i]) is counted -- t and the new EQ partition the old EQ, and t is
//      disjoint from GT / LT, so |EQ'| = |EQ| - |t| and |GT'| = |GT| + |t|.  Each
//      thread stores its share (<= 64, a byte) in an LDS row per count; no
//      barrier inside the circuit;
//   4. sum shares |bA[x] & result| from the same registers (no second read);
//      then the next key's slices start loading;
//   3. the rows are summed, and one wave replays the reference's type rule of
//      every step from those cardinalities (wave-uniform, no bits needed).  A
//      step whose type needs a run count (EFF: run containers in AND / OR / ...)
//      cannot be replayed so: such keys go to k_bsi_defer, which redoes them
//      with bsi_task_streamed.
// Results that are absent, clones or bitmap containers are written here (a
// bitmap is one coalesced 8 B store per thread); array / run results are left
// as raw bitmaps for k_bsi_defer to stage with the 256-thread helpers.
constexpr int kBsiRegSlices = 32;
constexpr int kNT1 = 1024;  // threads of k_bsi_reg
constexpr int kBsiRows = 1 + 2 * kBsiRegSlices + 4 + kBsiRegSlices;  // |ebM|, counted steps, finish, sum shares
constexpr int kRowB = kNT1 + 16;  // row stride in bytes: row sums of a wave spread over the banks

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
// row sums of rows [0, nk) -> tot[], one wave per row (a 16 B vector per lane,
// then a DPP reduction); ends with a barrier
__device__ __forceinline__ void sum_rows1(const uint8_t* rows, int nk, int* tot) {
  lds_barrier();
  const int lane = threadIdx.x & 63;
  for (int r = threadIdx.x >> 6; r < nk; r += kNT1 / 64) {
    const uint4 x = reinterpret_cast<const uint4*>(rows + r * kRowB)[lane];
    // 16 bytes: sum the byte lanes pairwise into 16-bit fields (each <= 8 * 64)
    const uint32_t a = (x.x & 0x00FF00FFu) + ((x.x >> 8) & 0x00FF00FFu) + (x.y & 0x00FF00FFu) +
                       ((x.y >> 8) & 0x00FF00FFu) + (x.z & 0x00FF00FFu) + ((x.z >> 8) & 0x00FF00FFu) +
                       (x.w & 0x00FF00FFu) + ((x.w >> 8) & 0x00FF00FFu);
    const int c = wave_sum((int)((a & 0xFFFF) + (a >> 16)));
    if (lane == 0) tot[r] = c;
  }
  lds_barrier();
}
// count k of this thread's key: the tables are transposed (row k of every key is
// contiguous), so a wave reads 64 keys' count k with one coalesced load
struct CountRows {
  const int* p;  // cnts + key index
  size_t stride;
  __device__ __forceinline__ int operator()(int k) const { return p[(size_t)k * stride]; }
};

// Type replay of a step / finish, in the order of the bits.  c* are the exact
// cardinalities of the bits (0 for an absent bitmap).
struct CircuitT {
  TB gt, lt, eq;
  int cgt, clt, ceq;
};
__device__ __forceinline__ void types_step(int bit, const TB& s, CircuitT& z, int& k, const CountRows& tv,
                                           int& slow) {
  const int ct = tv(k++);
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
// BSI/:453-467 on types: counted are fixed & EQ and the NEQ / GT / LT results;
// LE / GE are disjoint unions
__device__ __forceinline__ TB types_finish(int op, const TB& fixed, CircuitT& z, int& k, const CountRows& tv,
                                           int& slow) {
  const int ce = tv(k++);
  z.eq = tb_op<OPR_AND>(fixed, z.eq, ce, slow);
  z.ceq = ce;
  switch (op) {
    case BSI_EQ: return z.eq;
    case BSI_NEQ: return tb_op<OPR_ANDNOT>(fixed, z.eq, tv(k++), slow);
    case BSI_GT: return tb_op<OPR_AND>(z.gt, fixed, tv(k++), slow);
    case BSI_LT: return tb_op<OPR_AND>(z.lt, fixed, tv(k++), slow);
    case BSI_LE: return tb_op<OPR_OR>(z.lt, z.eq, z.clt + ce, slow);
    default: return tb_op<OPR_OR>(z.gt, z.eq, z.cgt + ce, slow);  // GE
  }
}
// the same on bits (thread's word), recording the counted steps
__device__ __forceinline__ uint64_t bits_finish1(int op, uint64_t fixed, uint64_t gt, uint64_t lt, uint64_t& eq, int& k,
                                                 uint8_t* rows) {
  eq &= fixed;
  rec1(eq, k++, rows);
  uint64_t out;
  switch (op) {
    case BSI_EQ: return eq;
    case BSI_NEQ: out = fixed & ~eq; break;
    case BSI_GT: out = gt & fixed; break;
    case BSI_LT: out = lt & fixed; break;
    case BSI_LE: return lt | eq;
    default: return gt | eq;  // GE
  }
  rec1(out, k++, rows);
  return out;
}

// wave-uniform (SGPR) copy of a type state
__device__ __forceinline__ TB tb_uni(const TB& x) {
  return TB{(int)uni((uint32_t)x.kind), (int)uni((uint32_t)x.card), (int)uni((uint32_t)x.src), 0};
}

// Thread t's word of a container; non-bitmap ones through the 8 KiB LDS scratch `lds`:
// arrays scattered; runs as toggles (run start, end + 1) whose prefix XOR is
// taken inside each word and carried across words by a workgroup parity scan
// (wpar: 16 ints).  All threads; contains barriers.
__device__ __forceinline__ uint64_t mat_word1(const CDesc& d, const uint8_t* payload, uint32_t* lds, int* wpar) {
  const int t = threadIdx.x;
  const uint8_t* slot = payload + d.slot;
  if (d.kind == DK_B) return reinterpret_cast<const uint64_t*>(slot)[t];
  lds_barrier();
  reinterpret_cast<uint64_t*>(lds)[t] = 0;
  lds_barrier();
  if (d.kind == DK_A) {
    const int card = (int)d.card;
    const int nvec = (card + 7) >> 3;
    const uint4* v4 = reinterpret_cast<const uint4*>(slot);
    for (int i = t; i < nvec; i += kNT1) {
      const uint4 v = v4[i];
      const uint32_t w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int j = 0; j < 8; j++) {
        if (8 * i + j < card) {
          const uint32_t x = (w[j >> 1] >> ((j & 1) * 16)) & 0xFFFF;
          atomicOr(&lds[x >> 5], 1u << (x & 31));
        }
      }
    }
    lds_barrier();
    return reinterpret_cast<const uint64_t*>(lds)[t];
  }
  const int nr = *reinterpret_cast<const uint16_t*>(slot + 2);
  const uint32_t* pairs = reinterpret_cast<const uint32_t*>(slot + 4);
  for (int i = t; i < nr; i += kNT1) {
    const uint32_t p = pairs[i];
    const uint32_t st = p & 0xFFFF, e1 = st + (p >> 16) + 1;
    atomicXor(&lds[st >> 5], 1u << (st & 31));
    if (e1 < 65536) atomicXor(&lds[e1 >> 5], 1u << (e1 & 31));
  }
  lds_barrier();
  uint64_t w = reinterpret_cast<const uint64_t*>(lds)[t];
  const uint32_t par = (uint32_t)popc64(w) & 1u;
  w = prefix_xor64(w);
  const uint64_t m = __ballot(par);
  const int lane = t & 63, wv = t >> 6;
  uint32_t c = (uint32_t)__popcll(m & ((1ull << lane) - 1)) & 1u;
  if (lane == 0) wpar[wv] = __popcll(m) & 1;
  lds_barrier();
  for (int j = 0; j < wv; j++) c ^= (uint32_t)wpar[j];
  lds_barrier();
  return c ? ~w : w;
}

// Diagnostic build only (-DRBG_BSI_STAMPS=1): per-phase shader-clock totals of
// k_bsi_reg (thread 0 of every workgroup), read back with rbg_debug_stamps when
// RBG_DEBUG_BSI is set.
#if RBG_BSI_STAMPS
__device__ unsigned long long g_bsi_stamp[20];
#define BST_DECL                                   \
  uint64_t bst_prev = __builtin_amdgcn_s_memtime(); \
  uint64_t bst[10] = {};
#define BST(ph)                                            \
  do {                                                     \
    const uint64_t bst_now = __builtin_amdgcn_s_memtime(); \
    bst[ph] += bst_now - bst_prev;                         \
    bst_prev = bst_now;                                    \
  } while (0)
#define BST_FLUSH()                                                                          \
  do {                                                                                       \
    if (threadIdx.x == 0)                                                                    \
      for (int i_ = 0; i_ < 10; i_++) atomicAdd(&g_bsi_stamp[i_], (unsigned long long)bst[i_]); \
  } while (0)
void debug_bsi_stamps(uint64_t* out20, bool reset) {
  (void)hipDeviceSynchronize();
  (void)hipMemcpyFromSymbol(out20, HIP_SYMBOL(g_bsi_stamp), 20 * 8, 0, hipMemcpyDeviceToHost);
  if (reset) {
    unsigned long long z[20] = {};
    (void)hipMemcpyToSymbol(HIP_SYMBOL(g_bsi_stamp), z, sizeof(z), 0, hipMemcpyHostToDevice);
  }
}
#else
#define BST_DECL
#define BST(ph) \
  do {          \
  } while (0)
#define BST_FLUSH() \
  do {              \
  } while (0)
void debug_bsi_stamps(uint64_t* out20, bool) {
  for (int i = 0; i < 20; i++) out20[i] = 0;
}
#endif

// Per-key LDS state of k_bsi_reg (double-buffered: the next key's is set up while
// the current key finishes)
struct BsiKeyBuf {
  int pos[kBsiMaxInputs];  // desc index of each input's container of the key, or -1
  TB stype[kBsiRegSlices];
  uint64_t sslot[kBsiRegSlices];
  uint32_t mask;  // slices that are bitmap containers
};

// positions of the key's inputs and its slice descriptors (wave 0, one lane per
// slice: one memory round trip); returns the bitmap-slice mask.  Contains barriers.
__device__ __forceinline__ uint32_t bsi_key_setup(const Task& tk, const WideArgs& A, int nb, BsiKeyBuf& kb) {
  const uint32_t s = uni((uint32_t)tk.a), n = uni((uint32_t)tk.b);
  if ((int)threadIdx.x < kBsiMaxInputs) kb.pos[threadIdx.x] = -1;
  lds_barrier();
  for (uint32_t j = threadIdx.x; j < n; j += kNT1) kb.pos[A.bm[s + j]] = (int)(s + j);
  lds_barrier();
  if (threadIdx.x < 64) {
    const int i = threadIdx.x;
    const int p = i < nb ? kb.pos[1 + i] : -1;
    CDesc d{};
    if (p >= 0) d = A.desc[p];
    if (i < kBsiRegSlices) {
      kb.stype[i] = p >= 0 ? TB{d.kind, (int)d.card, p, 0} : tb_absent();
      kb.sslot[i] = d.slot;
    }
    const uint64_t m = __ballot(p >= 0 && d.kind == DK_B);
    if (i == 0) kb.mask = (uint32_t)m;
  }
  lds_barrier();
  return uni(kb.mask);
}

// bitmap slices straight to registers (thread t: word t); all loads of the key in flight at once
__device__ __forceinline__ void bsi_issue_loads(const WideArgs& A, const BsiKeyBuf& kb, uint32_t mask,
                                                uint64_t sl[kBsiRegSlices]) {
#pragma unroll
  for (int i = 0; i < kBsiRegSlices; i++)
    sl[i] = ((mask >> i) & 1) ? reinterpret_cast<const uint64_t*>(A.payload + kb.sslot[i])[threadIdx.x] : 0;
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

// compare ops (BSI_EQ .. BSI_RANGE) with nbits <= kBsiRegSlices: one 1,024-thread
// workgroup per key computes the bits and the counts; k_bsi_types (a wave per key)
// replays the types and writes the records.  cnts: kBsiCnt rows of one int per task; kin:
// kBsiKin input types per task (slices, ebM, the fixed found set).
constexpr int kBsiCnt = 128;
constexpr int kBsiKin = kBsiRegSlices + 2;
static_assert(kBsiRows <= kBsiCnt, "count rows");
__global__ __launch_bounds__(1024, 1) void k_bsi_reg(const Task* __restrict__ tasks,
                                                     const uint32_t* __restrict__ n_tasks, WideArgs A, BsiArgs P,
                                                     OutCtx oc, bool want_sum, int* __restrict__ cnts,
                                                     TB* __restrict__ kin, size_t tstride) {
  __shared__ __align__(16) uint32_t tmp[2048];
  __shared__ __align__(16) uint8_t rows[kBsiRows * kRowB];
  __shared__ int tot[128];
  __shared__ BsiKeyBuf kbuf[2];
  __shared__ int wpar[16];
  const uint32_t nt = *n_tasks;
  const int nb = P.nbits;
  const bool two = P.op == BSI_RANGE;
  const int tid = threadIdx.x;
  uint32_t t = blockIdx.x;
  if (t >= nt) return;
  uint64_t sl[kBsiRegSlices];
  int cb = 0;
  Task tk = tasks[t];
  bsi_issue_loads(A, kbuf[0], bsi_key_setup(tk, A, nb, kbuf[0]), sl);
  BST_DECL
  while (true) {
    BsiKeyBuf& kb = kbuf[cb];
    // the next key's positions and slice descriptors, while this key's slices load
    const uint32_t tn = t + gridDim.x;
    Task tkn;
    uint32_t maskn = 0;
    if (tn < nt) {
      tkn = tasks[tn];
      maskn = bsi_key_setup(tkn, A, nb, kbuf[cb ^ 1]);
    }
    const uint64_t ebm = mat_word1(A.desc[kb.pos[0]], A.payload, tmp, wpar);  // a task exists only where ebM has the key
    uint64_t fixed = ebm;
    if (P.has_found) fixed = kb.pos[nb + 1] >= 0 ? mat_word1(A.desc[kb.pos[nb + 1]], A.payload, tmp, wpar) : 0;
    BST(0);
    // array / run slices through the LDS scratch
#pragma unroll
    for (int i = 0; i < kBsiRegSlices; i++) {
      if (i < nb && kb.stype[i].card > 0 && kb.stype[i].kind != DK_B)
        sl[i] = mat_word1(A.desc[kb.pos[1 + i]], A.payload, tmp, wpar);
    }
    // 2. bits of the whole circuit
    uint64_t eq0 = ebm, gt0 = 0, lt0 = 0, eq1 = ebm, gt1 = 0, lt1 = 0, res;
    int k = 0;
    rec1(ebm, k++, rows);  // |ebM| of the bits: the start of the derived cardinalities
    // predicate bits i = 31 .. 0 as the top bit of running copies; the asm keeps the
    // compiler from precomputing 64 per-step flags (SGPR spills)
    uint32_t p0 = P.pred0, p1 = P.pred1;
    int live = 32 - nb;  // steps i >= nb are skipped
#pragma unroll
    for (int i = kBsiRegSlices - 1; i >= 0; i--) {
      asm volatile("" : "+s"(p0), "+s"(p1), "+s"(live));
      if (live <= 0) {
        const uint64_t m0 = (uint64_t)(int64_t)((int32_t)p0 >> 31);  // all ones iff bit i of pred0
        const uint64_t tv = eq0 & (sl[i] ^ m0);                     // EQ & ~bA[i] / EQ & bA[i]
        rec1(tv, k++, rows);
        lt0 |= tv & m0;
        gt0 |= tv & ~m0;
        eq0 ^= tv;
        if (two) {
          const uint64_t m1 = (uint64_t)(int64_t)((int32_t)p1 >> 31);
          const uint64_t tw = eq1 & (sl[i] ^ m1);
          rec1(tw, k++, rows);
          lt1 |= tw & m1;
          gt1 |= tw & ~m1;
          eq1 ^= tw;
        }
      }
      p0 <<= 1;
      p1 <<= 1;
      live--;
    }
    if (two) {  // RANGE = and(GE(start), LE(end)), BSI/:503-507
      const uint64_t left = bits_finish1(BSI_GE, fixed, gt0, lt0, eq0, k, rows);
      const uint64_t right = bits_finish1(BSI_LE, fixed, gt1, lt1, eq1, k, rows);
      res = left & right;
      rec1(res, k++, rows);
    } else {
      res = bits_finish1(P.op, fixed, gt0, lt0, eq0, k, rows);
    }
    BST(1);
    // 4. sum shares |bA[x] & result| (an absent result has no bits: all zero)
    if (want_sum) {
#pragma unroll
      for (int x = 0; x < kBsiRegSlices; x++)
        if (x < nb) rec1(sl[x] & res, k + x, rows);
    }
    BST(2);
    // the slices of this key are dead: the next key's start loading now
    if (tn < nt) bsi_issue_loads(A, kbuf[cb ^ 1], maskn, sl);
    BST(3);
    // the result bits to the task's scratch slot: the container itself when it is a
    // bitmap, else the input k_bsi_types stages it from
    reinterpret_cast<uint64_t*>(oc.scratch + (size_t)t * kSlotBytes)[tid] = res;
    sum_rows1(rows, k + (want_sum ? nb : 0), tot);
    BST(4);
    // counts and the input types of the key for k_bsi_types (transposed: row r of
    // every key contiguous)
    if (tid < k + (want_sum ? nb : 0)) cnts[(size_t)tid * tstride + t] = tot[tid];
    if (tid >= 64 && tid < 64 + kBsiKin) {
      const int i = tid - 64;
      TB x = tb_absent();
      if (i < kBsiRegSlices) {
        x = kb.stype[i];
      } else {
        const int p = i == kBsiRegSlices ? kb.pos[0] : (P.has_found ? kb.pos[nb + 1] : kb.pos[0]);
        if (p >= 0) {
          const CDesc d = A.desc[p];
          x = TB{d.kind, (int)d.card, p, 0};
        }
      }
      kin[(size_t)i * tstride + t] = x;
    }
    BST(5);
    if (tn >= nt) break;
    lds_barrier();
    t = tn;
    tk = tkn;
    cb ^= 1;
  }
  BST_FLUSH();
}

// w_place for k_bsi_types: a staged result (LDS) to the task's scratch slot and its record
__device__ __forceinline__ void bsi_wave_place(uint32_t t, const uint32_t* lds, uint32_t len, uint32_t card,
                                               uint32_t key, int kind, const OutCtx& oc) {
  uint8_t* slot = oc.scratch + (size_t)t * kSlotBytes + (kind == DK_R ? 2 : 0);
  copy_lds_to_global<64>(slot, lds, len, lane_id());
  if (lane_id() == 0) bsi_rec(t, oc, true, slot, len, card, key, kind);
}

// Types of the keys k_bsi_reg computed, one THREAD per key: the reference's type
// rule of every step is replayed from the counts (branch-free selects; the counts
// and input types are read as transposed rows, coalesced across the keys of a
// wave), then the result record.  A bitmap result is already in the scratch slot;
// array / run results (staged from it by a wave) and keys whose replay needs a run
// count go to k_bsi_defer.  Sums: per slice one wave reduction, one atomic.
__global__ __launch_bounds__(256) void k_bsi_types(const Task* __restrict__ tasks,
                                                   const uint32_t* __restrict__ n_tasks, WideArgs A, BsiArgs P,
                                                   OutCtx oc, unsigned long long* __restrict__ sums,
                                                   const int* __restrict__ cnts, const TB* __restrict__ kin,
                                                   size_t tstride, uint32_t* __restrict__ defer) {
  const uint32_t nt = *n_tasks;
  const int nb = P.nbits;
  const bool two = P.op == BSI_RANGE;
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (uni(blockIdx.x * blockDim.x + (threadIdx.x & ~63u)) >= nt) return;  // whole waves past the end
  const bool live = t < nt;
  const uint32_t tt = live ? t : 0;
  const CountRows tv{cnts + tt, tstride};
  const TB ebmT = kin[(size_t)kBsiRegSlices * tstride + tt];
  const TB fixT = kin[(size_t)(kBsiRegSlices + 1) * tstride + tt];
  int slow = 0;
  int kk = 0;
  const int cebm = tv(kk++);
  CircuitT z0{tb_absent(), tb_absent(), ebmT, 0, 0, cebm}, z1 = z0;
#pragma unroll 1
  for (int i = nb - 1; i >= 0; i--) {
    const TB sT = kin[(size_t)i * tstride + tt];
    types_step((P.pred0 >> i) & 1, sT, z0, kk, tv, slow);
    if (two) types_step((P.pred1 >> i) & 1, sT, z1, kk, tv, slow);
  }
  TB rt;
  if (two) {
    const TB left = types_finish(BSI_GE, fixT, z0, kk, tv, slow);
    const TB right = types_finish(BSI_LE, fixT, z1, kk, tv, slow);
    rt = tb_op<OPR_AND>(left, right, tv(kk++), slow);
  } else {
    rt = types_finish(P.op, fixT, z0, kk, tv, slow);
  }
  const bool ok = live && !slow;
  // sums: the sum shares follow the counted steps (kk of them); one atomic per slice per wave
  if (sums) {
    const bool add = ok && rt.card > 0;
    for (int x = 0; x < nb; x++) {
      const int c = wave_sum(add ? tv(kk + x) : 0);
      if ((threadIdx.x & 63) == 0 && c) atomicAdd(&sums[x], (unsigned long long)(uint32_t)c);
    }
    const int cc = wave_sum(add ? rt.card : 0);
    if ((threadIdx.x & 63) == 0 && cc) atomicAdd(&sums[kBsiMaxInputs], (unsigned long long)(uint32_t)cc);
  }
  if (!live) return;
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

void launch_plan_bsi(hipStream_t s, const uint32_t* key_off, const uint32_t* bm, uint32_t need, Task* by_key,
                     uint8_t* flag, uint32_t* wg_count, uint64_t* zlb, uint64_t* ztile) {
  hipLaunchKernelGGL(k_plan_bsi, dim3(256), dim3(256), 0, s, key_off, bm, need, by_key, flag, wg_count, zlb, ztile);
}

void launch_bsi(hipStream_t s, int grid, const Task* tasks, const uint32_t* nt, WideArgs args, BsiArgs p, OutCtx oc,
                unsigned long long* sums, BsiScratch* sc) {
  if (p.op <= BSI_RANGE && p.nbits <= kBsiRegSlices && sc) {
    (void)hipMemsetAsync(sc->defer, 0, 4, s);
    const int g = std::max(1, std::min(grid, resident_grid((const void*)&k_bsi_reg)));
    hipLaunchKernelGGL(k_bsi_reg, dim3(g), dim3(kNT1), 0, s, tasks, nt, args, p, oc, sums != nullptr, sc->cnts,
                       reinterpret_cast<TB*>(sc->kin), sc->stride);
    const int g2 = (int)((sc->stride + 255) / 256);
    hipLaunchKernelGGL(k_bsi_types, dim3(g2), dim3(256), 0, s, tasks, nt, args, p, oc, sums, sc->cnts,
                       reinterpret_cast<const TB*>(sc->kin), sc->stride, sc->defer);
    const int g3 = std::max(1, std::min(grid, resident_grid((const void*)&k_bsi_defer)));
    hipLaunchKernelGGL(k_bsi_defer, dim3(g3), dim3(256), 0, s, tasks, sc->defer, args, p, oc, sums);
    return;
  }
  const int g = std::max(1, std::min(grid, resident_grid((const void*)&k_bsi)));
  hipLaunchKernelGGL(k_bsi, dim3(g), dim3(256), 0, s, tasks, nt, args, p, oc, sums);
}

}  // namespace rbg
