// Bit-sliced index query on the MI355X: RoaringBitmapSliceIndex.compare + sum
// (bsi/src/main/java/org/roaringbitmap/bsi/RoaringBitmapSliceIndex.java, BSI/
// below) as ONE fused pass per key.
//
// The reference runs the O'Neil circuit (BSI/:432-468) as a chain of whole-bitmap
// pairwise ops, about 4 per slice. Each op is independent per high-16 key, so one
// workgroup takes one key. It keeps every bitmap of the circuit (EQ, GT, LT, for
// one or two predicates) in registers (4 words per thread) and streams each slice
// container of the key once. The result container types must be the reference's,
// so every step replays the pairwise type rule of the op it stands for (App. A,
// device.hpp): present / absent (an unmatched container is cloned, an empty result
// dropped), kind, cardinality, and the run count where EFF decides. sum
// (BSI/:581-592) is fused: after the result container of the key is known, each
// slice is re-read and |slice & found| is added to a per-slice total.
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
  const int nb = P.nbits;
  for (uint32_t t = blockIdx.x; t < nt; t += gridDim.x) {
    const Task tk = tasks[t];
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
    if (P.op == BSI_SUM_ONLY) continue;
    if (!res.present) {
      wg_place(t, false, nullptr, true, tmp, 0, 0, tk.key, DK_A, oc, nullptr);
    } else if (res.src >= 0) {
      wg_passthrough(t, A.desc[res.src], A.payload, oc, nullptr);
    } else {
      const uint32_t len = stage_container(res.kind, res.r, res.card, acc, tmp, sh);
      wg_place(t, true, nullptr, true, tmp, len, (uint32_t)res.card, tk.key, res.kind, oc, nullptr);
    }
  }
}

void launch_plan_bsi(hipStream_t s, const uint32_t* key_off, const uint32_t* bm, uint32_t need, Task* by_key,
                     uint8_t* flag, uint32_t* wg_count, uint64_t* zlb, uint64_t* ztile) {
  hipLaunchKernelGGL(k_plan_bsi, dim3(256), dim3(256), 0, s, key_off, bm, need, by_key, flag, wg_count, zlb, ztile);
}

void launch_bsi(hipStream_t s, int grid, const Task* tasks, const uint32_t* nt, WideArgs args, BsiArgs p, OutCtx oc,
                unsigned long long* sums) {
  const int g = std::max(1, std::min(grid, resident_grid((const void*)&k_bsi)));
  hipLaunchKernelGGL(k_bsi, dim3(g), dim3(256), 0, s, tasks, nt, args, p, oc, sums);
}

}  // namespace rbg
