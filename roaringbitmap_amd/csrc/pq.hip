// FastAggregation.priorityqueue_or / priorityqueue_xor (RB/FastAggregation.java:677-812)
// on the MI355X.  RB/ = reference RoaringBitmap/src/main/java/org/roaringbitmap/.
//
// The reference pairs whole bitmaps in a java.util.PriorityQueue ordered by
// getLongSizeInBytes, so every step's operands depend on the sizes of earlier
// intermediate results over all keys.  The host replays the queue (engine.cpp:
// ctx_pq); each step here is one launch over the union keys of the batch (one
// workgroup per key) that combines two nodes -- an input bitmap (leaf) or an
// intermediate (temp) -- with the step's whole-bitmap op, keeps the per-key
// result in a temp slot and adds its getSizeInBytes to the step's size word.
//
// Per key a temp holds a PQState (kind, cardinality, run count) and either the
// index of the input container it is an unchanged clone of, or the container's
// set as an 8 KiB bitmap.  Kinds follow the reference's lazy algebra
// (RB/Container.java:717-774 lazyIOR / lazyOR): a lazy bitmap (card -1 in the
// reference) is kept apart from an exact one, because repairAfterLazy converts
// only the lazy one (RB/BitmapContainer.java:1205-1215).
#include <algorithm>

#include "kernels.hpp"
#include "wave.hpp"

namespace rbg {

__device__ __forceinline__ int block_card4(const uint64_t r[4], int* sh) {
  int c = popc64(r[0]) + popc64(r[1]) + popc64(r[2]) + popc64(r[3]);
  int u = 0;
  block_sum2(c, u, sh);
  return (int)uni((uint32_t)c);
}

// lazy OR of a run and an array container: RunContainer.lazyorToRun +
// convertToLazyBitmapIfNeeded (RB/RunContainer.java:1769-1813, 861-875): a full
// result is RunContainer.full(); more than 4096 runs a lazy bitmap; else runs
__device__ __forceinline__ int pq_run_lazyor_kind(bool r_full, int c, int nr) {
  if (r_full || c == 65536) return PK_R;
  return nr > 4096 ? PK_BL : PK_R;
}

struct PQNode {
  int present;
  int kind;  // PK_*
  int card;
  int nruns;
  int src;   // >= 0: desc index of the input container this one is a clone of
};

// Node of `ref` at task t (segment [s, s + n) of the key-major batch).  A leaf's
// container is found by a workgroup-wide scan of the segment's input indices
// (ascending); `found` is one int of LDS.  Contains barriers.
__device__ __forceinline__ PQNode pq_load(const PQRef& ref, const PQArgs& A, uint32_t t, uint32_t s, uint32_t n,
                                          int* found) {
  PQNode x{0, PK_A, 0, 0, -1};
  if (ref.leaf >= 0) {
    if (threadIdx.x == 0) *found = -1;
    lds_barrier();
    for (uint32_t j = threadIdx.x; j < n; j += NT)
      if (A.bm[s + j] == (uint32_t)ref.leaf) *found = (int)(s + j);
    lds_barrier();
    const int j = *found;
    lds_barrier();
    if (j >= 0) {
      const CDesc d = A.desc[j];
      x.present = 1;
      x.kind = d.kind;  // DK_A / DK_B (= PK_BE) / DK_R
      x.card = (int)d.card;
      x.nruns = d.kind == DK_R ? *reinterpret_cast<const uint16_t*>(A.payload + d.slot + 2) : 0;
      x.src = j;
    }
  } else {
    const PQState st = ref.st[t];
    x.present = st.present;
    x.kind = st.kind;
    x.card = (int)st.card;
    x.nruns = st.nruns;
    x.src = st.src;
  }
  return x;
}

__device__ __forceinline__ void pq_materialize(const PQNode& x, const PQRef& ref, const PQArgs& A, uint32_t t,
                                               uint32_t* lds, int* q, uint64_t r[4]) {
  if (x.src >= 0) materialize(A.desc[x.src], A.payload, lds, q, r);
  else load_bitmap_owned(reinterpret_cast<const uint8_t*>(ref.set + (size_t)t * 1024), r);
}

__device__ __forceinline__ int pq_size(int kind, int card, int nruns) {  // getSizeInBytes + the 2 B key
  return 2 + (kind == PK_A ? 2 * card + 4 : kind == PK_R ? 4 * nruns + 4 : 8192);
}

// The kind of one step's result where both operands hold the key.  `a` is the
// receiver of the reference's call, `b` its argument; r is the union (OR) or the
// symmetric difference (XOR).  *c / *nr: cardinality / runs of r as needed.
__device__ __forceinline__ int pq_kind(int op, const PQNode& a, const PQNode& b, const uint64_t r[4], uint32_t* lds,
                                       int* sh, int* c, int* nr) {
  *c = block_card4(r, sh);
  *nr = 0;
  if (op == PQ_XOR) {  // RoaringBitmap.xor(x1, x2): the pairwise XOR types (App. A)
    if (*c == 0) return -1;  // dropped
    const int ka = a.kind == PK_BL ? DK_B : a.kind, kb = b.kind == PK_BL ? DK_B : b.kind;
    if (pairwise_needs_runs(OPR_XOR, ka, a.card, kb, b.card)) {
      *nr = count_runs(r, lds, sh);
      return eff(*c, *nr);
    }
    return by_card(*c);
  }
  const bool a_bm = a.kind == PK_BE || a.kind == PK_BL, b_bm = b.kind == PK_BE || b.kind == PK_BL;
  if (op == PQ_LOR) {
    // Container.lazyOR (RB/Container.java:752-774); both operands are input containers
    if (a.kind == PK_A && b.kind == PK_A) return a.card + b.card > 1024 ? PK_BL : PK_A;  // ArrayContainer.lazyor
    if (a_bm || b_bm) return PK_BL;  // BitmapContainer.lazyor(A|B|R) / A|R lazyor(B): a lazy bitmap clone
    if (a.kind == PK_R && b.kind == PK_R) {  // RunContainer.or(RunContainer) (:1952-1986)
      if (a.card == 65536 || b.card == 65536) return PK_R;
      *nr = count_runs(r, lds, sh);
      return eff(*c, *nr);
    }
    *nr = count_runs(r, lds, sh);  // A|R, R|A: lazyorToRun
    return pq_run_lazyor_kind((a.kind == PK_R ? a.card : b.card) == 65536, *c, *nr);
  }
  // Container.lazyIOR (RB/Container.java:717-740), receiver a.  lazyorfromlazyinputs
  // (RB/RoaringBitmap.java:769-818) has already put a bitmap operand first.
  if (a_bm) return PK_BL;  // BitmapContainer.ilazyor
  if (a.kind == PK_A) {
    if (b.kind == PK_A) return a.card + b.card > 1024 ? PK_BL : PK_A;  // ArrayContainer.lazyor
    if (b_bm) return *c == 65536 ? PK_R : PK_BE;  // ior(BitmapContainer) = b.or(this), exact (:1064-1085)
    *nr = count_runs(r, lds, sh);                 // b.lazyor(this)
    return pq_run_lazyor_kind(b.card == 65536, *c, *nr);
  }
  // a is a run container
  if (a.card == 65536) return PK_R;  // a full run container returns itself (RB/RunContainer.java:1198-1240,1500-1550)
  if (b_bm) return *c == 65536 ? PK_R : PK_BE;  // RunContainer.or(BitmapContainer), exact (:1932-1949)
  if (b.kind == PK_A) {
    *nr = count_runs(r, lds, sh);  // ilazyorToRun
    return pq_run_lazyor_kind(false, *c, *nr);
  }
  if (b.card == 65536) return PK_R;  // RunContainer.or(RunContainer)
  *nr = count_runs(r, lds, sh);
  return eff(*c, *nr);
}

// One step of the queue over every union key: out = op(a, b).  out may be a's temp
// slot (the in-place RoaringBitmap.lazyor and lazyorfromlazyinputs).
__global__ __launch_bounds__(256) void k_pq_step(const Task* __restrict__ tasks, const uint32_t* __restrict__ n_tasks,
                                                 PQArgs A, int op, PQRef a_ref, PQRef b_ref, PQRef o_ref,
                                                 unsigned long long* size) {
  __shared__ __align__(16) uint32_t lds[2048];
  __shared__ int q[257];
  __shared__ int sh[8];
  __shared__ int found;
  const uint32_t nt = *n_tasks;
  unsigned long long acc = 0;
  for (uint32_t t = blockIdx.x; t < nt; t += gridDim.x) {
    const Task tk = tasks[t];
    const uint32_t s = (uint32_t)tk.a, n = (uint32_t)tk.b;
    PQNode a = pq_load(a_ref, A, t, s, n, &found);
    PQNode b = pq_load(b_ref, A, t, s, n, &found);
    PQRef ar = a_ref, br = b_ref;
    // lazyorfromlazyinputs: a bitmap container goes first (RB/RoaringBitmap.java:782-788)
    if (op == PQ_LFL && a.present && b.present && (b.kind == PK_BE || b.kind == PK_BL) &&
        !(a.kind == PK_BE || a.kind == PK_BL)) {
      const PQNode x = a;
      a = b;
      b = x;
      const PQRef y = ar;
      ar = br;
      br = y;
    }
    __syncthreads();  // every thread has read the states before the output state is written
    PQState out{0, 0, 0, 0, -1, 0};
    bool write_set = false, copy_set = false;
    const PQRef* copy_from = nullptr;
    uint64_t r[4] = {0, 0, 0, 0};
    if (a.present && b.present) {
      uint64_t x[4];
      pq_materialize(a, ar, A, t, lds, q, r);
      pq_materialize(b, br, A, t, lds, q, x);
#pragma unroll
      for (int i = 0; i < 4; i++) r[i] = op == PQ_XOR ? (r[i] ^ x[i]) : (r[i] | x[i]);
      int c, nr;
      const int kind = pq_kind(op, a, b, r, lds, sh, &c, &nr);
      if (kind >= 0) {
        if (kind == PK_R && nr == 0) nr = c == 65536 ? 1 : count_runs(r, lds, sh);
        out = PQState{(uint32_t)c, (uint16_t)nr, (uint8_t)kind, 1, -1, 0};
        write_set = true;
      }
    } else if (a.present || b.present) {
      // unmatched key: a clone of the operand that holds it
      const PQNode& x = a.present ? a : b;
      const PQRef& xr = a.present ? ar : br;
      out = PQState{(uint32_t)x.card, (uint16_t)x.nruns, (uint8_t)x.kind, 1, x.src, 0};
      if (x.src < 0 && xr.set != o_ref.set) {
        copy_set = true;
        copy_from = &xr;
      }
    }
    if (write_set) store_bitmap_owned(reinterpret_cast<uint8_t*>(o_ref.set + (size_t)t * 1024), r);
    if (copy_set) {
      load_bitmap_owned(reinterpret_cast<const uint8_t*>(copy_from->set + (size_t)t * 1024), r);
      store_bitmap_owned(reinterpret_cast<uint8_t*>(o_ref.set + (size_t)t * 1024), r);
    }
    if (threadIdx.x == 0) {
      o_ref.st[t] = out;
      if (out.present) acc += (unsigned long long)pq_size(out.kind, (int)out.card, out.nruns);
    }
  }
  if (threadIdx.x == 0 && acc) atomicAdd(size, acc);
}

// The root of the queue as the result: priorityqueue_or repairs it
// (RoaringBitmap.repairAfterLazy, RB/RoaringBitmap.java:2752-2757: A kept, R
// toEfficientContainer, a lazy bitmap BY_CARD with 65536 -> RunContainer.full, an exact
// bitmap kept); priorityqueue_xor returns it as is.
__global__ __launch_bounds__(256) void k_pq_final(const Task* __restrict__ tasks, const uint32_t* __restrict__ n_tasks,
                                                  PQArgs A, int repair, PQRef root, OutCtx oc) {
  __shared__ __align__(16) uint32_t acc[2048];
  __shared__ __align__(16) uint32_t tmp[2048];
  __shared__ int q[257];
  __shared__ int sh[8];
  __shared__ int found;
  __shared__ Prefix shp;
  const uint32_t nt = *n_tasks;
  for (uint32_t t = blockIdx.x; t < nt; t += gridDim.x) {
    __syncthreads();
    const Task tk = tasks[t];
    const PQNode x = pq_load(root, A, t, (uint32_t)tk.a, (uint32_t)tk.b, &found);
    if (!x.present) {
      wg_place(t, false, nullptr, true, tmp, 0, 0, tk.key, DK_A, oc, &shp);
      continue;
    }
    uint64_t r[4];
    int kind, c = x.card;
    if (x.src >= 0) {
      const CDesc d = A.desc[x.src];
      if (!repair || d.kind != DK_R || eff((int)d.card, x.nruns) == DK_R) {
        wg_passthrough(t, d, A.payload, oc, &shp);
        continue;
      }
      materialize(d, A.payload, tmp, q, r);  // RunContainer.toEfficientContainer -> A / B
      kind = by_card(c);
    } else {
      load_bitmap_owned(reinterpret_cast<const uint8_t*>(root.set + (size_t)t * 1024), r);
      if (!repair) kind = x.kind == PK_BL ? DK_B : x.kind;
      else if (x.kind == PK_BL) kind = c == 65536 ? DK_R : by_card(c);
      else if (x.kind == PK_R) kind = eff(c, x.nruns);
      else kind = x.kind;  // A, exact B
    }
    const uint32_t len = stage_container(kind, r, c, acc, tmp, sh);
    wg_place(t, true, nullptr, true, tmp, len, (uint32_t)c, tk.key, kind, oc, &shp);
  }
}

// getLongSizeInBytes of every input bitmap (RB/RoaringBitmap.java:2212-2219) without the
// constant 8: sizes[bm] += 2 + getSizeInBytes of each container
__global__ __launch_bounds__(256) void k_pq_leaf_sizes(const CDesc* __restrict__ desc, const uint32_t* __restrict__ bm,
                                                       const uint8_t* __restrict__ payload, uint64_t n,
                                                       unsigned long long* __restrict__ sizes) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const CDesc d = desc[i];
    const int nr = d.kind == DK_R ? *reinterpret_cast<const uint16_t*>(payload + d.slot + 2) : 0;
    atomicAdd(sizes + bm[i], (unsigned long long)pq_size(d.kind, (int)d.card, nr));
  }
}

void launch_pq_leaf_sizes(hipStream_t s, const CDesc* desc, const uint32_t* bm, const uint8_t* payload, uint64_t n,
                          unsigned long long* sizes) {
  if (n == 0) return;
  const unsigned g = (unsigned)std::min<uint64_t>((n + 255) / 256, 4096);
  hipLaunchKernelGGL(k_pq_leaf_sizes, dim3(g), dim3(256), 0, s, desc, bm, payload, n, sizes);
}

void launch_pq_step(hipStream_t s, int grid, const Task* tasks, const uint32_t* nt, PQArgs args, int op, PQRef a,
                    PQRef b, PQRef out, unsigned long long* size) {
  grid = std::max(1, std::min(grid, resident_grid((const void*)&k_pq_step)));
  hipLaunchKernelGGL(k_pq_step, dim3(grid), dim3(256), 0, s, tasks, nt, args, op, a, b, out, size);
}

void launch_pq_final(hipStream_t s, int grid, const Task* tasks, const uint32_t* nt, PQArgs args, int repair,
                     PQRef root, OutCtx oc) {
  grid = std::max(1, std::min(grid, resident_grid((const void*)&k_pq_final)));
  hipLaunchKernelGGL(k_pq_final, dim3(grid), dim3(256), 0, s, tasks, nt, args, repair, root, oc);
}

}  // namespace rbg
