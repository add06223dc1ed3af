// FastAggregation.priorityqueue_or / priorityqueue_xor (RB/FastAggregation.java:677-812)
// on the MI355X.  RB/ = reference RoaringBitmap/src/main/java/org/roaringbitmap/.
//
// The reference pairs whole bitmaps in a java.util.PriorityQueue ordered by
// getLongSizeInBytes, so every step's operands depend on the sizes of earlier
// intermediate results over all keys.  The queue lives in device memory: the host
// adds the inputs and plans the first step (engine.cpp: ctx_pq), then enqueues N - 1
// launches of k_pq_step.  Each combines the two nodes its step record names -- an input
// bitmap (leaf) or an intermediate (temp) -- over every union key (one workgroup per
// key), keeps the per-key result in the output temp and adds its getSizeInBytes to the
// step's size word; the launch's last workgroup folds that size into the queue and
// polls the next pair (pq_finish / pq_plan, kernels.hpp) with one wave, reading the
// heap a six-level subtree per round trip.  No host read-back between steps.
//
// Per key a temp holds a PQState (kind, cardinality, run count) and either the
// index of the input container it is an unchanged clone of, or an 8 KiB block of the
// set arena holding the container as a bitmap.  Blocks move with the data: a step's
// result reuses an operand temp's block at that key (every operand temp is consumed by
// its step -- updated in place or released), a fresh block comes off the key's own pool
// only where neither operand has one, and blocks left over go back to it.  A block at key
// t holds the combination of at least two of the key's input containers and live temps
// cover disjoint sets of inputs, so a pool of floor(n_t / 2) blocks (n_t = the inputs
// holding key t) never runs out, and no two workgroups share a pool (no atomics).
// Kinds follow the reference's lazy algebra
// (RB/Container.java:717-774 lazyIOR / lazyOR): a lazy bitmap (card -1 in the
// reference) is kept apart from an exact one, because repairAfterLazy converts
// only the lazy one (RB/BitmapContainer.java:1205-1215).
#include <algorithm>

#include "kernels.hpp"
#include "wave.hpp"

namespace rbg {

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
  int blk;   // temp: set arena block (-1: none)
};

__device__ __forceinline__ PQState* pq_states(const PQDev& D, int ref) {
  return D.states + (uint64_t)(-1 - ref) * D.stride;
}
__device__ __forceinline__ uint8_t* pq_block(const PQDev& D, int blk) {
  return reinterpret_cast<uint8_t*>(D.arena + (uint64_t)blk * 1024);
}

// Positions of inputs ra and rb (< 0: a temp, not searched) in the segment's ascending
// input indices bm[s, s + n), n when absent: a 64-way search by each wave (lane i samples
// position lo + i * step; the samples below ref are a prefix, so their count brackets
// it), one dependent load round per factor of 64 -- two rounds up to 4,096 inputs at the
// key -- and both searches' loads issued together in each round.
__device__ __forceinline__ void leaf_find2(const uint32_t* bm, uint32_t s, uint32_t n, int ra, int rb, uint32_t* at) {
  const uint32_t lane = (uint32_t)lane_id();
  const uint32_t ref[2] = {(uint32_t)ra, (uint32_t)rb};
  uint32_t lo[2] = {0, 0}, hi[2] = {n, n};
  bool done[2] = {ra < 0, rb < 0};
  at[0] = at[1] = n;
  while (!(done[0] && done[1])) {
    uint32_t v[2], step[2];
#pragma unroll
    for (int i = 0; i < 2; i++) {  // every load of the round first
      step[i] = hi[i] - lo[i] <= 64 ? 1 : (hi[i] - lo[i] + 63) >> 6;
      const uint32_t p = lo[i] + lane * step[i];
      v[i] = !done[i] && p < hi[i] ? bm[s + p] : 0xFFFFFFFFu;
    }
#pragma unroll
    for (int i = 0; i < 2; i++) {
      if (done[i]) continue;
      const uint32_t k = (uint32_t)__popcll(__ballot(v[i] < ref[i]));
      if (step[i] == 1 || k == 0) {  // the lower bound is lo + k (k == 0: lane 0 sampled lo)
        const uint32_t p = step[i] == 1 ? lo[i] + k : lo[i];
        uint32_t x;
        if (p < hi[i]) x = (uint32_t)__builtin_amdgcn_readlane((int)v[i], step[i] == 1 ? (int)k : 0);
        else x = p < n ? bm[s + p] : 0xFFFFFFFFu;
        at[i] = x == ref[i] ? p : n;
        done[i] = true;
      } else {
        const uint32_t nlo = lo[i] + (k - 1) * step[i] + 1;
        hi[i] = min(hi[i], lo[i] + k * step[i]);
        lo[i] = nlo;
      }
    }
  }
}

// Node `ref` at task t (segment [s, s + n) of the key-major batch); `pos`: a leaf's
// position in the segment (leaf_find2).
__device__ __forceinline__ PQNode pq_load(int ref, uint32_t pos, const PQDev& D, const PQArgs& A, uint32_t t,
                                          uint32_t s, uint32_t n) {
  PQNode x{0, PK_A, 0, 0, -1, -1};
  if (ref >= 0) {
    if (pos < n) {
      const uint32_t j = s + pos;
      const CDesc d = A.desc[j];
      x.present = 1;
      x.kind = d.kind;  // DK_A / DK_B (= PK_BE) / DK_R
      x.card = (int)d.card;
      x.nruns = d.kind == DK_R ? *reinterpret_cast<const uint16_t*>(A.payload + d.slot + 2) : 0;
      x.src = (int)j;
    }
  } else {
    const PQState st = pq_states(D, ref)[t];
    x.present = st.present;
    x.kind = st.kind;
    x.card = (int)st.card;
    x.nruns = st.nruns;
    x.src = st.src;
    x.blk = st.present ? st.blk : -1;
  }
  return x;
}

// a node's container into one wave's registers / combined into them (OR or XOR); `lds` is
// the wave's 8 KiB bitmap
__device__ __forceinline__ void w_pq_materialize(const PQNode& x, const PQDev& D, const PQArgs& A, uint32_t* lds,
                                                 WCtr& r) {
  if (x.src >= 0) w_materialize(A.desc[x.src], A.payload, lds, r);
  else if (x.blk >= 0) w_load_bitmap(pq_block(D, x.blk), r);
  else w_zero(r);  // a pool ran out in an earlier step (reported through ctl->err)
}
template <int OP>  // 1 or, 2 xor (wave.hpp w_op)
__device__ __forceinline__ void w_pq_combine(const PQNode& x, const PQDev& D, const PQArgs& A, uint32_t* lds,
                                             WCtr& r) {
  if (x.src >= 0) {
    w_combine<OP>(A.desc[x.src], A.payload, lds, r);
  } else if (x.blk >= 0) {
    const CDesc d{0, 0, 0, (uint8_t)DK_B, 0};
    w_combine<OP>(d, pq_block(D, x.blk), lds, r);
  }
}

__device__ __forceinline__ void pq_materialize(const PQNode& x, const PQDev& D, const PQArgs& A, uint32_t* lds, int* q,
                                               uint64_t r[4]) {
  if (x.src >= 0) {
    materialize(A.desc[x.src], A.payload, lds, q, r);
  } else if (x.blk >= 0) {
    load_bitmap_owned(pq_block(D, x.blk), r);
  } else {  // the arena ran out in an earlier step (reported through ctl->err)
    r[0] = r[1] = r[2] = r[3] = 0;
  }
}

__device__ __forceinline__ int pq_size(int kind, int card, int nruns) {  // getSizeInBytes + the 2 B key
  return 2 + (kind == PK_A ? 2 * card + 4 : kind == PK_R ? 4 * nruns + 4 : 8192);
}

// The kind of one step's result where both operands hold the key.  `a` is the
// receiver of the reference's call, `b` its argument; x (one wave's registers) is the
// union (OR) or the symmetric difference (XOR).  *c / *nr: cardinality / runs of x as needed.
__device__ __forceinline__ int pq_kind(int op, const PQNode& a, const PQNode& b, const WCtr& x, int* c, int* nr) {
  *c = w_card(x);
  *nr = 0;
  if (op == PQ_XOR) {  // RoaringBitmap.xor(x1, x2): the pairwise XOR types (App. A)
    if (*c == 0) return -1;  // dropped
    const int ka = a.kind == PK_BL ? DK_B : a.kind, kb = b.kind == PK_BL ? DK_B : b.kind;
    if (pairwise_needs_runs(OPR_XOR, ka, a.card, kb, b.card)) {
      *nr = w_runs(x);
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
      *nr = w_runs(x);
      return eff(*c, *nr);
    }
    *nr = w_runs(x);  // A|R, R|A: lazyorToRun
    return pq_run_lazyor_kind((a.kind == PK_R ? a.card : b.card) == 65536, *c, *nr);
  }
  // Container.lazyIOR (RB/Container.java:717-740), receiver a.  lazyorfromlazyinputs
  // (RB/RoaringBitmap.java:769-818) has already put a bitmap operand first.
  if (a_bm) return PK_BL;  // BitmapContainer.ilazyor
  if (a.kind == PK_A) {
    if (b.kind == PK_A) return a.card + b.card > 1024 ? PK_BL : PK_A;  // ArrayContainer.lazyor
    if (b_bm) return *c == 65536 ? PK_R : PK_BE;  // ior(BitmapContainer) = b.or(this), exact (:1064-1085)
    *nr = w_runs(x);                 // b.lazyor(this)
    return pq_run_lazyor_kind(b.card == 65536, *c, *nr);
  }
  // a is a run container
  if (a.card == 65536) return PK_R;  // a full run container returns itself (RB/RunContainer.java:1198-1240,1500-1550)
  if (b_bm) return *c == 65536 ? PK_R : PK_BE;  // RunContainer.or(BitmapContainer), exact (:1932-1949)
  if (b.kind == PK_A) {
    *nr = w_runs(x);  // ilazyorToRun
    return pq_run_lazyor_kind(false, *c, *nr);
  }
  if (b.card == 65536) return PK_R;  // RunContainer.or(RunContainer)
  *nr = w_runs(x);
  return eff(*c, *nr);
}

// ---- the queue on the device ----------------------------------------------------
// Loads and stores of the queue go through the vector memory path (atomic loads and
// stores, relaxed): the scheduling wave rereads entries it has just written.
template <class T>
__device__ __forceinline__ T pq_ld(const T* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
template <class T>
__device__ __forceinline__ void pq_st(T* p, T v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ int64_t rl64(int64_t v, int lane) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v, lane);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)((uint64_t)v >> 32), lane);
  return (int64_t)(((uint64_t)hi << 32) | lo);
}

// The queue operations run by one whole wave with uniform control flow; lane 0 stores.
// The heap is java.util.PriorityQueue's array: siftUp / siftDown as OpenJDK, each
// round trip fetching up to five levels of the path at once.
struct PQWave {
  const PQDev& D;
  int lane;
  __device__ void st_ent(int k, const PQEnt& e) {
    if (lane == 0) {
      pq_st(&D.heap[k].size, e.size);
      pq_st(&D.heap[k].node, e.node);
    }
  }
  __device__ PQEnt ld_ent(int k) { return PQEnt{pq_ld(&D.heap[k].size), pq_ld(&D.heap[k].node), 0}; }
  __device__ void add(PQStep& c, PQEnt x) {
    int k = c.heap_n++;
    // ancestor L + 1 levels up of position k, one per lane
    const int up = (k + 1) >> (lane + 1);
    int64_t asz = 0;
    int32_t and_ = 0;
    if (lane < 31 && up >= 1) {
      asz = pq_ld(&D.heap[up - 1].size);
      and_ = pq_ld(&D.heap[up - 1].node);
    }
    for (int L = 0; k > 0; L++) {
      const int64_t esz = rl64(asz, L);
      const int32_t end = __builtin_amdgcn_readlane(and_, L);
      if (pq_cmp(x.size, esz) >= 0) break;
      st_ent(k, PQEnt{esz, end, 0});
      k = (k - 1) >> 1;
    }
    st_ent(k, x);
    __threadfence_block();
  }
  __device__ PQEnt poll(PQStep& c) {
    const PQEnt r = ld_ent(0);
    const int n = --c.heap_n;
    if (n == 0) return r;
    const PQEnt x = ld_ent(n);
    // lane -> depth d (1..5) below the round trip's root, index j within that depth
    const int d = 31 - __builtin_clz((unsigned)lane + 2);
    const int j = lane + 2 - (1 << d);
    const int half = n >> 1;
    int k = 0;
    bool done = k >= half;
    while (!done) {
      const int pos = ((k + 1) << d) - 1 + j;
      int64_t sz = 0;
      int32_t nd = 0;
      if (d <= 5 && pos < n) {
        sz = pq_ld(&D.heap[pos].size);
        nd = pq_ld(&D.heap[pos].node);
      }
      int rel = 0;
      for (int dd = 0; dd < 5; dd++) {
        if (k >= half) {
          done = true;
          break;
        }
        int child = 2 * k + 1;
        int cl = (2 << dd) - 2 + 2 * rel;
        int64_t csz = rl64(sz, cl);
        int32_t cnd = __builtin_amdgcn_readlane(nd, cl);
        int nrel = 2 * rel;
        if (child + 1 < n) {
          const int64_t rsz = rl64(sz, cl + 1);
          if (pq_cmp(csz, rsz) > 0) {
            csz = rsz;
            cnd = __builtin_amdgcn_readlane(nd, cl + 1);
            child++;
            nrel++;
          }
        }
        if (pq_cmp(x.size, csz) <= 0) {
          done = true;
          break;
        }
        st_ent(k, PQEnt{csz, cnd, 0});
        k = child;
        rel = nrel;
      }
    }
    st_ent(k, x);
    __threadfence_block();
    return r;
  }
  __device__ int32_t node(int i) { return pq_ld(&D.node[i]); }
  __device__ void set_node(int i, int32_t v) {
    if (lane == 0) pq_st(&D.node[i], v);
    __threadfence_block();
  }
  __device__ bool istmp(int i) { return pq_ld(&D.istmp[i]) != 0; }
  __device__ void set_istmp(int i) {
    if (lane == 0) pq_st(&D.istmp[i], (uint8_t)1);
    __threadfence_block();
  }
  __device__ int slot_pop(PQStep& c) { return pq_ld(&D.slots[--c.slot_top]); }
  __device__ void slot_push(PQStep& c, int s) {
    if (lane == 0) pq_st(&D.slots[c.slot_top], s);
    c.slot_top++;
    __threadfence_block();
  }
};

// One step of the queue over every union key: out = op(a, b), the step record's operands.
// out may be a's temp (the in-place x1.lazyor and lazyorfromlazyinputs).  One wave per key
// (grid-stride over the resident grid's waves; a key's chain of dependent loads -- task,
// leaf search, descriptor, payload or block -- is latency, so the more keys in flight the
// better: a wave per key keeps 4x the keys of a workgroup per key in flight per CU).  The
// launch's last workgroup plans the next step.
__global__ __launch_bounds__(256) void k_pq_step(const Task* __restrict__ tasks, const uint32_t* __restrict__ n_tasks,
                                                 PQArgs A, PQDev D) {
  __shared__ __align__(16) uint32_t lds_w[4][2048];
  __shared__ unsigned long long acc_w[4];
  __shared__ int last;
  const int wv = (int)(threadIdx.x >> 6), lane = lane_id();
  uint32_t* lds = lds_w[wv];
  const int op = D.ctl->step.op;
  const int a_ref = D.ctl->step.a, b_ref = D.ctl->step.b, o_ref = D.ctl->step.o;
  PQState* const o_st = pq_states(D, o_ref);
  const uint32_t nt = *n_tasks;
  unsigned long long acc = 0;
  for (uint32_t t = uni(blockIdx.x * 4 + (uint32_t)wv); t < nt; t += gridDim.x * 4) {
    const Task tk = tasks[t];
    const uint32_t s = (uint32_t)tk.a, n = (uint32_t)tk.b;
    // lane 0: the key's pool top and its next free block, in flight during the search
    int32_t pool_top = 0, pool_blk = -1;
    uint32_t pool_base = 0;
    if (lane == 0) {
      pool_base = D.kbase[t];
      pool_top = D.ktop[t];
      if (pool_top > 0) pool_blk = D.kstack[pool_base + pool_top - 1];
    }
    uint32_t pos[2];
    leaf_find2(A.bm, s, n, a_ref, b_ref, pos);
    PQNode a = pq_load(a_ref, pos[0], D, A, t, s, n);
    PQNode b = pq_load(b_ref, pos[1], D, A, t, s, n);
    // lazyorfromlazyinputs: a bitmap container goes first (RB/RoaringBitmap.java:782-788)
    if (op == PQ_LFL && a.present && b.present && (b.kind == PK_BE || b.kind == PK_BL) &&
        !(a.kind == PK_BE || a.kind == PK_BL)) {
      const PQNode x = a;
      a = b;
      b = x;
    }
    PQState out{0, 0, 0, 0, -1, -1};
    // every operand temp is consumed by the step, so its blocks are the result's to
    // reuse; the ones not reused go back to the key's pool
    int spare0 = a.blk, spare1 = b.blk;
    bool write_set = false;
    WCtr r;
    if (a.present && b.present) {
      w_pq_materialize(a, D, A, lds, r);
      if (op == PQ_XOR) w_pq_combine<2>(b, D, A, lds, r);
      else w_pq_combine<1>(b, D, A, lds, r);
      int c, nr;
      const int kind = pq_kind(op, a, b, r, &c, &nr);
      if (kind >= 0) {
        if (kind == PK_R && nr == 0) nr = c == 65536 ? 1 : w_runs(r);
        out = PQState{(uint32_t)c, (uint16_t)nr, (uint8_t)kind, 1, -1, -1};
        write_set = true;
      }
    } else if (a.present || b.present) {
      // unmatched key: the operand's container moves over unchanged (a clone of an input
      // container, or the temp's block itself)
      const PQNode& x = a.present ? a : b;
      out = PQState{(uint32_t)x.card, (uint16_t)x.nruns, (uint8_t)x.kind, 1, x.src, x.blk};
      if (x.blk >= 0) {
        if (spare0 == x.blk) spare0 = -1;
        else spare1 = -1;
      }
    }
    int blk = -1;
    if (lane == 0) {
      // the key's own block pool (no other wave touches it during the step)
      int top = pool_top;
      if (write_set) {
        if (spare0 >= 0) {
          blk = spare0;
          spare0 = -1;
        } else if (spare1 >= 0) {
          blk = spare1;
          spare1 = -1;
        } else {
          blk = pool_blk;
          top--;
          if (blk < 0) atomicOr(&D.ctl->err, 1u);
        }
      }
      if (spare0 >= 0) D.kstack[pool_base + top++] = spare0;
      if (spare1 >= 0) D.kstack[pool_base + top++] = spare1;
      if (top != pool_top) D.ktop[t] = max(top, 0);
    }
    if (write_set) {
      out.blk = __builtin_amdgcn_readfirstlane(blk);
      if (out.blk >= 0) w_store_bitmap(pq_block(D, out.blk), r);
    }
    if (lane == 0) {  // the operand states were read above (their values are in registers)
      o_st[t] = out;
      if (out.present) acc += (unsigned long long)pq_size(out.kind, (int)out.card, out.nruns);
    }
  }
  if (lane == 0) acc_w[wv] = acc;
  __syncthreads();
  if (threadIdx.x == 0) acc = acc_w[0] + acc_w[1] + acc_w[2] + acc_w[3];
  // the last workgroup to finish schedules: each workgroup adds its size to its group's
  // word and counts in (release); the group's last one counts the group in; the last
  // group's last workgroup acquires every size
  const int g = (int)(blockIdx.x % kPQGroups);
  const uint32_t n_groups = min(gridDim.x, (uint32_t)kPQGroups);
  const uint32_t in_group = (gridDim.x - (uint32_t)g + kPQGroups - 1) / kPQGroups;
  if (threadIdx.x == 0) {
    if (acc) atomicAdd(&D.ctl->grp[g].size, acc);
    bool l = __hip_atomic_fetch_add(&D.ctl->grp[g].done, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) ==
             in_group - 1;
    if (l) l = __hip_atomic_fetch_add(&D.ctl->done, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT) == n_groups - 1;
    last = l;
  }
  __syncthreads();
  if (!last) return;
  __threadfence();
  if (threadIdx.x >= 64) return;
  PQWave m{D, (int)threadIdx.x};
  PQStep c;
  c.op = pq_ld(&D.ctl->step.op);
  c.final_step = pq_ld(&D.ctl->step.final_step);
  c.a = pq_ld(&D.ctl->step.a);
  c.b = pq_ld(&D.ctl->step.b);
  c.o = pq_ld(&D.ctl->step.o);
  c.target = pq_ld(&D.ctl->step.target);
  c.rel1 = pq_ld(&D.ctl->step.rel1);
  c.rel2 = pq_ld(&D.ctl->step.rel2);
  c.heap_n = pq_ld(&D.ctl->step.heap_n);
  c.n_nodes = pq_ld(&D.ctl->step.n_nodes);
  c.slot_top = pq_ld(&D.ctl->step.slot_top);
  c.or_mode = pq_ld(&D.ctl->step.or_mode);
  unsigned long long size = 0;
  for (int k = 0; k < kPQGroups; k++) size += pq_ld(&D.ctl->grp[k].size);
  pq_finish(m, c, 8 + (int64_t)size);
  pq_plan(m, c);
  if (threadIdx.x == 0) {
    pq_st(&D.ctl->step.op, c.op);
    pq_st(&D.ctl->step.final_step, c.final_step);
    pq_st(&D.ctl->step.a, c.a);
    pq_st(&D.ctl->step.b, c.b);
    pq_st(&D.ctl->step.o, c.o);
    pq_st(&D.ctl->step.target, c.target);
    pq_st(&D.ctl->step.rel1, c.rel1);
    pq_st(&D.ctl->step.rel2, c.rel2);
    pq_st(&D.ctl->step.heap_n, c.heap_n);
    pq_st(&D.ctl->step.n_nodes, c.n_nodes);
    pq_st(&D.ctl->step.slot_top, c.slot_top);
    pq_st(&D.ctl->done, 0u);
  }
  if (threadIdx.x < (unsigned)kPQGroups) {
    pq_st(&D.ctl->grp[threadIdx.x].size, 0ull);
    pq_st(&D.ctl->grp[threadIdx.x].done, 0u);
  }
}

// The root of the queue as the result: priorityqueue_or repairs it
// (RoaringBitmap.repairAfterLazy, RB/RoaringBitmap.java:2752-2757: A kept, R
// toEfficientContainer, a lazy bitmap BY_CARD with 65536 -> RunContainer.full, an exact
// bitmap kept); priorityqueue_xor returns it as is.
__global__ __launch_bounds__(256) void k_pq_final(const Task* __restrict__ tasks, const uint32_t* __restrict__ n_tasks,
                                                  PQArgs A, int repair, PQDev D, OutCtx oc) {
  __shared__ __align__(16) uint32_t acc[2048];
  __shared__ __align__(16) uint32_t tmp[2048];
  __shared__ int q[257];
  __shared__ int sh[8];
  __shared__ Prefix shp;
  const int root = D.ctl->step.a;
  const uint32_t nt = *n_tasks;
  for (uint32_t t = blockIdx.x; t < nt; t += gridDim.x) {
    __syncthreads();
    const Task tk = tasks[t];
    uint32_t pos[2];
    leaf_find2(A.bm, (uint32_t)tk.a, (uint32_t)tk.b, root, -1, pos);
    const PQNode x = pq_load(root, pos[0], D, A, t, (uint32_t)tk.a, (uint32_t)tk.b);
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
      pq_materialize(x, D, A, tmp, q, r);
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

void launch_pq_step(hipStream_t s, int grid, const Task* tasks, const uint32_t* nt, PQArgs args, PQDev D) {
  grid = std::max(1, std::min(grid, resident_grid((const void*)&k_pq_step)));
  hipLaunchKernelGGL(k_pq_step, dim3(grid), dim3(256), 0, s, tasks, nt, args, D);
}

void launch_pq_final(hipStream_t s, int grid, const Task* tasks, const uint32_t* nt, PQArgs args, int repair,
                     PQDev D, OutCtx oc) {
  grid = std::max(1, std::min(grid, resident_grid((const void*)&k_pq_final)));
  hipLaunchKernelGGL(k_pq_final, dim3(grid), dim3(256), 0, s, tasks, nt, args, repair, D, oc);
}

}  // namespace rbg
