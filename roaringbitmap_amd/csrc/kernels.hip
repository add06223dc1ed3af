// HIP kernels of the MI355X Roaring engine (gfx950).  RB/ = reference
// RoaringBitmap/src/main/java/org/roaringbitmap/.
//
// Every op runs as one pipeline on the context stream, with no host sync:
//   plan    : per-key (65536 threads) decide whether key k produces a task
//   compact : one workgroup scans the per-key flags into a dense task list
//   compute : one 256-thread workgroup per task computes the result container
//             in registers/LDS and writes it to a fixed 8208 B scratch slot
//   finalize: one workgroup scans the kept outputs, writes the header prefix
//   emit    : descriptors, offset table and payload copies into the
//             portable-format output buffer
#include "kernels.hpp"

namespace rbg {

// ===========================================================================
// plan / compact
// ===========================================================================
__device__ __forceinline__ int lower_bound_u16(const uint16_t* keys, int n, uint32_t k) {
  int lo = 0, hi = n;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (keys[mid] < k) lo = mid + 1;
    else hi = mid;
  }
  return lo;
}

// Key alignment of two sorted key arrays (RoaringArray.advanceUntil walk of
// RB/RoaringBitmap.java:382-400, :864-896, :1076-1113, :449-471), one thread per key.
__global__ __launch_bounds__(256) void k_plan_pairwise(int op, const uint16_t* __restrict__ ka, int na,
                                                       const uint16_t* __restrict__ kb, int nb,
                                                       Task* __restrict__ by_key, uint8_t* __restrict__ flag) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= 65536) return;
  const int pa = lower_bound_u16(ka, na, k);
  const int pb = lower_bound_u16(kb, nb, k);
  const int ia = (pa < na && ka[pa] == k) ? pa : -1;
  const int ib = (pb < nb && kb[pb] == k) ? pb : -1;
  int f;
  switch (op) {
    case OP_OR:
    case OP_XOR: f = (ia >= 0) || (ib >= 0); break;
    case OP_ANDNOT: f = ia >= 0; break;
    default: f = (ia >= 0) && (ib >= 0); break;  // AND and every cardinality op
  }
  flag[k] = (uint8_t)f;
  by_key[k] = Task{k, ia, ib, 0};
}

// Wide plan from the key-major CSR: n_k = key_off[k+1] - key_off[k].
// mode 0: n_k > 0 (or / xor / orCardinality); mode 1: n_k == n_req (and).
__global__ __launch_bounds__(256) void k_plan_wide(int mode, const uint32_t* __restrict__ key_off,
                                                   uint32_t n_req, int key_lo, int key_hi,
                                                   Task* __restrict__ by_key, uint8_t* __restrict__ flag) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k >= 65536) return;
  const uint32_t s = key_off[k], n = key_off[k + 1] - s;
  int f = (mode == 0) ? (n > 0) : (n == n_req && n > 0);
  if ((int)k < key_lo || (int)k >= key_hi) f = 0;
  flag[k] = (uint8_t)f;
  by_key[k] = Task{k, (int32_t)s, (int32_t)n, 0};
}

// One 1024-thread workgroup compacts 65536 flags (64 per thread, in key order).
__global__ __launch_bounds__(1024) void k_compact(const uint8_t* __restrict__ flag, const Task* __restrict__ by_key,
                                                  Task* __restrict__ tasks, uint32_t* __restrict__ n_tasks) {
  __shared__ int wsum[16];
  const int t = threadIdx.x;
  const uint4* f4 = reinterpret_cast<const uint4*>(flag + 64 * t);
  uint4 f[4] = {f4[0], f4[1], f4[2], f4[3]};
  const uint8_t* fb = reinterpret_cast<const uint8_t*>(f);
  int cnt = 0;
#pragma unroll
  for (int i = 0; i < 64; i++) cnt += fb[i];
  // block exclusive scan of cnt
  const int lane = t & 63, w = t >> 6;
  const int inc = wave_incl_scan(cnt);
  if (lane == 63) wsum[w] = inc;
  __syncthreads();
  int off = 0, tot = 0;
  for (int i = 0; i < 16; i++) {
    if (i < w) off += wsum[i];
    tot += wsum[i];
  }
  int p = off + inc - cnt;
  for (int i = 0; i < 64; i++)
    if (fb[i]) tasks[p++] = by_key[64 * t + i];
  if (t == 0) *n_tasks = (uint32_t)tot;
}

// ===========================================================================
// pairwise compute
// ===========================================================================
// Result container type of the static pairwise ops, as a function of the
// operand kinds and the result's cardinality c and run count r (DESIGN.md
// §Type contract; derived from RB/{Array,Bitmap,Run}Container.java):
//   AND   : R&R -> EFF(c,r) (RB/RunContainer.java:381-456); else BY_CARD(c)
//   OR    : A|R, R|A, R|R -> EFF(c,r) (:1926-1986); A|A -> BY_CARD(c)
//           (RB/ArrayContainer.java:949-963); B|x, x|B -> c==65536 ? R.full : B
//           (RB/BitmapContainer.java:1064-1096, RB/RunContainer.java:1932-1949)
//   XOR   : R^R -> EFF; R^A, A^R with |A| < 32 -> EFF (RB/RunContainer.java:2410-2424);
//           else BY_CARD (RB/BitmapContainer.java:1372-1408)
//   ANDNOT: R\R -> EFF (:637-692); R\A with |A| < 32 -> EFF (:574-591); else BY_CARD
__device__ __forceinline__ bool pairwise_needs_runs(int op, int ka, int ca, int kb, int cb) {
  switch (op) {
    case OP_AND: return ka == DK_R && kb == DK_R;
    case OP_OR: return (ka == DK_R && kb != DK_B) || (kb == DK_R && ka != DK_B);
    case OP_XOR:
      return (ka == DK_R && kb == DK_R) || (ka == DK_R && kb == DK_A && cb < 32) ||
             (kb == DK_R && ka == DK_A && ca < 32);
    default:  // ANDNOT
      return ka == DK_R && (kb == DK_R || (kb == DK_A && cb < 32));
  }
}
__device__ __forceinline__ int pairwise_kind(int op, int ka, int kb, bool use_eff, int c, int r) {
  if (use_eff) return eff(c, r);
  if (op == OP_OR && (ka == DK_B || kb == DK_B)) return c == 65536 ? DK_R : DK_B;
  return by_card(c);
}

template <int OP>
__device__ __forceinline__ uint64_t apply_op(uint64_t x, uint64_t y) {
  if (OP == OP_AND) return x & y;
  if (OP == OP_OR) return x | y;
  if (OP == OP_XOR) return x ^ y;
  return x & ~y;
}

struct OperandView {
  const CDesc* desc;
  const uint8_t* payload;
};

__device__ __forceinline__ void passthrough(const CDesc& d, const uint8_t* payload, ODesc* o) {
  ODesc r;
  r.src = reinterpret_cast<uint64_t>(payload + d.slot + (d.kind == DK_R ? 2 : 0));
  r.card = d.card;
  r.key = d.key;
  r.kind = d.kind;
  r.keep = 1;
  if (d.kind == DK_A) r.ser_len = 2 * d.card;
  else if (d.kind == DK_B) r.ser_len = 8192;
  else r.ser_len = 2 + 4 * (uint32_t)(*reinterpret_cast<const uint16_t*>(payload + d.slot + 2));
  r.pad0 = 0;
  r.pad1 = 0;
  *o = r;
}

// MODE 0: materialise results.  MODE 1: cardinality only (task_card[t]).
template <int OP, int MODE>
__global__ __launch_bounds__(256) void k_pairwise(const Task* __restrict__ tasks, const uint32_t* __restrict__ n_tasks,
                                                  OperandView A, OperandView B, ODesc* __restrict__ out,
                                                  uint8_t* __restrict__ scratch, uint32_t* __restrict__ task_card) {
  __shared__ __align__(16) uint32_t lds_a[2048];
  __shared__ __align__(16) uint32_t lds_b[2048];
  __shared__ int q[257];
  __shared__ int sh[8];
  const uint32_t nt = *n_tasks;
  for (uint32_t t = blockIdx.x; t < nt; t += gridDim.x) {
    const Task tk = tasks[t];
    if (tk.a < 0 || tk.b < 0) {  // unmatched key: clone (appendCopy), RB/RoaringArray.java:184-205
      if (MODE == 0 && threadIdx.x == 0) {
        if (tk.a >= 0) passthrough(A.desc[tk.a], A.payload, out + t);
        else passthrough(B.desc[tk.b], B.payload, out + t);
      }
      continue;
    }
    const CDesc da = A.desc[tk.a];
    const CDesc db = B.desc[tk.b];
    uint64_t x[4], y[4];
    materialize(da, A.payload, lds_a, q, x);
    materialize(db, B.payload, lds_b, q, y);
    uint64_t r[4];
#pragma unroll
    for (int i = 0; i < 4; i++) r[i] = apply_op<OP>(x[i], y[i]);
    int c = popc64(r[0]) + popc64(r[1]) + popc64(r[2]) + popc64(r[3]);
    int unused = 0;
    block_sum2(c, unused, sh);
    if (MODE == 1) {
      if (threadIdx.x == 0) task_card[t] = (uint32_t)c;
      continue;
    }
    if (c == 0) {  // empty results are dropped (RB/RoaringBitmap.java:389,456,1084)
      if (threadIdx.x == 0) {
        ODesc o = {};
        o.keep = 0;
        out[t] = o;
      }
      continue;
    }
    const bool use_eff = pairwise_needs_runs(OP, da.kind, (int)da.card, db.kind, (int)db.card);
    const int nr = use_eff ? count_runs(r, lds_a, sh) : 0;
    const int kind = pairwise_kind(OP, da.kind, db.kind, use_eff, c, nr);
    uint8_t* slot = scratch + (size_t)t * kSlotBytes;
    uint64_t src;
    uint32_t len;
    emit_container(kind, r, c, slot, lds_a, lds_b, sh, &src, &len);
    if (threadIdx.x == 0) {
      ODesc o;
      o.src = src;
      o.ser_len = len;
      o.card = (uint32_t)c;
      o.key = (uint16_t)tk.key;
      o.kind = (uint8_t)kind;
      o.keep = 1;
      o.pad0 = 0;
      o.pad1 = 0;
      out[t] = o;
    }
  }
}

// ===========================================================================
// finalize / emit (portable format, RB/RoaringArray.java:896-940)
// ===========================================================================
__global__ __launch_bounds__(1024) void k_finalize(const ODesc* __restrict__ out, const uint32_t* __restrict__ n_tasks,
                                                   uint32_t* __restrict__ out_idx, uint64_t* __restrict__ out_off,
                                                   ResultInfo* __restrict__ info, uint8_t* __restrict__ buf) {
  __shared__ uint32_t runflags[2048];  // 65536 bits
  __shared__ int wsum[16];
  __shared__ unsigned long long wbytes[16];
  __shared__ int wrun[16];
  __shared__ unsigned long long wcard[16];
  const int t = threadIdx.x;
  const uint32_t nt = *n_tasks;
  for (int i = t; i < 2048; i += 1024) runflags[i] = 0;
  // each thread handles 64 consecutive tasks
  const uint32_t t0 = 64u * t;
  int cnt = 0, run = 0;
  unsigned long long bytes = 0, card = 0;
  for (uint32_t i = t0; i < t0 + 64 && i < nt; i++) {
    const ODesc o = out[i];
    if (o.keep) {
      cnt++;
      bytes += o.ser_len;
      card += o.card;
      run |= (o.kind == DK_R);
    }
  }
  const int lane = t & 63, w = t >> 6;
  const int inc = wave_incl_scan(cnt);
  // 64-bit byte scan inside the wave
  unsigned long long binc = bytes;
  for (int o = 1; o < 64; o <<= 1) {
    unsigned long long u = __shfl_up(binc, o, 64);
    if (lane >= o) binc += u;
  }
  unsigned long long csum = card;
  for (int o = 32; o > 0; o >>= 1) csum += __shfl_xor(csum, o, 64);
  int rany = __any(run) ? 1 : 0;
  if (lane == 63) {
    wsum[w] = inc;
    wbytes[w] = binc;
  }
  if (lane == 0) {
    wrun[w] = rany;
    wcard[w] = csum;
  }
  __syncthreads();
  int off = 0, tot = 0, has_run = 0;
  unsigned long long boff = 0, btot = 0, ctot = 0;
  for (int i = 0; i < 16; i++) {
    if (i < w) {
      off += wsum[i];
      boff += wbytes[i];
    }
    tot += wsum[i];
    btot += wbytes[i];
    has_run |= wrun[i];
    ctot += wcard[i];
  }
  int p = off + inc - cnt;
  unsigned long long bp = boff + binc - bytes;
  for (uint32_t i = t0; i < t0 + 64 && i < nt; i++) {
    const ODesc o = out[i];
    if (o.keep) {
      out_idx[i] = (uint32_t)p;
      out_off[i] = bp;
      if (o.kind == DK_R) atomicOr(&runflags[p >> 5], 1u << (p & 31));
      p++;
      bp += o.ser_len;
    } else {
      out_idx[i] = 0xFFFFFFFFu;
    }
  }
  __syncthreads();
  const uint32_t size = (uint32_t)tot;
  uint64_t header;
  if (has_run) header = (size < 4) ? 4 + (size + 7) / 8 + 4 * (uint64_t)size : 4 + (size + 7) / 8 + 8 * (uint64_t)size;
  else header = 8 + 8 * (uint64_t)size;
  if (t == 0) {
    ResultInfo r;
    r.n_out = size;
    r.has_run = (uint32_t)has_run;
    r.header = header;
    r.payload = btot;
    r.total = header + btot;
    r.long_card = (int64_t)ctot;
    r.card32 = (uint32_t)ctot;
    r.any = size > 0;
    *info = r;
    // cookie (+ size)
    uint32_t* b32 = reinterpret_cast<uint32_t*>(buf);
    if (has_run) {
      b32[0] = 12347u | ((size - 1) << 16);
    } else {
      b32[0] = 12346u;
      b32[1] = size;
    }
  }
  if (has_run) {
    const uint32_t nflag = (size + 7) / 8;
    const uint8_t* rf = reinterpret_cast<const uint8_t*>(runflags);
    for (uint32_t i = t; i < nflag; i += 1024) buf[4 + i] = rf[i];
  }
}

// Writes descriptors, offsets and payloads; one workgroup per task (grid-stride).
__global__ __launch_bounds__(256) void k_emit(const ODesc* __restrict__ out, const uint32_t* __restrict__ n_tasks,
                                              const uint32_t* __restrict__ out_idx, const uint64_t* __restrict__ out_off,
                                              const ResultInfo* __restrict__ info, uint8_t* __restrict__ buf) {
  const uint32_t nt = *n_tasks;
  const ResultInfo ri = *info;
  const uint32_t size = ri.n_out;
  const uint64_t desc_base = ri.has_run ? 4 + (size + 7) / 8 : 8;
  const bool offsets = !ri.has_run || size >= 4;
  const uint64_t off_base = desc_base + 4ull * size;
  for (uint32_t i = blockIdx.x; i < nt; i += gridDim.x) {
    const uint32_t idx = out_idx[i];
    if (idx == 0xFFFFFFFFu) continue;
    const ODesc o = out[i];
    const uint64_t poff = ri.header + out_off[i];
    if (threadIdx.x < 4) {
      const uint32_t d = (uint32_t)o.key | ((o.card - 1) << 16);
      buf[desc_base + 4ull * idx + threadIdx.x] = (uint8_t)(d >> (8 * threadIdx.x));
    } else if (offsets && threadIdx.x < 8) {
      const int b = threadIdx.x - 4;
      buf[off_base + 4ull * idx + b] = (uint8_t)((uint32_t)poff >> (8 * b));
    }
    group_copy<NT>(buf + poff, reinterpret_cast<const uint8_t*>(o.src), o.ser_len, threadIdx.x);
  }
}

// Java-int sum of task cardinalities (mod 2^32) plus "any nonzero" for intersects.
__global__ __launch_bounds__(1024) void k_reduce_card(const uint32_t* __restrict__ task_card,
                                                      const uint32_t* __restrict__ n_tasks, ResultInfo* __restrict__ info) {
  __shared__ unsigned long long ws[16];
  __shared__ int wa[16];
  const uint32_t nt = *n_tasks;
  unsigned long long s = 0;
  int any = 0;
  for (uint32_t i = threadIdx.x; i < nt; i += 1024) {
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
    *info = r;
  }
}

// ===========================================================================
// ingest: raw serialized buffers -> slotted payload arena (one wave per container)
// ===========================================================================
__global__ __launch_bounds__(256) void k_ingest(const uint8_t* __restrict__ raw, const IngestItem* __restrict__ items,
                                                uint64_t n_items, uint8_t* __restrict__ payload) {
  const int lane = threadIdx.x & 63;
  const uint64_t wave = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
  const uint64_t nw = (uint64_t)gridDim.x * 4;
  for (uint64_t i = wave; i < n_items; i += nw) {
    const IngestItem it = items[i];
    uint8_t* dst = payload + it.dst + (it.kind == DK_R ? 2 : 0);
    group_copy<64>(dst, raw + it.src, it.len, lane);
  }
}

// ===========================================================================
// host launchers
// ===========================================================================
void launch_plan_pairwise(hipStream_t s, int op, const uint16_t* ka, int na, const uint16_t* kb, int nb, Task* by_key,
                          uint8_t* flag) {
  hipLaunchKernelGGL(k_plan_pairwise, dim3(256), dim3(256), 0, s, op, ka, na, kb, nb, by_key, flag);
}
void launch_plan_wide(hipStream_t s, int mode, const uint32_t* key_off, uint32_t n_req, int key_lo, int key_hi,
                      Task* by_key, uint8_t* flag) {
  hipLaunchKernelGGL(k_plan_wide, dim3(256), dim3(256), 0, s, mode, key_off, n_req, key_lo, key_hi, by_key, flag);
}
void launch_compact(hipStream_t s, const uint8_t* flag, const Task* by_key, Task* tasks, uint32_t* n_tasks) {
  hipLaunchKernelGGL(k_compact, dim3(1), dim3(1024), 0, s, flag, by_key, tasks, n_tasks);
}

template <int OP>
static void launch_pw(hipStream_t s, int mode, int grid, const Task* tasks, const uint32_t* nt, const CDesc* da,
                      const uint8_t* pa, const CDesc* db, const uint8_t* pb, ODesc* out, uint8_t* scratch,
                      uint32_t* task_card) {
  OperandView A{da, pa}, B{db, pb};
  if (mode == 0)
    hipLaunchKernelGGL((k_pairwise<OP, 0>), dim3(grid), dim3(256), 0, s, tasks, nt, A, B, out, scratch, task_card);
  else
    hipLaunchKernelGGL((k_pairwise<OP, 1>), dim3(grid), dim3(256), 0, s, tasks, nt, A, B, out, scratch, task_card);
}

void launch_pairwise(hipStream_t s, int op, int mode, int grid, const Task* tasks, const uint32_t* nt, const CDesc* da,
                     const uint8_t* pa, const CDesc* db, const uint8_t* pb, ODesc* out, uint8_t* scratch,
                     uint32_t* task_card) {
  switch (op) {
    case OP_AND: launch_pw<OP_AND>(s, mode, grid, tasks, nt, da, pa, db, pb, out, scratch, task_card); break;
    case OP_OR: launch_pw<OP_OR>(s, mode, grid, tasks, nt, da, pa, db, pb, out, scratch, task_card); break;
    case OP_XOR: launch_pw<OP_XOR>(s, mode, grid, tasks, nt, da, pa, db, pb, out, scratch, task_card); break;
    default: launch_pw<OP_ANDNOT>(s, mode, grid, tasks, nt, da, pa, db, pb, out, scratch, task_card); break;
  }
}

void launch_finalize(hipStream_t s, const ODesc* out, const uint32_t* nt, uint32_t* out_idx, uint64_t* out_off,
                     ResultInfo* info, uint8_t* buf) {
  hipLaunchKernelGGL(k_finalize, dim3(1), dim3(1024), 0, s, out, nt, out_idx, out_off, info, buf);
}
void launch_emit(hipStream_t s, int grid, const ODesc* out, const uint32_t* nt, const uint32_t* out_idx,
                 const uint64_t* out_off, const ResultInfo* info, uint8_t* buf) {
  hipLaunchKernelGGL(k_emit, dim3(grid), dim3(256), 0, s, out, nt, out_idx, out_off, info, buf);
}
void launch_reduce_card(hipStream_t s, const uint32_t* task_card, const uint32_t* nt, ResultInfo* info) {
  hipLaunchKernelGGL(k_reduce_card, dim3(1), dim3(1024), 0, s, task_card, nt, info);
}
void launch_ingest(hipStream_t s, const uint8_t* raw, const IngestItem* items, uint64_t n, uint8_t* payload) {
  uint64_t g = (n + 3) / 4;
  if (g > 8192) g = 8192;
  if (g == 0) return;
  hipLaunchKernelGGL(k_ingest, dim3((unsigned)g), dim3(256), 0, s, raw, items, n, payload);
}

}  // namespace rbg
