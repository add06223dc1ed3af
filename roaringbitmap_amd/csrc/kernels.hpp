// Kernel launch interface of the engine (host side <-> kernels.hip / wide.hip).
#pragma once
#include <hip/hip_runtime.h>

#include "device.hpp"

namespace rbg {

enum OpCode : int { OP_AND = 0, OP_OR = 1, OP_XOR = 2, OP_ANDNOT = 3 };

// wide-op flavours (wide.hip)
enum WideMode : int {
  WIDE_OR = 0,         // FastAggregation.naive_or
  WIDE_OR_CARD = 1,    // horizontalOrCardinality
  WIDE_XOR = 2,        // naive_xor
  WIDE_AND_SHY = 3,    // workShyAnd
  WIDE_AND_SHY_CARD = 4,  // workShyAndCardinality
  WIDE_AND_NAIVE = 5,  // naive_and chain (WideArgs::buffer: BufferFastAggregation's)
  WIDE_LAZY_CHAIN = 6,  // lazyIOR chain + repairAfterLazy: ParallelAggregation.or, BufferFastAggregation.or(Mutable...),
                        // horizontal_or
  WIDE_XOR_CHAIN = 7,   // clone + ixor chain without restart: ParallelAggregation.xor, horizontal_xor
};

// WideArgs::chain flags
constexpr uint32_t kChainLimit16 = 1;  // ParallelAggregation.or: 16+ containers per key take the lazy-bitmap branch
constexpr uint32_t kChainN1Clone = 2;  // a key of one container is a plain clone (no repairAfterLazy)
constexpr uint32_t kChainKeepEmpty = 4;  // horizontal_xor appends empty results

struct WideArgs {
  const CDesc* desc;      // key-major container table
  const uint32_t* bm;     // input bitmap index per container
  const uint8_t* payload; // arena
  const uint8_t* skip;    // naive_and: per input bitmap, 1 = skip (identity with the start)
  uint32_t start_bm;      // naive_and: input bitmap the chain starts from
  uint32_t all_array;     // every container is an array: a key segment is one contiguous u16 value stream
  uint32_t slot32;        // every slot offset / 16 fits 32 bits (payload < 64 GiB)
  const uint32_t* order;  // chain modes: container index at chain position j of a key segment (null: input order)
  uint32_t chain;         // chain modes: kChain* flags
  unsigned long long* rd_bytes;  // workShyAnd: payload + 4 B per container it read, summed (null: not counted)
  uint32_t buffer;        // naive_and: the buffer package's chain (MappeableRunContainer.iand(R) keeps the merged runs)
  BigRuns big;            // naive_and (buffer): results of more than 2047 runs
};

// priority-queue aggregations (pq.hip): the size-ordered queue runs on the device.  Each
// step launch combines two nodes (an input bitmap of the batch, or an intermediate temp)
// over every union key; the launch's last workgroup folds the result size into the
// queue and writes the next step, so the host only enqueues N - 1 launches.
//   PQ_XOR  RoaringBitmap.xor(x1, x2)                 (priorityqueue_xor)
//   PQ_LOR  RoaringBitmap.lazyor(x1, x2), static      (priorityqueue_or, two inputs)
//   PQ_LIOR x1.lazyor(x2), in place on the temp x1    (one temp)
//   PQ_LFL  RoaringBitmap.lazyorfromlazyinputs(x1, x2) (two temps)
enum PQOp : int { PQ_XOR = 0, PQ_LOR = 1, PQ_LIOR = 2, PQ_LFL = 3 };
// container kinds of a node: DK_A / DK_B (exact) / DK_R, and a lazy bitmap (card -1 in the reference)
enum PQKind : int { PK_A = 0, PK_BE = 1, PK_R = 2, PK_BL = 3 };
struct __align__(16) PQState {  // per key of a temp
  uint32_t card;
  uint16_t nruns;
  uint8_t kind;     // PQKind
  uint8_t present;  // the temp holds this key
  int32_t src;      // >= 0: an unchanged clone of this input container (desc index)
  int32_t blk;      // else: the 8 KiB block of the set arena holding the container
};
// A queue entry: the node's getLongSizeInBytes is fixed while it is queued.
struct PQEnt {
  int64_t size;
  int32_t node;
  int32_t pad;
};
// The step the next launch runs, and the queue's scalar state.  Node references:
// >= 0 input bitmap of the batch, < 0 temp slot -1 - ref.
struct PQStep {
  int32_t op, final_step, a, b, o;
  int32_t target;      // node index whose size the step's result gives
  int32_t rel1, rel2;  // temp slots freed after the step (-1: none)
  int32_t heap_n, n_nodes, slot_top, or_mode;
};
// A step's workgroups report in kPQGroups groups (blockIdx % kPQGroups), each counter and
// size word in a cache line of its own: one contended address serialises its atomics
// (~12 ns each), so a launch of G workgroups pays G / kPQGroups of them on the longest chain.
constexpr int kPQGroups = 8;
struct __align__(128) PQLine {
  uint32_t done;  // workgroups of the group finished in the running step
  uint32_t pad;
  unsigned long long size;  // the group's share of the step's result size
  uint8_t pad2[112];
};
struct PQCtl {
  PQStep step;
  uint32_t done;  // groups finished in the running step
  uint32_t err;   // a key's block pool ran out (cannot happen: see ctx_pq)
  uint8_t pad[72];
  PQLine grp[kPQGroups];
};
struct PQDev {
  PQCtl* ctl;
  PQEnt* heap;        // java.util.PriorityQueue array order
  int32_t* node;      // node index -> reference
  uint8_t* istmp;     // priorityqueue_or: node holds a temp
  int32_t* slots;     // free temp slots (stack)
  PQState* states;    // temp slot s: states[s * stride + task]
  uint64_t stride;
  uint64_t* arena;    // 8 KiB blocks (1024 words)
  // Per key, a private pool of arena blocks: the free blocks of key t are
  // kstack[kbase[t] .. kbase[t] + ktop[t]).  Only the workgroup of key t touches them.
  int32_t* kstack;
  const uint32_t* kbase;
  int32_t* ktop;
};
struct PQArgs {
  const CDesc* desc;
  const uint32_t* bm;
  const uint8_t* payload;
};

// The queue (RB/FastAggregation.java:758-781 / :799-811) after the host has added every
// input: pq_finish folds a step's result size in, pq_plan polls the next pair.  M gives
// the heap operations and node table: sequential on the host (the first step), a wave of
// the scheduling workgroup on the device.
template <class M>
__host__ __device__ inline void pq_finish(M& m, PQStep& c, int64_t size) {
  m.add(c, PQEnt{size, c.target, 0});
  if (c.rel1 >= 0) m.slot_push(c, c.rel1);
  if (c.rel2 >= 0) m.slot_push(c, c.rel2);
}
template <class M>
__host__ __device__ inline void pq_plan(M& m, PQStep& c) {
  if (c.heap_n <= 1) {
    c.final_step = 1;
    c.a = c.heap_n ? m.node(m.poll(c).node) : 0;
    return;
  }
  const int x1 = m.poll(c).node;
  const int x2 = m.poll(c).node;
  c.rel1 = c.rel2 = -1;
  if (c.or_mode) {
    const bool t1 = m.istmp(x1), t2 = m.istmp(x2);
    if (t1 && t2) {  // lazyorfromlazyinputs(buffer[x1], buffer[x2]) into x1's temp
      c.op = PQ_LFL;
      c.a = m.node(x1);
      c.b = m.node(x2);
      c.o = c.a;
      c.target = x1;
      c.rel1 = -1 - c.b;
    } else if (t2) {  // buffer[x2].lazyor(buffer[x1])
      c.op = PQ_LIOR;
      c.a = m.node(x2);
      c.b = m.node(x1);
      c.o = c.a;
      c.target = x2;
    } else if (t1) {  // buffer[x1].lazyor(buffer[x2])
      c.op = PQ_LIOR;
      c.a = m.node(x1);
      c.b = m.node(x2);
      c.o = c.a;
      c.target = x1;
    } else {  // RoaringBitmap.lazyor(buffer[x1], buffer[x2]) into a new temp
      c.op = PQ_LOR;
      c.a = m.node(x1);
      c.b = m.node(x2);
      c.o = -1 - m.slot_pop(c);
      m.set_node(x1, c.o);
      m.set_istmp(x1);
      c.target = x1;
    }
  } else {  // pq.add(RoaringBitmap.xor(x1, x2))
    c.op = PQ_XOR;
    c.a = m.node(x1);
    c.b = m.node(x2);
    c.o = -1 - m.slot_pop(c);
    c.target = c.n_nodes++;
    m.set_node(c.target, c.o);
    if (c.a < 0) c.rel1 = -1 - c.a;
    if (c.b < 0) c.rel2 = -1 - c.b;
  }
}
// java.util.PriorityQueue's comparator over getLongSizeInBytes: (int)(sizes[a] - sizes[b])
__host__ __device__ inline int pq_cmp(int64_t a, int64_t b) { return (int)(int32_t)(uint32_t)(uint64_t)(a - b); }

// sizes[bm] += 2 + getSizeInBytes over the batch's containers (sizes zeroed by the caller)
void launch_pq_leaf_sizes(hipStream_t s, const CDesc* desc, const uint32_t* bm, const uint8_t* payload, uint64_t n,
                          unsigned long long* sizes);
// one step of the queue (the step record in D.ctl), then the next step's plan
void launch_pq_step(hipStream_t s, int grid, const Task* tasks, const uint32_t* nt, PQArgs args, PQDev D);
// the root node as the op's result records (repair: priorityqueue_or's repairAfterLazy)
void launch_pq_final(hipStream_t s, int grid, const Task* tasks, const uint32_t* nt, PQArgs args, int repair,
                     PQDev D, OutCtx oc);

// bit-sliced index (bsi.hip); ops in the order of BitmapSliceIndex.Operation
// (bsi/src/main/java/org/roaringbitmap/bsi/BitmapSliceIndex.java:23-38)
// BSI_ALL: compareUsingMinMax's "all" (BSI/:516: ebM, or and(ebM, foundSet));
// BSI_SUM_ONLY: sum(foundSet) alone
enum BsiOp : int { BSI_EQ = 0, BSI_NEQ = 1, BSI_LE = 2, BSI_LT = 3, BSI_GE = 4, BSI_GT = 5, BSI_RANGE = 6,
                   BSI_ALL = 7, BSI_SUM_ONLY = 8 };
constexpr int kBsiMaxInputs = 34;  // ebM + up to 32 slices + foundSet
// BSI sum words (u64): per-slice |bA[x] & found| at [x], the found count at [kBsiMaxInputs],
// then sum(found) = (sum, count) as Java longs at [kBsiSumOut], [kBsiSumOut + 1]
constexpr int kBsiSumOut = kBsiMaxInputs + 1;
constexpr int kBsiSumWords = kBsiSumOut + 2;
// k_bsi_types adds its per-block sums into one of kBsiSumReps replicas of 64 words after
// those (block b: replica b % kBsiSumReps), so no sum word takes more than a few dozen
// atomics; k_bsi_sum_final adds the replicas.  All of it is zeroed by the plan kernel.
constexpr int kBsiSumReps = 16;
constexpr int kBsiSumAll = kBsiSumWords + 64 * kBsiSumReps;
constexpr int kOwenOrder = 64;  // bytes per task of an owenGreatEqual chain order
struct BsiArgs {
  int op;         // BsiOp
  int nbits;      // slices
  int has_found;  // input nbits+1 is the foundSet
  uint32_t pred0;  // predicate (RANGE: start)
  uint32_t pred1;  // RANGE: end
  // buffer package (bsi/.../bsi/buffer/BitSliceIndexBase.java): its own compare circuit and
  // ImmutableRoaringBitmap's pairwise types (bsi.hip, "Buffer-package BSI")
  int buffer;
  int found_input;      // input index of the found set (nbits + 1 of the batch; the buffer kernel may run
                        // with nbits = 0 over the same batch)
  uint32_t owen_zeros;  // GE / RANGE: slice positions of owenGreatEqual's orInputs (0 bits of start - 1)
  uint32_t owen_ones;   //   and of its spine ANDs (1 bits), both within [leastSignifZero, nbits)
  const uint8_t* owen_order;  // per task kOwenOrder bytes: [0] = n, [1 + k] = orInput of chain position k
                              // (the horizontal_or queue's poll order); null: top-down order
  void* owen_tb;              // per task 32 x 16 B: each orInput's (kind, card, src) (k_bsi_owen_pre)
  uint32_t* task_keys;        // k_bsi_owen_pre: key of each task
  BigRuns big;
};

// Workgroups of `kernel` (256 threads) that are resident on the whole device at
// once: CUs x occupancy.  Task kernels launch at most this many workgroups and
// stride over their tasks, so no workgroup waits for a dispatch slot and no
// wave pays a launch per task (cached per kernel).
int resident_grid(const void* kernel, int block = 256);  // workgroups of `block` threads resident at once

// plan kernels also zero the op's look-back header (zlb, 32 u64) and tile statuses (ztile, 128 u64)
void launch_plan_wide(hipStream_t s, int mode, const uint32_t* key_off, uint32_t n_req, int key_lo, int key_hi,
                      Task* by_key, uint8_t* flag, uint32_t* wg_count, uint64_t* zlb, uint64_t* ztile);
void launch_compact(hipStream_t s, const uint8_t* flag, const Task* by_key, const uint32_t* wg_count, Task* tasks,
                    uint32_t* n_tasks);
// pairwise.hip: plan (key alignment + descriptor resolution) and the wave-per-key compute
// plan + compaction in one launch: tasks[] in key order, *n_tasks.  wg_epoch: 256 u64
// (zeroed once per context), epoch: unique per op of the context; only keys in [key_lo, key_hi).
void launch_plan_pairwise(hipStream_t s, int op, int key_lo, int key_hi, const uint32_t* koa, const CDesc* da,
                          const uint8_t* pa, const uint32_t* kob, const CDesc* db, const uint8_t* pb,
                          uint64_t* wg_epoch, uint32_t epoch, PTask* tasks, uint32_t* n_tasks, uint64_t* zlb,
                          uint64_t* ztile, uint32_t* err);
// mode 0: materialise results (task slots + records); mode 1: andCardinality into task_card
// Direct mode of the pairwise compute kernel (no plan launch): task t = key key_lo + t over
// nkeys keys, resolved by the kernel through both operands' key CSR; it also writes the task
// count (n_tasks_out) and zeroes the op's look-back state (zlb, ztile), as the plan would.
struct PwDirect {
  const uint32_t* koa;
  const CDesc* da;
  const uint32_t* kob;
  const CDesc* db;
  int key_lo;
  uint32_t nkeys;
  uint32_t* n_tasks_out;
  uint64_t* zlb;
  uint64_t* ztile;
  uint32_t n_tasks_write;  // the task count block 0 writes to n_tasks_out (a pipelined op's total over its ranges)
};
// direct: null = tasks / nt from launch_plan_pairwise; balanced (with direct): tasks / nt[0..1] from
// launch_plan_balanced, records at key positions (direct->key_lo)
// balanced: k_plan_balanced's list (dense ranges), run by k_pair_cu (one 16-wave workgroup per CU, tasks
// claimed from the CU's share)
void launch_pairwise(hipStream_t s, int op, int mode, int grid, const PTask* tasks, const uint32_t* nt,
                     const uint8_t* pa, const uint8_t* pb, OutCtx oc, uint32_t* task_card, const PwDirect* direct,
                     bool balanced = false);
// dense key ranges: every key's task resolved and ordered by estimated cost within its 256-key segment
// (heaviest first, rotated by the segment index) into tasks[]; n_tasks[0] = n_tasks[1] = nkeys (records
// and list positions, one per key: keys without a task are marked, with an empty record / a zero count)
void launch_plan_balanced(hipStream_t s, int op, int mode, int key_lo, uint32_t nkeys, const uint32_t* koa,
                          const CDesc* da, const uint8_t* pa, const uint32_t* kob, const CDesc* db, const uint8_t* pb,
                          PTask* tasks, uint32_t* n_tasks, OutCtx oc, uint32_t* task_card, uint64_t* zlb,
                          uint64_t* ztile);
// retired diagnostic (per-phase clock totals of the pairwise kernel): zeroes
void debug_stamps(uint64_t* out20, bool reset);
// retired diagnostic (per-workgroup clocks of k_bsi_reg): zeroes
void debug_bsi_stamps(uint64_t* out20, bool reset);
void launch_wide(hipStream_t s, int mode, int grid, const Task* tasks, const uint32_t* nt, WideArgs args, OutCtx oc,
                 uint32_t* task_card);
// result materialisation: k_place = compaction scan over the task records
// (container index + payload offset per kept container, ResultInfo); the
// portable serialization (payload copies, descriptors, offsets, run flags,
// cookie) runs only when the result is fetched
void launch_place(hipStream_t s, const uint32_t* nt, OutCtx oc, ResultInfo* info);
// placement + serialization in one launch from the compute kernel's per-tile sums (OutCtx::tile_agg):
// one workgroup per kAggTile records, no look-back; also writes info, the totals word and the result's
// cardinality like k_place.  max_tasks: an upper bound of *nt (the grid)
void launch_serialize_agg(hipStream_t s, const uint32_t* nt, OutCtx oc, ResultInfo* info, size_t max_tasks);
// the placement tiles covering tasks [t_lo, t_hi) (t_lo a multiple of the 1,024-record tile), for a
// pipelined op whose key ranges are placed one launch each, in order
void launch_place_tiles(hipStream_t s, const uint32_t* nt, OutCtx oc, ResultInfo* info, uint32_t t_lo, uint32_t t_hi);
constexpr uint32_t kPlaceTile = 1024;
// one part of k_serialize: part 1 = the header (cookie, run flags, descriptors, offsets; every record
// placed), part 2 = the payload copies of records [t_lo, t_hi); grid: workgroups to launch (clamped)
void launch_serialize_part(hipStream_t s, const uint32_t* nt, OutCtx oc, int part, uint32_t t_lo, uint32_t t_hi,
                           int grid);
void launch_spec_fix(hipStream_t s, const uint32_t* nt, OutCtx oc);
void launch_serialize(hipStream_t s, const uint32_t* nt, OutCtx oc);
// key shard of a global bitmap: payloads into payload_dst, 4 B descriptors into desc, global
// offsets (off0 + local offset) into offs (nullable), one run-flag byte per container into runb (nullable)
void launch_serialize_shard(hipStream_t s, int grid, const uint32_t* nt, OutCtx oc, uint8_t* payload_dst, uint64_t off0,
                            uint8_t* desc, uint8_t* offs, uint8_t* runb);
// the same with the global layout in device memory (lay: world x {containers, payload bytes, has_run}
// int64); out is laid out as the whole global bitmap, runb one byte per global container (nullable);
// rank 0 also writes the cookie.  emit = false: the payload is already in place.
void launch_serialize_shard_dyn(hipStream_t s, int grid, const uint32_t* nt, OutCtx oc, const int64_t* lay, int rank,
                                int world, uint8_t* out, uint8_t* runb, bool emit);
// in-place OR's types after an OR (x1.or(x2), RB/RoaringBitmap.java:2481-2523): a full result of
// bitmap x1 | array x2 stays a bitmap (ones: 8192 bytes of 0xFF)
void launch_ior_fix(hipStream_t s, const uint32_t* nt, ORec* recs, const uint32_t* koa, const CDesc* da,
                    const uint32_t* kob, const CDesc* db, const uint8_t* ones);
// dst[0..2] = the pending result's (containers, payload bytes, has_run) from k_place's ResultInfo
void launch_layout_out(hipStream_t s, const ResultInfo* info, int64_t* dst);
void launch_reduce_card(hipStream_t s, const uint32_t* task_card, const uint32_t* nt, ResultInfo* info,
                        const uint32_t* err);
void launch_batch_bytes(hipStream_t s, const CDesc* desc, uint64_t n, const uint8_t* payload, unsigned long long* out);
// dst[it.dst .. +it.len) = src[it.src .. +it.len) for every item (wave per item; src needs 16 B read slack)
struct GatherItem {
  uint64_t src, dst, len;
};
void launch_gather(hipStream_t s, const GatherItem* items, uint64_t n, const uint8_t* src, uint8_t* dst);

// block 0 also zeroes zsums (kBsiSumWords u64) and zdefer[0] (either may be null)
void launch_plan_bsi(hipStream_t s, const uint32_t* key_off, const uint32_t* bm, uint32_t need, Task* by_key,
                     uint8_t* flag, uint32_t* wg_count, uint64_t* zlb, uint64_t* ztile, unsigned long long* zsums,
                     uint32_t* zdefer);
// sums: kBsiSumWords u64 (per-slice |bA[x] & found|, the found count, then the final (sum, count)
// written by k_bsi_sum_final); null = no sum
// scratch of the register-resident compare kernels (bsi.hip), per task of the op
// (stride = task capacity; the tables are transposed, row-major over the tasks):
// defer: 1 + stride u32, cnts: 128 x 4 rows of stride ints, kin: 34 rows of stride x 16 B.
// Null: the streamed kernel only.
struct BsiScratch {
  uint32_t* defer;
  int* cnts;
  void* kin;
  size_t stride;
  void* table;  // 34 x 16 B per task: each input's container of the key
  // The task list and the input table depend on the batch only: a batch keeps them across queries
  // (table_ready: k_bsi_table skipped).  The zeroing the plan kernel does per query is then done by
  // block 0 of k_bsi_reg (zlb / ztile: placement look-back, zsums: sum words, zdefer: defer count),
  // and the batch's task count is copied to nt_dst (the context's, which k_place reads).
  bool table_ready;
  uint64_t* zlb;
  uint64_t* ztile;
  unsigned long long* zsums;
  const uint32_t* nt_src;
  uint32_t* nt_dst;
  // k_bsi_reg's unit pools: one counter per group of kBsiGroup workgroups, 64 B apart (kBsiClaimWords
  // words, zero before every query: k_bsi_types zeroes them after k_bsi_reg)
  unsigned int* claims;
};
#ifndef RBG_BSI_GROUP
#define RBG_BSI_GROUP 128
#endif
constexpr int kBsiGroup = RBG_BSI_GROUP;  // workgroups per k_bsi_reg unit pool
constexpr int kBsiMaxGroups = 1024;  // groups of a resident k_bsi_reg grid (at most 4 workgroups per CU)
constexpr int kBsiClaimWords = 16 * kBsiMaxGroups;
// true: compare `op` over `nbits` slices runs the register-resident kernels (k_bsi_table, k_bsi_reg, ...)
bool bsi_reg_path(int op, int nbits);
void launch_bsi_table(hipStream_t s, const Task* tasks, const uint32_t* nt, WideArgs args, void* table, size_t stride);
void launch_bsi_sums_out(hipStream_t s, const unsigned long long* sums, void* dst);  // 2 x u64 at kBsiSumOut
// sums_dst (nullable): (sum, count) also written there by the final sum kernel (two int64, device memory)
void launch_bsi(hipStream_t s, int grid, const Task* tasks, const uint32_t* nt, WideArgs args, BsiArgs p, OutCtx oc,
                unsigned long long* sums, BsiScratch* sc, void* sums_dst = nullptr);
// buffer-package compare (p.buffer): k_bsi_owen_pre writes the orInput types of owenGreatEqual per
// task (p.owen_tb, p.task_keys) for the host's horizontal_or queue replay; k_bsi_buf runs the circuit
void launch_bsi_owen_pre(hipStream_t s, int grid, const Task* tasks, const uint32_t* nt, WideArgs args, BsiArgs p);
void launch_bsi_buf(hipStream_t s, int grid, const Task* tasks, const uint32_t* nt, WideArgs args, BsiArgs p, OutCtx oc);
// ImmutableRoaringBitmap.and / andNot (op OP_AND / OP_ANDNOT) over the pairwise plan's task list, the
// buffer package's container types (workgroup per task; run results above 2047 runs to `big`)
void launch_pair_buf(hipStream_t s, int op, int grid, const PTask* tasks, const uint32_t* nt, const uint8_t* pa,
                     const uint8_t* pb, OutCtx oc, BigRuns big);

// static add / remove / flip(rb, rangeStart, rangeEnd) (rangemut.hip); hbs > hbl: no key in the range
// RMUT_ADD_INPLACE: x.add(rangeStart, rangeEnd) (RB/RoaringBitmap.java:1181), Container.iadd on every key
// RMUT_DERUN: removeRunCompression (RB/RoaringBitmap.java:2738-2749), every run container by cardinality
// RMUT_LIMIT: limit(maxcardinality) (RB/RoaringBitmap.java:2457-2476): keys below hbs cloned, key hbs cut to its
// first lbs values (lbs = 0: none), the rest dropped
// RMUT_RANGE: bitmapOfRange(min, max) (RB/RoaringBitmap.java:588-615), add over an empty bitmap whose
// containers are all RunContainer.rangeOfOnes (run containers even for one or two values)
enum RmutOp : int { RMUT_ADD = 0, RMUT_REMOVE = 1, RMUT_FLIP = 2, RMUT_ADD_INPLACE = 3, RMUT_DERUN = 4, RMUT_LIMIT = 5,
                    RMUT_RANGE = 6 };
struct RmutArgs {
  int op, hbs, lbs, hbl, lbl;
};
// RoaringBitmap.addOffset (RB/RoaringBitmap.java:230-288), addoffset.hip: offset = 65536 co + off, off in
// [0, 65535]; none: a container offset outside [-65536, 65535] (an empty result)
struct AoffArgs {
  int co, off, none;
};
void launch_aoff(hipStream_t s, const uint32_t* koa, const CDesc* da, const uint8_t* pa, AoffArgs aa,
                 uint64_t* wg_epoch, uint32_t epoch, PTask* tasks, uint32_t* n_tasks, OutCtx oc, uint64_t* zlb,
                 uint64_t* ztile, int grid);
void launch_rmut(hipStream_t s, const uint32_t* koa, const CDesc* da, const uint8_t* pa, RmutArgs ra, bool buf,
                 uint64_t* wg_epoch, uint32_t epoch, PTask* tasks, uint32_t* n_tasks, OutCtx oc, uint64_t* zlb,
                 uint64_t* ztile, BigRuns big, int grid);

// RoaringBitmap.orNot (ornot.hip): the reference's key-loop bound, computed on the device
struct OrNotPlan {
  int32_t k_end;       // keys [0, k_end) the loop reaches
  int32_t neg;         // maxSize < 0 (the reference's NegativeArraySizeException)
  int32_t max_size;
  int32_t correction;
};
// k_ornot_scan -> k_plan_ornot -> k_ornot over single-bitmap batches A (x1) and B (x2); flags: 1 in place,
// 2 the buffer package's types (RBG_ORNOT_INPLACE / RBG_ORNOT_BUFFER)
void launch_ornot(hipStream_t s, const uint32_t* koa, const CDesc* da, const uint8_t* pa, int na, const uint32_t* kob,
                  const CDesc* db, const uint8_t* pb, int nb, int max_key, int last_run, int flags, OrNotPlan* plan,
                  uint64_t* wg_epoch, uint32_t epoch, PTask* tasks, uint32_t* n_tasks, OutCtx oc, uint64_t* zlb,
                  uint64_t* ztile, int grid);

// batched andCardinality over pairs (2i, 2i+1) of a bitmap-major batch: per-pair key
// alignment (count, scan, emit), then one wave per matched key; pairs of more than 64
// keys take one wave per pair.  Scratch: cnt (n_pairs u64), part (scan_parts(n_pairs)
// u64), tot (u64: items | large pairs << 32), items (batch_pair_items_cap), large (n_pairs).
struct PairItem {  // one matched key of a pair: both descriptors resolved (32 B, scalar-loaded)
  uint64_t slot_a, slot_b;
  uint32_t card_a, card_b;
  uint32_t pair;
  uint8_t kind_a, kind_b, pad0, pad1;
};
void launch_batch_and_card(hipStream_t s, uint64_t n_pairs, const uint32_t* bm_off, const uint16_t* keys,
                           const CDesc* desc, const uint8_t* payload, int32_t* out, uint64_t* cnt, uint64_t* part,
                           uint64_t* tot, PairItem* items, uint32_t* large);
uint64_t batch_pair_items_cap(const uint32_t* h_bm_nctr, uint64_t n_pairs);

// synthetic generators (synth.hip)
// C3 uniform key slice [key_lo, key_lo + nkeys): pass 0 writes per-key slot bytes,
// pass 1 (given the exclusive per-key byte offsets) fills desc/keys/bm/payload
void launch_synth_c3u(hipStream_t s, uint64_t seed, uint32_t n, int key_lo, int nkeys, unsigned long long* key_bytes,
                      const unsigned long long* key_base, CDesc* desc, uint16_t* keys, uint32_t* bm,
                      uint8_t* payload, int pass);
// C3 clustered: keys/bm of every container given (host CSR); fills desc + 8192 B bitmap slots
void launch_synth_c3c(hipStream_t s, uint64_t seed, uint64_t n_ctr, const uint16_t* keys, const uint32_t* bm,
                      CDesc* desc, uint8_t* payload);
void launch_sum_cards(hipStream_t s, const CDesc* desc, uint64_t n, unsigned long long* out);
// C5 BSI rows 0..rows-1 (nbits slices): pass 0 cards[(key, input)] + minmax, pass 1 fills at pos[(key, input)]
void launch_synth_c5(hipStream_t s, uint64_t seed, uint64_t rows, int key_lo, int nbits, int nkeys, int pass,
                     uint32_t* cards,
                     const uint32_t* pos, unsigned int* minmax, CDesc* desc, uint16_t* keys, uint32_t* bm,
                     uint8_t* payload);
// array payloads for host-built descriptors (C4 pairs)
void launch_synth_arrays(hipStream_t s, uint64_t seed, const CDesc* desc, uint64_t n, uint8_t* payload);
// force < 0: C2 mix (kind drawn per key); force = DK_A/DK_B/DK_R: every key drawn from that family
void launch_synth_c2(hipStream_t s, uint64_t seed, int force, CDesc* desc, uint16_t* keys, uint8_t* payload);

// runopt.hip: device-wide exclusive scan of u64 (part: scan_parts(n) u64 scratch;
// *total = sum), and RoaringBitmap.runOptimize over a batch
uint64_t scan_parts(uint64_t n);
void launch_exclusive_scan(hipStream_t s, const uint64_t* in, uint64_t* out, uint64_t n, uint64_t* part,
                           uint64_t* total);
// the arrays the new batch shares with the input (keys, input index, key CSR, bitmap CSR), copied by
// the write kernel
struct RoCopy {
  const uint16_t* keys;
  uint16_t* out_keys;
  const uint32_t* bm;
  uint32_t* out_bm;
  const uint32_t* koff;
  uint32_t* out_koff;
  uint64_t n_koff;
  const uint32_t* boff;
  uint32_t* out_boff;
  uint64_t n_boff;
};
// runOptimize of every container, each written at its own slot offset of the new payload (the input's
// layout; a converted container is never larger); per workgroup g (of runopt_groups(n)) wstat[4 g + k] =
// {#A, #B, #R, serialized payload bytes} of its containers
uint64_t runopt_groups(uint64_t n);
void launch_runopt(hipStream_t s, const CDesc* desc, const uint8_t* payload, uint64_t n, CDesc* out_desc,
                   uint8_t* out_payload, RoCopy cp, unsigned long long* wstat);
// flags[bitmap] = 1 where the (new) batch holds a run container; flags zeroed by the caller
void launch_runopt_flags(hipStream_t s, const CDesc* desc, const uint32_t* bm, uint64_t n, uint32_t* flags);

// runopt.hip: selectRangeWithoutCopy of every bitmap of a batch (range-restricted aggregations): the
// range's first / last key and low bits (lbs..lbl kept on those keys)
struct RselArgs {
  int hbs, lbs, hbl, lbl;
  int buf;  // the buffer package's cut: MappeableBitmapContainer.remove makes an array below 4096 values
};
void launch_rsel_plan(hipStream_t s, const CDesc* desc, const uint32_t* bm, const uint8_t* payload, uint64_t n,
                      RselArgs ra, uint32_t* info, uint32_t* card, uint64_t* size, uint64_t* keep,
                      unsigned long long* bm_cnt, unsigned long long* bm_card, unsigned long long* totals);
void launch_rsel_write(hipStream_t s, const CDesc* desc, const uint32_t* bm, const uint8_t* payload, uint64_t n,
                       RselArgs ra, const uint32_t* info, const uint32_t* card, const uint64_t* off,
                       const uint64_t* idx, CDesc* out_desc, uint16_t* out_keys, uint32_t* out_bm,
                       uint8_t* out_payload);

// decode.hip: portable-format decode on the device
enum DecErr : uint32_t {
  DEC_OK = 0,
  DEC_TRUNC_COOKIE,
  DEC_BAD_COOKIE,
  DEC_TRUNC_SIZE,
  DEC_SIZE_LARGE,
  DEC_SIZE_NEG,
  DEC_TRUNC_FLAGS,
  DEC_TRUNC_DESC,
  DEC_KEY_ORDER,
  DEC_TRUNC_OFFSETS,
  DEC_TRUNC_RUNS,
  DEC_TRUNC_PAYLOAD,
};
struct DecHead {  // per input: table geometry (byte positions within the input)
  uint64_t pay_pos;
  uint32_t desc_pos, flags_pos, off_pos;
  int32_t size;
  uint32_t flags;
  uint32_t pad;
};
struct DecCtr {  // per container, input order
  uint64_t src;  // payload byte offset in the raw upload
  uint32_t len;  // serialized payload bytes
  uint32_t card;
  uint32_t bm;
  uint32_t kind;
};
void launch_dec_head(hipStream_t s, const uint8_t* raw, const uint64_t* in_off, const uint64_t* in_len, uint64_t n,
                     DecHead* hd, uint64_t* nctr, uint64_t* nch, uint32_t* err, uint32_t* any_err);
// bm_card and bm_flag zeroed by the caller; *n_chunks = sum of nch (device), max_chunks its host bound
void launch_dec_ctrs(hipStream_t s, const uint8_t* raw, const uint64_t* in_off, const uint64_t* in_len, uint64_t n,
                     const DecHead* hd, const uint64_t* ctr_base, const uint64_t* nch, const uint64_t* ch_base,
                     const uint64_t* n_chunks, uint64_t max_chunks, uint32_t* map, DecCtr* q, uint16_t* qkey,
                     uint64_t* bm_card, uint32_t* bm_flag, uint64_t* consumed, uint32_t* err, uint32_t* any_err);
size_t dec_sort_temp_bytes(uint64_t C);
// stable sort of the container keys: perm[p] = input-order index of key-major position p
int launch_dec_sort(hipStream_t s, void* temp, size_t temp_bytes, const uint16_t* qkey, uint16_t* skey,
                    uint32_t* iota, uint32_t* perm, uint64_t C);
void launch_dec_key_off(hipStream_t s, const uint16_t* skey, uint64_t C, uint32_t* key_off);
// perm null: input order.  totals (may be null) += {#A, #B, #R, bytes of payloads above 8194 B}.
// packed: array payloads at their exact length (2 B granularity, as in the portable format) instead of
// 16 B slots -- only for batches of arrays alone (every other slot stays 16 B aligned that way)
void launch_dec_sizes(hipStream_t s, const DecCtr* q, const uint32_t* perm, uint64_t C, uint64_t* size,
                      unsigned long long* totals, bool packed = false);
void launch_dec_fill(hipStream_t s, const uint8_t* raw, const DecCtr* q, const uint16_t* qkey, const uint32_t* perm,
                     const uint64_t* slot, uint64_t C, CDesc* desc, uint16_t* keys, uint32_t* bm, uint8_t* payload,
                     uint64_t* bm_card, bool packed = false);  // bm_card: run cardinalities are re-derived from the runs

}  // namespace rbg
