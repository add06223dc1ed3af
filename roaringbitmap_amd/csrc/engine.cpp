// Host side of the MI355X Roaring engine: device contexts, batch upload
// (staged H2D of the serialized bytes -> device decode into the slotted arena,
// decode.hip), op pipelines and
// the exported C ABI of include/roaring_mi355x.h.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <chrono>
#include <unordered_map>
#include <vector>

#include <sys/mman.h>

#include "../../include/roaring_mi355x.h"
#include "format.hpp"
#include "kernels.hpp"

namespace rbg {

static thread_local std::string g_err;
static void set_err(const std::string& s) { g_err = s; }

#define HIPCHK(x)                                                            \
  do {                                                                       \
    hipError_t e_ = (x);                                                     \
    if (e_ != hipSuccess) {                                                  \
      set_err(std::string(#x) + " failed: " + hipGetErrorString(e_));        \
      return e_ == hipErrorOutOfMemory ? RBG_ERR_OUT_OF_MEMORY : RBG_ERR_DEVICE; \
    }                                                                        \
  } while (0)

#define CHK(x)              \
  do {                      \
    int st_ = (x);          \
    if (st_ != RBG_OK) return st_; \
  } while (0)

constexpr size_t kSlack = 256;  // every device buffer carries read slack (group_copy)
constexpr int kMaxKeys = 65536;
constexpr size_t kLbHeader = 256;  // look-back state: error @64, result card @96
// tile statuses (kMaxTiles, device.hpp) follow the 65536 task statuses, tile cardinalities them

// RBG_DEBUG_SYNC=1: synchronise and report after every pipeline stage (debugging aid)
static bool debug_sync() {
  static int v = -1;
  if (v < 0) {
    const char* e = std::getenv("RBG_DEBUG_SYNC");
    v = (e && e[0] == '1') ? 1 : 0;
  }
  return v == 1;
}
static void dbg(hipStream_t s, const char* what) {
  if (!debug_sync()) return;
  static auto last = std::chrono::steady_clock::now();
  hipError_t e = hipStreamSynchronize(s);
  const auto now = std::chrono::steady_clock::now();
  std::fprintf(stderr, "[rbg] %s done: %s (+%.3f ms)\n", what, hipGetErrorString(e),
               std::chrono::duration<double, std::milli>(now - last).count());
  last = now;
  std::fflush(stderr);
}  // look-back state: ticket @0, error word @64, statuses @256

// On an out-of-memory hipMalloc, the device buffers kept for reuse (Ctx::pool) are freed and the
// allocation retried: first the pool of the context the calling thread works on, then, if that was
// not enough, those of every other context on the device (defined after Ctx).  Every pooled buffer
// freed this way is counted (rbg_pool_evictions), so memory pressure shows.
static size_t release_pools_on(int device, int stage);

struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
  DevBuf() = default;
  DevBuf(const DevBuf&) = delete;
  DevBuf& operator=(const DevBuf&) = delete;
  DevBuf(DevBuf&& o) noexcept : p(o.p), cap(o.cap) {
    o.p = nullptr;
    o.cap = 0;
  }
  DevBuf& operator=(DevBuf&& o) noexcept {
    if (this != &o) {
      if (p) (void)hipFree(p);
      p = o.p;
      cap = o.cap;
      o.p = nullptr;
      o.cap = 0;
    }
    return *this;
  }
  ~DevBuf() {
    if (p) (void)hipFree(p);
  }
  int ensure(size_t bytes) {
    if (cap >= bytes && p) return RBG_OK;
    if (p) (void)hipFree(p);
    p = nullptr;
    cap = 0;
    hipError_t e = hipMalloc(&p, bytes + kSlack);
    if (e == hipErrorOutOfMemory) {
      int dev = 0;
      (void)hipGetLastError();
      for (int stage = 0; stage < 2 && e == hipErrorOutOfMemory; stage++) {
        if (hipGetDevice(&dev) != hipSuccess) break;
        if (release_pools_on(dev, stage) > 0) {
          e = hipMalloc(&p, bytes + kSlack);
          if (e == hipErrorOutOfMemory) (void)hipGetLastError();
        }
      }
    }
    if (e != hipSuccess) {
      p = nullptr;
      set_err(std::string("hipMalloc(") + std::to_string(bytes) + ") failed: " + hipGetErrorString(e));
      return e == hipErrorOutOfMemory ? RBG_ERR_OUT_OF_MEMORY : RBG_ERR_DEVICE;
    }
    cap = bytes;
    return RBG_OK;
  }
  template <class T>
  T* as() const {
    return reinterpret_cast<T*>(p);
  }
};

// runOptimize's device statistics (Batch::ro_stats): from byte 64 the k_runopt workgroups' partial
// counts (4 u64 each), from ro_flags_off(groups) the per-bitmap run flags, computed only when the host
// asks (ensure_stats).
static size_t ro_flags_off(size_t groups) { return (64 + 32 * groups + 255) & ~(size_t)255; }
struct Batch {
  bool live = false;
  bool key_major = false;  // containers sorted by (key, input); else by (input, key)
  bool gapped = false;     // slots not back to back (runOptimize result: a hole after a shrunk container)
  bool packed = false;     // array payloads packed at 2 B granularity (C3 uniform synthetic
                           // batches): wide ops and fetches only
  size_t n_bm = 0, n_ctr = 0;
  DevBuf keys, desc, bm, key_off, bm_off, payload;
  size_t payload_bytes = 0;
  std::vector<uint32_t> h_bm_off;   // bitmap-major container ranges (n_bm + 1), or counts prefix
  std::vector<uint32_t> h_bm_nctr;  // containers per input bitmap
  std::vector<int64_t> h_bm_card;   // long cardinality per input bitmap
  int64_t n_kind[3] = {0, 0, 0};
  int64_t ser_bytes = 0;
  int64_t long_card = 0;
  size_t max_ser = 0;  // Σ serialized payload of containers larger than 8194 B (long run inputs)
  int32_t bsi_min = 0, bsi_max = 0;  // synthetic C5: min / max of the indexed values
  bool pair_cap_known = false;        // batched andCardinality: item capacity computed
  // made by runOptimize: kinds / payload bytes / run flags still in ro_stats (device: 5 u64 totals,
  // plan partial counts, run flags: ro_flags_off) until ensure_stats derives them
  bool stats_pending = false;
  DevBuf ro_stats;
  size_t ro_groups = 0;  // plan workgroups whose partial counts ro_stats holds
  std::vector<uint8_t> h_has_run;
  // BSI compare over this batch (ebM = input 0): the task list (keys of ebM) and the per-key input
  // table, planned by the first query and kept (ctx_bsi)
  bool bsi_cached = false;
  DevBuf bsi_tasks, bsi_nt, bsi_table;
  uint64_t pair_items_cap = 0;
  // host copy of the container table for fetches (batches are immutable once loaded):
  // h_desc in container order, h_pos[h_pos_off[i] .. h_pos_off[i+1]) = bitmap i's containers
  bool h_index = false;
  bool h_chain_identity = false;  // horizontal_order found the batch order to be the chain order
  std::vector<CDesc> h_desc;
  std::vector<uint32_t> h_pos, h_pos_off;
};

struct DecBufs {  // scratch of the device decode (decode.hip), reused across loads
  DevBuf meta, head, nctr, base, nch, chbase, chmap, flag, err, card, cons, part, q, qkey, sort, skey, iota, perm,
      size, cpart;
};

constexpr int kPipeMax = 16;  // key ranges of a pipelined pairwise op + serialization

struct Ctx {
  int device = 0;
  DecBufs dec;
  DevBuf wg_epoch;         // pairwise plan: per-workgroup task counts tagged with the op epoch
  uint32_t epoch = 0;
  DevBuf pc_cnt, pc_part, pc_items, pc_large;  // batched andCardinality scratch
  hipStream_t stream = nullptr;
  // pipelined op + serialization (ctx_pairwise_ser): placement and payload copies of key range r
  // run on stream2 while range r + 1 computes on stream
  hipStream_t stream2 = nullptr;
  hipEvent_t pipe_ev[kPipeMax + 1] = {};
  std::vector<std::unique_ptr<Batch>> batches;
  uint64_t* zlb = nullptr;    // look-back state the next plan kernel zeroes (null: none)
  uint64_t* ztile = nullptr;
  DevBuf bsi_defer, bsi_cnts, bsi_kin, bsi_table;  // scratch of the register-resident BSI kernels
  DevBuf bsi_claims;  // k_bsi_reg's unit-pool counters (zero between queries)
  DevBuf bsi_sums;  // kBsiMaxInputs + 1 u64: per-slice |bA[x] & found|, found count
  void* bsi_sums_dst = nullptr;  // rbg_ctx_bsi_sums_target: (sum, count) also written here by every sum
  // buffer-package BSI: owenGreatEqual's orInput types / task keys / chain order, and the arena of
  // result run containers above 2047 runs (BigRuns; big_ctl = {bytes used, overflow})
  DevBuf owen_tb, owen_keys, owen_ord, big, big_ctl;
  DevBuf ones;  // 8192 bytes of 0xFF: the full bitmap container of an in-place OR (k_ior_fix)
  DevBuf ornot_plan;  // OrNotPlan of the last orNot
  DevBuf gather_items, gather_out;  // batch fetch: slot gather list and download buffer
  DevBuf order;                     // horizontal_*: chain order of every key segment
  DevBuf ro_info, ro_size, ro_part;  // range selection scratch (kept: no allocation per call)
  DevBuf rs_card, rs_keep, rs_bm;
  // device buffers of released batches kept for the next batch of a similar size (hipMalloc /
  // hipFree of a 0.36 GB payload cost more than runOptimize's kernels); bounded by kPoolMax
  std::vector<DevBuf> pool;
  size_t pool_bytes = 0;
  std::mutex pool_mu;  // the pool may be emptied by another thread's out-of-memory allocation
  ResultInfo last_ri{};   // the pending result's facts, once ctx_info has read them (fetch_shard_device)
  bool ri_valid = false;
  int bsi_nbits = 0;
  DevBuf by_key, flag, tasks, ntasks, wg_count, lb, recs, kind_by_out, info, task_card, result, cards, skip, raw,
      scalar, scratch;
  size_t result_cap = 0;
  OutCtx pending{};         // output state of the last materialising op
  std::vector<int32_t> pending_src;  // batches the pending result's pass-through records point into
  size_t pending_ub = 0;
  bool serialized = false;  // pending result already in the portable layout
  bool place_pending = false;  // the op's k_place not launched yet (serialization then places too)
  // the pending result's records were summed per tile by its compute kernel (OutCtx::tile_agg): its
  // serialization places and copies in one launch (k_serialize_agg) instead of k_place + k_serialize
  bool agg_ok = false;
  size_t n_cards = 0;
  int last = 0;  // 0 none, 1 serialized result, 2 cardinality, 3 batch cardinalities
  void* pinned = nullptr;
  size_t pinned_cap = 0;
  // HIP-event phase timing: 4 events per op (start, after plan+compact, after
  // compute, after finalize+emit); read back without per-op host syncs.
  std::vector<hipEvent_t> prof_ev;
  size_t prof_cap = 0, prof_n = 0;
  DevBuf rd_ctr;  // while profiling: bytes the early-exit workShyAnd kernels read (rbg_ctx_profile_bytes)
  void prof_free() {
    for (hipEvent_t e : prof_ev) (void)hipEventDestroy(e);
    prof_ev.clear();
    prof_cap = prof_n = 0;
  }
  bool prof_compute_only = false;  // events around the compute launch only (rbg_ctx_profile_compute)
  void mark(int phase) {
    if (prof_compute_only && (phase == 0 || phase == 3)) {
      if (phase == 3 && prof_n < prof_cap) prof_n++;  // the op's record is complete
      return;
    }
    if (prof_n < prof_cap) (void)hipEventRecord(prof_ev[4 * prof_n + phase], stream);
    if (phase == 3 && prof_n < prof_cap) prof_n++;
  }
  ~Ctx();
};

// every live context, for release_pools_on
static std::mutex g_ctx_mu;
static std::vector<Ctx*> g_ctxs;

Ctx::~Ctx() {
  {
    std::lock_guard<std::mutex> g(g_ctx_mu);
    g_ctxs.erase(std::remove(g_ctxs.begin(), g_ctxs.end(), this), g_ctxs.end());
  }
  prof_free();
  if (pinned) (void)hipHostFree(pinned);
  batches.clear();
  for (hipEvent_t e : pipe_ev)
    if (e) (void)hipEventDestroy(e);
  if (stream2) (void)hipStreamDestroy(stream2);
  if (stream) (void)hipStreamDestroy(stream);
}

static size_t pool_clear(Ctx* c) {
  std::lock_guard<std::mutex> g(c->pool_mu);
  const size_t n = c->pool.size();
  c->pool.clear();
  c->pool_bytes = 0;
  return n;
}

// the context the calling thread works on (set by tl_ctx / enter), for release_pools_on's first stage
static thread_local Ctx* t_cur_ctx = nullptr;
static std::atomic<uint64_t> g_pool_evictions{0};

static size_t release_pools_on(int device, int stage) {
  std::lock_guard<std::mutex> g(g_ctx_mu);
  size_t n = 0;
  const bool own = t_cur_ctx && std::find(g_ctxs.begin(), g_ctxs.end(), t_cur_ctx) != g_ctxs.end();
  if (stage == 0) {
    if (own && t_cur_ctx->device == device) n = pool_clear(t_cur_ctx);
  } else {
    for (Ctx* c : g_ctxs)
      if (c->device == device && !(own && c == t_cur_ctx)) n += pool_clear(c);
  }
  g_pool_evictions += n;
  return n;
}

// entry of a session call: the context's device, and the context out-of-memory retries empty first
static int enter(Ctx* c) {
  t_cur_ctx = c;
  HIPCHK(hipSetDevice(c->device));
  return RBG_OK;
}

static int ctx_init(Ctx* c, int device) {
  int n = 0;
  HIPCHK(hipGetDeviceCount(&n));
  if (device < 0 || device >= n) {
    set_err("no HIP device " + std::to_string(device));
    return RBG_ERR_DEVICE;
  }
  HIPCHK(hipSetDevice(device));
  hipDeviceProp_t prop;
  HIPCHK(hipGetDeviceProperties(&prop, device));
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0) {
    set_err(std::string("engine is built for gfx950, device is ") + prop.gcnArchName);
    return RBG_ERR_DEVICE;
  }
  c->device = device;
  {
    std::lock_guard<std::mutex> g(g_ctx_mu);
    g_ctxs.push_back(c);
  }
  HIPCHK(hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking));
  CHK(c->by_key.ensure(sizeof(PTask) * kMaxKeys));  // Task (wide) or PTask (pairwise) records
  CHK(c->flag.ensure(kMaxKeys));
  // (+ 32768: the pairwise direct mode lays its tasks out wave-major in regions of a multiple of
  // 4 records, at most 4 per resident wave (<= 8192 waves) past the task count)
  CHK(c->tasks.ensure(sizeof(PTask) * (kMaxKeys + 32768)));
  CHK(c->ntasks.ensure(64));
  CHK(c->wg_count.ensure(4 * 256));
  CHK(c->wg_epoch.ensure(8 * 256));
  HIPCHK(hipMemset(c->wg_epoch.p, 0, 8 * 256));
  CHK(c->lb.ensure(kLbHeader + 8 * (kMaxKeys + 2 * kMaxTiles + kMaxAggTiles)));  // + the pairwise tile aggregates
  CHK(c->recs.ensure(sizeof(ORec) * kMaxKeys));
  CHK(c->kind_by_out.ensure(kMaxKeys));
  CHK(c->scalar.ensure(64));
  CHK(c->info.ensure(sizeof(ResultInfo)));
  CHK(c->task_card.ensure(4 * kMaxKeys));
  return RBG_OK;
}

static int pinned_ensure(Ctx* c, size_t bytes) {
  if (c->pinned_cap >= bytes) return RBG_OK;
  if (c->pinned) (void)hipHostFree(c->pinned);
  c->pinned = nullptr;
  c->pinned_cap = 0;
  HIPCHK(hipHostMalloc(&c->pinned, bytes, hipHostMallocDefault));
  c->pinned_cap = bytes;
  return RBG_OK;
}

static inline uint64_t round16(uint64_t x) { return (x + 15) & ~15ULL; }
static inline uint64_t slot_bytes(uint8_t kind, uint32_t ser_len) {
  return kind == KR ? round16(ser_len + 2) : round16(ser_len);
}

// epoch of the next pairwise plan (never 0, the value the tags start from)
static uint32_t next_epoch(Ctx* c) {
  if (++c->epoch == 0) ++c->epoch;
  return c->epoch;
}

static int find_batch(Ctx* c, int32_t id, Batch** out) {
  if (id < 0 || (size_t)id >= c->batches.size() || !c->batches[id] || !c->batches[id]->live) {
    set_err("invalid batch id " + std::to_string(id));
    return RBG_ERR_ILLEGAL_ARGUMENT;
  }
  *out = c->batches[id].get();
  return RBG_OK;
}

// A batch made by runOptimize on the device has its statistics (container kinds, payload bytes, the
// per-bitmap run flags) in device memory until something on the host needs them: read them then.
static int ensure_stats(Ctx* c, Batch* b) {
  if (!b->stats_pending) return RBG_OK;
  const size_t n = b->n_bm, g = b->ro_groups, foff = ro_flags_off(g);
  uint32_t* flags = reinterpret_cast<uint32_t*>(b->ro_stats.as<uint8_t>() + foff);
  if (n) {
    HIPCHK(hipMemsetAsync(flags, 0, 4 * n, c->stream));
    launch_runopt_flags(c->stream, b->desc.as<CDesc>(), b->bm.as<uint32_t>(), b->n_ctr, flags);
  }
  std::vector<unsigned long long> hs(8 + 4 * g);
  std::vector<uint32_t> hf(n);
  HIPCHK(hipMemcpyAsync(hs.data(), b->ro_stats.p, 8 * hs.size(), hipMemcpyDeviceToHost, c->stream));
  if (n) HIPCHK(hipMemcpyAsync(hf.data(), flags, 4 * n, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  b->stats_pending = false;
  unsigned long long h[4] = {0, 0, 0, 0};
  for (size_t w = 0; w < g; w++)
    for (int k = 0; k < 4; k++) h[k] += hs[8 + 4 * w + k];
  for (int k = 0; k < 3; k++) b->n_kind[k] = (int64_t)h[k];
  int64_t ser = (int64_t)h[3];
  b->h_has_run.assign(n, 0);
  for (size_t i = 0; i < n; i++) {
    const size_t nc = b->h_bm_nctr.empty() ? 0 : b->h_bm_nctr[i];
    ser += (int64_t)header_size(nc, hf[i] != 0);
    b->h_has_run[i] = hf[i] != 0;
  }
  if (b->ser_bytes) b->ser_bytes = ser;  // batches built on the device carry no serialized size
  return RBG_OK;
}

static int get_batch(Ctx* c, int32_t id, Batch** out) {
  CHK(find_batch(c, id, out));
  return ensure_stats(c, *out);
}

static int32_t new_batch(Ctx* c) {
  for (size_t i = 0; i < c->batches.size(); i++)
    if (!c->batches[i]) {
      c->batches[i].reset(new Batch());
      return (int32_t)i;
    }
  c->batches.emplace_back(new Batch());
  return (int32_t)(c->batches.size() - 1);
}

constexpr size_t kPoolMax = 2ull << 30;    // bytes of released buffers a context keeps
constexpr size_t kPoolMaxBuf = 1ull << 30;  // larger buffers are freed at once

// a released batch buffer into the context's pool (reused only by later work on the same stream)
static void pool_put(Ctx* c, DevBuf& b) {
  if (!b.p) return;
  std::lock_guard<std::mutex> g(c->pool_mu);
  if (b.cap > kPoolMaxBuf) {
    b = DevBuf();
    return;
  }
  while (!c->pool.empty() && c->pool_bytes + b.cap > kPoolMax) {  // oldest first
    c->pool_bytes -= c->pool.front().cap;
    c->pool.erase(c->pool.begin());
  }
  c->pool_bytes += b.cap;
  c->pool.push_back(std::move(b));
}

// dst sized for `bytes`: the smallest pooled buffer that holds it (at most twice as large),
// else a fresh allocation
static int pool_take(Ctx* c, DevBuf& dst, size_t bytes) {
  if (dst.p && dst.cap >= bytes) return RBG_OK;
  std::unique_lock<std::mutex> lk(c->pool_mu);
  size_t best = c->pool.size();
  for (size_t i = 0; i < c->pool.size(); i++) {
    const size_t cap = c->pool[i].cap;
    if (cap >= bytes && cap <= 2 * bytes + (1u << 20) && (best == c->pool.size() || cap < c->pool[best].cap))
      best = i;
  }
  if (best == c->pool.size()) {
    lk.unlock();  // ensure may empty the pools (out of memory)
    return dst.ensure(bytes);
  }
  c->pool_bytes -= c->pool[best].cap;
  dst = std::move(c->pool[best]);
  c->pool.erase(c->pool.begin() + (std::ptrdiff_t)best);
  return RBG_OK;
}

// drops the listed batches on scope exit
struct BatchGuard {
  Ctx* c;
  std::vector<int32_t> ids;
  ~BatchGuard() {
    for (int32_t id : ids)
      if (id >= 0 && (size_t)id < c->batches.size()) c->batches[id].reset();
  }
};

// ---------------------------------------------------------------------------
// upload: the host concatenates the serialized inputs (16 B aligned) and copies
// them once; decode.hip parses every header and places every payload on the GPU
// ---------------------------------------------------------------------------
static const char* dec_message(uint32_t e, int* status) {
  *status = RBG_ERR_TRUNCATED;
  switch (e) {
    case DEC_TRUNC_COOKIE: return "truncated input: cookie";
    case DEC_BAD_COOKIE: *status = RBG_ERR_INVALID_FORMAT; return "I failed to find one of the right cookies.";
    case DEC_TRUNC_SIZE: return "truncated input: size";
    case DEC_SIZE_LARGE: *status = RBG_ERR_INVALID_FORMAT; return "Size too large";
    case DEC_SIZE_NEG: *status = RBG_ERR_INVALID_FORMAT; return "negative container count";
    case DEC_TRUNC_FLAGS: return "truncated input: run flags";
    case DEC_TRUNC_DESC: return "truncated input: descriptors";
    case DEC_KEY_ORDER: *status = RBG_ERR_INVALID_FORMAT; return "container keys are not strictly increasing";
    case DEC_TRUNC_OFFSETS: return "truncated input: offsets";
    case DEC_TRUNC_RUNS: return "truncated input: run count";
    default: return "truncated input: container payload";
  }
}

static int dec_report(Ctx* c, size_t n) {
  std::vector<uint32_t> e(n);
  HIPCHK(hipMemcpy(e.data(), c->dec.err.p, 4 * n, hipMemcpyDeviceToHost));
  for (size_t i = 0; i < n; i++)
    if (e[i]) {
      int st;
      const char* m = dec_message(e[i], &st);
      set_err("input " + std::to_string(i) + ": " + m);
      return st;
    }
  set_err("decode reported an error but no input carries one");
  return RBG_ERR_DEVICE;
}

// Host side of an upload: the inputs are copied into pinned staging (worker
// threads over <= 4 MiB pieces, in offset order) and each ~32 MiB group goes to the
// device as soon as its pieces are staged, so the copies overlap the DMA.
static int stage_upload(Ctx* c, const uint8_t* const* bufs, const size_t* lens, size_t n, const uint64_t* dst_off,
                        uint64_t raw_bytes) {
  uint8_t* pin = reinterpret_cast<uint8_t*>(c->pinned);
  uint8_t* dev = c->raw.as<uint8_t>();
  hipStream_t s = c->stream;
  constexpr uint64_t kPiece = 4ull << 20, kGroup = 32ull << 20;
  if (raw_bytes <= kGroup) {
    for (size_t i = 0; i < n; i++)
      if (lens[i]) std::memcpy(pin + dst_off[i], bufs[i], lens[i]);
    if (raw_bytes) HIPCHK(hipMemcpyAsync(dev, pin, raw_bytes, hipMemcpyHostToDevice, s));
    return RBG_OK;
  }
  struct Piece {
    uint64_t dst;
    const uint8_t* src;
    uint64_t len;
    uint32_t g0, g1;  // groups the piece touches (pieces are smaller than a group)
  };
  std::vector<Piece> pieces;
  for (size_t i = 0; i < n; i++)
    for (uint64_t o = 0; o < lens[i]; o += kPiece) {
      const uint64_t d = dst_off[i] + o;
      const uint64_t l = std::min<uint64_t>(kPiece, lens[i] - o);
      pieces.push_back(Piece{d, bufs[i] + o, l, (uint32_t)(d / kGroup), (uint32_t)((d + l - 1) / kGroup)});
    }
  const uint32_t groups = (uint32_t)((raw_bytes + kGroup - 1) / kGroup);
  std::unique_ptr<std::atomic<int>[]> left(new std::atomic<int>[groups]);
  for (uint32_t g = 0; g < groups; g++) left[g].store(0);
  for (const Piece& p : pieces) {
    left[p.g0].fetch_add(1);
    if (p.g1 != p.g0) left[p.g1].fetch_add(1);
  }
  std::atomic<size_t> next{0};
  const int nthr = (int)std::min<unsigned>(16, std::max(1u, std::thread::hardware_concurrency()));
  std::vector<std::thread> th;
  for (int t = 0; t < nthr; t++)
    th.emplace_back([&]() {
      for (size_t k; (k = next.fetch_add(1)) < pieces.size();) {
        std::memcpy(pin + pieces[k].dst, pieces[k].src, pieces[k].len);
        left[pieces[k].g0].fetch_sub(1, std::memory_order_release);
        if (pieces[k].g1 != pieces[k].g0) left[pieces[k].g1].fetch_sub(1, std::memory_order_release);
      }
    });
  int st = RBG_OK;
  for (uint32_t g = 0; g < groups; g++) {
    while (left[g].load(std::memory_order_acquire) > 0) std::this_thread::yield();
    const uint64_t lo = (uint64_t)g * kGroup, hi = std::min<uint64_t>(raw_bytes, lo + kGroup);
    if (st == RBG_OK && hipMemcpyAsync(dev + lo, pin + lo, hi - lo, hipMemcpyHostToDevice, s) != hipSuccess) {
      set_err("host-to-device copy of the upload failed");
      st = RBG_ERR_DEVICE;
    }
  }
  for (auto& x : th) x.join();
  return st;
}

// The serialized inputs at 16 B aligned offsets of one upload into c->raw: off[i] (host)
static int ctx_upload_raw(Ctx* c, const uint8_t* const* bufs, const size_t* lens, size_t n,
                          std::vector<uint64_t>* off) {
  if (n && (!bufs || !lens)) return RBG_ERR_ILLEGAL_ARGUMENT;
  for (size_t i = 0; i < n; i++)
    if (!bufs[i] && lens[i]) return RBG_ERR_ILLEGAL_ARGUMENT;
  off->assign(n, 0);
  uint64_t raw_bytes = 0;
  for (size_t i = 0; i < n; i++) {
    (*off)[i] = raw_bytes;
    raw_bytes = round16(raw_bytes + lens[i]);
  }
  CHK(c->raw.ensure(raw_bytes + 64));
  CHK(pinned_ensure(c, raw_bytes + 64));
  CHK(stage_upload(c, bufs, lens, n, off->data(), raw_bytes));
  dbg(c->stream, "load: host staging copy");
  return RBG_OK;
}

// Device decode of n uploaded inputs (c->raw at off[i], len[i] bytes) into one batch.
// key_major: containers sorted by (key, input) with a key CSR (operands of every op);
// otherwise input order (bitmap-major, batched andCardinality)
static int ctx_decode_raw(Ctx* c, const uint64_t* off, const size_t* lens, size_t n, bool key_major,
                          int32_t* out_id, bool pack_arrays = false) {
  DecBufs& d = c->dec;
  hipStream_t s = c->stream;
  std::vector<uint64_t> meta(2 * n + 2, 0);  // in_off[n], in_len[n]
  for (size_t i = 0; i < n; i++) {
    meta[i] = off[i];
    meta[n + i] = lens[i];
  }
  CHK(d.meta.ensure(8 * (2 * n + 2)));
  CHK(d.head.ensure(sizeof(DecHead) * n + 16));
  CHK(d.nctr.ensure(8 * n + 16));
  CHK(d.base.ensure(8 * n + 16));
  CHK(d.nch.ensure(8 * n + 16));
  CHK(d.chbase.ensure(8 * n + 16));
  CHK(d.flag.ensure(4 * n + 16));
  CHK(d.err.ensure(4 * n + 16));
  CHK(d.card.ensure(8 * n + 16));
  CHK(d.cons.ensure(8 * n + 16));
  CHK(d.part.ensure(8 * (scan_parts(std::max<size_t>(n, 1)) + 1)));
  CHK(c->scalar.ensure(64));
  const uint64_t* in_off = d.meta.as<uint64_t>();
  const uint64_t* in_len = in_off + n;
  unsigned long long* sc = c->scalar.as<unsigned long long>();  // [0] any error, [1] C, [2..5] totals, [6] bytes,
                                                                // [7] chunks
  HIPCHK(hipMemcpyAsync(d.meta.p, meta.data(), 8 * (2 * n + 2), hipMemcpyHostToDevice, s));
  HIPCHK(hipMemsetAsync(sc, 0, 64, s));
  dbg(s, "load: H2D");
  uint32_t* any_err = reinterpret_cast<uint32_t*>(sc);
  launch_dec_head(s, c->raw.as<uint8_t>(), in_off, in_len, n, d.head.as<DecHead>(), d.nctr.as<uint64_t>(),
                  d.nch.as<uint64_t>(), d.err.as<uint32_t>(), any_err);
  launch_exclusive_scan(s, d.nctr.as<uint64_t>(), d.base.as<uint64_t>(), n, d.part.as<uint64_t>(),
                        reinterpret_cast<uint64_t*>(sc + 1));
  launch_exclusive_scan(s, d.nch.as<uint64_t>(), d.chbase.as<uint64_t>(), n, d.part.as<uint64_t>(),
                        reinterpret_cast<uint64_t*>(sc + 7));
  HIPCHK(hipGetLastError());
  unsigned long long h[8] = {};
  HIPCHK(hipMemcpyAsync(h, sc, 64, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  if (h[0]) return dec_report(c, n);
  const uint64_t C = h[1];
  if (C > 0x7FFFFFFFull) {
    set_err("a batch holds at most 2^31 - 1 containers");
    return RBG_ERR_ILLEGAL_ARGUMENT;
  }
  dbg(s, "load: headers");
  const uint64_t n_chunks = h[7];
  CHK(d.q.ensure(sizeof(DecCtr) * C + 16));
  CHK(d.qkey.ensure(2 * C + 16));
  CHK(d.chmap.ensure(4 * n_chunks + 16));
  HIPCHK(hipMemsetAsync(d.card.p, 0, 8 * n + 16, s));
  HIPCHK(hipMemsetAsync(d.flag.p, 0, 4 * n + 16, s));
  launch_dec_ctrs(s, c->raw.as<uint8_t>(), in_off, in_len, n, d.head.as<DecHead>(), d.base.as<uint64_t>(),
                  d.nch.as<uint64_t>(), d.chbase.as<uint64_t>(), reinterpret_cast<uint64_t*>(sc + 7), n_chunks,
                  d.chmap.as<uint32_t>(), d.q.as<DecCtr>(), d.qkey.as<uint16_t>(), d.card.as<uint64_t>(),
                  d.flag.as<uint32_t>(), d.cons.as<uint64_t>(), d.err.as<uint32_t>(), any_err);
  const int32_t id = new_batch(c);
  Batch& b = *c->batches[id];
  BatchGuard guard{c, {id}};  // dropped unless the load completes
  b.n_bm = n;
  b.n_ctr = C;
  b.key_major = key_major;
  CHK(b.keys.ensure(2 * C + 16));
  CHK(b.desc.ensure(sizeof(CDesc) * C + 16));
  CHK(b.bm.ensure(4 * C + 16));
  CHK(b.bm_off.ensure(4 * (n + 1)));
  const uint32_t* perm = nullptr;
  if (key_major) {
    CHK(b.key_off.ensure(4 * (kMaxKeys + 1)));
    const uint16_t* sorted = d.qkey.as<uint16_t>();
    if (n > 1 && C > 0) {  // one bitmap is key-sorted already
      const size_t tb = dec_sort_temp_bytes(C);
      CHK(d.sort.ensure(tb + 16));
      CHK(d.skey.ensure(2 * C + 16));
      CHK(d.iota.ensure(4 * C + 16));
      CHK(d.perm.ensure(4 * C + 16));
      if (launch_dec_sort(s, d.sort.p, tb, d.qkey.as<uint16_t>(), d.skey.as<uint16_t>(), d.iota.as<uint32_t>(),
                          d.perm.as<uint32_t>(), C) != 0) {
        set_err("radix sort of the container keys failed");
        return RBG_ERR_DEVICE;
      }
      sorted = d.skey.as<uint16_t>();
      perm = d.perm.as<uint32_t>();
    }
    launch_dec_key_off(s, sorted, C, b.key_off.as<uint32_t>());
  }
  dbg(s, "load: containers + sort");
  CHK(d.size.ensure(8 * C + 16));
  CHK(d.cpart.ensure(8 * (scan_parts(std::max<uint64_t>(C, 1)) + 1)));
  launch_dec_sizes(s, d.q.as<DecCtr>(), perm, C, d.size.as<uint64_t>(), sc + 2);
  launch_exclusive_scan(s, d.size.as<uint64_t>(), d.size.as<uint64_t>(), C, d.cpart.as<uint64_t>(),
                        reinterpret_cast<uint64_t*>(sc + 6));
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(h, sc, 64, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  if (h[0]) return dec_report(c, n);
  for (int k = 0; k < 3; k++) b.n_kind[k] = (int64_t)h[2 + k];
  b.max_ser = h[5];
  // a key-major batch of arrays alone, for the wide ops: the array payloads packed as in the portable
  // format (2 B granularity) instead of 16 B slots -- the wide kernels' fastest layout
  const bool packed = pack_arrays && key_major && C > 0 && b.n_kind[DK_B] == 0 && b.n_kind[DK_R] == 0;
  if (packed) {
    launch_dec_sizes(s, d.q.as<DecCtr>(), perm, C, d.size.as<uint64_t>(), nullptr, true);
    launch_exclusive_scan(s, d.size.as<uint64_t>(), d.size.as<uint64_t>(), C, d.cpart.as<uint64_t>(),
                          reinterpret_cast<uint64_t*>(sc + 6));
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(h, sc, 64, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    b.packed = true;
  }
  b.payload_bytes = h[6];
  CHK(b.payload.ensure(b.payload_bytes + 64));
  dbg(s, "load: sizes + payload alloc");
  launch_dec_fill(s, c->raw.as<uint8_t>(), d.q.as<DecCtr>(), d.qkey.as<uint16_t>(), perm, d.size.as<uint64_t>(), C,
                  b.desc.as<CDesc>(), b.keys.as<uint16_t>(), b.bm.as<uint32_t>(), b.payload.as<uint8_t>(),
                  d.card.as<uint64_t>(), packed);
  HIPCHK(hipGetLastError());
  std::vector<uint64_t> nctr(n), card(n), cons(n);
  if (n) {
    HIPCHK(hipMemcpyAsync(nctr.data(), d.nctr.p, 8 * n, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(card.data(), d.card.p, 8 * n, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(cons.data(), d.cons.p, 8 * n, hipMemcpyDeviceToHost, s));
  }
  HIPCHK(hipStreamSynchronize(s));
  b.h_bm_off.assign(n + 1, 0);
  b.h_bm_nctr.resize(n);
  b.h_bm_card.resize(n);
  for (size_t i = 0; i < n; i++) {
    b.h_bm_nctr[i] = (uint32_t)nctr[i];
    b.h_bm_off[i + 1] = b.h_bm_off[i] + (uint32_t)nctr[i];
    b.h_bm_card[i] = (int64_t)card[i];
    b.long_card += (int64_t)card[i];
    b.ser_bytes += (int64_t)cons[i];
  }
  HIPCHK(hipMemcpyAsync(b.bm_off.p, b.h_bm_off.data(), 4 * (n + 1), hipMemcpyHostToDevice, s));
  HIPCHK(hipStreamSynchronize(s));
  dbg(s, "load: fill + readback");
  guard.ids.clear();
  b.live = true;
  *out_id = id;
  return RBG_OK;
}

static int ctx_load_impl(Ctx* c, const uint8_t* const* bufs, const size_t* lens, size_t n, bool key_major,
                         int32_t* out_id, bool pack_arrays = false) {
  std::vector<uint64_t> off;
  CHK(ctx_upload_raw(c, bufs, lens, n, &off));
  return ctx_decode_raw(c, off.data(), lens, n, key_major, out_id, pack_arrays);
}

// pack_arrays: a batch of arrays alone is decoded packed (wide ops and fetches only, see Batch::packed)
static int ctx_load(Ctx* c, const uint8_t* const* bufs, const size_t* lens, size_t n, int32_t* out_id,
                    bool pack_arrays = false) {
  return ctx_load_impl(c, bufs, lens, n, true, out_id, pack_arrays);
}

// n serialized bitmaps in ONE upload, each decoded into a batch of its own (the operands of a
// pairwise op: one staging pass and DMA for both); ids[i] = batch of bitmap i
static int ctx_load_separate(Ctx* c, const uint8_t* const* bufs, const size_t* lens, size_t n, int32_t* ids) {
  std::vector<uint64_t> off;
  CHK(ctx_upload_raw(c, bufs, lens, n, &off));
  BatchGuard g{c, {}};
  for (size_t i = 0; i < n; i++) {
    CHK(ctx_decode_raw(c, &off[i], &lens[i], 1, true, &ids[i]));
    g.ids.push_back(ids[i]);
  }
  g.ids.clear();
  return RBG_OK;
}

// ---------------------------------------------------------------------------
// op pipelines
// ---------------------------------------------------------------------------
// Result buffer: [header reserve P0][payload region].  The header (whose size
// depends on the final container count and run flag) is written right in front
// of the payload, so the serialized bitmap starts at P0 - header.
static uint64_t header_reserve(size_t max_tasks) {
  return round16(8 + (max_tasks + 7) / 8 + 8 * (uint64_t)max_tasks + 16);
}

static int grid_for(size_t tasks, size_t cap = 4096) {
  size_t g = std::min(tasks, cap);
  return (int)std::max<size_t>(g, 1);
}

// Output state of a materialising op: per-task records + scratch slots (the
// device-resident result), and the portable-format buffer the serialization
// writes into on fetch.  Card-only ops need no output state.
static int prepare_output(Ctx* c, size_t max_tasks, size_t max_payload, OutCtx* oc, bool card_only) {
  uint8_t* lb = c->lb.as<uint8_t>();
  *oc = OutCtx{};
  oc->err = reinterpret_cast<uint32_t*>(lb + 64);
  oc->status = reinterpret_cast<uint64_t*>(lb + kLbHeader);
  oc->tile_status = reinterpret_cast<uint64_t*>(lb + kLbHeader + 8 * kMaxKeys);
  oc->tile_card = reinterpret_cast<uint64_t*>(lb + kLbHeader + 8 * (kMaxKeys + kMaxTiles));
  oc->recs = c->recs.as<ORec>();
  c->serialized = false;
  c->place_pending = false;
  c->agg_ok = false;
  c->ri_valid = false;
  c->pending_ub = 0;
  c->zlb = c->ztile = nullptr;
  c->pending_src.clear();
  if (card_only) {
    c->zlb = reinterpret_cast<uint64_t*>(lb);  // the error word must not carry over from an earlier op
    return RBG_OK;
  }
  const uint64_t P0 = header_reserve(max_tasks);
  CHK(c->result.ensure(P0 + max_payload + 64));
  c->result_cap = P0 + max_payload;
  CHK(c->scratch.ensure((size_t)kSlotBytes * std::max<size_t>(max_tasks, 1) + 64));
  // the look-back header and tile statuses are zeroed by the op's plan kernel
  c->zlb = reinterpret_cast<uint64_t*>(lb);
  c->ztile = reinterpret_cast<uint64_t*>(lb + kLbHeader + 8 * kMaxKeys);
  oc->out = c->result.as<uint8_t>();
  oc->payload_base = P0;
  oc->scratch = c->scratch.as<uint8_t>();
  oc->kind_by_out = c->kind_by_out.as<uint8_t>();
  c->pending = *oc;
  c->pending_ub = max_tasks;
  return RBG_OK;
}

// Placement of a materialising op's result (k_place) is deferred until something needs it
// (serialization, result statistics, a key-shard fetch): an op whose caller only wants the
// result to exist on the device (a BSI query followed by its sum) does not pay for it.
static void defer_place(Ctx* c) {
  c->place_pending = true;
  c->last = 1;
}
static int ensure_placed(Ctx* c) {
  if (!c->place_pending) return RBG_OK;
  launch_place(c->stream, c->ntasks.as<uint32_t>(), c->pending, c->info.as<ResultInfo>());
  HIPCHK(hipGetLastError());
  c->place_pending = false;
  return RBG_OK;
}

// Portable serialization of the pending result (RB/RoaringArray.java:896-940),
// on the device, once per result.
static int ctx_serialize(Ctx* c) {
  if (c->last != 1) {
    set_err("no materialised result pending");
    return RBG_ERR_ILLEGAL_ARGUMENT;
  }
  if (c->serialized) return RBG_OK;
  if (c->place_pending && c->agg_ok && !c->pending.spec && c->pending_ub <= (size_t)kMaxAggTiles * kAggTile) {
    // placement from the compute kernel's tile sums and the serialization in one launch
    launch_serialize_agg(c->stream, c->ntasks.as<uint32_t>(), c->pending, c->info.as<ResultInfo>(), c->pending_ub);
    HIPCHK(hipGetLastError());
    c->place_pending = false;
    c->serialized = true;
    return RBG_OK;
  }
  CHK(ensure_placed(c));
  if (c->pending.spec) launch_spec_fix(c->stream, c->ntasks.as<uint32_t>(), c->pending);
  launch_serialize(c->stream, c->ntasks.as<uint32_t>(), c->pending);
  HIPCHK(hipGetLastError());
  c->serialized = true;
  return RBG_OK;
}


// operand range of bitmap i of a batch (must be contiguous: one-bitmap batch)
static int operand(Batch* b, size_t i, const uint16_t** keys, const CDesc** desc, int* n) {
  if (i >= b->n_bm) {
    set_err("bitmap index out of range");
    return RBG_ERR_ILLEGAL_ARGUMENT;
  }
  if (b->n_bm != 1 || !b->key_major || b->packed) {
    set_err("pairwise operands must be single-bitmap key-major batches with slot-aligned payloads");
    return RBG_ERR_ILLEGAL_ARGUMENT;
  }
  *keys = b->keys.as<uint16_t>();
  *desc = b->desc.as<CDesc>();
  *n = (int)b->n_ctr;
  return RBG_OK;
}

// op RBG_OR_INPLACE: x1.or(x2) in place (RB/RoaringBitmap.java:2481-2523), the OR with Container.ior's
// types (k_ior_fix)
// RoaringBitmap.and / or / xor / andNot + serialize of a dense key range as K key ranges in one
// pipeline (ctx_pairwise with pipe_k > 1): range r's compute launch runs on the context stream; its
// placement tiles (k_place: the look-back reads the tiles the earlier ranges published, so every record
// gets its global output index and payload offset) and its payload copies (k_serialize part 2) run on
// stream2 while range r + 1 computes.  The header (cookie, run flags, descriptors, offsets) follows the
// last range; the context stream then waits for stream2.  Same records, same bytes as the op followed
// by ctx_serialize: only the order of the launches differs.  Ranges are whole placement tiles.
// RBG_PIPE_PW_WG / RBG_PIPE_COPY_WG: workgroups per CU of the compute / copy launches (defaults:
// resident maximum, 1).
static int pairwise_pipelined(Ctx* c, int op, int K, PwDirect pd, Batch* A, Batch* B, OutCtx oc) {
  hipStream_t s = c->stream;
  if (!c->stream2) {
    HIPCHK(hipStreamCreateWithFlags(&c->stream2, hipStreamNonBlocking));
    for (hipEvent_t& e : c->pipe_ev) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  }
  hipStream_t s2 = c->stream2;
  K = std::min(K, kPipeMax);
  const uint32_t n = pd.nkeys;
  // range bounds in whole tiles
  const uint32_t tiles = (n + kPlaceTile - 1) / kPlaceTile;
  K = (int)std::max<uint32_t>(1, std::min<uint32_t>((uint32_t)K, tiles));
  const int pw_wg = getenv("RBG_PIPE_PW_WG") ? atoi(getenv("RBG_PIPE_PW_WG")) : 0;
  const int cp_wg = getenv("RBG_PIPE_COPY_WG") ? atoi(getenv("RBG_PIPE_COPY_WG")) : 1;
  int cus = 256;
  (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, c->device);
  c->mark(0);
  c->mark(1);
  // the first range's record -> the previous op's stream2 work (a pending header of the last
  // pipelined op) is complete before this op reuses the records: stream waits for it at the end of
  // every pipelined op, so nothing is needed here
  uint32_t t_lo = 0;
  for (int r = 0; r < K; r++) {
    const uint32_t t_hi = r == K - 1 ? n : (uint32_t)(((uint64_t)tiles * (r + 1) / K) * kPlaceTile);
    PwDirect d = pd;
    d.key_lo = pd.key_lo + (int)t_lo;
    d.nkeys = t_hi - t_lo;
    if (r) d.zlb = d.ztile = nullptr;  // zeroed once, by the first range's launch
    OutCtx o = oc;
    o.recs = oc.recs + t_lo;
    o.scratch = oc.scratch + (size_t)t_lo * kSlotBytes;
    const int want = grid_for((d.nkeys + 3) / 4, 16384);
    const int grid = pw_wg > 0 ? std::min(want, pw_wg * cus) : want;
    launch_pairwise(s, op, 0, grid, c->tasks.as<PTask>(), c->ntasks.as<uint32_t>(), A->payload.as<uint8_t>(),
                    B->payload.as<uint8_t>(), o, c->task_card.as<uint32_t>(), &d);
    HIPCHK(hipEventRecord(c->pipe_ev[r], s));
    HIPCHK(hipStreamWaitEvent(s2, c->pipe_ev[r], 0));
    launch_place_tiles(s2, c->ntasks.as<uint32_t>(), oc, c->info.as<ResultInfo>(), t_lo, t_hi);
    launch_serialize_part(s2, c->ntasks.as<uint32_t>(), oc, 2, t_lo, t_hi, cp_wg * cus);
    t_lo = t_hi;
  }
  c->mark(2);
  launch_serialize_part(s2, c->ntasks.as<uint32_t>(), oc, 1, 0, 0xFFFFFFFFu, 256);
  HIPCHK(hipEventRecord(c->pipe_ev[kPipeMax], s2));
  HIPCHK(hipStreamWaitEvent(s, c->pipe_ev[kPipeMax], 0));
  c->place_pending = false;
  c->serialized = true;
  c->last = 1;
  c->mark(3);
  HIPCHK(hipGetLastError());
  return RBG_OK;
}

// key ranges of a pipelined op + serialization (RBG_SER_PIPE; default 1 = the op, then the serialization: pipelining
// off, measured slower at every split)
static int pipe_ranges() {
  const char* e = getenv("RBG_SER_PIPE");  // read per call (tests vary it)
  return e ? std::max(1, atoi(e)) : 1;  // measured: 2-16 ranges are slower than the two calls
}
// ImmutableRoaringBitmap.and / andNot and MutableRoaringBitmap's static and / andNot
// (RB/buffer/ImmutableRoaringBitmap.java:299-325, 441-471; RB/buffer/MutableRoaringBitmap.java:235-301):
// the pairwise plan, then k_pair_buf (the buffer package's container types).  A run result above
// 2047 runs goes to the big-run arena; the arena is checked after the op and the op rerun once with
// the size the first pass reserved (as the buffer naive_and chain, ctx_wide).
static int ctx_pairwise_buffer(Ctx* c, int op, int32_t ia, size_t ma, int32_t ib, size_t mb, int key_lo, int key_hi) {
  key_lo = std::max(0, key_lo);
  key_hi = std::min(kMaxKeys, key_hi);
  Batch *A, *B;
  CHK(get_batch(c, ia, &A));
  CHK(get_batch(c, ib, &B));
  const uint16_t *ka, *kb;
  const CDesc *da, *db;
  int na, nb;
  CHK(operand(A, ma, &ka, &da, &na));
  CHK(operand(B, mb, &kb, &db, &nb));
  hipStream_t s = c->stream;
  const size_t ub = std::max<size_t>(1, op == OP_AND ? (size_t)std::min(na, nb) : (size_t)na);
  if (!c->big_ctl.p) CHK(c->big_ctl.ensure(16));
  if (!c->big.p) CHK(c->big.ensure(16ull << 20));
  for (int attempt = 0;; attempt++) {
    OutCtx oc;
    CHK(prepare_output(c, ub, A->payload_bytes + B->payload_bytes + (size_t)8194 * ub + c->big.cap, &oc, false));
    c->pending_src = {ia, ib};
    c->mark(0);
    launch_plan_pairwise(s, op, key_lo, key_hi, A->key_off.as<uint32_t>(), da, A->payload.as<uint8_t>(),
                         B->key_off.as<uint32_t>(), db, B->payload.as<uint8_t>(), c->wg_epoch.as<uint64_t>(),
                         next_epoch(c), c->tasks.as<PTask>(), c->ntasks.as<uint32_t>(), c->zlb, c->ztile, oc.err);
    HIPCHK(hipMemsetAsync(c->big_ctl.p, 0, 16, s));
    c->mark(1);
    launch_pair_buf(s, op, grid_for(ub, 65536), c->tasks.as<PTask>(), c->ntasks.as<uint32_t>(),
                    A->payload.as<uint8_t>(), B->payload.as<uint8_t>(), oc,
                    BigRuns{c->big.as<uint8_t>(), c->big_ctl.as<unsigned long long>(), c->big.cap});
    c->mark(2);
    defer_place(c);
    c->mark(3);
    HIPCHK(hipGetLastError());
    unsigned long long used[2] = {0, 0};
    HIPCHK(hipMemcpyAsync(used, c->big_ctl.p, 16, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if (!used[1]) return RBG_OK;
    if (attempt) {
      set_err("buffer and / andNot: the run-container arena overflowed twice");
      return RBG_ERR_DEVICE;
    }
    CHK(c->big.ensure(used[0] + (used[0] >> 3) + 4096));
  }
}

// RoaringBitmap.orNot(x1, x2, rangeEnd) (static, RB/RoaringBitmap.java:1521-1603) and x1.orNot(x2,
// rangeEnd) (in place, :1431-1506), ornot.hip.  rangeSanityCheck(0, rangeEnd) (:204-213).  The
// reference's maxSize is negative only for rangeEnd == 0 (maxKey = -1) with x1 empty and x2's first
// container full (new char[-1] throws): only that case reads the plan back before returning.
static int ctx_ornot(Ctx* c, int32_t ia, size_t ma, int32_t ib, size_t mb, int64_t range_end, int flags) {
  if (range_end < 0 || range_end > (int64_t)0x100000000ll) {
    set_err("rangeEnd should be in [0, 0xffffffff + 1]");
    return RBG_ERR_ILLEGAL_ARGUMENT;
  }
  Batch *A, *B;
  CHK(get_batch(c, ia, &A));
  CHK(get_batch(c, ib, &B));
  const uint16_t *ka, *kb;
  const CDesc *da, *db;
  int na, nb;
  CHK(operand(A, ma, &ka, &da, &na));
  CHK(operand(B, mb, &kb, &db, &nb));
  const int max_key = range_end == 0 ? -1 : (int)((range_end - 1) >> 16);
  const int last_run = (range_end & 0xFFFF) == 0 ? 0x10000 : (int)(range_end & 0xFFFF);
  hipStream_t s = c->stream;
  const size_t ub = std::max<size_t>(1, std::min<size_t>(kMaxKeys, (size_t)(max_key + 1) + (size_t)na));
  if (!c->ornot_plan.p) CHK(c->ornot_plan.ensure(sizeof(OrNotPlan)));
  OutCtx oc;
  CHK(prepare_output(c, ub, A->payload_bytes + B->payload_bytes + (size_t)8194 * ub, &oc, false));
  c->pending_src = {ia, ib};
  c->mark(0);
  c->mark(1);
  launch_ornot(s, A->key_off.as<uint32_t>(), da, A->payload.as<uint8_t>(), na, B->key_off.as<uint32_t>(), db,
               B->payload.as<uint8_t>(), nb, max_key, last_run, flags, c->ornot_plan.as<OrNotPlan>(),
               c->wg_epoch.as<uint64_t>(), next_epoch(c), c->tasks.as<PTask>(), c->ntasks.as<uint32_t>(), oc, c->zlb,
               c->ztile, grid_for(ub, 65536));
  c->mark(2);
  defer_place(c);
  c->mark(3);
  HIPCHK(hipGetLastError());
  if (max_key < 0 && na == 0 && nb > 0) {
    OrNotPlan pl;
    HIPCHK(hipMemcpyAsync(&pl, c->ornot_plan.p, sizeof(pl), hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if (pl.neg) {
      c->last = 0;
      set_err("orNot: negative maxSize (the reference throws NegativeArraySizeException)");
      return RBG_ERR_ILLEGAL_ARGUMENT;
    }
  }
  return RBG_OK;
}

// static add / remove / flip(rb, rangeStart, rangeEnd) (RB/RoaringBitmap.java:298-345, 995-1040, 626-668;
// buf: MutableRoaringBitmap's, RB/buffer/MutableRoaringBitmap.java:152-205, 649-700, 455-505), rangemut.hip.
// rangeSanityCheck (:204-213); rangeEnd <= rangeStart gives a clone.  A run result above 2047 runs goes
// to the big-run arena; the arena is checked after the op and the op rerun once with the size the first
// pass reserved (as ctx_pairwise_buffer).
static int ctx_range_mut(Ctx* c, int op, int32_t ia, size_t ma, int64_t start, int64_t end, bool buf) {
  if (op < RMUT_ADD || (op > RMUT_ADD_INPLACE && op != RMUT_RANGE)) return RBG_ERR_ILLEGAL_ARGUMENT;
  if (start < 0 || start > 0xFFFFFFFFll || end < 0 || end > 0x100000000ll) {
    set_err("rangeStart=" + std::to_string(start) + " should be in [0, 0xffffffff], rangeEnd=" + std::to_string(end) +
            " in [0, 0xffffffff + 1]");
    return RBG_ERR_ILLEGAL_ARGUMENT;
  }
  Batch* A;
  CHK(get_batch(c, ia, &A));
  const uint16_t* ka;
  const CDesc* da;
  int na;
  CHK(operand(A, ma, &ka, &da, &na));
  RmutArgs ra{op, 1, 0, 0, 0};  // end <= start: no key in the range, every container cloned
  if (end > start) {  // (char) casts: Util.highbits / lowbits
    ra.hbs = (int)((uint64_t)start >> 16 & 0xFFFF);
    ra.lbs = (int)(start & 0xFFFF);
    ra.hbl = (int)((uint64_t)(end - 1) >> 16 & 0xFFFF);
    ra.lbl = (int)((end - 1) & 0xFFFF);
  }
  const size_t in_range = end > start ? (size_t)(ra.hbl - ra.hbs + 1) : 0;
  const size_t ub = std::max<size_t>(1, std::min<size_t>(kMaxKeys, (size_t)na + in_range));
  hipStream_t s = c->stream;
  if (!c->big_ctl.p) CHK(c->big_ctl.ensure(16));
  if (!c->big.p) CHK(c->big.ensure(16ull << 20));
  for (int attempt = 0;; attempt++) {
    OutCtx oc;
    CHK(prepare_output(c, ub, A->payload_bytes + (size_t)8194 * ub + c->big.cap, &oc, false));
    c->pending_src = {ia};
    c->mark(0);
    HIPCHK(hipMemsetAsync(c->big_ctl.p, 0, 16, s));
    c->mark(1);
    launch_rmut(s, A->key_off.as<uint32_t>(), da, A->payload.as<uint8_t>(), ra, buf, c->wg_epoch.as<uint64_t>(),
                next_epoch(c), c->tasks.as<PTask>(), c->ntasks.as<uint32_t>(), oc, c->zlb, c->ztile,
                BigRuns{c->big.as<uint8_t>(), c->big_ctl.as<unsigned long long>(), c->big.cap}, grid_for(ub, 65536));
    c->mark(2);
    defer_place(c);
    c->mark(3);
    HIPCHK(hipGetLastError());
    unsigned long long used[2] = {0, 0};
    HIPCHK(hipMemcpyAsync(used, c->big_ctl.p, 16, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if (!used[1]) return RBG_OK;
    if (attempt) {
      set_err("range add / remove: the run-container arena overflowed twice");
      return RBG_ERR_DEVICE;
    }
    CHK(c->big.ensure(used[0] + (used[0] >> 3) + 4096));
  }
}

// x.removeRunCompression() (RB/RoaringBitmap.java:2738-2749; the buffer package's alike): every run
// container through toBitmapOrArrayContainer (RB/RunContainer.java:2300-2323), the rest cloned; rangemut.hip
static int ctx_remove_run_compression(Ctx* c, int32_t ia, size_t ma) {
  Batch* A;
  CHK(get_batch(c, ia, &A));
  const uint16_t* ka;
  const CDesc* da;
  int na;
  CHK(operand(A, ma, &ka, &da, &na));
  const RmutArgs ra{RMUT_DERUN, 1, 0, 0, 0};
  const size_t ub = std::max<size_t>(1, (size_t)na);
  hipStream_t s = c->stream;
  OutCtx oc;
  CHK(prepare_output(c, ub, A->payload_bytes + (size_t)8194 * ub, &oc, false));
  c->pending_src = {ia};
  c->mark(0);
  c->mark(1);
  // RunContainer.toBitmapOrArrayContainer never makes a run container: no big-run arena (RMUT_DERUN's kernel
  // has no path to it)
  launch_rmut(s, A->key_off.as<uint32_t>(), da, A->payload.as<uint8_t>(), ra, false, c->wg_epoch.as<uint64_t>(),
              next_epoch(c), c->tasks.as<PTask>(), c->ntasks.as<uint32_t>(), oc, c->zlb, c->ztile,
              BigRuns{nullptr, nullptr, 0}, grid_for(ub, 65536));
  c->mark(2);
  defer_place(c);
  c->mark(3);
  HIPCHK(hipGetLastError());
  return RBG_OK;
}

// RoaringBitmap.addOffset(x, offset) (RB/RoaringBitmap.java:230-288; MutableRoaringBitmap.addOffset,
// RB/buffer/MutableRoaringBitmap.java:84-142, the same bytes), addoffset.hip.  The container offset is
// the floor of offset / 65536 (:233-234); outside [-65536, 65535] the result is empty (:235-237).
static int ctx_add_offset(Ctx* c, int32_t ia, size_t ma, int64_t offset) {
  Batch* A;
  CHK(get_batch(c, ia, &A));
  const uint16_t* ka;
  const CDesc* da;
  int na;
  CHK(operand(A, ma, &ka, &da, &na));
  const int64_t co = offset < 0 ? (offset - 65535) / 65536 : offset / 65536;
  AoffArgs aa{0, 0, 1};
  if (co >= -65536 && co < 65536) aa = AoffArgs{(int)co, (int)(offset - co * 65536), 0};
  // each input container gives at most two output containers, each staged (<= 8194 B) or a clone
  const size_t ub = std::max<size_t>(1, std::min<size_t>(kMaxKeys, 2 * (size_t)na));
  hipStream_t s = c->stream;
  OutCtx oc;
  CHK(prepare_output(c, ub, A->payload_bytes + (size_t)8194 * ub, &oc, false));
  c->pending_src = {ia};
  c->mark(0);
  c->mark(1);
  launch_aoff(s, A->key_off.as<uint32_t>(), da, A->payload.as<uint8_t>(), aa, c->wg_epoch.as<uint64_t>(),
              next_epoch(c), c->tasks.as<PTask>(), c->ntasks.as<uint32_t>(), oc, c->zlb, c->ztile,
              grid_for(ub, 65536));
  c->mark(2);
  defer_place(c);
  c->mark(3);
  HIPCHK(hipGetLastError());
  return RBG_OK;
}

static int ctx_pairwise(Ctx* c, int op, int32_t ia, size_t ma, int32_t ib, size_t mb, bool card_only, int key_lo = 0,
                        int key_hi = kMaxKeys, int pipe_k = 0) {
  if (op == RBG_AND_BUFFER || op == RBG_ANDNOT_BUFFER) {
    if (card_only) return RBG_ERR_ILLEGAL_ARGUMENT;
    return ctx_pairwise_buffer(c, op == RBG_AND_BUFFER ? OP_AND : OP_ANDNOT, ia, ma, ib, mb, key_lo, key_hi);
  }
  if (op == RBG_OR_INPLACE && !card_only) {
    CHK(ctx_pairwise(c, OP_OR, ia, ma, ib, mb, false, key_lo, key_hi));
    if (!c->ones.p) {
      CHK(c->ones.ensure(8192));
      HIPCHK(hipMemsetAsync(c->ones.p, 0xFF, 8192, c->stream));
    }
    Batch *A, *B;
    CHK(get_batch(c, ia, &A));
    CHK(get_batch(c, ib, &B));
    launch_ior_fix(c->stream, c->ntasks.as<uint32_t>(), c->recs.as<ORec>(), A->key_off.as<uint32_t>(),
                   A->desc.as<CDesc>(), B->key_off.as<uint32_t>(), B->desc.as<CDesc>(), c->ones.as<uint8_t>());
    HIPCHK(hipGetLastError());
    c->agg_ok = false;  // k_ior_fix changed records after the compute kernel summed them
    return RBG_OK;
  }
  if (op < 0 || op > 3) return RBG_ERR_ILLEGAL_ARGUMENT;
  key_lo = std::max(0, key_lo);
  key_hi = std::min(kMaxKeys, key_hi);
  Batch *A, *B;
  CHK(get_batch(c, ia, &A));
  CHK(get_batch(c, ib, &B));
  const uint16_t *ka, *kb;
  const CDesc *da, *db;
  int na, nb;
  CHK(operand(A, ma, &ka, &da, &na));
  CHK(operand(B, mb, &kb, &db, &nb));
  hipStream_t s = c->stream;
  const int plan_op = card_only ? OP_AND : op;
  size_t ub;
  switch (plan_op) {
    case OP_AND: ub = std::min(na, nb); break;
    case OP_ANDNOT: ub = na; break;
    default: ub = std::min<size_t>((size_t)na + nb, kMaxKeys); break;
  }
  // Dense key ranges (the op's task bound covers at least half of the range) skip the plan
  // launch: the compute kernel takes key key_lo + t as task t and resolves it itself (one
  // record and scratch slot per key of the range).  Sparse ones are planned and compacted
  // first, so the kernel sees only keys with work.  RBG_PAIRWISE_PLAN=1 always plans.
  static const bool force_plan = getenv("RBG_PAIRWISE_PLAN") != nullptr;
  const size_t nkeys = key_hi > key_lo ? (size_t)(key_hi - key_lo) : 0;
  const bool direct = nkeys > 0 && 2 * ub >= nkeys && !force_plan;
  OutCtx oc;
  CHK(prepare_output(c, direct ? std::max(ub, nkeys) : ub, A->payload_bytes + B->payload_bytes + (size_t)8194 * ub,
                     &oc, card_only));
  c->pending_src = {ia, ib};
  c->mark(0);
  PwDirect pd{A->key_off.as<uint32_t>(), da, B->key_off.as<uint32_t>(), db, key_lo, (uint32_t)nkeys,
              c->ntasks.as<uint32_t>(), c->zlb, c->ztile, (uint32_t)nkeys};
  if (direct && pipe_k > 1 && !card_only) return pairwise_pipelined(c, op, pipe_k, pd, A, B, oc);
  if (!direct) {
    launch_plan_pairwise(s, plan_op, key_lo, key_hi, A->key_off.as<uint32_t>(), da, A->payload.as<uint8_t>(),
                         B->key_off.as<uint32_t>(), db, B->payload.as<uint8_t>(), c->wg_epoch.as<uint64_t>(),
                         next_epoch(c), c->tasks.as<PTask>(), c->ntasks.as<uint32_t>(), c->zlb, c->ztile, oc.err);
    dbg(s, "plan");
  }
  // dense ranges: tasks binned by estimated cost so every wave draws the same mix (k_plan_balanced;
  // RBG_PW_BALANCE=0: the direct form, tasks in key order)
  const char* bal_env = getenv("RBG_PW_BALANCE");
  const bool balanced = direct && (!bal_env || atoi(bal_env) != 0);
  // ... run by one 16-wave workgroup per CU that claims the CU's tasks through LDS (k_pair_cu)
  if (balanced)
    launch_plan_balanced(s, plan_op, card_only ? 1 : 0, key_lo, (uint32_t)nkeys, A->key_off.as<uint32_t>(), da,
                         A->payload.as<uint8_t>(), B->key_off.as<uint32_t>(), db, B->payload.as<uint8_t>(),
                         c->tasks.as<PTask>(), c->ntasks.as<uint32_t>(), oc, c->task_card.as<uint32_t>(), c->zlb,
                         c->ztile);
  c->mark(1);
  // the compute kernel sums its kept results per tile for the serialization (k_serialize_agg) when a
  // plan kernel has zeroed the sums first: the balanced (dense) and planned (sparse) forms; the direct
  // form zeroes inside the compute kernel itself
  if (!card_only && (balanced || !direct)) {
    oc.tile_agg = reinterpret_cast<unsigned long long*>(oc.tile_status + 2 * kMaxTiles);
    c->pending.tile_agg = oc.tile_agg;
    c->agg_ok = true;
  }
  // 4 waves (tasks) per workgroup, clamped to the resident grid
  const int grid = grid_for(((direct ? nkeys : ub) + 3) / 4, 16384);
  launch_pairwise(s, op, card_only ? 1 : 0, grid, c->tasks.as<PTask>(), c->ntasks.as<uint32_t>(),
                  A->payload.as<uint8_t>(), B->payload.as<uint8_t>(), oc, c->task_card.as<uint32_t>(),
                  direct ? &pd : nullptr, balanced);
  dbg(s, "pairwise");
  c->mark(2);
  if (card_only) {
    launch_reduce_card(s, c->task_card.as<uint32_t>(), c->ntasks.as<uint32_t>(), c->info.as<ResultInfo>(), oc.err);
    c->last = 2;
  } else {
    defer_place(c);
  }
  c->mark(3);
  HIPCHK(hipGetLastError());
  return RBG_OK;
}

static int batch_host_index(Ctx* c, Batch* b);

// Chain order of horizontal_or / horizontal_xor (RB/FastAggregation.java:124-289): the
// reference drains a java.util.PriorityQueue of one container pointer per bitmap, ordered
// by key, then larger cardinality first (RB/RoaringArray.java:708-713), with the heap's own
// tie order.  The heap is replayed here over the container table (keys and cardinalities
// only -- no payload); order[key_off[k] + j] = the j-th container of key k's chain.
namespace {
struct HPtr {
  uint32_t bm, i, key, card, pos;
};
static int hcmp(const HPtr& x, const HPtr& y) {  // ContainerPointer.compareTo
  if (x.key != y.key) return (int)x.key - (int)y.key;
  return (int)y.card - (int)x.card;
}
struct JHeap {  // java.util.PriorityQueue siftUp / siftDown (OpenJDK)
  std::vector<HPtr> q;
  void add(const HPtr& x) {
    size_t k = q.size();
    q.push_back(x);
    while (k > 0) {
      const size_t p = (k - 1) >> 1;
      if (hcmp(x, q[p]) >= 0) break;
      q[k] = q[p];
      k = p;
    }
    q[k] = x;
  }
  HPtr poll() {
    const HPtr r = q[0];
    const HPtr x = q.back();
    q.pop_back();
    const size_t n = q.size();
    if (n) {
      size_t k = 0;
      const size_t half = n >> 1;
      while (k < half) {
        size_t ch = 2 * k + 1;
        if (ch + 1 < n && hcmp(q[ch], q[ch + 1]) > 0) ch++;
        if (hcmp(x, q[ch]) <= 0) break;
        q[k] = q[ch];
        k = ch;
      }
      q[k] = x;
    }
    return r;
  }
};
}  // namespace

// *identity: the chain order is the batch's own (no key needed sorting): no order table
static int horizontal_order(Ctx* c, Batch* B, bool* identity) {
  *identity = B->h_chain_identity;
  if (*identity) return RBG_OK;
  CHK(batch_host_index(c, B));
  std::vector<uint32_t> order;
  // Within a key the heap pops by larger cardinality first; only equal cardinalities pop in
  // the heap's tie order, which depends on everything polled before.  The chain's order
  // matters only at keys holding a run container (the wide kernel types run-free keys from
  // the result alone, wide.hip), so unless such a key has two containers of equal
  // cardinality the order is the per-key sort by cardinality and the replay is skipped.
  if (B->key_major || B->n_bm == 1) {
    const std::vector<CDesc>& D = B->h_desc;
    const size_t n = B->n_ctr;
    std::vector<std::pair<uint32_t, uint32_t>> rkeys;  // segments of keys holding a run container
    std::vector<uint32_t> seg;
    bool tie = false;
    for (size_t p = 0; p < n && !tie;) {
      size_t e = p;
      bool has_r = false;
      while (e < n && D[e].key == D[p].key) has_r |= D[e++].kind == DK_R;
      if (has_r && e - p > 1) {
        seg.resize(e - p);
        for (size_t q = p; q < e; q++) seg[q - p] = D[q].card;
        std::sort(seg.begin(), seg.end());
        tie = std::adjacent_find(seg.begin(), seg.end()) != seg.end();
        rkeys.emplace_back((uint32_t)p, (uint32_t)e);
      }
      p = e;
    }
    if (!tie && rkeys.empty()) {
      *identity = B->h_chain_identity = true;
      return RBG_OK;
    }
    if (!tie) {
      order.resize(n);
      for (size_t q = 0; q < n; q++) order[q] = (uint32_t)q;
      for (const auto& pe : rkeys)
        std::sort(order.begin() + pe.first, order.begin() + pe.second,
                  [&](uint32_t x, uint32_t y) { return D[x].card > D[y].card; });
      CHK(c->order.ensure(4 * std::max<size_t>(n, 1)));
      if (n) HIPCHK(hipMemcpyAsync(c->order.p, order.data(), 4 * n, hipMemcpyHostToDevice, c->stream));
      HIPCHK(hipStreamSynchronize(c->stream));  // `order` is a stack vector
      return RBG_OK;
    }
    order.clear();
  }
  order.reserve(B->n_ctr);
  auto ptr = [&](uint32_t bm, uint32_t i) {
    const uint32_t pos = B->h_pos[B->h_pos_off[bm] + i];
    const CDesc& d = B->h_desc[pos];
    return HPtr{bm, i, d.key, d.card, pos};
  };
  auto has = [&](uint32_t bm, uint32_t i) { return B->h_pos_off[bm] + i < B->h_pos_off[bm + 1]; };
  JHeap pq;
  for (uint32_t b = 0; b < B->n_bm; b++)
    if (has(b, 0)) pq.add(ptr(b, 0));
  auto advance_add = [&](const HPtr& x) {
    if (has(x.bm, x.i + 1)) pq.add(ptr(x.bm, x.i + 1));
  };
  while (!pq.q.empty()) {
    const HPtr x1 = pq.poll();
    order.push_back(x1.pos);
    if (pq.q.empty() || pq.q[0].key != x1.key) {
      advance_add(x1);
      continue;
    }
    const HPtr x2 = pq.poll();
    order.push_back(x2.pos);
    while (!pq.q.empty() && pq.q[0].key == x1.key) {
      const HPtr x = pq.poll();
      order.push_back(x.pos);
      if (has(x.bm, x.i + 1)) pq.add(ptr(x.bm, x.i + 1));
      else if (pq.q.empty()) break;
    }
    advance_add(x1);
    advance_add(x2);
  }
  if (order.size() != B->n_ctr) {
    set_err("horizontal order: container table inconsistent");
    return RBG_ERR_DEVICE;
  }
  CHK(c->order.ensure(4 * std::max<size_t>(order.size(), 1)));
  if (!order.empty())
    HIPCHK(hipMemcpyAsync(c->order.p, order.data(), 4 * order.size(), hipMemcpyHostToDevice, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));  // `order` is a stack vector
  return RBG_OK;
}

// FastAggregation.priorityqueue_or / priorityqueue_xor (RB/FastAggregation.java:677-812).
// The reference keeps a java.util.PriorityQueue of bitmaps ordered by
// (int)(sizes[a] - sizes[b]) over getLongSizeInBytes.  The host adds the inputs and plans
// the first step; the queue then runs on the device (pq.hip): N - 1 step launches, each
// planning the next, with no host read-back in between.
namespace {
// host side of the queue for the first step (same operations as pq.hip's PQWave)
struct PQHost {
  std::vector<PQEnt>& heap;
  std::vector<int32_t>& nodes;
  std::vector<uint8_t>& tmp;
  std::vector<int32_t>& slots;
  void add(PQStep& c, PQEnt x) {  // OpenJDK PriorityQueue.siftUp
    int k = c.heap_n++;
    while (k > 0) {
      const int p = (k - 1) >> 1;
      if (pq_cmp(x.size, heap[p].size) >= 0) break;
      heap[k] = heap[p];
      k = p;
    }
    heap[k] = x;
  }
  PQEnt poll(PQStep& c) {  // PriorityQueue.poll + siftDown
    const PQEnt r = heap[0];
    const int n = --c.heap_n;
    if (n == 0) return r;
    const PQEnt x = heap[n];
    int k = 0;
    const int half = n >> 1;
    while (k < half) {
      int ch = 2 * k + 1;
      if (ch + 1 < n && pq_cmp(heap[ch].size, heap[ch + 1].size) > 0) ch++;
      if (pq_cmp(x.size, heap[ch].size) <= 0) break;
      heap[k] = heap[ch];
      k = ch;
    }
    heap[k] = x;
    return r;
  }
  int32_t node(int i) { return nodes[i]; }
  void set_node(int i, int32_t v) { nodes[i] = v; }
  bool istmp(int i) { return tmp[i] != 0; }
  void set_istmp(int i) { tmp[i] = 1; }
  int slot_pop(PQStep& c) { return slots[--c.slot_top]; }
  void slot_push(PQStep& c, int s) { slots[c.slot_top++] = s; }
};
}  // namespace

static int ctx_pq(Ctx* c, int op, Batch* B, int32_t id, int key_lo, int key_hi) {
  if (key_lo != 0 || key_hi != kMaxKeys) {
    set_err("priorityqueue aggregations need the full key range (the queue order depends on every key)");
    return RBG_ERR_ILLEGAL_ARGUMENT;
  }
  hipStream_t s = c->stream;
  const size_t N = B->n_bm;
  const size_t ub = std::min<size_t>(kMaxKeys, std::max<size_t>(B->n_ctr, 1));
  OutCtx oc;
  CHK(prepare_output(c, ub, (size_t)8194 * ub + B->max_ser, &oc, false));
  c->pending_src = {id};
  c->mark(0);
  // one task per union key (an empty aggregate has none: new RoaringBitmap())
  launch_plan_wide(s, N ? 0 : 1, B->key_off.as<uint32_t>(), N ? (uint32_t)N : 0xFFFFFFFFu, 0, kMaxKeys,
                   c->by_key.as<Task>(), c->flag.as<uint8_t>(), c->wg_count.as<uint32_t>(), c->zlb, c->ztile);
  launch_compact(s, c->flag.as<uint8_t>(), c->by_key.as<Task>(), c->wg_count.as<uint32_t>(), c->tasks.as<Task>(),
                 c->ntasks.as<uint32_t>());
  c->mark(1);
  if (!N) {
    c->mark(2);
    launch_place(s, c->ntasks.as<uint32_t>(), oc, c->info.as<ResultInfo>());
    c->last = 1;
    c->mark(3);
    HIPCHK(hipGetLastError());
    return RBG_OK;
  }
  uint32_t h_nt = 0;
  HIPCHK(hipMemcpyAsync(&h_nt, c->ntasks.p, 4, hipMemcpyDeviceToHost, s));
  std::vector<unsigned long long> leaf(N);
  DevBuf dsz;
  CHK(dsz.ensure(8 * N));
  HIPCHK(hipMemsetAsync(dsz.p, 0, 8 * N, s));
  launch_pq_leaf_sizes(s, B->desc.as<CDesc>(), B->bm.as<uint32_t>(), B->payload.as<uint8_t>(), B->n_ctr,
                       dsz.as<unsigned long long>());
  HIPCHK(hipMemcpyAsync(leaf.data(), dsz.p, 8 * N, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));

  // Temps: at most N/2 + 1 are live at once (every priorityqueue_or temp starts from two
  // inputs; a priorityqueue_xor step allocates one while its operands are still queued).
  // Each has one 16 B state per union key; containers that are not input clones live in
  // 8 KiB arena blocks from the key's own pool: floor(n_t / 2) blocks for a key held by
  // n_t inputs (pq.hip), at most half the batch's containers in all.
  const size_t n_slots = N / 2 + 2;
  const size_t stride = std::max<uint32_t>(h_nt, 1);
  const size_t st_bytes = n_slots * stride * sizeof(PQState);
  std::vector<Task> h_tasks(h_nt);
  if (h_nt) HIPCHK(hipMemcpyAsync(h_tasks.data(), c->tasks.p, sizeof(Task) * h_nt, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  std::vector<uint32_t> kbase(stride, 0);
  std::vector<int32_t> ktop(stride, 0);
  size_t free_b = 0, total_b = 0;
  pool_clear(c);  // pooled buffers would count as used
  HIPCHK(hipMemGetInfo(&free_b, &total_b));
  const size_t budget = free_b / 10 * 9;
  // pools of floor(n_t / 2) blocks never run out; when they do not all fit, every pool is
  // capped at the largest size that fits (a key that needs more ends the op with
  // RBG_ERR_OUT_OF_MEMORY, as a full arena did)
  auto pool_blocks = [&](int32_t cap) {
    size_t n = 0;
    for (uint32_t t = 0; t < h_nt; t++) n += (size_t)std::min(h_tasks[t].b / 2, cap);
    return n;
  };
  int32_t cap = 0;
  for (uint32_t t = 0; t < h_nt; t++) cap = std::max(cap, h_tasks[t].b / 2);
  if (st_bytes + pool_blocks(cap) * 8192 > budget) {
    int32_t lo = 0, hi = cap;  // the largest cap that fits
    while (lo < hi) {
      const int32_t mid = lo + (hi - lo + 1) / 2;
      if (st_bytes + pool_blocks(mid) * 8192 <= budget) lo = mid;
      else hi = mid - 1;
    }
    if (lo < 1 && cap >= 1) {
      set_err("priorityqueue: " + std::to_string(n_slots) + " temps x " + std::to_string(stride) +
              " union keys need more than the free device memory; use FastAggregation.or / xor");
      return RBG_ERR_OUT_OF_MEMORY;
    }
    cap = lo;
  }
  size_t n_blk = 0;
  for (uint32_t t = 0; t < h_nt; t++) {
    kbase[t] = (uint32_t)n_blk;
    ktop[t] = std::min(h_tasks[t].b / 2, cap);
    n_blk += (size_t)ktop[t];
  }
  n_blk = std::max<size_t>(n_blk, 1);
  // host: add every input, plan the first step
  std::vector<PQEnt> heap(N);
  std::vector<int32_t> nodes(2 * N);
  std::vector<uint8_t> tmp(2 * N, 0);
  std::vector<int32_t> slots(n_slots);
  for (size_t k = 0; k < N; k++) nodes[k] = (int32_t)k;
  for (size_t k = 0; k < n_slots; k++) slots[k] = (int32_t)(n_slots - 1 - k);
  PQCtl ctl{};
  ctl.step.or_mode = op == RBG_WIDE_PQ_OR;
  ctl.step.n_nodes = (int32_t)N;
  ctl.step.slot_top = (int32_t)n_slots;
  ctl.step.rel1 = ctl.step.rel2 = -1;
  PQHost hm{heap, nodes, tmp, slots};
  for (size_t k = 0; k < N; k++) hm.add(ctl.step, PQEnt{8 + (int64_t)leaf[k], (int32_t)k, 0});
  pq_plan(hm, ctl.step);
  // Block ids level-major: pool position j of key t is block lvl[j] + rank[t], with the keys
  // ranked by pool size (largest first, stable), so level j holds the keys with more than j
  // blocks contiguously.  Keys pop their positions 0, 1, ... in order, so the workgroups of
  // neighbouring keys write neighbouring blocks (uniform data: one contiguous level per
  // step instead of blocks a pool apart).
  std::vector<uint32_t> order(h_nt);
  for (uint32_t t = 0; t < h_nt; t++) order[t] = t;
  std::stable_sort(order.begin(), order.end(), [&](uint32_t x, uint32_t y) { return ktop[x] > ktop[y]; });
  std::vector<uint32_t> rank(h_nt);
  for (uint32_t i = 0; i < h_nt; i++) rank[order[i]] = i;
  const int32_t max_cap = h_nt ? ktop[order[0]] : 0;
  std::vector<size_t> lvl(max_cap + 1, 0);
  for (int32_t j = 0, i = (int32_t)h_nt; j < max_cap; j++) {  // keys with more than j blocks: the first i
    while (i > 0 && ktop[order[i - 1]] <= j) i--;
    lvl[j + 1] = lvl[j] + (size_t)i;
  }
  std::vector<int32_t> stack(n_blk);
  for (uint32_t t = 0; t < h_nt; t++)
    for (int32_t i = 0; i < ktop[t]; i++) stack[kbase[t] + i] = (int32_t)(lvl[ktop[t] - 1 - i] + rank[t]);
  // device copies
  auto al = [](size_t x) { return (x + 255) & ~(size_t)255; };
  const size_t o_heap = al(sizeof(PQCtl)), o_node = o_heap + al(16 * N), o_tmp = o_node + al(8 * N),
               o_slots = o_tmp + al(2 * N), o_stack = o_slots + al(4 * n_slots), o_base = o_stack + al(4 * n_blk),
               o_top = o_base + al(4 * stride), o_end = o_top + al(4 * stride);
  DevBuf meta, states, arena;
  CHK(meta.ensure(o_end));
  CHK(states.ensure(st_bytes));
  CHK(arena.ensure(n_blk * 8192));
  uint8_t* mb = meta.as<uint8_t>();
  HIPCHK(hipMemcpyAsync(mb, &ctl, sizeof(ctl), hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(mb + o_heap, heap.data(), 16 * N, hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(mb + o_node, nodes.data(), 8 * N, hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(mb + o_tmp, tmp.data(), 2 * N, hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(mb + o_slots, slots.data(), 4 * n_slots, hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(mb + o_stack, stack.data(), 4 * n_blk, hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(mb + o_base, kbase.data(), 4 * stride, hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(mb + o_top, ktop.data(), 4 * stride, hipMemcpyHostToDevice, s));
  const PQDev D{reinterpret_cast<PQCtl*>(mb), reinterpret_cast<PQEnt*>(mb + o_heap),
                reinterpret_cast<int32_t*>(mb + o_node), mb + o_tmp, reinterpret_cast<int32_t*>(mb + o_slots),
                states.as<PQState>(), stride, arena.as<uint64_t>(), reinterpret_cast<int32_t*>(mb + o_stack),
                reinterpret_cast<const uint32_t*>(mb + o_base), reinterpret_cast<int32_t*>(mb + o_top)};
  const PQArgs pa{B->desc.as<CDesc>(), B->bm.as<uint32_t>(), B->payload.as<uint8_t>()};
  const int grid = grid_for(h_nt, 65536);
  for (size_t k = 0; k + 1 < N; k++) {
    launch_pq_step(s, grid, c->tasks.as<Task>(), c->ntasks.as<uint32_t>(), pa, D);
    if ((k & 1023) == 1023) HIPCHK(hipGetLastError());
  }
  c->mark(2);
  launch_pq_final(s, grid, c->tasks.as<Task>(), c->ntasks.as<uint32_t>(), pa, op == RBG_WIDE_PQ_OR ? 1 : 0, D, oc);
  HIPCHK(hipGetLastError());
  launch_place(s, c->ntasks.as<uint32_t>(), oc, c->info.as<ResultInfo>());
  PQCtl done{};
  HIPCHK(hipMemcpyAsync(&done, mb, sizeof(done), hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));  // the temps are freed on return
  if (done.err || !done.step.final_step) {
    set_err(done.err ? "priorityqueue: a key's block pool ran out (" + std::to_string(n_blk) + " x 8 KiB in all)"
                     : std::string("priorityqueue: the device queue did not finish"));
    return done.err ? RBG_ERR_OUT_OF_MEMORY : RBG_ERR_DEVICE;
  }
  c->last = 1;
  c->mark(3);
  HIPCHK(hipGetLastError());
  return RBG_OK;
}

// FastAggregation dispatch (RB/FastAggregation.java:26-101,653-666,823-836)
// start_override >= 0: naive_and starts from that input (key-range shards pass the
// input with the fewest containers over the WHOLE universe, RB/FastAggregation.java:333-339)
// Wide ops whose kernels read array payloads at any 2 B alignment (a packed batch): every op that runs
// the per-key OR / XOR kernels or workShyAnd (k_wide, k_shy_wave, and the queue / horizontal / parallel
// forms, which reduce to them on a batch without run containers).  naive_and's chains (N <= 10, the
// Iterator forms, the buffer package's and chains) materialise through the slot-aligned helpers.
static bool wide_reads_packed(int op, size_t n) {
  switch (op) {
    case RBG_WIDE_OR:
    case RBG_WIDE_XOR:
    case RBG_WIDE_WORKSHY_AND:
    case RBG_WIDE_PARALLEL_OR:
    case RBG_WIDE_PARALLEL_XOR:
    case RBG_WIDE_BUFFER_OR_MUTABLE:
    case RBG_WIDE_HORIZONTAL_OR:
    case RBG_WIDE_HORIZONTAL_XOR:
    case RBG_WIDE_PQ_OR:
    case RBG_WIDE_PQ_XOR: return true;
    case RBG_WIDE_AND: return n > 10;  // FastAggregation.and: workShyAnd above 10 inputs (RB/FastAggregation.java:38)
    default: return false;
  }
}

static int ctx_wide(Ctx* c, int op, int32_t id, int key_lo, int key_hi, const int32_t* ids, bool card_only,
                    int* host_card_out, bool* host_card_valid, int32_t start_override = -1) {
  Batch* B;
  CHK(get_batch(c, id, &B));
  if (!B->key_major) {
    set_err("wide ops need a key-major batch");
    return RBG_ERR_ILLEGAL_ARGUMENT;
  }
  if (B->packed && !card_only && !wide_reads_packed(op, B->n_bm)) {
    set_err("this wide op needs slot-aligned payloads (load the batch without packing)");
    return RBG_ERR_ILLEGAL_ARGUMENT;
  }
  key_lo = std::max(0, key_lo);
  key_hi = std::min(kMaxKeys, key_hi);
  *host_card_valid = false;
  if (!card_only && (op == RBG_WIDE_PQ_OR || op == RBG_WIDE_PQ_XOR)) {
    // Without run containers the queue's order cannot show in the bytes: every container of
    // its algebra ends BY_CARD of its set (pq.hip: lazy bitmaps are repaired to BY_CARD or
    // RunContainer.full; an exact bitmap only comes from an input bitmap, over 4096 values;
    // an array from ArrayContainer.lazyor holds at most 1024; the pairwise XOR types are
    // BY_CARD), and a key held by one input is that input's container, as in naive_or /
    // naive_xor, which then give the same bytes.
    if (B->n_kind[DK_R] != 0 || key_lo != 0 || key_hi != kMaxKeys) return ctx_pq(c, op, B, id, key_lo, key_hi);
    op = op == RBG_WIDE_PQ_OR ? RBG_WIDE_OR : RBG_WIDE_XOR;
  }
  // BufferFastAggregation's and chains: the heap forms' dispatch, with the buffer package's run AND run
  bool buffer = false;
  if (!card_only && op >= RBG_WIDE_BUFFER_AND && op <= RBG_WIDE_BUFFER_AND_ITER) {
    buffer = true;
    op = op == RBG_WIDE_BUFFER_AND ? RBG_WIDE_AND : op == RBG_WIDE_BUFFER_NAIVE_AND ? RBG_WIDE_NAIVE_AND : RBG_WIDE_AND_ITER;
  }
  hipStream_t s = c->stream;
  const size_t N = B->n_bm;
  int mode = WIDE_OR, plan_mode = 0;
  uint32_t start_bm = 0, chain = 0;
  const uint32_t* order = nullptr;
  std::vector<uint8_t> skip;
  if (card_only) {
    // andCardinality: 0 -> 0, 1 -> card, >= 2 -> per-key AND sum (== andCardinality / workShyAndCardinality)
    // orCardinality : 0 -> 0, 1 -> card, >= 2 -> per-key OR sum (== orCardinality / horizontalOrCardinality)
    if (op != RBG_WIDE_CARD_AND && op != RBG_WIDE_CARD_OR) return RBG_ERR_ILLEGAL_ARGUMENT;
    const bool full_range = key_lo == 0 && key_hi == kMaxKeys;
    if (N == 0 || (N == 1 && full_range)) {
      const int64_t cc = N ? B->h_bm_card[0] : 0;
      *host_card_out = (int32_t)(uint32_t)(uint64_t)cc;
      *host_card_valid = true;
      c->last = 2;
      return RBG_OK;
    }
    if (op == RBG_WIDE_CARD_AND && N >= 2) {
      mode = WIDE_AND_SHY_CARD;
      plan_mode = 1;
    } else {
      mode = WIDE_OR_CARD;  // also a single input restricted to a key range
    }
  } else {
    switch (op) {
      case RBG_WIDE_OR: mode = WIDE_OR; break;
      case RBG_WIDE_XOR: mode = WIDE_XOR; break;
      case RBG_WIDE_AND:
      case RBG_WIDE_AND_ITER:
      case RBG_WIDE_NAIVE_AND:
      case RBG_WIDE_WORKSHY_AND:
        plan_mode = 1;
        if (op == RBG_WIDE_WORKSHY_AND && N == 0) {
          set_err("workShyAnd needs at least one bitmap");  // bitmaps[0] on an empty array
          return RBG_ERR_ILLEGAL_ARGUMENT;
        }
        if ((op == RBG_WIDE_AND && N > 10) || op == RBG_WIDE_WORKSHY_AND) {
          mode = WIDE_AND_SHY;
        } else {
          mode = WIDE_AND_NAIVE;
          skip.assign(std::max<size_t>(N, 1), 0);
          if (op != RBG_WIDE_AND_ITER) {
            // the input with the fewest containers, first on ties (:333-339)
            if (start_override >= 0 && (size_t)start_override < N) {
              start_bm = (uint32_t)start_override;
            } else {
              for (size_t i = 1; i < N; i++)
                if (B->h_bm_nctr[i] < B->h_bm_nctr[start_bm]) start_bm = (uint32_t)i;
            }
            for (size_t i = 0; i < N; i++)
              skip[i] = (i == start_bm) || (ids && ids[i] == ids[start_bm]);  // :341 identity skip
          } else {
            start_bm = 0;  // naive_and(Iterator): clone of the first input, :309-313
            skip[0] = 1;
          }
        }
        break;
      case RBG_WIDE_PARALLEL_OR: mode = WIDE_LAZY_CHAIN; chain = kChainLimit16; break;
      case RBG_WIDE_PARALLEL_XOR: mode = WIDE_XOR_CHAIN; break;
      case RBG_WIDE_BUFFER_OR_MUTABLE: mode = WIDE_LAZY_CHAIN; break;
      case RBG_WIDE_HORIZONTAL_OR:
      case RBG_WIDE_HORIZONTAL_XOR:
        mode = op == RBG_WIDE_HORIZONTAL_OR ? WIDE_LAZY_CHAIN : WIDE_XOR_CHAIN;
        chain = op == RBG_WIDE_HORIZONTAL_OR ? kChainN1Clone : kChainKeepEmpty;
        bool identity;
        CHK(horizontal_order(c, B, &identity));
        order = identity ? nullptr : c->order.as<uint32_t>();
        break;
      default: return RBG_ERR_ILLEGAL_ARGUMENT;
    }
  }
  if (N == 0) {
    // empty aggregate: empty bitmap (:329-331 for and; naive_or/xor of nothing)
    plan_mode = 2;
  }
  // the buffer naive_and chain may keep run containers of more than 2047 runs: they go to the
  // big-run arena, checked after the op (rerun once with the size the first pass reserved)
  const bool big_runs = buffer && mode == WIDE_AND_NAIVE && N > 0;
  if (big_runs) {
    if (!c->big_ctl.p) CHK(c->big_ctl.ensure(16));
    if (!c->big.p) CHK(c->big.ensure(16ull << 20));
  }
  for (int attempt = 0;; attempt++) {
    const size_t ub = std::min<size_t>(kMaxKeys, std::max<size_t>(B->n_ctr, 1));
    OutCtx oc;
    // each result container is staged (<= 8194 B) or a clone of one input container
    CHK(prepare_output(c, ub, (size_t)8194 * ub + B->max_ser + (big_runs ? c->big.cap : 0), &oc, card_only));
    // OR results are bitmaps whenever more than 4096 values survive: write those in place
    // (8192 t < 8194 ub, inside the payload region)
    if (!card_only && (mode == WIDE_OR || mode == WIDE_LAZY_CHAIN)) oc.spec = c->pending.spec = 1;
    c->pending_src = {id};
    if (!skip.empty()) {
      CHK(c->skip.ensure(skip.size()));
      HIPCHK(hipMemcpyAsync(c->skip.p, skip.data(), skip.size(), hipMemcpyHostToDevice, s));
    }
    const uint32_t n_req = plan_mode == 2 ? 0xFFFFFFFFu : (uint32_t)N;
    c->mark(0);
    launch_plan_wide(s, plan_mode == 0 ? 0 : 1, B->key_off.as<uint32_t>(), n_req, key_lo, key_hi,
                     c->by_key.as<Task>(), c->flag.as<uint8_t>(), c->wg_count.as<uint32_t>(), c->zlb, c->ztile);
    launch_compact(s, c->flag.as<uint8_t>(), c->by_key.as<Task>(), c->wg_count.as<uint32_t>(), c->tasks.as<Task>(),
                   c->ntasks.as<uint32_t>());
    WideArgs wa{};
    wa.desc = B->desc.as<CDesc>();
    wa.bm = B->bm.as<uint32_t>();
    wa.payload = B->payload.as<uint8_t>();
    wa.skip = skip.empty() ? nullptr : c->skip.as<uint8_t>();
    wa.start_bm = start_bm;
    // (the all-array path streams a key's slots as one run of values: they must be back to back)
    wa.all_array = (B->n_kind[DK_B] == 0 && B->n_kind[DK_R] == 0 && !B->gapped) ? 1u : 0u;
    wa.slot32 = B->payload_bytes < (1ull << 36) ? 1u : 0u;
    wa.order = order;
    wa.chain = chain;
    wa.rd_bytes = c->prof_cap > 0 && c->rd_ctr.p ? c->rd_ctr.as<unsigned long long>() : nullptr;
    wa.buffer = buffer ? 1u : 0u;
    if (big_runs) {
      HIPCHK(hipMemsetAsync(c->big_ctl.p, 0, 16, s));
      wa.big = BigRuns{c->big.as<uint8_t>(), c->big_ctl.as<unsigned long long>(), c->big.cap};
    }
    c->mark(1);
    launch_wide(s, mode, grid_for(ub, 65536), c->tasks.as<Task>(), c->ntasks.as<uint32_t>(), wa, oc,
                c->task_card.as<uint32_t>());
    c->mark(2);
    if (card_only) {
      launch_reduce_card(s, c->task_card.as<uint32_t>(), c->ntasks.as<uint32_t>(), c->info.as<ResultInfo>(), oc.err);
      c->last = 2;
    } else {
      defer_place(c);
    }
    c->mark(3);
    HIPCHK(hipGetLastError());
    if (!big_runs) break;
    unsigned long long used[2] = {0, 0};
    HIPCHK(hipMemcpyAsync(used, c->big_ctl.p, 16, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if (!used[1]) break;
    if (attempt) {
      set_err("naive_and: the run-container arena overflowed twice");
      return RBG_ERR_DEVICE;
    }
    CHK(c->big.ensure(used[0] + (used[0] >> 3) + 4096));  // the first pass counted every reservation
  }
  return RBG_OK;
}

// compareUsingMinMax (BSI/:515-579): 0 = run the circuit, 1 = all, 2 = empty
static int bsi_minmax(int op, int32_t s, int32_t e, int32_t lo, int32_t hi) {
  switch (op) {
    case BSI_LT: return s > hi ? 1 : s <= lo ? 2 : 0;
    case BSI_LE: return s >= hi ? 1 : s < lo ? 2 : 0;
    case BSI_GT: return s < lo ? 1 : s >= hi ? 2 : 0;
    case BSI_GE: return s <= lo ? 1 : s > hi ? 2 : 0;
    case BSI_EQ:
      if (lo == hi && lo == s) return 1;
      return (s < lo || s > hi) ? 2 : 0;
    case BSI_NEQ:
      if (lo == hi) return lo == s ? 2 : 1;
      return 0;
    case BSI_RANGE:
      if (s <= lo && e >= hi) return 1;
      return (s > hi || e < lo) ? 2 : 0;
    default: return 0;
  }
}

// RoaringBitmapSliceIndex.compare (BSI/:482-513) and / or sum (BSI/:581-592) over a
// key-major batch [ebM, bA[0..nbits-1], foundSet?]; the result is materialised like a
// wide op's, the sums land in c->bsi_sums.
static int ctx_bsi(Ctx* c, int32_t id, int op, int nbits, int has_found, int32_t start, int32_t end,
                   int32_t min_value, int32_t max_value, int want_sum) {
  Batch* B;
  CHK(get_batch(c, id, &B));
  if (!B->key_major || B->packed || nbits < 0 || nbits + 2 > kBsiMaxInputs || B->n_bm != (size_t)(1 + nbits + (has_found ? 1 : 0)) ||
      op < 0 || op > BSI_SUM_ONLY || (op == BSI_SUM_ONLY && !has_found)) {
    set_err("bsi: batch must hold ebM, nbits slices and the optional foundSet; bad op");
    return RBG_ERR_ILLEGAL_ARGUMENT;
  }
  hipStream_t s = c->stream;
  CHK(c->bsi_sums.ensure(8 * kBsiSumAll));  // zeroed by the plan kernel
  c->bsi_nbits = nbits;
  int mode = op;
  if (op != BSI_SUM_ONLY) {
    const int mm = bsi_minmax(op, start, end, min_value, max_value);
    if (mm == 1) mode = BSI_ALL;
    if (mm == 2) mode = -1;  // empty result
  }
  const size_t ub = std::min<size_t>(kMaxKeys, std::max<size_t>(B->n_ctr, 1));
  OutCtx oc;
  CHK(prepare_output(c, ub, (size_t)8194 * ub + B->max_ser, &oc, op == BSI_SUM_ONLY));
  c->pending_src = {id};
  const uint32_t need = mode == -1 ? 0xFFFFFFFFu : (op == BSI_SUM_ONLY ? (uint32_t)(nbits + 1) : 0u);
  BsiScratch sc{};
  if (mode >= 0 && mode <= BSI_RANGE) {
    CHK(c->bsi_defer.ensure(4 * (ub + 1)));
    CHK(c->bsi_cnts.ensure((size_t)4 * 128 * 4 * ub));  // count rows (< 128) x 4 units
    CHK(c->bsi_kin.ensure((size_t)16 * 34 * ub));
    CHK(c->bsi_table.ensure((size_t)16 * 34 * ub));
    sc = BsiScratch{c->bsi_defer.as<uint32_t>(), c->bsi_cnts.as<int>(), c->bsi_kin.p, ub, c->bsi_table.p};
    if (!c->bsi_claims.p) {  // zeroed once here, then by k_bsi_types after every query that claims
      CHK(c->bsi_claims.ensure(4 * kBsiClaimWords));
      HIPCHK(hipMemsetAsync(c->bsi_claims.p, 0, 4 * kBsiClaimWords, s));
    }
    sc.claims = c->bsi_claims.as<unsigned int>();
  }
  WideArgs wa{};
  wa.desc = B->desc.as<CDesc>();
  wa.bm = B->bm.as<uint32_t>();
  wa.payload = B->payload.as<uint8_t>();
  c->mark(0);
  Task* tasks = c->tasks.as<Task>();
  uint32_t* nt = c->ntasks.as<uint32_t>();
  if (sc.defer && bsi_reg_path(mode, nbits)) {
    // The task list (keys where ebM has a container) and the input table depend on the batch
    // only: planned once per batch, kept with it (RoaringBitmapSliceIndex queries on one index,
    // BSI/:482-513, re-walk the same keys every time).
    if (!B->bsi_cached) {
      CHK(B->bsi_tasks.ensure(sizeof(Task) * kMaxKeys));
      CHK(B->bsi_nt.ensure(64));
      CHK(B->bsi_table.ensure((size_t)16 * 34 * ub));
      launch_plan_bsi(s, B->key_off.as<uint32_t>(), B->bm.as<uint32_t>(), need, c->by_key.as<Task>(),
                      c->flag.as<uint8_t>(), c->wg_count.as<uint32_t>(), nullptr, nullptr, nullptr, nullptr);
      launch_compact(s, c->flag.as<uint8_t>(), c->by_key.as<Task>(), c->wg_count.as<uint32_t>(),
                     B->bsi_tasks.as<Task>(), B->bsi_nt.as<uint32_t>());
      launch_bsi_table(s, B->bsi_tasks.as<Task>(), B->bsi_nt.as<uint32_t>(), wa, B->bsi_table.p, ub);
      B->bsi_cached = true;
    }
    tasks = B->bsi_tasks.as<Task>();
    nt = B->bsi_nt.as<uint32_t>();
    sc.table = B->bsi_table.p;
    sc.table_ready = true;
    sc.zlb = c->zlb;
    sc.ztile = c->ztile;
    sc.zsums = c->bsi_sums.as<unsigned long long>();
    sc.nt_src = nt;
    sc.nt_dst = c->ntasks.as<uint32_t>();
  } else {
    launch_plan_bsi(s, B->key_off.as<uint32_t>(), B->bm.as<uint32_t>(), need, c->by_key.as<Task>(),
                    c->flag.as<uint8_t>(), c->wg_count.as<uint32_t>(), c->zlb, c->ztile,
                    c->bsi_sums.as<unsigned long long>(), sc.defer);
    launch_compact(s, c->flag.as<uint8_t>(), c->by_key.as<Task>(), c->wg_count.as<uint32_t>(), tasks, nt);
  }
  c->mark(1);
  BsiArgs p{mode < 0 ? BSI_EQ : mode, nbits, has_found, (uint32_t)start, (uint32_t)end};
  launch_bsi(s, grid_for(ub, 65536), tasks, nt, wa, p, oc, want_sum ? c->bsi_sums.as<unsigned long long>() : nullptr,
             sc.defer ? &sc : nullptr, want_sum ? c->bsi_sums_dst : nullptr);
  c->mark(2);
  if (op == BSI_SUM_ONLY) {
    c->last = 0;
  } else {
    defer_place(c);
  }
  c->mark(3);
  HIPCHK(hipGetLastError());
  return RBG_OK;
}

// ---------------------------------------------------------------------------
// Buffer-package BSI: BitSliceIndexBase.compare (bsi/src/main/java/org/roaringbitmap/bsi/buffer/
// BitSliceIndexBase.java, BBSI/ below), bsi.hip's k_bsi_buf
// ---------------------------------------------------------------------------

// horizontal_or's chain order for owenGreatEqual (BBSI/:266, RB/buffer/BufferFastAggregation.java:187-235):
// the queue holds one container pointer per orInput bitmap (in orInputs order, top down,
// BBSI/:247-264); each walks the keys where its orInput has a container, ordered by key, then
// larger cardinality first (RB/buffer/MutableRoaringArray.java:476-481), ties in the heap's
// order.  The poll order of a key's pointers is that key's chain: ord[t * kOwenOrder] = n,
// then the n orInput indices.
static int owen_order(Ctx* c, int M, uint32_t nt) {
  hipStream_t s = c->stream;
  std::vector<uint32_t> keys(nt);
  std::vector<int32_t> tb((size_t)nt * 32 * 4);  // TB: kind, card, src, pad
  if (nt) {
    HIPCHK(hipMemcpyAsync(keys.data(), c->owen_keys.p, 4 * (size_t)nt, hipMemcpyDeviceToHost, s));
    HIPCHK(hipMemcpyAsync(tb.data(), c->owen_tb.p, 16 * 32 * (size_t)nt, hipMemcpyDeviceToHost, s));
  }
  HIPCHK(hipStreamSynchronize(s));
  std::vector<std::vector<uint32_t>> lists(M);  // tasks (ascending keys) where orInput j has a container
  for (uint32_t t = 0; t < nt; t++)
    for (int j = 0; j < M; j++)
      if (tb[((size_t)t * 32 + j) * 4 + 1] > 0) lists[j].push_back(t);
  std::vector<uint8_t> ord((size_t)std::max<uint32_t>(nt, 1) * kOwenOrder, 0);
  auto ptr = [&](uint32_t j, uint32_t i) {
    const uint32_t t = lists[j][i];
    return HPtr{j, i, keys[t], (uint32_t)tb[((size_t)t * 32 + j) * 4 + 1], t};
  };
  auto push = [&](const HPtr& x) {
    uint8_t* o = ord.data() + (size_t)x.pos * kOwenOrder;
    o[1 + o[0]++] = (uint8_t)x.bm;
  };
  JHeap pq;
  for (int j = 0; j < M; j++)
    if (!lists[j].empty()) pq.add(ptr((uint32_t)j, 0));
  auto advance_add = [&](const HPtr& x) {
    if (x.i + 1 < lists[x.bm].size()) pq.add(ptr(x.bm, x.i + 1));
  };
  while (!pq.q.empty()) {
    const HPtr x1 = pq.poll();
    push(x1);
    if (pq.q.empty() || pq.q[0].key != x1.key) {
      advance_add(x1);
      continue;
    }
    const HPtr x2 = pq.poll();
    push(x2);
    while (!pq.q.empty() && pq.q[0].key == x1.key) {
      const HPtr x = pq.poll();
      push(x);
      if (x.i + 1 < lists[x.bm].size()) pq.add(ptr(x.bm, x.i + 1));
      else if (pq.q.empty()) break;
    }
    advance_add(x1);
    advance_add(x2);
  }
  CHK(c->owen_ord.ensure(ord.size()));
  HIPCHK(hipMemcpyAsync(c->owen_ord.p, ord.data(), ord.size(), hipMemcpyHostToDevice, s));
  HIPCHK(hipStreamSynchronize(s));  // `ord` is a stack vector
  return RBG_OK;
}

// op: RBG_BSI_* (compare) or RBG_BSI_RANGE_NEQ_DIRECT; the batch is [ebM, bA[0..nbits-1], foundSet?].
// Synchronous: the big-run arena is checked after the op (and the op rerun with a larger arena).
static int ctx_bsi_buffer(Ctx* c, int32_t id, int op, int nbits, int has_found, int32_t start, int32_t end,
                          int32_t min_value, int32_t max_value) {
  Batch* B;
  CHK(get_batch(c, id, &B));
  if (!B->key_major || B->packed || nbits < 0 || nbits + 2 > kBsiMaxInputs ||
      B->n_bm != (size_t)(1 + nbits + (has_found ? 1 : 0)) || op < 0 || op > RBG_BSI_RANGE_NEQ_DIRECT) {
    set_err("bsi: batch must hold ebM, nbits slices and the optional foundSet; bad op");
    return RBG_ERR_ILLEGAL_ARGUMENT;
  }
  hipStream_t s = c->stream;
  // compareUsingMinMax (BBSI/:455-519, as the heap one) and the op's own dispatch (BBSI/:422-453)
  int mode, nb_eff = nbits, found_eff = has_found;
  if (op == RBG_BSI_RANGE_NEQ_DIRECT || op == BSI_NEQ) {
    const int mm = op == BSI_NEQ ? bsi_minmax(BSI_NEQ, start, end, min_value, max_value) : 0;
    if (mm) {
      mode = mm == 1 ? BSI_ALL : -1;
    } else {  // andNot(ebM, rangeEQ(foundSet, value)); rangeEQ checks compareUsingMinMax(EQ) itself
      const int em = bsi_minmax(BSI_EQ, start, 0, min_value, max_value);
      mode = BSI_NEQ;
      if (em == 2) {  // andNot(ebM, empty): ebM's clone
        mode = BSI_ALL;
        found_eff = 0;
      } else if (em == 1) {  // andNot(ebM, ebM.clone() or and(ebM, foundSet)): the chain without slices
        nb_eff = 0;
      }
    }
  } else {
    const int mm = bsi_minmax(op, start, end, min_value, max_value);
    mode = mm == 1 ? BSI_ALL : mm == 2 ? -1 : op;
  }
  // owenGreatEqual (BBSI/:245-264): beGtrThan = start - 1, leastSignifZero =
  // Long.numberOfTrailingZeros(~beGtrThan) (64 when start - 1 == -1: no orInput at all)
  uint32_t zeros = 0, ones = 0;
  if (mode == BSI_GE || mode == BSI_RANGE) {
    const int32_t b = (int32_t)((uint32_t)start - 1u);
    const uint32_t nbx = ~(uint32_t)b;
    const int lsz = nbx == 0 ? 64 : __builtin_ctz(nbx);
    for (int w = nbits - 1; w >= lsz; w--) {
      if ((((uint32_t)b >> w) & 1u) == 0) zeros |= 1u << w;
      else ones |= 1u << w;
    }
  }
  const int M = __builtin_popcount(zeros);
  const size_t ub = std::min<size_t>(kMaxKeys, std::max<size_t>(B->n_ctr, 1));
  if (!c->big_ctl.p) CHK(c->big_ctl.ensure(16));
  if (!c->big.p) CHK(c->big.ensure(16ull << 20));
  for (int attempt = 0;; attempt++) {
    OutCtx oc;
    CHK(prepare_output(c, ub, (size_t)8194 * ub + B->max_ser + c->big.cap, &oc, false));
    c->pending_src = {id};
    const uint32_t need = mode == -1 ? 0xFFFFFFFFu : 0xFFFFFFFEu;  // every key of any input
    c->mark(0);
    launch_plan_bsi(s, B->key_off.as<uint32_t>(), B->bm.as<uint32_t>(), need, c->by_key.as<Task>(),
                    c->flag.as<uint8_t>(), c->wg_count.as<uint32_t>(), c->zlb, c->ztile, nullptr, nullptr);
    launch_compact(s, c->flag.as<uint8_t>(), c->by_key.as<Task>(), c->wg_count.as<uint32_t>(), c->tasks.as<Task>(),
                   c->ntasks.as<uint32_t>());
    HIPCHK(hipMemsetAsync(c->big_ctl.p, 0, 16, s));
    c->mark(1);
    WideArgs wa{};
    wa.desc = B->desc.as<CDesc>();
    wa.bm = B->bm.as<uint32_t>();
    wa.payload = B->payload.as<uint8_t>();
    BsiArgs p{};
    p.op = mode < 0 ? BSI_EQ : mode;
    p.nbits = nb_eff;
    p.has_found = found_eff;
    p.pred0 = (uint32_t)start;
    p.pred1 = (uint32_t)end;
    p.buffer = 1;
    p.found_input = nbits + 1;
    p.owen_zeros = zeros;
    p.owen_ones = ones;
    p.big = BigRuns{c->big.as<uint8_t>(), c->big_ctl.as<unsigned long long>(), c->big.cap};
    const int grid = grid_for(ub, 65536);
    if (mode >= 0 && M >= 3) {  // the chain order needs horizontal_or's queue: every orInput's type first
      CHK(c->owen_tb.ensure((size_t)16 * 32 * ub));
      CHK(c->owen_keys.ensure(4 * ub));
      p.owen_tb = c->owen_tb.p;
      p.task_keys = c->owen_keys.as<uint32_t>();
      launch_bsi_owen_pre(s, grid, c->tasks.as<Task>(), c->ntasks.as<uint32_t>(), wa, p);
      HIPCHK(hipGetLastError());
      uint32_t nt = 0;
      HIPCHK(hipMemcpyAsync(&nt, c->ntasks.p, 4, hipMemcpyDeviceToHost, s));
      HIPCHK(hipStreamSynchronize(s));
      CHK(owen_order(c, M, nt));
      p.owen_order = c->owen_ord.as<uint8_t>();
    }
    if (mode >= 0) launch_bsi_buf(s, grid, c->tasks.as<Task>(), c->ntasks.as<uint32_t>(), wa, p, oc);
    c->mark(2);
    defer_place(c);
    c->mark(3);
    HIPCHK(hipGetLastError());
    unsigned long long used[2] = {0, 0};
    HIPCHK(hipMemcpyAsync(used, c->big_ctl.p, 16, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if (!used[1]) return RBG_OK;
    if (attempt) {
      set_err("bsi: the run-container arena overflowed twice");
      return RBG_ERR_DEVICE;
    }
    CHK(c->big.ensure(used[0] + (used[0] >> 3) + 4096));  // the first pass counted every reservation
  }
}

// (sum, count) of the last BSI call: k_bsi_sum_final's Java longs, read back
static int ctx_bsi_sums(Ctx* c, int64_t* out2) {
  if (!c->bsi_sums.p) {
    out2[0] = out2[1] = 0;
    return RBG_OK;
  }
  HIPCHK(hipMemcpyAsync(out2, c->bsi_sums.as<uint64_t>() + kBsiSumOut, 16, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return RBG_OK;
}

static int ctx_info(Ctx* c, ResultInfo* ri) {
  if (c->last == 1) CHK(ensure_placed(c));
  HIPCHK(hipMemcpyAsync(ri, c->info.p, sizeof(ResultInfo), hipMemcpyDeviceToHost, c->stream));
  uint64_t card = 0;
  uint32_t err = 0;
  if (c->last == 1)  // materialised result: k_place / the pairwise placer accumulated its cardinality
    HIPCHK(hipMemcpyAsync(&card, c->lb.as<uint8_t>() + 64 + 8 * kCardWord, 8, hipMemcpyDeviceToHost, c->stream));
  if (c->last == 1 || c->last == 2)  // spin timeouts of any kernel of the op
    HIPCHK(hipMemcpyAsync(&err, c->lb.as<uint8_t>() + 64, 4, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  if (c->last == 1) {
    ri->long_card = (int64_t)card;
    ri->card32 = (uint32_t)card;
  }
  ri->err |= err;
  if ((c->last == 1 || c->last == 2) && ri->err) {
    set_err("a look-back spin of the op's plan or placement timed out: the result is invalid");
    return RBG_ERR_DEVICE;
  }
  if (c->last == 1) {
    c->last_ri = *ri;
    c->ri_valid = true;
  }
  return RBG_OK;
}

// Device -> host copy of a large result into caller (pageable) memory: 32 MiB groups DMA'd into
// the context's pinned staging, each copied out by worker threads as soon as its event fires, so
// the DMA of the next groups overlaps the host copies (the mirror of stage_upload).
static int download_staged(Ctx* c, const uint8_t* dev, uint64_t bytes, uint8_t* dst) {
  constexpr uint64_t kGroup = 32ull << 20;
  hipStream_t s = c->stream;
  if (bytes <= kGroup) {
    HIPCHK(hipMemcpyAsync(dst, dev, bytes, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    return RBG_OK;
  }
  CHK(pinned_ensure(c, bytes + 64));
  uint8_t* pin = reinterpret_cast<uint8_t*>(c->pinned);
  const uint32_t groups = (uint32_t)((bytes + kGroup - 1) / kGroup);
  std::vector<hipEvent_t> ev(groups);
  for (auto& e : ev) HIPCHK(hipEventCreateWithFlags(&e, hipEventDisableTiming));
  int st = RBG_OK;
  for (uint32_t g = 0; g < groups; g++) {
    const uint64_t lo = (uint64_t)g * kGroup, hi = std::min<uint64_t>(bytes, lo + kGroup);
    if (hipMemcpyAsync(pin + lo, dev + lo, hi - lo, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipEventRecord(ev[g], s) != hipSuccess) {
      set_err("device-to-host copy of the result failed");
      st = RBG_ERR_DEVICE;
      break;
    }
  }
  if (st == RBG_OK) {
    std::atomic<uint32_t> next{0};
    std::atomic<int> bad{0};
    const int nthr = (int)std::min<unsigned>(8, std::max(1u, std::thread::hardware_concurrency()));
    std::vector<std::thread> th;
    for (int t = 0; t < nthr; t++)
      th.emplace_back([&]() {
        for (uint32_t g; (g = next.fetch_add(1)) < groups;) {
          if (hipEventSynchronize(ev[g]) != hipSuccess) {
            bad.store(1);
            continue;
          }
          const uint64_t lo = (uint64_t)g * kGroup, hi = std::min<uint64_t>(bytes, lo + kGroup);
          std::memcpy(dst + lo, pin + lo, hi - lo);
        }
      });
    for (auto& x : th) x.join();
    if (bad.load()) {
      set_err("device-to-host copy of the result failed");
      st = RBG_ERR_DEVICE;
    }
  }
  (void)hipStreamSynchronize(s);
  for (auto& e : ev) (void)hipEventDestroy(e);
  return st;
}

// Large result buffers (a serialized C2 AND result is 0.25 GB): 2 MiB-aligned with transparent
// huge pages, so first touch faults once per 2 MiB instead of once per 4 KiB, and rbg_free keeps up
// to two of them for the next large result (a fresh buffer's pages are faulted and zeroed by the
// kernel on first touch: tens of ms for 0.25 GB, more than its PCIe download).
static std::mutex g_out_mu;
static std::unordered_map<void*, size_t> g_out_live;        // large buffers handed out -> capacity
static std::vector<std::pair<void*, size_t>> g_out_cache;   // freed ones kept for reuse
// The cache holds at most two buffers and 1 GiB; rbg_trim releases it.
constexpr size_t kOutLarge = 8ull << 20, kOutCacheMax = 2, kOutCacheBytes = 1ull << 30, kOutAlign = 2ull << 20;
static size_t out_cache_bytes() {
  size_t b = 0;
  for (const auto& e : g_out_cache) b += e.second;
  return b;
}
static uint8_t* out_alloc(size_t n) {
  if (n < kOutLarge) return (uint8_t*)std::malloc(n ? n : 1);
  std::lock_guard<std::mutex> g(g_out_mu);
  for (size_t i = 0; i < g_out_cache.size(); i++) {
    const auto e = g_out_cache[i];
    if (e.second >= n && e.second <= 2 * n + kOutAlign) {
      g_out_cache.erase(g_out_cache.begin() + (std::ptrdiff_t)i);
      g_out_live[e.first] = e.second;
      return (uint8_t*)e.first;
    }
  }
  const size_t cap = (n + kOutAlign - 1) & ~(kOutAlign - 1);
  void* p = nullptr;
  if (posix_memalign(&p, kOutAlign, cap) != 0) return nullptr;
  (void)madvise(p, cap, MADV_HUGEPAGE);
  g_out_live[p] = cap;
  return (uint8_t*)p;
}

static int ctx_fetch(Ctx* c, rbg_buffer* out) {
  if (c->last != 1) {
    set_err("no serialized result pending");
    return RBG_ERR_ILLEGAL_ARGUMENT;
  }
  CHK(ctx_serialize(c));
  ResultInfo ri;
  CHK(ctx_info(c, &ri));
  uint8_t* p = out_alloc(ri.total);
  if (!p) return RBG_ERR_OUT_OF_MEMORY;
  out->data = p;
  out->len = ri.total;
  const int st = download_staged(c, c->result.as<uint8_t>() + ri.start, ri.total, p);
  if (st != RBG_OK) {
    rbg_free(out);
    return st;
  }
  return RBG_OK;
}

// ---------------------------------------------------------------------------
// thread-local one-shot contexts
// ---------------------------------------------------------------------------
static std::mutex g_dev_mu;
static uint64_t g_dev_mask = 1;

struct TLCtx {
  std::unique_ptr<Ctx> ctx;
  int device = -1;
};
static thread_local TLCtx tl;

static int tl_ctx(Ctx** out) {
  int dev;
  {
    std::lock_guard<std::mutex> g(g_dev_mu);
    uint64_t m = g_dev_mask;
    dev = m ? __builtin_ctzll(m) : 0;
  }
  if (!tl.ctx || tl.device != dev) {
    std::unique_ptr<Ctx> c(new Ctx());
    CHK(ctx_init(c.get(), dev));
    tl.ctx = std::move(c);
    tl.device = dev;
  }
  CHK(enter(tl.ctx.get()));
  *out = tl.ctx.get();
  return RBG_OK;
}


}  // namespace rbg

using namespace rbg;

struct rbg_ctx {
  Ctx c;
};

extern "C" {

int rbg_version(void) { return 1; }

void rbg_trim(void) {
  std::lock_guard<std::mutex> g(g_out_mu);
  for (const auto& e : g_out_cache) std::free(e.first);
  g_out_cache.clear();
}

uint64_t rbg_pool_evictions(void) { return g_pool_evictions.load(); }
const char* rbg_last_error(void) { return g_err.c_str(); }

void rbg_free(rbg_buffer* buf) {
  if (!buf) return;
  if (buf->data) {
    std::lock_guard<std::mutex> g(g_out_mu);
    const auto it = g_out_live.find(buf->data);
    if (it != g_out_live.end()) {  // a large result buffer: kept for reuse (the oldest kept one freed)
      g_out_cache.emplace_back(it->first, it->second);
      g_out_live.erase(it);
      while (g_out_cache.size() > kOutCacheMax || (!g_out_cache.empty() && out_cache_bytes() > kOutCacheBytes)) {
        std::free(g_out_cache.front().first);
        g_out_cache.erase(g_out_cache.begin());
      }
      buf->data = nullptr;
      buf->len = 0;
      return;
    }
  }
  std::free(buf->data);
  buf->data = nullptr;
  buf->len = 0;
}

int rbg_set_devices(uint64_t mask) {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || n == 0) {
    set_err("no HIP device");
    return RBG_ERR_DEVICE;
  }
  uint64_t usable = mask & ((n >= 64) ? ~0ULL : ((1ULL << n) - 1));
  if (!usable) {
    set_err("device mask selects no present device");
    return RBG_ERR_DEVICE;
  }
  std::lock_guard<std::mutex> g(g_dev_mu);
  g_dev_mask = usable;
  return __builtin_popcountll(usable);
}

int rbg_pairwise(int op, const uint8_t* a, size_t a_len, const uint8_t* b, size_t b_len, rbg_buffer* out) {
  if (!out || op < 0 || op > RBG_ANDNOT_BUFFER) return RBG_ERR_ILLEGAL_ARGUMENT;
  Ctx* c;
  CHK(tl_ctx(&c));
  BatchGuard g{c, {}};
  const uint8_t* bufs[2] = {a, b};
  const size_t lens[2] = {a_len, b_len};
  int32_t ids[2];
  CHK(ctx_load_separate(c, bufs, lens, 2, ids));  // one upload for both operands
  g.ids = {ids[0], ids[1]};
  CHK(ctx_pairwise(c, op, ids[0], 0, ids[1], 0, false, 0, kMaxKeys, op <= RBG_ANDNOT ? pipe_ranges() : 0));
  return ctx_fetch(c, out);
}

static int ctx_batch_fetch(Ctx* c, int32_t batch, size_t i, rbg_buffer* out);
int rbg_pairwise_inplace(int op, const uint8_t* a, size_t a_len, const uint8_t* b, size_t b_len, int same_object,
                         rbg_buffer* out) {
  if (!out || op < 0 || op > 3) return RBG_ERR_ILLEGAL_ARGUMENT;
  if (same_object) {
    // x1.and(x1) / x1.or(x1) return at once (x1 unchanged); x1.xor(x1) / x1.andNot(x1) clear it
    // (RB/RoaringBitmap.java:1271, 2482, 3297-3300, 1347-1350)
    if (op == RBG_XOR || op == RBG_ANDNOT) {
      static const uint8_t kEmpty[8] = {0x3A, 0x30, 0, 0, 0, 0, 0, 0};
      uint8_t* p = (uint8_t*)std::malloc(8);
      if (!p) return RBG_ERR_OUT_OF_MEMORY;
      std::memcpy(p, kEmpty, 8);
      out->data = p;
      out->len = 8;
      return RBG_OK;
    }
    // x1 unchanged: validated on the host like any input, then its own bytes back (no device call)
    HostBitmap hb;
    std::string err;
    const int st = parse(a, a_len, &hb, &err);
    if (st) {
      set_err(err);
      return st;
    }
    uint8_t* p = out_alloc(hb.consumed);
    if (!p) return RBG_ERR_OUT_OF_MEMORY;
    std::memcpy(p, a, hb.consumed);
    out->data = p;
    out->len = hb.consumed;
    return RBG_OK;
  }
  // x1.and / xor / andNot(x2) in place type like the static ops (Container.iand / ixor / iandNot
  // end in the same container types); x1.or(x2) is Container.ior's
  return rbg_pairwise(op == RBG_OR ? RBG_OR_INPLACE : op, a, a_len, b, b_len, out);
}

int rbg_ornot(const uint8_t* a, size_t a_len, const uint8_t* b, size_t b_len, int64_t range_end, int flags,
              rbg_buffer* out) {
  if (!out || flags < 0 || flags > 3) return RBG_ERR_ILLEGAL_ARGUMENT;
  Ctx* c;
  CHK(tl_ctx(&c));
  BatchGuard g{c, {}};
  const uint8_t* bufs[2] = {a, b};
  const size_t lens[2] = {a_len, b_len};
  int32_t ids[2];
  CHK(ctx_load_separate(c, bufs, lens, 2, ids));
  g.ids = {ids[0], ids[1]};
  CHK(ctx_ornot(c, ids[0], 0, ids[1], 0, range_end, flags));
  return ctx_fetch(c, out);
}

int rbg_ctx_ornot(rbg_ctx* ctx, int32_t a, size_t ia, int32_t b, size_t ib, int64_t range_end, int flags) {
  if (!ctx || flags < 0 || flags > 3) return RBG_ERR_ILLEGAL_ARGUMENT;
  CHK(enter(&ctx->c));
  return ctx_ornot(&ctx->c, a, ia, b, ib, range_end, flags);
}

int rbg_range_mut(int op, const uint8_t* a, size_t a_len, int64_t range_start, int64_t range_end, rbg_buffer* out) {
  if (!out || op < 0 || op > (RBG_RMUT_ADD_INPLACE | RBG_RMUT_BUFFER))
    return RBG_ERR_ILLEGAL_ARGUMENT;
  Ctx* c;
  CHK(tl_ctx(&c));
  BatchGuard g{c, {}};
  int32_t id;
  CHK(ctx_load_separate(c, &a, &a_len, 1, &id));
  g.ids = {id};
  CHK(ctx_range_mut(c, op & 3, id, 0, range_start, range_end, (op & RBG_RMUT_BUFFER) != 0));
  return ctx_fetch(c, out);
}

int rbg_ctx_range_mut(rbg_ctx* ctx, int op, int32_t batch, size_t i, int64_t range_start, int64_t range_end) {
  if (!ctx || op < 0 || op > (RBG_RMUT_ADD_INPLACE | RBG_RMUT_BUFFER))
    return RBG_ERR_ILLEGAL_ARGUMENT;
  CHK(enter(&ctx->c));
  return ctx_range_mut(&ctx->c, op & 3, batch, i, range_start, range_end, (op & RBG_RMUT_BUFFER) != 0);
}

int rbg_add_offset(const uint8_t* a, size_t a_len, int64_t offset, rbg_buffer* out) {
  if (!out) return RBG_ERR_ILLEGAL_ARGUMENT;
  Ctx* c;
  CHK(tl_ctx(&c));
  BatchGuard g{c, {}};
  int32_t id;
  CHK(ctx_load_separate(c, &a, &a_len, 1, &id));
  g.ids = {id};
  CHK(ctx_add_offset(c, id, 0, offset));
  return ctx_fetch(c, out);
}

// x.limit(maxcardinality) (RB/RoaringBitmap.java:2457-2476).  The cut is planned from the serialized
// header's cardinalities on the host (the reference's own loop walks getCardinality per container):
// keys before it cloned, its container cut to the leftover by k_rmut<RMUT_LIMIT>, the rest dropped.
int rbg_limit(const uint8_t* a, size_t a_len, int32_t maxcard, rbg_buffer* out) {
  if (!out) return RBG_ERR_ILLEGAL_ARGUMENT;
  HostBitmap hb;
  std::string err;
  const int pst = parse(a, a_len, &hb, &err);
  if (pst) {
    set_err(err);
    return pst;
  }
  int cut_key = 65536, leftover = 0;
  int64_t cur = 0;
  for (size_t i = 0; cur < maxcard && i < hb.ctrs.size(); i++) {
    const int64_t cc = hb.ctrs[i].card;
    if (cc + cur <= maxcard) {
      cur += cc;
    } else {
      cut_key = hb.ctrs[i].key;
      leftover = (int)(maxcard - cur);
      break;
    }
  }
  if (leftover == 0) {  // the containers that fit whole: those before the first that does not
    cut_key = 0;
    for (size_t i = 0, acc = 0; i < hb.ctrs.size() && (int64_t)(acc + hb.ctrs[i].card) <= (int64_t)maxcard; i++) {
      acc += hb.ctrs[i].card;
      cut_key = hb.ctrs[i].key + 1;
    }
  }
  Ctx* c;
  CHK(tl_ctx(&c));
  BatchGuard g{c, {}};
  int32_t id;
  CHK(ctx_load_separate(c, &a, &a_len, 1, &id));
  g.ids = {id};
  Batch* A;
  CHK(get_batch(c, id, &A));
  const uint16_t* ka;
  const CDesc* da;
  int na;
  CHK(operand(A, 0, &ka, &da, &na));
  const RmutArgs ra{RMUT_LIMIT, cut_key, leftover, 0, 0};
  const size_t ub = std::max<size_t>(1, (size_t)na);
  hipStream_t s = c->stream;
  if (!c->big_ctl.p) CHK(c->big_ctl.ensure(16));
  if (!c->big.p) CHK(c->big.ensure(16ull << 20));
  for (int attempt = 0;; attempt++) {
    OutCtx oc;
    CHK(prepare_output(c, ub, A->payload_bytes + (size_t)8194 * ub + c->big.cap, &oc, false));
    c->pending_src = {id};
    c->mark(0);
    HIPCHK(hipMemsetAsync(c->big_ctl.p, 0, 16, s));
    c->mark(1);
    launch_rmut(s, A->key_off.as<uint32_t>(), da, A->payload.as<uint8_t>(), ra, false, c->wg_epoch.as<uint64_t>(),
                next_epoch(c), c->tasks.as<PTask>(), c->ntasks.as<uint32_t>(), oc, c->zlb, c->ztile,
                BigRuns{c->big.as<uint8_t>(), c->big_ctl.as<unsigned long long>(), c->big.cap}, grid_for(ub, 65536));
    c->mark(2);
    defer_place(c);
    c->mark(3);
    HIPCHK(hipGetLastError());
    unsigned long long used[2] = {0, 0};
    HIPCHK(hipMemcpyAsync(used, c->big_ctl.p, 16, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    if (!used[1]) break;
    if (attempt) {
      set_err("limit: the run-container arena overflowed twice");
      return RBG_ERR_DEVICE;
    }
    CHK(c->big.ensure(used[0] + (used[0] >> 3) + 4096));
  }
  return ctx_fetch(c, out);
}

// RoaringBitmap.bitmapOfRange(min, max) (RB/RoaringBitmap.java:588-615): k_rmut<RMUT_RANGE> over an empty
// bitmap (every container written as a run container)
int rbg_bitmap_of_range(int64_t min, int64_t max, rbg_buffer* out) {
  if (!out) return RBG_ERR_ILLEGAL_ARGUMENT;
  static const uint8_t kEmpty[8] = {0x3A, 0x30, 0, 0, 0, 0, 0, 0};
  const uint8_t* a = kEmpty;
  size_t a_len = 8;
  Ctx* c;
  CHK(tl_ctx(&c));
  BatchGuard g{c, {}};
  int32_t id;
  CHK(ctx_load_separate(c, &a, &a_len, 1, &id));
  g.ids = {id};
  CHK(ctx_range_mut(c, RMUT_RANGE, id, 0, min, max, false));
  return ctx_fetch(c, out);
}

int rbg_remove_run_compression(const uint8_t* a, size_t a_len, rbg_buffer* out) {
  if (!out) return RBG_ERR_ILLEGAL_ARGUMENT;
  Ctx* c;
  CHK(tl_ctx(&c));
  BatchGuard g{c, {}};
  int32_t id;
  CHK(ctx_load_separate(c, &a, &a_len, 1, &id));
  g.ids = {id};
  CHK(ctx_remove_run_compression(c, id, 0));
  return ctx_fetch(c, out);
}

int rbg_ctx_add_offset(rbg_ctx* ctx, int32_t batch, size_t i, int64_t offset) {
  if (!ctx) return RBG_ERR_ILLEGAL_ARGUMENT;
  CHK(enter(&ctx->c));
  return ctx_add_offset(&ctx->c, batch, i, offset);
}

int rbg_pairwise_card(int op, const uint8_t* a, size_t a_len, const uint8_t* b, size_t b_len, int32_t* out) {
  if (!out || op < 0 || op > RBG_CONTAINS) return RBG_ERR_ILLEGAL_ARGUMENT;
  Ctx* c;
  CHK(tl_ctx(&c));
  BatchGuard g{c, {}};
  int32_t ia, ib;
  CHK(ctx_load(c, &a, &a_len, 1, &ia));
  g.ids.push_back(ia);
  CHK(ctx_load(c, &b, &b_len, 1, &ib));
  g.ids.push_back(ib);
  CHK(ctx_pairwise(c, OP_AND, ia, 0, ib, 0, true));
  ResultInfo ri;
  CHK(ctx_info(c, &ri));
  const uint32_t ac = ri.card32;
  const uint32_t ca = (uint32_t)(uint64_t)c->batches[ia]->long_card;  // RoaringBitmap.getCardinality (int)
  const uint32_t cb = (uint32_t)(uint64_t)c->batches[ib]->long_card;
  switch (op) {
    case RBG_CARD_AND: *out = (int32_t)ac; break;
    case RBG_CARD_OR: *out = (int32_t)(ca + cb - ac); break;         // RB/RoaringBitmap.java:916-920
    case RBG_CARD_XOR: *out = (int32_t)(ca + cb - 2u * ac); break;   // :931-933
    case RBG_CARD_ANDNOT: *out = (int32_t)(ca - ac); break;          // :944-985 (both branches, mod 2^32)
    case RBG_CONTAINS:  // b is a subset of a (:2781-2802): every value of b in a AND b, counted in 64 bits
      *out = ri.long_card == c->batches[ib]->long_card ? 1 : 0;
      break;
    default: *out = ri.any ? 1 : 0; break;                           // intersects :698-720
  }
  return RBG_OK;
}

int rbg_wide(int op, const uint8_t* const* bufs, const size_t* lens, const int32_t* ids, size_t n, rbg_buffer* out) {
  if (!out || op < 0 || op > RBG_WIDE_BUFFER_AND_ITER) return RBG_ERR_ILLEGAL_ARGUMENT;
  Ctx* c;
  CHK(tl_ctx(&c));
  BatchGuard g{c, {}};
  int32_t id;
  CHK(ctx_load(c, bufs, lens, n, &id, wide_reads_packed(op, n)));
  g.ids.push_back(id);
  int hc;
  bool hv;
  CHK(ctx_wide(c, op, id, 0, 65536, ids, false, &hc, &hv));
  return ctx_fetch(c, out);
}

static int ctx_select_range(Ctx* c, int32_t id, int64_t start, int64_t end, int32_t* out_id, bool buf = false);
// rangeSanityCheck (RB/RoaringBitmap.java:204-213)
static int check_range(int64_t start, int64_t end) {
  if (start < 0 || start > 0xFFFFFFFFll || end < 0 || end > 0x100000000ll) {
    set_err("rangeStart=" + std::to_string(start) + " should be in [0, 0xffffffff], rangeEnd=" + std::to_string(end) +
            " in [0, 0xffffffff + 1]");
    return RBG_ERR_ILLEGAL_ARGUMENT;
  }
  return RBG_OK;
}

int rbg_range_op(int op, const uint8_t* const* bufs, const size_t* lens, size_t n, int64_t range_start,
                 int64_t range_end, rbg_buffer* out) {
  if (!out || op < RBG_RANGE_AND || op > RBG_RANGE_BUFFER_ANDNOT ||
      ((op == RBG_RANGE_ANDNOT || op == RBG_RANGE_BUFFER_ANDNOT) && n != 2))
    return RBG_ERR_ILLEGAL_ARGUMENT;
  const bool buf = op >= RBG_RANGE_BUFFER_AND;
  const int base = buf ? op - RBG_RANGE_BUFFER_AND : op;
  if (buf && base == RBG_RANGE_AND && n == 0) {
    // BufferFastAggregation.and(long[], Iterator) with no input: an empty bitmap (:81-88)
    CHK(check_range(range_start, range_end));
    static const uint8_t kEmpty[8] = {0x3A, 0x30, 0, 0, 0, 0, 0, 0};
    uint8_t* p = (uint8_t*)std::malloc(8);
    if (!p) return RBG_ERR_OUT_OF_MEMORY;
    std::memcpy(p, kEmpty, 8);
    out->data = p;
    out->len = 8;
    return RBG_OK;
  }
  Ctx* c;
  CHK(tl_ctx(&c));
  BatchGuard g{c, {}};
  CHK(check_range(range_start, range_end));  // rangeSanityCheck before the selections (RB/RoaringBitmap.java:204-213)
  if (base == RBG_RANGE_ANDNOT) {  // andNot(x1, x2, start, end): both operands selected, then andNot
    int32_t ids[2], sel[2];
    CHK(ctx_load_separate(c, bufs, lens, 2, ids));
    g.ids = {ids[0], ids[1]};
    for (int i = 0; i < 2; i++) {
      CHK(ctx_select_range(c, ids[i], range_start, range_end, &sel[i], buf));
      g.ids.push_back(sel[i]);
    }
    // the buffer package's andNot keeps R \ R's merged run container (ImmutableRoaringBitmap.andNot)
    CHK(ctx_pairwise(c, buf ? RBG_ANDNOT_BUFFER : OP_ANDNOT, sel[0], 0, sel[1], 0, false));
    return ctx_fetch(c, out);
  }
  int32_t id, sel;
  CHK(ctx_load(c, bufs, lens, n, &id));
  g.ids.push_back(id);
  CHK(ctx_select_range(c, id, range_start, range_end, &sel, buf));
  g.ids.push_back(sel);
  // heap: and -> FastAggregation.and(Iterator) = naive_and(Iterator); or / xor -> naive_or / naive_xor.
  // buffer: and -> BufferFastAggregation.and(Iterator) = workShyAnd for any count (no input: empty);
  // or / xor -> naive_or / naive_xor, typed like the heap's
  const int wop = base == RBG_RANGE_AND ? (buf ? RBG_WIDE_WORKSHY_AND : RBG_WIDE_AND_ITER)
                  : base == RBG_RANGE_OR ? RBG_WIDE_OR
                                         : RBG_WIDE_XOR;
  int hc;
  bool hv;
  CHK(ctx_wide(c, wop, sel, 0, 65536, nullptr, false, &hc, &hv));
  return ctx_fetch(c, out);
}

int rbg_select_range(const uint8_t* a, size_t a_len, int64_t range_start, int64_t range_end, int buffer,
                     rbg_buffer* out) {
  if (!out) return RBG_ERR_ILLEGAL_ARGUMENT;
  Ctx* c;
  CHK(tl_ctx(&c));
  BatchGuard g{c, {}};
  int32_t id, sel;
  CHK(ctx_load_separate(c, &a, &a_len, 1, &id));
  g.ids = {id};
  CHK(ctx_select_range(c, id, range_start, range_end, &sel, buffer != 0));
  g.ids.push_back(sel);
  return ctx_batch_fetch(c, sel, 0, out);
}

int rbg_ctx_select_range(rbg_ctx* ctx, int32_t batch, int64_t range_start, int64_t range_end, int32_t* out_batch) {
  if (!ctx || !out_batch) return RBG_ERR_ILLEGAL_ARGUMENT;
  CHK(enter(&ctx->c));
  return ctx_select_range(&ctx->c, batch, range_start, range_end, out_batch);
}

int rbg_wide_card(int op, const uint8_t* const* bufs, const size_t* lens, size_t n, int32_t* out) {
  if (!out || op < 0 || op > 1) return RBG_ERR_ILLEGAL_ARGUMENT;
  Ctx* c;
  CHK(tl_ctx(&c));
  BatchGuard g{c, {}};
  int32_t id;
  CHK(ctx_load(c, bufs, lens, n, &id));
  g.ids.push_back(id);
  int hc = 0;
  bool hv = false;
  CHK(ctx_wide(c, op, id, 0, 65536, nullptr, true, &hc, &hv));
  if (hv) {
    *out = hc;
    return RBG_OK;
  }
  ResultInfo ri;
  CHK(ctx_info(c, &ri));
  *out = (int32_t)ri.card32;
  return RBG_OK;
}

static int ctx_batch_card(Ctx* c, int32_t id) {
  Batch* B;
  CHK(get_batch(c, id, &B));
  if (B->packed) {
    set_err("batched andCardinality needs slot-aligned payloads");
    return RBG_ERR_ILLEGAL_ARGUMENT;
  }
  if (B->n_bm % 2 != 0) {
    set_err("batched andCardinality needs an even number of bitmaps");
    return RBG_ERR_ILLEGAL_ARGUMENT;
  }
  const size_t np = B->n_bm / 2;
  CHK(c->cards.ensure(4 * std::max<size_t>(np, 1)));
  if (B->key_major && B->n_bm > 1) {
    // pairs need bitmap-major ranges: permuted view of a key-major batch is not supported
    set_err("batched andCardinality needs a bitmap-major batch");
    return RBG_ERR_ILLEGAL_ARGUMENT;
  }
  c->mark(0);
  c->mark(1);
  if (!B->pair_cap_known) {
    B->pair_items_cap = batch_pair_items_cap(B->h_bm_nctr.data(), np);
    B->pair_cap_known = true;
  }
  CHK(c->pc_cnt.ensure(8 * ((np + 255) / 256) + std::max<size_t>(np, 1) + 16));  // workgroup totals + a count byte per pair
  CHK(c->pc_part.ensure(8 * (scan_parts(std::max<size_t>(np, 1)) + 1)));
  CHK(c->pc_items.ensure(sizeof(PairItem) * std::max<uint64_t>(B->pair_items_cap, 1)));
  CHK(c->pc_large.ensure(4 * std::max<size_t>(np, 1)));
  CHK(c->scalar.ensure(64));
  launch_batch_and_card(c->stream, np, B->bm_off.as<uint32_t>(), B->keys.as<uint16_t>(), B->desc.as<CDesc>(),
                        B->payload.as<uint8_t>(), c->cards.as<int32_t>(), c->pc_cnt.as<uint64_t>(),
                        c->pc_part.as<uint64_t>(), c->scalar.as<uint64_t>() + 7, c->pc_items.as<PairItem>(),
                        c->pc_large.as<uint32_t>());
  c->mark(2);
  c->mark(3);
  HIPCHK(hipGetLastError());
  c->n_cards = np;
  c->last = 3;
  return RBG_OK;
}

// bitmap-major upload used by batched andCardinality (pairs kept adjacent)
static int ctx_load_bitmap_major(Ctx* c, const uint8_t* const* bufs, const size_t* lens, size_t n, int32_t* out_id) {
  return ctx_load_impl(c, bufs, lens, n, false, out_id);
}

int rbg_batch_and_card(size_t n_pairs, const uint8_t* const* a_bufs, const size_t* a_lens,
                       const uint8_t* const* b_bufs, const size_t* b_lens, int32_t* out) {
  if (n_pairs && (!a_bufs || !a_lens || !b_bufs || !b_lens || !out)) return RBG_ERR_ILLEGAL_ARGUMENT;
  if (n_pairs == 0) return RBG_OK;
  Ctx* c;
  CHK(tl_ctx(&c));
  std::vector<const uint8_t*> bufs(2 * n_pairs);
  std::vector<size_t> lens(2 * n_pairs);
  for (size_t i = 0; i < n_pairs; i++) {
    bufs[2 * i] = a_bufs[i];
    lens[2 * i] = a_lens[i];
    bufs[2 * i + 1] = b_bufs[i];
    lens[2 * i + 1] = b_lens[i];
  }
  BatchGuard g{c, {}};
  int32_t id;
  CHK(ctx_load_bitmap_major(c, bufs.data(), lens.data(), 2 * n_pairs, &id));
  g.ids.push_back(id);
  CHK(ctx_batch_card(c, id));
  HIPCHK(hipMemcpyAsync(out, c->cards.p, 4 * n_pairs, hipMemcpyDeviceToHost, c->stream));
  HIPCHK(hipStreamSynchronize(c->stream));
  return RBG_OK;
}

// ---- host-side format utilities ----
static int emit_host(const std::vector<uint8_t>& v, rbg_buffer* out) {
  uint8_t* p = (uint8_t*)std::malloc(v.size() ? v.size() : 1);
  if (!p) return RBG_ERR_OUT_OF_MEMORY;
  if (!v.empty()) std::memcpy(p, v.data(), v.size());
  out->data = p;
  out->len = v.size();
  return RBG_OK;
}

int rbg_from_values(const uint32_t* values, size_t n, int run_optimize, rbg_buffer* out) {
  if (!out || (n && !values)) return RBG_ERR_ILLEGAL_ARGUMENT;
  return emit_host(build_from_values(values, n, run_optimize != 0), out);
}

// RoaringBitmap.runOptimize() (RB/RoaringBitmap.java:2764-2774): the device pass
// (runopt.hip) over a one-bitmap batch, like rbg_run_optimize_many.
int rbg_run_optimize(const uint8_t* buf, size_t len, rbg_buffer* out) {
  if (!out || (!buf && len)) return RBG_ERR_ILLEGAL_ARGUMENT;
  uint8_t answer = 0;
  return rbg_run_optimize_many(&buf, &len, 1, out, &answer);
}

int rbg_to_values(const uint8_t* buf, size_t len, rbg_buffer* out) {
  if (!out) return RBG_ERR_ILLEGAL_ARGUMENT;
  std::vector<uint32_t> v;
  std::string err;
  int st = values_of_serialized(buf, len, &v, &err);
  if (st) {
    set_err(err);
    return st;
  }
  uint8_t* p = (uint8_t*)std::malloc(v.size() * 4 + 4);
  if (!p) return RBG_ERR_OUT_OF_MEMORY;
  std::memcpy(p, v.data(), v.size() * 4);
  out->data = p;
  out->len = v.size() * 4;
  return RBG_OK;
}

int rbg_inspect(const uint8_t* buf, size_t len, size_t* consumed, int64_t* cardinality, int64_t* stats3) {
  HostBitmap hb;
  std::string err;
  int st = parse(buf, len, &hb, &err);
  if (st) {
    set_err(err);
    return st;
  }
  if (consumed) *consumed = hb.consumed;
  if (cardinality) *cardinality = hb.card;
  if (stats3) {
    stats3[0] = stats3[1] = stats3[2] = 0;
    for (const HostCtr& c : hb.ctrs) stats3[c.kind]++;
  }
  return RBG_OK;
}

// ---- session API ----
int rbg_ctx_create(int device, rbg_ctx** out) {
  if (!out) return RBG_ERR_ILLEGAL_ARGUMENT;
  std::unique_ptr<rbg_ctx> c(new rbg_ctx());
  CHK(ctx_init(&c->c, device));
  *out = c.release();
  return RBG_OK;
}
void rbg_ctx_destroy(rbg_ctx* ctx) {
  if (!ctx) return;
  (void)hipSetDevice(ctx->c.device);
  delete ctx;
}
void* rbg_ctx_stream(rbg_ctx* ctx) { return ctx ? (void*)ctx->c.stream : nullptr; }
static int ctx_profile(rbg_ctx* ctx, int max_ops, bool compute_only) {
  CHK(enter(&ctx->c));
  HIPCHK(hipStreamSynchronize(ctx->c.stream));
  ctx->c.prof_free();
  ctx->c.prof_compute_only = compute_only;
  if (max_ops <= 0) return RBG_OK;
  ctx->c.prof_ev.resize(4 * (size_t)max_ops);
  for (hipEvent_t& e : ctx->c.prof_ev) HIPCHK(hipEventCreate(&e));
  ctx->c.prof_cap = (size_t)max_ops;
  ctx->c.prof_n = 0;
  CHK(ctx->c.rd_ctr.ensure(8));
  HIPCHK(hipMemsetAsync(ctx->c.rd_ctr.p, 0, 8, ctx->c.stream));
  return RBG_OK;
}
int rbg_ctx_profile(rbg_ctx* ctx, int max_ops) { return ctx_profile(ctx, max_ops, false); }
int rbg_ctx_profile_compute(rbg_ctx* ctx, int max_ops) { return ctx_profile(ctx, max_ops, true); }
int rbg_ctx_profile_bytes(rbg_ctx* ctx, int64_t* bytes) {
  if (!ctx || !bytes) {
    set_err("profile_bytes: null argument");
    return RBG_ERR_ILLEGAL_ARGUMENT;
  }
  Ctx& c = ctx->c;
  CHK(enter(&c));
  HIPCHK(hipStreamSynchronize(c.stream));
  unsigned long long v = 0;
  if (c.rd_ctr.p) HIPCHK(hipMemcpy(&v, c.rd_ctr.p, 8, hipMemcpyDeviceToHost));
  *bytes = (int64_t)v;
  return RBG_OK;
}
int rbg_ctx_profile_read(rbg_ctx* ctx, double* ms3, int* n_ops) {
  Ctx& c = ctx->c;
  CHK(enter(&c));
  HIPCHK(hipStreamSynchronize(c.stream));
  ms3[0] = ms3[1] = ms3[2] = 0.0;
  for (size_t i = 0; i < c.prof_n; i++) {
    for (int ph = 0; ph < 3; ph++) {
      if (c.prof_compute_only && ph != 1) continue;  // only the compute launch was bracketed
      float ms = 0.f;
      HIPCHK(hipEventElapsedTime(&ms, c.prof_ev[4 * i + ph], c.prof_ev[4 * i + ph + 1]));
      ms3[ph] += ms;
    }
  }
  *n_ops = (int)c.prof_n;
  c.prof_n = 0;
  return RBG_OK;
}
int rbg_ctx_sync(rbg_ctx* ctx) {
  CHK(enter(&ctx->c));
  HIPCHK(hipStreamSynchronize(ctx->c.stream));
  return RBG_OK;
}
int rbg_ctx_load_separate(rbg_ctx* ctx, const uint8_t* const* bufs, const size_t* lens, size_t n, int32_t* ids) {
  if (!ctx || !ids) return RBG_ERR_ILLEGAL_ARGUMENT;
  CHK(enter(&ctx->c));
  return ctx_load_separate(&ctx->c, bufs, lens, n, ids);
}
int rbg_ctx_load(rbg_ctx* ctx, const uint8_t* const* bufs, const size_t* lens, size_t n, int32_t* batch) {
  CHK(enter(&ctx->c));
  return ctx_load(&ctx->c, bufs, lens, n, batch);
}
int rbg_ctx_load_packed(rbg_ctx* ctx, const uint8_t* const* bufs, const size_t* lens, size_t n, int32_t* batch) {
  if (!ctx || !batch) return RBG_ERR_ILLEGAL_ARGUMENT;
  CHK(enter(&ctx->c));
  return ctx_load(&ctx->c, bufs, lens, n, batch, true);
}
int rbg_ctx_release(rbg_ctx* ctx, int32_t batch) {
  Ctx& c = ctx->c;
  Batch* b;
  CHK(find_batch(&c, batch, &b));  // no statistics read-back for a batch that goes
  CHK(enter(&c));
  // A materialised result references pass-through containers inside its operand
  // batches (ORec::src) until it is serialized: serialize it before an operand goes.
  if (c.last == 1 && !c.serialized &&
      std::find(c.pending_src.begin(), c.pending_src.end(), batch) != c.pending_src.end())
    CHK(ctx_serialize(&c));
  // No host sync: the buffers go to this context's pool, and whatever reuses them is enqueued on
  // the same stream after every launch that reads them (a pipelined op's second stream is joined
  // back into it at the op's end); a pooled buffer that is freed goes through hipFree, which waits
  // for the device.
  for (DevBuf* d : {&b->keys, &b->desc, &b->bm, &b->key_off, &b->bm_off, &b->payload, &b->ro_stats,
                    &b->bsi_tasks, &b->bsi_nt, &b->bsi_table})
    pool_put(&c, *d);
  c.batches[batch].reset();
  return RBG_OK;
}
int rbg_ctx_batch_stats(rbg_ctx* ctx, int32_t batch, int64_t* st) {
  Batch* b;
  CHK(get_batch(&ctx->c, batch, &b));
  st[0] = (int64_t)b->n_bm;
  st[1] = (int64_t)b->n_ctr;
  st[2] = b->n_kind[0];
  st[3] = b->n_kind[1];
  st[4] = b->n_kind[2];
  st[5] = 0;  // payload bytes (serialized form)
  st[6] = b->long_card;
  st[7] = b->ser_bytes;
  if (b->n_ctr) {
    CHK(enter(&ctx->c));
    hipStream_t s = ctx->c.stream;
    HIPCHK(hipMemsetAsync(ctx->c.scalar.p, 0, 8, s));
    launch_batch_bytes(s, b->desc.as<CDesc>(), b->n_ctr, b->payload.as<uint8_t>(),
                       ctx->c.scalar.as<unsigned long long>());
    unsigned long long pay = 0;
    HIPCHK(hipMemcpyAsync(&pay, ctx->c.scalar.p, 8, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    st[5] = (int64_t)pay;
  }
  return RBG_OK;
}
static int ctx_batch_fetch(Ctx* c, int32_t batch, size_t i, rbg_buffer* out);
static int ctx_batch_fetch_range(Ctx* c, int32_t batch, size_t i0, size_t i1, rbg_buffer* outs);
int rbg_ctx_batch_fetch(rbg_ctx* ctx, int32_t batch, size_t i, rbg_buffer* out) {
  if (!ctx) return RBG_ERR_ILLEGAL_ARGUMENT;
  CHK(enter(&ctx->c));
  return ctx_batch_fetch(&ctx->c, batch, i, out);
}
int rbg_ctx_batch_fetch_range(rbg_ctx* ctx, int32_t batch, size_t first, size_t count, rbg_buffer* outs) {
  if (!ctx) return RBG_ERR_ILLEGAL_ARGUMENT;
  CHK(enter(&ctx->c));
  return ctx_batch_fetch_range(&ctx->c, batch, first, first + count, outs);
}
}  // extern "C"

namespace rbg {
// Host index of a batch's containers, built once per batch: the container table and,
// per input bitmap, its container positions (in key order).
static int batch_host_index(Ctx* c, Batch* b) {
  if (b->h_index) return RBG_OK;
  HIPCHK(hipStreamSynchronize(c->stream));
  b->h_desc.resize(b->n_ctr);
  if (b->n_ctr) HIPCHK(hipMemcpy(b->h_desc.data(), b->desc.p, sizeof(CDesc) * b->n_ctr, hipMemcpyDeviceToHost));
  b->h_pos_off.assign(b->n_bm + 1, 0);
  b->h_pos.resize(b->n_ctr);
  if ((b->n_bm == 1 || !b->key_major) && b->h_bm_off.size() == b->n_bm + 1) {
    for (size_t i = 0; i <= b->n_bm; i++) b->h_pos_off[i] = b->h_bm_off[i];
    for (size_t p = 0; p < b->n_ctr; p++) b->h_pos[p] = (uint32_t)p;
  } else {  // key-major: counting sort of the positions by input bitmap (stable, so key order)
    std::vector<uint32_t> bm(b->n_ctr);
    if (b->n_ctr) HIPCHK(hipMemcpy(bm.data(), b->bm.p, 4 * b->n_ctr, hipMemcpyDeviceToHost));
    for (uint32_t x : bm) b->h_pos_off[x + 1]++;
    for (size_t i = 0; i < b->n_bm; i++) b->h_pos_off[i + 1] += b->h_pos_off[i];
    std::vector<uint32_t> fill(b->h_pos_off.begin(), b->h_pos_off.end() - 1);
    for (size_t p = 0; p < b->n_ctr; p++) b->h_pos[fill[bm[p]]++] = (uint32_t)p;
  }
  b->h_index = true;
  return RBG_OK;
}

}  // namespace rbg

// Download bitmaps [i0, i1) of a batch as portable serialized bytes: their slots are
// gathered on the device into one buffer (one D2H copy), the headers built here.
static int ctx_batch_fetch_range(Ctx* c, int32_t batch, size_t i0, size_t i1, rbg_buffer* outs) {
  Batch* b;
  CHK(get_batch(c, batch, &b));
  if (i0 > i1 || i1 > b->n_bm || (i1 > i0 && !outs)) return RBG_ERR_ILLEGAL_ARGUMENT;
  CHK(batch_host_index(c, b));
  const std::vector<CDesc>& D = b->h_desc;
  // slots are consecutive in container order: a slot ends where the next one starts
  auto slot_end = [&](uint32_t p) -> uint64_t { return p + 1 < b->n_ctr ? D[p + 1].slot : b->payload_bytes; };
  std::vector<GatherItem> items;
  uint64_t tot = 0;
  for (size_t i = i0; i < i1; i++)
    for (uint32_t k = b->h_pos_off[i]; k < b->h_pos_off[i + 1]; k++) {
      const uint32_t p = b->h_pos[k];
      const uint64_t len = slot_end(p) - D[p].slot;
      items.push_back(GatherItem{D[p].slot, tot, len});
      tot = round16(tot + len);
    }
  std::vector<uint8_t> pay(tot + 16);
  if (!items.empty()) {
    CHK(c->gather_items.ensure(sizeof(GatherItem) * items.size()));
    CHK(c->gather_out.ensure(tot + 16));
    HIPCHK(hipMemcpyAsync(c->gather_items.p, items.data(), sizeof(GatherItem) * items.size(), hipMemcpyHostToDevice,
                          c->stream));
    launch_gather(c->stream, c->gather_items.as<GatherItem>(), items.size(), b->payload.as<uint8_t>(),
                  c->gather_out.as<uint8_t>());
    HIPCHK(hipGetLastError());
    HIPCHK(hipMemcpyAsync(pay.data(), c->gather_out.p, tot, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(hipStreamSynchronize(c->stream));
  }
  size_t it = 0;
  for (size_t i = i0; i < i1; i++) {
    const uint32_t k0 = b->h_pos_off[i], n = b->h_pos_off[i + 1] - k0;
    bool has_run = false;
    std::vector<uint32_t> lens(n);
    for (uint32_t k = 0; k < n; k++) {
      const CDesc& d = D[b->h_pos[k0 + k]];
      has_run |= d.kind == KR;
      if (d.kind == KA) lens[k] = 2 * d.card;
      else if (d.kind == KB) lens[k] = 8192;
      else {
        const uint8_t* q = pay.data() + items[it + k].dst + 2;
        lens[k] = 2 + 4 * (uint32_t)(q[0] | (q[1] << 8));
      }
    }
    std::vector<uint8_t> o;
    auto put16 = [&](uint32_t v) { o.push_back((uint8_t)v); o.push_back((uint8_t)(v >> 8)); };
    auto put32 = [&](uint32_t v) { for (int j = 0; j < 4; j++) o.push_back((uint8_t)(v >> (8 * j))); };
    if (has_run) {
      put32(12347u | (uint32_t)((n - 1) << 16));
      std::vector<uint8_t> fl((n + 7) / 8, 0);
      for (uint32_t k = 0; k < n; k++)
        if (D[b->h_pos[k0 + k]].kind == KR) fl[k / 8] |= (uint8_t)(1u << (k % 8));
      o.insert(o.end(), fl.begin(), fl.end());
    } else {
      put32(12346u);
      put32(n);
    }
    for (uint32_t k = 0; k < n; k++) {
      const CDesc& d = D[b->h_pos[k0 + k]];
      put16(d.key);
      put16(d.card - 1);
    }
    if (!has_run || n >= 4) {
      uint32_t start = (uint32_t)header_size(n, has_run);
      for (uint32_t k = 0; k < n; k++) {
        put32(start);
        start += lens[k];
      }
    }
    for (uint32_t k = 0; k < n; k++) {
      const uint8_t* q = pay.data() + items[it + k].dst + (D[b->h_pos[k0 + k]].kind == KR ? 2 : 0);
      o.insert(o.end(), q, q + lens[k]);
    }
    it += n;
    const int st = emit_host(o, &outs[i - i0]);
    if (st != RBG_OK) {
      for (size_t j = i0; j < i; j++) rbg_free(&outs[j - i0]);
      return st;
    }
  }
  return RBG_OK;
}

static int ctx_batch_fetch(Ctx* c, int32_t batch, size_t i, rbg_buffer* out) {
  if (!out) return RBG_ERR_ILLEGAL_ARGUMENT;
  return ctx_batch_fetch_range(c, batch, i, i + 1, out);
}

extern "C" {
int rbg_ctx_pairwise(rbg_ctx* ctx, int op, int32_t a, size_t ia, int32_t b, size_t ib) {
  CHK(enter(&ctx->c));
  return ctx_pairwise(&ctx->c, op, a, ia, b, ib, false);
}
int rbg_ctx_pairwise_serialized(rbg_ctx* ctx, int op, int32_t a, size_t ia, int32_t b, size_t ib) {
  if (!ctx) return RBG_ERR_ILLEGAL_ARGUMENT;
  CHK(enter(&ctx->c));
  if (op < 0 || op > 3) return RBG_ERR_ILLEGAL_ARGUMENT;
  CHK(ctx_pairwise(&ctx->c, op, a, ia, b, ib, false, 0, kMaxKeys, pipe_ranges()));
  return ctx_serialize(&ctx->c);  // no-op after the pipelined form
}
int rbg_ctx_pairwise_range(rbg_ctx* ctx, int op, int32_t a, size_t ia, int32_t b, size_t ib, int key_lo, int key_hi) {
  if (!ctx || key_lo > key_hi) return RBG_ERR_ILLEGAL_ARGUMENT;
  CHK(enter(&ctx->c));
  return ctx_pairwise(&ctx->c, op, a, ia, b, ib, false, key_lo, key_hi);
}
int rbg_ctx_pairwise_card(rbg_ctx* ctx, int op, int32_t a, size_t ia, int32_t b, size_t ib) {
  CHK(enter(&ctx->c));
  if (op != RBG_CARD_AND) {
    set_err("the session API computes andCardinality; derive the others from the input cardinalities");
    return RBG_ERR_ILLEGAL_ARGUMENT;
  }
  return ctx_pairwise(&ctx->c, OP_AND, a, ia, b, ib, true);
}
int rbg_ctx_wide(rbg_ctx* ctx, int op, int32_t batch, int key_lo, int key_hi, const int32_t* ids) {
  CHK(enter(&ctx->c));
  int hc;
  bool hv;
  return ctx_wide(&ctx->c, op, batch, key_lo, key_hi, ids, false, &hc, &hv);
}
int rbg_ctx_wide_start(rbg_ctx* ctx, int op, int32_t batch, int key_lo, int key_hi, const int32_t* ids,
                       int32_t start_bm) {
  CHK(enter(&ctx->c));
  int hc;
  bool hv;
  return ctx_wide(&ctx->c, op, batch, key_lo, key_hi, ids, false, &hc, &hv, start_bm);
}
int rbg_ctx_batch_counts(rbg_ctx* ctx, int32_t batch, uint32_t* out, size_t n) {
  Batch* b;
  CHK(get_batch(&ctx->c, batch, &b));
  if (!out || n != b->n_bm) return RBG_ERR_ILLEGAL_ARGUMENT;
  for (size_t i = 0; i < n; i++) out[i] = b->h_bm_nctr[i];
  return RBG_OK;
}
int rbg_synth_key_bytes(int kind, uint64_t seed, size_t n, uint64_t* out) {
  if (!out || (kind != 1 && kind != 2)) return RBG_ERR_ILLEGAL_ARGUMENT;
  for (int k = 0; k < kMaxKeys; k++) out[k] = 0;
  for (size_t i = 0; i < n; i++) {
    if (kind == 1) {
      for (int k = 0; k < kMaxKeys; k++) out[k] += 4 + 2 * (uint64_t)c3u_card(seed, (uint32_t)i, (uint32_t)k);
    } else {
      const uint32_t b0 = c3c_base(seed, (uint32_t)i);
      for (uint32_t k = b0; k < b0 + 16; k++) out[k] += 4 + 8192;
    }
  }
  return RBG_OK;
}
int rbg_ctx_bsi(rbg_ctx* ctx, int32_t batch, int op, int nbits, int has_found, int32_t start, int32_t end,
                int32_t min_value, int32_t max_value, int want_sum) {
  CHK(enter(&ctx->c));
  return ctx_bsi(&ctx->c, batch, op, nbits, has_found, start, end, min_value, max_value, want_sum);
}
int rbg_ctx_bsi_sums(rbg_ctx* ctx, int64_t* out2) {
  if (!out2) return RBG_ERR_ILLEGAL_ARGUMENT;
  CHK(enter(&ctx->c));
  return ctx_bsi_sums(&ctx->c, out2);
}
int rbg_ctx_bsi_sums_target(rbg_ctx* ctx, void* dst2) {
  if (!ctx) return RBG_ERR_ILLEGAL_ARGUMENT;
  ctx->c.bsi_sums_dst = dst2;
  return RBG_OK;
}
int rbg_ctx_bsi_sums_device(rbg_ctx* ctx, void* dst2) {
  if (!ctx || !dst2 || !ctx->c.bsi_sums.p) return RBG_ERR_ILLEGAL_ARGUMENT;
  CHK(enter(&ctx->c));
  launch_bsi_sums_out(ctx->c.stream, ctx->c.bsi_sums.as<unsigned long long>(), dst2);
  HIPCHK(hipGetLastError());
  return RBG_OK;
}
static int bsi_load(Ctx* c, const uint8_t* ebm, size_t ebm_len, const uint8_t* const* slices, const size_t* lens,
                    size_t nbits, const uint8_t* found, size_t found_len, int32_t* id) {
  if (!ebm || (nbits && (!slices || !lens)) || nbits + 2 > (size_t)kBsiMaxInputs) return RBG_ERR_ILLEGAL_ARGUMENT;
  std::vector<const uint8_t*> bufs{ebm};
  std::vector<size_t> ls{ebm_len};
  for (size_t i = 0; i < nbits; i++) {
    bufs.push_back(slices[i]);
    ls.push_back(lens[i]);
  }
  if (found) {
    bufs.push_back(found);
    ls.push_back(found_len);
  }
  return ctx_load(c, bufs.data(), ls.data(), bufs.size(), id);
}
int rbg_bsi_compare(int op, int32_t start, int32_t end, const uint8_t* ebm, size_t ebm_len,
                    const uint8_t* const* slices, const size_t* slice_lens, size_t nbits, int32_t min_value,
                    int32_t max_value, const uint8_t* found, size_t found_len, rbg_buffer* out) {
  if (!out || op < 0 || op > BSI_RANGE) return RBG_ERR_ILLEGAL_ARGUMENT;
  Ctx* c;
  CHK(tl_ctx(&c));
  BatchGuard g{c, {}};
  int32_t id;
  CHK(bsi_load(c, ebm, ebm_len, slices, slice_lens, nbits, found, found_len, &id));
  g.ids.push_back(id);
  CHK(ctx_bsi(c, id, op, (int)nbits, found ? 1 : 0, start, end, min_value, max_value, 0));
  return ctx_fetch(c, out);
}
int rbg_bsi_compare_buffer(int op, int32_t start, int32_t end, const uint8_t* ebm, size_t ebm_len,
                           const uint8_t* const* slices, const size_t* slice_lens, size_t nbits, int32_t min_value,
                           int32_t max_value, const uint8_t* found, size_t found_len, rbg_buffer* out) {
  if (!out || op < 0 || op > RBG_BSI_RANGE_NEQ_DIRECT) return RBG_ERR_ILLEGAL_ARGUMENT;
  Ctx* c;
  CHK(tl_ctx(&c));
  BatchGuard g{c, {}};
  int32_t id;
  CHK(bsi_load(c, ebm, ebm_len, slices, slice_lens, nbits, found, found_len, &id));
  g.ids.push_back(id);
  CHK(ctx_bsi_buffer(c, id, op, (int)nbits, found ? 1 : 0, start, end, min_value, max_value));
  return ctx_fetch(c, out);
}
int rbg_ctx_bsi_buffer(rbg_ctx* ctx, int32_t batch, int op, int nbits, int has_found, int32_t start, int32_t end,
                       int32_t min_value, int32_t max_value) {
  CHK(enter(&ctx->c));
  return ctx_bsi_buffer(&ctx->c, batch, op, nbits, has_found, start, end, min_value, max_value);
}
int rbg_bsi_sum(const uint8_t* ebm, size_t ebm_len, const uint8_t* const* slices, const size_t* slice_lens,
                size_t nbits, const uint8_t* found, size_t found_len, int64_t* out2) {
  if (!out2) return RBG_ERR_ILLEGAL_ARGUMENT;
  if (!found) {  // BSI/:582: null foundSet -> (0, 0)
    out2[0] = out2[1] = 0;
    return RBG_OK;
  }
  Ctx* c;
  CHK(tl_ctx(&c));
  BatchGuard g{c, {}};
  int32_t id;
  CHK(bsi_load(c, ebm, ebm_len, slices, slice_lens, nbits, found, found_len, &id));
  g.ids.push_back(id);
  CHK(ctx_bsi(c, id, BSI_SUM_ONLY, (int)nbits, 1, 0, 0, 0, 0, 1));
  return ctx_bsi_sums(c, out2);
}
int rbg_debug_stamps(uint64_t* out20, int reset) {
  if (!out20) return RBG_ERR_ILLEGAL_ARGUMENT;
  if (getenv("RBG_DEBUG_BSI")) debug_bsi_stamps(out20, reset != 0);
  else debug_stamps(out20, reset != 0);
  return RBG_OK;
}
int rbg_ctx_pair_bytes(rbg_ctx* ctx, int32_t batch, int64_t* out2) {
  Batch* b;
  CHK(get_batch(&ctx->c, batch, &b));
  if (!out2 || b->key_major || b->n_bm % 2) {
    set_err("needs a bitmap-major batch of pairs");
    return RBG_ERR_ILLEGAL_ARGUMENT;
  }
  CHK(enter(&ctx->c));
  HIPCHK(hipStreamSynchronize(ctx->c.stream));
  std::vector<CDesc> d(b->n_ctr);
  if (b->n_ctr) HIPCHK(hipMemcpy(d.data(), b->desc.p, sizeof(CDesc) * b->n_ctr, hipMemcpyDeviceToHost));
  auto pay = [](const CDesc& x) -> int64_t { return x.kind == KA ? 2 * (int64_t)x.card : x.kind == KB ? 8192 : 0; };
  int64_t matched = 0, all = 0;
  for (size_t p = 0; p < b->n_bm / 2; p++) {
    uint32_t i = b->h_bm_off[2 * p], ie = b->h_bm_off[2 * p + 1], j = ie, je = b->h_bm_off[2 * p + 2];
    all += 4 * (int64_t)(je - i);
    while (i < ie && j < je) {
      if (d[i].key == d[j].key) {
        matched += pay(d[i++]) + pay(d[j++]);
      } else if (d[i].key < d[j].key) {
        i++;
      } else {
        j++;
      }
    }
  }
  out2[0] = matched + all;  // matched payload + descriptors
  int64_t tot = 0;
  for (const CDesc& x : d) tot += pay(x) + 4;
  out2[1] = tot;  // every payload + descriptors
  return RBG_OK;
}
int rbg_ctx_wide_card(rbg_ctx* ctx, int op, int32_t batch, int key_lo, int key_hi) {
  CHK(enter(&ctx->c));
  int hc;
  bool hv;
  CHK(ctx_wide(&ctx->c, op, batch, key_lo, key_hi, nullptr, true, &hc, &hv));
  if (hv) {
    ResultInfo ri = {};
    ri.card32 = (uint32_t)hc;
    ri.long_card = hc;
    HIPCHK(hipMemcpyAsync(ctx->c.info.p, &ri, sizeof(ri), hipMemcpyHostToDevice, ctx->c.stream));
    HIPCHK(hipStreamSynchronize(ctx->c.stream));
  }
  return RBG_OK;
}
int rbg_ctx_batch_and_card(rbg_ctx* ctx, int32_t batch) {
  CHK(enter(&ctx->c));
  return ctx_batch_card(&ctx->c, batch);
}
int rbg_ctx_card(rbg_ctx* ctx, int32_t* out) {
  CHK(enter(&ctx->c));
  ResultInfo ri;
  CHK(ctx_info(&ctx->c, &ri));
  *out = (int32_t)ri.card32;
  return RBG_OK;
}
int rbg_ctx_cards(rbg_ctx* ctx, int32_t* out, size_t n) {
  CHK(enter(&ctx->c));
  if (n > ctx->c.n_cards) return RBG_ERR_ILLEGAL_ARGUMENT;
  HIPCHK(hipMemcpyAsync(out, ctx->c.cards.p, 4 * n, hipMemcpyDeviceToHost, ctx->c.stream));
  HIPCHK(hipStreamSynchronize(ctx->c.stream));
  return RBG_OK;
}
int rbg_ctx_result_stats(rbg_ctx* ctx, int64_t* st) {
  CHK(enter(&ctx->c));
  ResultInfo ri;
  CHK(ctx_info(&ctx->c, &ri));
  st[0] = ri.n_out;
  st[1] = (int64_t)ri.payload;
  st[2] = ri.has_run;
  st[3] = ri.long_card;
  return RBG_OK;
}
int rbg_ctx_serialize(rbg_ctx* ctx) {
  CHK(enter(&ctx->c));
  return ctx_serialize(&ctx->c);
}
int rbg_ctx_fetch(rbg_ctx* ctx, rbg_buffer* out) {
  CHK(enter(&ctx->c));
  return ctx_fetch(&ctx->c, out);
}
// Key-shard placement of the pending result inside a global portable bitmap of
// total_containers containers, enqueued on the context stream.
static int ctx_fetch_shard_device(Ctx* c, int64_t total_containers, int has_run, int64_t payload_base, void* desc_dst,
                                  void* offsets_dst, void* runflag_dst, void* payload_dst) {
  if (c->last != 1) {
    set_err("no materialised result pending");
    return RBG_ERR_ILLEGAL_ARGUMENT;
  }
  if (total_containers < 0 || total_containers > kMaxKeys || payload_base < 0 || !desc_dst || !payload_dst) {
    set_err("fetch_shard: bad layout or null destination");
    return RBG_ERR_ILLEGAL_ARGUMENT;
  }
  const bool offsets = !has_run || total_containers >= 4;  // RB/RoaringArray.java:927-933
  if (offsets && !offsets_dst) {
    set_err("fetch_shard: the global bitmap has an offset table; offsets_dst is required");
    return RBG_ERR_ILLEGAL_ARGUMENT;
  }
  // the result's facts: read by the result_stats call that sized the global layout (which also
  // reported a timed-out spin as RBG_ERR_DEVICE), so the fetch stays asynchronous; without one,
  // ctx_info synchronises here
  ResultInfo ri;
  if (c->ri_valid) {
    ri = c->last_ri;
    CHK(ensure_placed(c));
  } else {
    CHK(ctx_info(c, &ri));
  }
  const uint64_t off0 = header_size((size_t)total_containers, has_run != 0) + (uint64_t)payload_base;
  if (off0 > 0xFFFFFFFFull) {
    set_err("fetch_shard: payload offsets exceed 32 bits");
    return RBG_ERR_ILLEGAL_ARGUMENT;
  }
  uint8_t* emit_dst = (uint8_t*)payload_dst;
  if (c->serialized) {
    // already serialized (possibly because an operand batch was released since): copy the
    // payload region rather than re-reading the operands' pass-through containers
    if (ri.payload)
      HIPCHK(hipMemcpyAsync(payload_dst, c->result.as<uint8_t>() + c->pending.payload_base, ri.payload,
                            hipMemcpyDeviceToDevice, c->stream));
    emit_dst = nullptr;
  }
  launch_serialize_shard(c->stream, grid_for((c->pending_ub + 255) / 256, 256), c->ntasks.as<uint32_t>(), c->pending,
                         emit_dst, off0, (uint8_t*)desc_dst, offsets ? (uint8_t*)offsets_dst : nullptr,
                         has_run ? (uint8_t*)runflag_dst : nullptr);
  HIPCHK(hipGetLastError());
  return RBG_OK;
}

int rbg_ctx_result_layout_device(rbg_ctx* ctx, void* dst3) {
  if (!ctx || !dst3) return RBG_ERR_ILLEGAL_ARGUMENT;
  Ctx* c = &ctx->c;
  CHK(enter(c));
  if (c->last != 1) {
    set_err("no materialised result pending");
    return RBG_ERR_ILLEGAL_ARGUMENT;
  }
  if (c->place_pending) {  // the placement writes the layout too (one launch fewer per sharded step)
    OutCtx o = c->pending;
    o.layout_out = reinterpret_cast<int64_t*>(dst3);
    launch_place(c->stream, c->ntasks.as<uint32_t>(), o, c->info.as<ResultInfo>());
    c->place_pending = false;
  } else {
    launch_layout_out(c->stream, c->info.as<ResultInfo>(), reinterpret_cast<int64_t*>(dst3));
  }
  HIPCHK(hipGetLastError());
  return RBG_OK;
}
int rbg_ctx_fetch_shard_device_dyn(rbg_ctx* ctx, const void* layout, int rank, int world, void* out, void* runb) {
  if (!ctx || !layout || !out || world < 1 || world > 1024 || rank < 0 || rank >= world)
    return RBG_ERR_ILLEGAL_ARGUMENT;
  Ctx* c = &ctx->c;
  CHK(enter(c));
  if (c->last != 1) {
    set_err("no materialised result pending");
    return RBG_ERR_ILLEGAL_ARGUMENT;
  }
  CHK(ensure_placed(c));
  // an already serialized result's pass-through records may point into released operands: copy its
  // payload region instead (like rbg_ctx_fetch_shard_device); not expected on the sharded path
  if (c->serialized) {
    set_err("fetch_shard_device_dyn: the result was already serialized; fetch it before releasing operands "
            "or use rbg_ctx_fetch_shard_device");
    return RBG_ERR_ILLEGAL_ARGUMENT;
  }
  launch_serialize_shard_dyn(c->stream, grid_for((c->pending_ub + 255) / 256, 256), c->ntasks.as<uint32_t>(), c->pending,
                             reinterpret_cast<const int64_t*>(layout), rank, world, (uint8_t*)out, (uint8_t*)runb, true);
  HIPCHK(hipGetLastError());
  return RBG_OK;
}
int rbg_ctx_fetch_shard_device(rbg_ctx* ctx, int64_t total_containers, int has_run, int64_t payload_base,
                               void* desc_dst, void* offsets_dst, void* runflag_dst, void* payload_dst) {
  if (!ctx) return RBG_ERR_ILLEGAL_ARGUMENT;
  CHK(enter(&ctx->c));
  return ctx_fetch_shard_device(&ctx->c, total_containers, has_run, payload_base, desc_dst, offsets_dst, runflag_dst,
                                payload_dst);
}

int rbg_ctx_fetch_shard(rbg_ctx* ctx, int64_t total_containers, int has_run, int64_t first_container,
                        int64_t payload_base, rbg_buffer* out_desc, rbg_buffer* out_offsets, rbg_buffer* out_payload) {
  if (!ctx || !out_desc || !out_offsets || !out_payload) return RBG_ERR_ILLEGAL_ARGUMENT;
  Ctx& c = ctx->c;
  CHK(enter(&c));
  (void)first_container;  // the shard's own buffers start at its first container
  ResultInfo ri;
  CHK(ctx_info(&c, &ri));
  const size_t n = ri.n_out;
  const bool offsets = !has_run || total_containers >= 4;
  DevBuf d;
  CHK(d.ensure(9 * n + ri.payload + 64));
  uint8_t* base = d.as<uint8_t>();
  CHK(ctx_fetch_shard_device(&c, total_containers, has_run, payload_base, base, base + 4 * n, base + 8 * n,
                             base + 9 * n));
  std::vector<uint8_t> h(9 * n + ri.payload);
  if (!h.empty()) HIPCHK(hipMemcpyAsync(h.data(), base, h.size(), hipMemcpyDeviceToHost, c.stream));
  HIPCHK(hipStreamSynchronize(c.stream));
  CHK(emit_host(std::vector<uint8_t>(h.begin(), h.begin() + 4 * n), out_desc));
  CHK(emit_host(offsets ? std::vector<uint8_t>(h.begin() + 4 * n, h.begin() + 8 * n) : std::vector<uint8_t>(),
                out_offsets));
  return emit_host(std::vector<uint8_t>(h.begin() + 9 * n, h.end()), out_payload);
}

// C3 synthetic key slice [key_lo, key_hi) of n bitmaps (kind 1 uniform, 2 clustered)
static int synth_c3(Ctx* c, int kind, uint64_t seed, size_t n, int key_lo, int key_hi, int32_t* out_id) {
  key_lo = std::max(0, key_lo);
  key_hi = std::min(kMaxKeys, key_hi);
  if (n == 0 || n > 0x7FFFFFFF || key_hi < key_lo) {
    set_err("synthetic C3 needs 0 < n and key_lo <= key_hi");
    return RBG_ERR_ILLEGAL_ARGUMENT;
  }
  const int nkeys = key_hi - key_lo;
  hipStream_t s = c->stream;
  std::vector<uint32_t> key_off(kMaxKeys + 1, 0);
  std::vector<uint16_t> h_keys;
  std::vector<uint32_t> h_bm, nctr(n, 0);
  if (kind == 1) {
    for (int k = 0; k < kMaxKeys; k++) {
      const bool in = k >= key_lo && k < key_hi;
      key_off[k + 1] = key_off[k] + (in ? (uint32_t)n : 0u);
    }
    for (size_t i = 0; i < n; i++) nctr[i] = (uint32_t)nkeys;
  } else {
    std::vector<uint32_t> base(n);
    for (size_t i = 0; i < n; i++) {
      base[i] = c3c_base(seed, (uint32_t)i);
      for (uint32_t k = base[i]; k < base[i] + 16; k++)
        if ((int)k >= key_lo && (int)k < key_hi) {
          key_off[k + 1]++;
          nctr[i]++;
        }
    }
    for (int k = 0; k < kMaxKeys; k++) key_off[k + 1] += key_off[k];
    h_keys.resize(key_off[kMaxKeys]);
    h_bm.resize(key_off[kMaxKeys]);
    std::vector<uint32_t> cur(key_off.begin(), key_off.end() - 1);
    for (size_t i = 0; i < n; i++)  // ascending i: input order within each key
      for (uint32_t k = base[i]; k < base[i] + 16; k++)
        if ((int)k >= key_lo && (int)k < key_hi) {
          h_keys[cur[k]] = (uint16_t)k;
          h_bm[cur[k]++] = (uint32_t)i;
        }
  }
  const size_t C = key_off[kMaxKeys];
  const int32_t id = new_batch(c);
  Batch& b = *c->batches[id];
  b.n_bm = n;
  b.n_ctr = C;
  b.key_major = true;
  b.h_bm_nctr = nctr;
  b.h_bm_card.assign(n, 0);
  CHK(b.keys.ensure(2 * C + 16));
  CHK(b.desc.ensure(sizeof(CDesc) * C + 16));
  CHK(b.bm.ensure(4 * C + 16));
  CHK(b.key_off.ensure(4 * (kMaxKeys + 1)));
  CHK(b.bm_off.ensure(8));
  HIPCHK(hipMemcpyAsync(b.key_off.p, key_off.data(), 4 * (kMaxKeys + 1), hipMemcpyHostToDevice, s));
  if (kind == 1) {
    CHK(c->scratch.ensure(16 * (size_t)kMaxKeys));
    unsigned long long* kb = c->scratch.as<unsigned long long>();
    launch_synth_c3u(s, seed, (uint32_t)n, key_lo, nkeys, kb, nullptr, nullptr, nullptr, nullptr, nullptr, 0);
    std::vector<unsigned long long> bytes(nkeys + 1, 0);
    if (nkeys) HIPCHK(hipMemcpyAsync(bytes.data(), kb, 8 * nkeys, hipMemcpyDeviceToHost, s));
    HIPCHK(hipStreamSynchronize(s));
    unsigned long long tot = 0;
    for (int k = 0; k < nkeys; k++) {
      const unsigned long long x = bytes[k];
      bytes[k] = tot;
      tot += x;
    }
    b.payload_bytes = tot;
    CHK(b.payload.ensure(tot + 64));
    HIPCHK(hipMemcpyAsync(kb, bytes.data(), 8 * std::max(nkeys, 1), hipMemcpyHostToDevice, s));
    launch_synth_c3u(s, seed, (uint32_t)n, key_lo, nkeys, nullptr, kb, b.desc.as<CDesc>(), b.keys.as<uint16_t>(),
                     b.bm.as<uint32_t>(), b.payload.as<uint8_t>(), 1);
    b.n_kind[DK_A] = (int64_t)C;
    b.packed = true;
  } else {
    b.payload_bytes = 8192 * C;
    CHK(b.payload.ensure(b.payload_bytes + 64));
    if (C) {
      HIPCHK(hipMemcpyAsync(b.keys.p, h_keys.data(), 2 * C, hipMemcpyHostToDevice, s));
      HIPCHK(hipMemcpyAsync(b.bm.p, h_bm.data(), 4 * C, hipMemcpyHostToDevice, s));
    }
    launch_synth_c3c(s, seed, C, b.keys.as<uint16_t>(), b.bm.as<uint32_t>(), b.desc.as<CDesc>(),
                     b.payload.as<uint8_t>());
    b.n_kind[DK_B] = (int64_t)C;
  }
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemsetAsync(c->scalar.p, 0, 8, s));
  launch_sum_cards(s, b.desc.as<CDesc>(), C, c->scalar.as<unsigned long long>());
  unsigned long long card = 0;
  HIPCHK(hipMemcpyAsync(&card, c->scalar.p, 8, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  b.long_card = (int64_t)card;
  b.ser_bytes = 0;
  b.live = true;
  *out_id = id;
  return RBG_OK;
}

// C4: n pairs = 2n small bitmaps, bitmap-major (pairs adjacent).  Each bitmap has
// K in [1,4] keys from [0,64), each an array container of card in [16,512].
static int synth_c4(Ctx* c, uint64_t seed, size_t n_pairs, int32_t* out_id) {
  const size_t nb = 2 * n_pairs;
  if (nb == 0 || nb > 0x7FFFFFFF) return RBG_ERR_ILLEGAL_ARGUMENT;
  const int32_t id = new_batch(c);
  Batch& b = *c->batches[id];
  b.n_bm = nb;
  b.key_major = false;
  b.h_bm_off.assign(nb + 1, 0);
  b.h_bm_nctr.resize(nb);
  b.h_bm_card.resize(nb);
  std::vector<CDesc> d;
  d.reserve(nb * 5 / 2 + 16);
  uint64_t off = 0;
  for (size_t j = 0; j < nb; j++) {
    const uint64_t h = splitmix64(seed ^ (0xC4000000ULL + j));
    const int K = 1 + (int)(h % 4);
    uint64_t used = 0;
    int got = 0;
    for (uint64_t t = 1; got < K; t++) {
      const int k = (int)(splitmix64(h + t) & 63);
      if (!((used >> k) & 1)) {
        used |= 1ULL << k;
        got++;
      }
    }
    int64_t card_sum = 0;
    for (int k = 0; k < 64; k++)
      if ((used >> k) & 1) {
        const uint32_t card = 16 + (uint32_t)(splitmix64(h ^ ((uint64_t)k << 40)) % 497);
        d.push_back(CDesc{off, card, (uint16_t)k, DK_A, 0});
        off += (2 * card + 15) & ~15ull;
        card_sum += card;
      }
    b.h_bm_nctr[j] = (uint32_t)K;
    b.h_bm_off[j + 1] = b.h_bm_off[j] + (uint32_t)K;
    b.h_bm_card[j] = card_sum;
    b.long_card += card_sum;
  }
  const size_t C = d.size();
  b.n_ctr = C;
  b.n_kind[DK_A] = (int64_t)C;
  b.payload_bytes = off;
  CHK(b.desc.ensure(sizeof(CDesc) * C + 16));
  CHK(b.keys.ensure(2 * C + 16));
  CHK(b.bm.ensure(4 * C + 16));
  CHK(b.bm_off.ensure(4 * (nb + 1)));
  CHK(b.payload.ensure(off + 64));
  hipStream_t s = c->stream;
  std::vector<uint16_t> hk(C);
  std::vector<uint32_t> hbm(C);
  for (size_t j = 0; j < nb; j++)
    for (uint32_t p = b.h_bm_off[j]; p < b.h_bm_off[j + 1]; p++) {
      hk[p] = d[p].key;
      hbm[p] = (uint32_t)j;
    }
  HIPCHK(hipMemcpyAsync(b.desc.p, d.data(), sizeof(CDesc) * C, hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(b.keys.p, hk.data(), 2 * C, hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(b.bm.p, hbm.data(), 4 * C, hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(b.bm_off.p, b.h_bm_off.data(), 4 * (nb + 1), hipMemcpyHostToDevice, s));
  launch_synth_arrays(s, seed, b.desc.as<CDesc>(), C, b.payload.as<uint8_t>());
  HIPCHK(hipGetLastError());
  HIPCHK(hipStreamSynchronize(s));
  b.live = true;
  *out_id = id;
  return RBG_OK;
}

// C5: a bit-sliced index over rows 0..rows-1 with 31 slices, as the key-major batch
// [ebM, bA[0..30]] of rbg_ctx_bsi; the value min / max go to b.bsi_min / bsi_max
static int synth_c5(Ctx* c, uint64_t seed, size_t rows, int key_lo, int key_hi, int32_t* out_id) {
  const int nbits = 31, nin = nbits + 1;
  if (rows == 0 || rows > (1ull << 32)) return RBG_ERR_ILLEGAL_ARGUMENT;
  key_lo = std::max(0, key_lo);
  key_hi = (int)std::min<uint64_t>((uint64_t)std::min(key_hi, kMaxKeys), (rows + 65535) / 65536);
  const int nkeys = std::max(0, key_hi - key_lo);
  hipStream_t s = c->stream;
  const size_t G = (size_t)nkeys * nin;
  CHK(c->scratch.ensure(8 * G + 64));
  uint32_t* cards = c->scratch.as<uint32_t>();
  uint32_t* pos = cards + G;
  unsigned int* mm = reinterpret_cast<unsigned int*>(c->scalar.p);
  const unsigned int mm0[2] = {0xFFFFFFFFu, 0u};
  HIPCHK(hipMemcpyAsync(mm, mm0, 8, hipMemcpyHostToDevice, s));
  launch_synth_c5(s, seed, rows, key_lo, nbits, nkeys, 0, cards, nullptr, mm, nullptr, nullptr, nullptr, nullptr);
  std::vector<uint32_t> h(G);
  unsigned int mmh[2];
  HIPCHK(hipMemcpyAsync(h.data(), cards, 4 * G, hipMemcpyDeviceToHost, s));
  HIPCHK(hipMemcpyAsync(mmh, mm, 8, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  std::vector<uint32_t> key_off(kMaxKeys + 1, 0), hp(G, 0);
  uint32_t C = 0;
  for (int k = 0; k < kMaxKeys; k++) {
    const int j = k - key_lo;
    if (j >= 0 && j < nkeys)
      for (int i = 0; i < nin; i++)
        if (h[(size_t)j * nin + i]) hp[(size_t)j * nin + i] = C++;
    key_off[k + 1] = C;
  }
  const int32_t id = new_batch(c);
  Batch& b = *c->batches[id];
  b.n_bm = nin;
  b.n_ctr = C;
  b.key_major = true;
  b.payload_bytes = (size_t)kSlotBytes * C;
  b.h_bm_nctr.assign(nin, 0);
  b.h_bm_card.assign(nin, 0);
  for (int k = 0; k < nkeys; k++)
    for (int i = 0; i < nin; i++)
      if (h[(size_t)k * nin + i]) {
        b.h_bm_nctr[i]++;
        b.h_bm_card[i] += h[(size_t)k * nin + i];
      }
  for (int i = 0; i < nin; i++) b.long_card += b.h_bm_card[i];
  CHK(b.keys.ensure(2 * (size_t)C + 16));
  CHK(b.desc.ensure(sizeof(CDesc) * (size_t)C + 16));
  CHK(b.bm.ensure(4 * (size_t)C + 16));
  CHK(b.key_off.ensure(4 * (kMaxKeys + 1)));
  CHK(b.bm_off.ensure(8));
  CHK(b.payload.ensure(b.payload_bytes + 64));
  HIPCHK(hipMemcpyAsync(b.key_off.p, key_off.data(), 4 * (kMaxKeys + 1), hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(pos, hp.data(), 4 * G, hipMemcpyHostToDevice, s));
  launch_synth_c5(s, seed, rows, key_lo, nbits, nkeys, 1, nullptr, pos, nullptr, b.desc.as<CDesc>(),
                  b.keys.as<uint16_t>(),
                  b.bm.as<uint32_t>(), b.payload.as<uint8_t>());
  HIPCHK(hipGetLastError());
  std::vector<CDesc> d(C);
  if (C) HIPCHK(hipMemcpyAsync(d.data(), b.desc.p, sizeof(CDesc) * C, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  for (const CDesc& x : d) b.n_kind[x.kind]++;
  b.bsi_min = (int32_t)mmh[0];
  b.bsi_max = (int32_t)mmh[1];
  b.live = true;
  *out_id = id;
  return RBG_OK;
}

// RoaringBitmap.runOptimize (RB/RoaringBitmap.java:2764-2774) over every bitmap of a
// batch, into a new batch: plan (new kind + slot size per container), scan of the
// slot sizes, write.  answers[i] = 1 iff bitmap i holds a run container afterwards.

static int ctx_run_optimize(Ctx* c, int32_t id, int32_t* out_id, uint8_t* answers) {
  Batch* a;
  CHK(get_batch(c, id, &a));
  if (a->packed) {
    set_err("runOptimize needs slot-aligned payloads (not a packed synthetic batch)");
    return RBG_ERR_ILLEGAL_ARGUMENT;
  }
  hipStream_t s = c->stream;
  const size_t C = a->n_ctr, n = a->n_bm;
  // one kernel: every container is written at its own slot offset (a conversion never makes a slot
  // larger), so the new batch has the input's payload size and layout and nothing waits on the host
  const int32_t bid = new_batch(c);
  Batch& b = *c->batches[bid];
  struct Drop {  // an error below frees the half-built batch
    Ctx* c;
    int32_t id;
    bool keep = false;
    ~Drop() {
      if (!keep) c->batches[id].reset();
    }
  } drop{c, bid};
  CHK(pool_take(c, b.desc, sizeof(CDesc) * C + 16));
  CHK(pool_take(c, b.payload, a->payload_bytes + 64));
  b.ro_groups = runopt_groups(C);
  CHK(pool_take(c, b.ro_stats, ro_flags_off(b.ro_groups) + 4 * n + 16));
  CHK(pool_take(c, b.keys, a->keys.cap));
  CHK(pool_take(c, b.bm, a->bm.cap));
  CHK(pool_take(c, b.key_off, a->key_off.cap));
  CHK(pool_take(c, b.bm_off, a->bm_off.cap));
  const RoCopy cp{a->keys.as<uint16_t>(), b.keys.as<uint16_t>(), a->bm.as<uint32_t>(), b.bm.as<uint32_t>(),
                  a->key_off.as<uint32_t>(), b.key_off.as<uint32_t>(), a->key_off.cap / 4,
                  a->bm_off.as<uint32_t>(), b.bm_off.as<uint32_t>(), a->bm_off.cap / 4};
  if (C)
    launch_runopt(s, a->desc.as<CDesc>(), a->payload.as<uint8_t>(), C, b.desc.as<CDesc>(), b.payload.as<uint8_t>(), cp,
                  b.ro_stats.as<unsigned long long>() + 8);
  HIPCHK(hipGetLastError());
  // no host read-back here: the new batch's statistics stay on the device until needed (ensure_stats)
  b.n_bm = n;
  b.n_ctr = C;
  b.key_major = a->key_major;
  b.h_bm_off = a->h_bm_off;
  b.h_bm_nctr = a->h_bm_nctr;
  b.h_bm_card = a->h_bm_card;
  b.long_card = a->long_card;
  b.bsi_min = a->bsi_min;
  b.bsi_max = a->bsi_max;
  b.payload_bytes = a->payload_bytes;  // the input's layout (holes after shrunk containers)
  b.gapped = a->gapped || a->n_kind[DK_R] > 0;  // only R -> A can leave an all-array batch with holes
  b.max_ser = 0;  // runOptimize leaves no container above 8194 serialized bytes
  b.ser_bytes = a->ser_bytes ? 1 : 0;  // nonzero: computed by ensure_stats
  b.stats_pending = true;
  b.live = true;
  drop.keep = true;
  *out_id = bid;
  if (answers) {  // runOptimize's boolean per bitmap: the statistics now
    CHK(ensure_stats(c, &b));
    for (size_t i = 0; i < n; i++) answers[i] = b.h_has_run[i];
  }
  return RBG_OK;
}

// selectRangeWithoutCopy (RB/RoaringBitmap.java:3160-3214) of every bitmap of a key-major batch into a
// new batch, on the device (runopt.hip: k_rsel_plan, two scans, k_rsel_write, the key CSR); one host
// read-back for the new batch's container counts.  rangeSanityCheck (:204-213) first.
// x.selectRange(rangeStart, rangeEnd) (RB/RoaringBitmap.java:3095-3147; buffer RB/buffer/ImmutableRoaringBitmap.java
// :701-757): no rangeSanityCheck (the range aggregations, which do check, call check_range first); the high and
// low bits are the reference's char casts of rangeStart and rangeEnd - 1 (Util.highbits / lowbits, RB/Util.java
// :436-438,481-483), so selectRange(x, Long.MAX_VALUE) keeps [start, 0xFFFFFFFF).  Divergences, raised as
// IllegalArgumentException: a negative bound (the reference's assert) and casts that put the last key below the
// first (the reference would append keys out of order).
static int ctx_select_range(Ctx* c, int32_t id, int64_t start, int64_t end, int32_t* out_id, bool buf) {
  if (start < 0 || end < 0) {
    set_err("selectRange: rangeStart and rangeEnd must not be negative");
    return RBG_ERR_ILLEGAL_ARGUMENT;
  }
  if (end > start && ((uint64_t)start >> 16 & 0xFFFF) > ((uint64_t)(end - 1) >> 16 & 0xFFFF)) {
    set_err("selectRange: the range's key casts are out of order (the reference would build an unsorted bitmap)");
    return RBG_ERR_ILLEGAL_ARGUMENT;
  }
  Batch* a;
  CHK(get_batch(c, id, &a));
  if (!a->key_major || a->packed) {
    set_err("range selection needs a key-major batch with slot-aligned payloads");
    return RBG_ERR_ILLEGAL_ARGUMENT;
  }
  hipStream_t s = c->stream;
  const size_t C = a->n_ctr, n = a->n_bm;
  RselArgs ra{1, 0, 0, 0, buf ? 1 : 0};  // end <= start: no key is kept
  if (end > start) {  // (char) casts: Util.highbits / lowbits
    ra.hbs = (int)((uint64_t)start >> 16 & 0xFFFF);
    ra.lbs = (int)(start & 0xFFFF);
    ra.hbl = (int)((uint64_t)(end - 1) >> 16 & 0xFFFF);
    ra.lbl = (int)((end - 1) & 0xFFFF);
  }
  CHK(c->ro_info.ensure(4 * C + 16));
  CHK(c->ro_size.ensure(8 * C + 16));
  CHK(c->ro_part.ensure(8 * (scan_parts(std::max<size_t>(C, 1)) + 1)));
  CHK(c->rs_card.ensure(4 * C + 16));
  CHK(c->rs_keep.ensure(8 * C + 16));
  CHK(c->rs_bm.ensure(16 * n + 64 + 16));  // per bitmap: kept containers, cardinality; then the totals
  const int32_t bid = new_batch(c);
  Batch& b = *c->batches[bid];
  BatchGuard guard{c, {bid}};  // dropped unless the selection completes
  CHK(pool_take(c, b.desc, sizeof(CDesc) * C + 16));
  CHK(pool_take(c, b.payload, a->payload_bytes + 64));
  CHK(b.keys.ensure(2 * C + 16));
  CHK(b.bm.ensure(4 * C + 16));
  CHK(b.key_off.ensure(4 * (kMaxKeys + 1)));
  CHK(b.bm_off.ensure(4 * (n + 1)));
  unsigned long long* bm_cnt = c->rs_bm.as<unsigned long long>();
  unsigned long long* bm_card = bm_cnt + n;
  unsigned long long* tot = bm_cnt + 2 * n;  // #A, #B, #R, big bytes, then the two scan totals
  HIPCHK(hipMemsetAsync(c->rs_bm.p, 0, 16 * n + 64, s));
  launch_rsel_plan(s, a->desc.as<CDesc>(), a->bm.as<uint32_t>(), a->payload.as<uint8_t>(), C, ra,
                   c->ro_info.as<uint32_t>(), c->rs_card.as<uint32_t>(), c->ro_size.as<uint64_t>(),
                   c->rs_keep.as<uint64_t>(), bm_cnt, bm_card, tot);
  launch_exclusive_scan(s, c->ro_size.as<uint64_t>(), c->ro_size.as<uint64_t>(), C, c->ro_part.as<uint64_t>(),
                        reinterpret_cast<uint64_t*>(tot + 4));
  launch_exclusive_scan(s, c->rs_keep.as<uint64_t>(), c->rs_keep.as<uint64_t>(), C, c->ro_part.as<uint64_t>(),
                        reinterpret_cast<uint64_t*>(tot + 5));
  launch_rsel_write(s, a->desc.as<CDesc>(), a->bm.as<uint32_t>(), a->payload.as<uint8_t>(), C, ra,
                    c->ro_info.as<uint32_t>(), c->rs_card.as<uint32_t>(), c->ro_size.as<uint64_t>(),
                    c->rs_keep.as<uint64_t>(), b.desc.as<CDesc>(), b.keys.as<uint16_t>(), b.bm.as<uint32_t>(),
                    b.payload.as<uint8_t>());
  HIPCHK(hipGetLastError());
  std::vector<unsigned long long> h(2 * n + 8);
  HIPCHK(hipMemcpyAsync(h.data(), c->rs_bm.p, 8 * (2 * n + 6), hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  const unsigned long long* t = h.data() + 2 * n;
  const uint64_t C2 = t[5];
  launch_dec_key_off(s, b.keys.as<uint16_t>(), C2, b.key_off.as<uint32_t>());
  b.n_bm = n;
  b.n_ctr = C2;
  b.key_major = true;
  for (int k = 0; k < 3; k++) b.n_kind[k] = (int64_t)t[k];
  b.max_ser = t[3];
  b.payload_bytes = t[4];
  b.h_bm_off.assign(n + 1, 0);
  b.h_bm_nctr.resize(n);
  b.h_bm_card.resize(n);
  for (size_t i = 0; i < n; i++) {
    b.h_bm_nctr[i] = (uint32_t)h[i];
    b.h_bm_off[i + 1] = b.h_bm_off[i] + (uint32_t)h[i];
    b.h_bm_card[i] = (int64_t)h[n + i];
    b.long_card += (int64_t)h[n + i];
  }
  HIPCHK(hipMemcpyAsync(b.bm_off.p, b.h_bm_off.data(), 4 * (n + 1), hipMemcpyHostToDevice, s));
  HIPCHK(hipStreamSynchronize(s));  // the host vector above goes out of scope
  HIPCHK(hipGetLastError());
  b.live = true;
  guard.ids.clear();
  *out_id = bid;
  return RBG_OK;
}

int rbg_run_optimize_many(const uint8_t* const* bufs, const size_t* lens, size_t n, rbg_buffer* outs,
                          uint8_t* answers) {
  if (n && !outs) return RBG_ERR_ILLEGAL_ARGUMENT;
  Ctx* c;
  CHK(tl_ctx(&c));
  BatchGuard g{c, {}};
  int32_t in = -1, opt = -1;
  CHK(ctx_load(c, bufs, lens, n, &in));
  g.ids.push_back(in);
  CHK(ctx_run_optimize(c, in, &opt, answers));
  g.ids.push_back(opt);
  for (size_t i = 0; i < n; i++) {
    outs[i] = rbg_buffer{};
    const int st = ctx_batch_fetch(c, opt, i, &outs[i]);
    if (st) {
      for (size_t j = 0; j < i; j++) rbg_free(&outs[j]);
      return st;
    }
  }
  return RBG_OK;
}

int rbg_ctx_run_optimize(rbg_ctx* ctx, int32_t batch, int32_t* out_batch, uint8_t* answers) {
  if (!ctx || !out_batch) return RBG_ERR_ILLEGAL_ARGUMENT;
  CHK(enter(&ctx->c));
  return ctx_run_optimize(&ctx->c, batch, out_batch, answers);
}

int rbg_ctx_batch_minmax(rbg_ctx* ctx, int32_t batch, int32_t* out2) {
  Batch* b;
  CHK(get_batch(&ctx->c, batch, &b));
  if (!out2) return RBG_ERR_ILLEGAL_ARGUMENT;
  out2[0] = b->bsi_min;
  out2[1] = b->bsi_max;
  return RBG_OK;
}

int rbg_ctx_synth(rbg_ctx* ctx, int kind, uint64_t seed, size_t n, int key_lo, int key_hi, int32_t* batch) {
  Ctx* c = &ctx->c;
  CHK(enter(c));
  if (kind == 4) return synth_c5(c, seed, n, key_lo, key_hi, batch);
  if (kind == 1 || kind == 2) return synth_c3(c, kind, seed, n, key_lo, key_hi, batch);
  if (kind == 3) return synth_c4(c, seed, n, batch);
  // kind 0: C2 mix; 16 + DK_A/DK_B/DK_R: the same generator with one container family
  if (kind != 0 && !(kind >= 16 && kind <= 18)) {
    set_err("synthetic kind not available");
    return RBG_ERR_ILLEGAL_ARGUMENT;
  }
  const int32_t id = new_batch(c);
  Batch& b = *c->batches[id];
  const size_t C = kMaxKeys;
  b.n_bm = 1;
  b.n_ctr = C;
  b.key_major = true;
  b.payload_bytes = (size_t)kSlotBytes * C;
  CHK(b.keys.ensure(2 * C + 16));
  CHK(b.desc.ensure(sizeof(CDesc) * C + 16));
  CHK(b.bm.ensure(4 * C + 16));
  CHK(b.key_off.ensure(4 * (kMaxKeys + 1)));
  CHK(b.bm_off.ensure(8));
  CHK(b.payload.ensure(b.payload_bytes + 64));
  std::vector<uint32_t> key_off(kMaxKeys + 1);
  for (int k = 0; k <= kMaxKeys; k++) key_off[k] = (uint32_t)k;
  b.h_bm_off = {0u, (uint32_t)C};
  b.h_bm_nctr = {(uint32_t)C};
  hipStream_t s = c->stream;
  HIPCHK(hipMemsetAsync(b.bm.p, 0, 4 * C, s));
  HIPCHK(hipMemcpyAsync(b.key_off.p, key_off.data(), 4 * (kMaxKeys + 1), hipMemcpyHostToDevice, s));
  HIPCHK(hipMemcpyAsync(b.bm_off.p, b.h_bm_off.data(), 8, hipMemcpyHostToDevice, s));
  launch_synth_c2(s, seed, kind == 0 ? -1 : kind - 16, b.desc.as<CDesc>(), b.keys.as<uint16_t>(), b.payload.as<uint8_t>());
  HIPCHK(hipGetLastError());
  std::vector<CDesc> d(C);
  HIPCHK(hipMemcpyAsync(d.data(), b.desc.p, sizeof(CDesc) * C, hipMemcpyDeviceToHost, s));
  HIPCHK(hipStreamSynchronize(s));
  int64_t card = 0;
  for (const CDesc& x : d) {
    b.n_kind[x.kind]++;
    card += x.card;
  }
  b.long_card = card;
  b.h_bm_card = {card};
  b.ser_bytes = 0;
  b.live = true;
  *batch = id;
  return RBG_OK;
}

}  // extern "C"
