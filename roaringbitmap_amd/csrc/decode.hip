// Portable-format decode on the device: the host only
// concatenates the serialized inputs; headers, descriptors, run counts and payload
// placement are all resolved here.
//
// Follows RoaringArray.deserialize (RB/RoaringArray.java:547-629) and the format
// of SURVEY App. B:
//   k_dec_head  : one thread per input: cookie, size, run-flag bitset and table
//                 geometry, with the reference's checks in its order (cookie,
//                 size, "Size too large", run flags, descriptors).
//   k_dec_ctrs  : one wave per input: key, card - 1 and kind of every container
//                 (keys must strictly increase), then each payload's position.
//                 The reference walks the payloads in order (it skips the offset
//                 table); a walk is serial through run containers (a run
//                 container's length is its first u16), so the wave reads the
//                 offset table instead and proves it equal to the walk: offset 0
//                 is the end of the header and each next offset is this one plus
//                 this container's length.  Inputs without a table (run cookie,
//                 size < 4) and any input whose table is not the walk are walked
//                 serially by one lane, exactly like the reference, which also
//                 yields the reference's error for malformed inputs.
//   key-major   : stable radix sort of the container keys (input order kept
//                 within a key), the key CSR, slot sizes, an exclusive scan of
//                 them, then k_dec_fill: one wave per container writes its
//                 descriptor and copies its payload into its slot (A slots padded
//                 with the last value, R slots with the u16 pad in front).  A batch of
//                 arrays alone can be decoded packed instead: array payloads back to back
//                 at 2 B granularity, exactly as in the portable format (RB/RoaringArray.java
//                 :547-629), the layout the wide kernels read fastest.
#include <hipcub/hipcub.hpp>

#include <algorithm>

#include "kernels.hpp"
#include "wave.hpp"

namespace rbg {

__device__ __forceinline__ uint32_t rd16b(const uint8_t* p) { return (uint32_t)p[0] | ((uint32_t)p[1] << 8); }
__device__ __forceinline__ uint32_t rd32b(const uint8_t* p) {
  return (uint32_t)p[0] | ((uint32_t)p[1] << 8) | ((uint32_t)p[2] << 16) | ((uint32_t)p[3] << 24);
}

constexpr uint32_t kDecChunk = 1024;  // containers per wave of k_dec_ctrs

// DecHead::flags
constexpr uint32_t kHdRun = 1, kHdOffsets = 2, kHdOffTrunc = 4;

__global__ __launch_bounds__(256) void k_dec_head(const uint8_t* __restrict__ raw, const uint64_t* __restrict__ in_off,
                                                  const uint64_t* __restrict__ in_len, uint64_t n,
                                                  DecHead* __restrict__ hd, uint64_t* __restrict__ nctr,
                                                  uint64_t* __restrict__ nch, uint32_t* __restrict__ err,
                                                  uint32_t* __restrict__ any_err) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint8_t* p = raw + in_off[i];
  const uint64_t len = in_len[i];
  DecHead h = {};
  uint32_t e = DEC_OK;
  int64_t size = 0;
  do {
    if (len < 4) {
      e = DEC_TRUNC_COOKIE;
      break;
    }
    const uint32_t cookie = rd32b(p);
    uint64_t pos = 4;
    if ((cookie & 0xFFFF) != 12347u && cookie != 12346u) {  // RB/RoaringArray.java:557-559
      e = DEC_BAD_COOKIE;
      break;
    }
    const bool hasrun = (cookie & 0xFFFF) == 12347u;
    if (hasrun) {
      size = (int64_t)(cookie >> 16) + 1;
    } else {
      if (len < pos + 4) {
        e = DEC_TRUNC_SIZE;
        break;
      }
      size = (int32_t)rd32b(p + pos);
      pos += 4;
    }
    if (size > 65536) {  // :564-566
      e = DEC_SIZE_LARGE;
      break;
    }
    if (size < 0) {
      e = DEC_SIZE_NEG;
      break;
    }
    if (hasrun) {
      const uint64_t fl = (uint64_t)(size + 7) / 8;
      if (len < pos + fl) {
        e = DEC_TRUNC_FLAGS;
        break;
      }
      h.flags_pos = (uint32_t)pos;
      pos += fl;
    }
    if (len < pos + 4 * (uint64_t)size) {
      e = DEC_TRUNC_DESC;
      break;
    }
    h.desc_pos = (uint32_t)pos;
    pos += 4 * (uint64_t)size;
    h.flags = hasrun ? kHdRun : 0;
    if (!hasrun || size >= 4) {  // offsets present (and skipped by the reference)
      h.flags |= kHdOffsets;
      if (len < pos + 4 * (uint64_t)size) h.flags |= kHdOffTrunc;  // reported after the key check
      h.off_pos = (uint32_t)pos;
      pos += 4 * (uint64_t)size;
    }
    h.pay_pos = pos;
    h.size = (int32_t)size;
  } while (0);
  hd[i] = h;
  nctr[i] = e ? 0 : (uint64_t)size;
  nch[i] = e ? 0 : ((uint64_t)size + kDecChunk - 1) / kDecChunk;
  err[i] = e;
  if (e) atomicOr(any_err, 1u);
}

// chunk -> input table (thread per input)
__global__ __launch_bounds__(256) void k_dec_chunk_map(const uint64_t* __restrict__ nch,
                                                       const uint64_t* __restrict__ ch_base, uint64_t n,
                                                       uint32_t* __restrict__ map) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint64_t b = ch_base[i], c = nch[i];
  for (uint64_t k = 0; k < c; k++) map[b + k] = (uint32_t)i;
}

// one wave per chunk of kDecChunk containers of one input: descriptors, key order,
// and the offset table checked against the payload walk; per-input verdicts are
// OR-ed into bm_flag (1: keys out of order, 2: offsets are not the walk)
__global__ __launch_bounds__(256) void k_dec_ctrs(const uint8_t* __restrict__ raw, const uint64_t* __restrict__ in_off,
                                                  const uint64_t* __restrict__ in_len, const uint32_t* __restrict__ map,
                                                  const uint64_t* __restrict__ ch_base, const uint64_t* __restrict__ tot,
                                                  const DecHead* __restrict__ hd,
                                                  const uint64_t* __restrict__ ctr_base, DecCtr* __restrict__ q,
                                                  uint16_t* __restrict__ qkey, uint64_t* __restrict__ bm_card,
                                                  uint32_t* __restrict__ bm_flag, uint64_t* __restrict__ consumed) {
  const uint64_t nw = (uint64_t)gridDim.x * 4;
  const uint64_t n_chunks = *tot;
  const int lane = lane_id();
  for (uint64_t ch = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6); ch < n_chunks; ch += nw) {
    const uint32_t i = map[ch];
    const DecHead h = hd[i];
    const uint8_t* p = raw + in_off[i];
    const uint64_t len = in_len[i];
    const int size = h.size;
    const int kbeg = (int)(ch - ch_base[i]) * (int)kDecChunk;
    const int kend = min(size, kbeg + (int)kDecChunk);
    const uint64_t qb = ctr_base[i];
    const bool hasrun = h.flags & kHdRun;
    bool fast = (h.flags & kHdOffsets) && !(h.flags & kHdOffTrunc);
    bool bad_key = false;
    uint64_t card_sum = 0, end = 0;
    for (int k0 = kbeg; k0 < kend; k0 += 64) {
      const int k = k0 + lane;
      if (k < kend) {
        const uint8_t* d = p + h.desc_pos + 4 * (uint64_t)k;
        const uint32_t key = rd16b(d), card = rd16b(d + 2) + 1;
        if (k > 0 && rd16b(d - 4) >= key) bad_key = true;
        const bool isrun = hasrun && ((p[h.flags_pos + k / 8] >> (k % 8)) & 1);
        const uint32_t kind = isrun ? DK_R : (card > 4096 ? DK_B : DK_A);
        card_sum += card;
        DecCtr c;
        c.card = card;
        c.kind = kind;
        c.bm = i;
        c.src = 0;
        c.len = 0;
        if (fast) {
          const uint64_t at = rd32b(p + h.off_pos + 4 * (uint64_t)k);
          uint32_t l = 0;
          bool ok = true;
          if (kind == DK_R) {
            ok = at + 2 <= len;
            l = ok ? 2 + 4 * rd16b(p + at) : 0;
          } else {
            l = kind == DK_B ? 8192u : 2u * card;
          }
          if (k == 0 && at != h.pay_pos) ok = false;
          if (k + 1 < size) {
            if (rd32b(p + h.off_pos + 4 * (uint64_t)(k + 1)) != at + l) ok = false;
          } else {
            if (at + l > len) ok = false;
            end = at + l;
          }
          if (!ok) fast = false;
          c.src = in_off[i] + at;
          c.len = l;
        }
        q[qb + k] = c;
        qkey[qb + k] = (uint16_t)key;
      }
      bad_key = __ballot(bad_key) != 0;
      fast = __ballot(!fast) == 0;
    }
    for (int o = 32; o > 0; o >>= 1) card_sum += (uint64_t)__shfl_xor((long long)card_sum, o, 64);
    const uint64_t e_last = (uint64_t)__shfl((long long)end, (size - 1) & 63, 64);
    if (lane == 0) {
      atomicAdd(reinterpret_cast<unsigned long long*>(&bm_card[i]), (unsigned long long)card_sum);
      const uint32_t f = (bad_key ? 1u : 0u) | (fast ? 0u : 2u);
      if (f) atomicOr(&bm_flag[i], f);
      if (kend == size && fast) consumed[i] = e_last;
    }
  }
}

// per input: the verdict in the reference's order, and the serial payload walk
// (RB/RoaringArray.java:593-629) wherever the offset table was absent or not the walk
__global__ __launch_bounds__(256) void k_dec_finish(const uint8_t* __restrict__ raw, const uint64_t* __restrict__ in_off,
                                                    const uint64_t* __restrict__ in_len, uint64_t n,
                                                    const DecHead* __restrict__ hd,
                                                    const uint64_t* __restrict__ ctr_base,
                                                    const uint32_t* __restrict__ bm_flag, DecCtr* __restrict__ q,
                                                    uint64_t* __restrict__ consumed, uint32_t* __restrict__ err,
                                                    uint32_t* __restrict__ any_err) {
  const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n || err[i]) return;
  const DecHead h = hd[i];
  const uint32_t f = bm_flag[i];
  uint32_t e = DEC_OK;
  if (f & 1) {
    e = DEC_KEY_ORDER;
  } else if (h.flags & kHdOffTrunc) {
    e = DEC_TRUNC_OFFSETS;
  } else if (h.size == 0) {
    consumed[i] = h.pay_pos;
  } else if (f & 2) {
    const uint8_t* p = raw + in_off[i];
    const uint64_t len = in_len[i];
    const uint64_t qb = ctr_base[i];
    uint64_t pos = h.pay_pos;
    for (int k = 0; k < h.size; k++) {
      DecCtr c = q[qb + k];
      uint32_t l;
      if (c.kind == DK_B) {
        l = 8192;
      } else if (c.kind == DK_R) {
        if (len < pos + 2) {
          e = DEC_TRUNC_RUNS;
          break;
        }
        l = 2 + 4 * rd16b(p + pos);
      } else {
        l = 2 * c.card;
      }
      if (len < pos + l) {
        e = DEC_TRUNC_PAYLOAD;
        break;
      }
      c.src = in_off[i] + pos;
      c.len = l;
      q[qb + k] = c;
      pos += l;
    }
    consumed[i] = pos;
  }
  if (e) {
    err[i] = e;
    atomicOr(any_err, 1u);
  }
}

// key CSR from the sorted keys (thread per key)
__global__ __launch_bounds__(256) void k_dec_key_off(const uint16_t* __restrict__ skey, uint64_t C,
                                                     uint32_t* __restrict__ key_off) {
  const uint32_t k = blockIdx.x * blockDim.x + threadIdx.x;
  if (k > 65536) return;
  uint64_t lo = 0, hi = C;
  while (lo < hi) {
    const uint64_t m = (lo + hi) >> 1;
    if (skey[m] < k) lo = m + 1;
    else hi = m;
  }
  key_off[k] = (uint32_t)lo;
}

__device__ __forceinline__ uint64_t dec_slot_bytes(uint32_t kind, uint32_t len) {
  return kind == DK_R ? (uint64_t)((len + 2 + 15) & ~15u) : (uint64_t)((len + 15) & ~15u);
}

__global__ __launch_bounds__(256) void k_dec_sizes(const DecCtr* __restrict__ q, const uint32_t* __restrict__ perm,
                                                   uint64_t C, uint64_t* __restrict__ size,
                                                   unsigned long long* __restrict__ totals, int packed) {
  uint64_t cnt[3] = {0, 0, 0}, big = 0;
  for (uint64_t p = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; p < C; p += (uint64_t)gridDim.x * blockDim.x) {
    const DecCtr c = q[perm ? perm[p] : p];
    size[p] = packed && c.kind == DK_A ? (uint64_t)c.len : dec_slot_bytes(c.kind, c.len);
    cnt[c.kind]++;
    if (c.len > 8194) big += c.len;
  }
  for (int o = 32; o > 0; o >>= 1) {
#pragma unroll
    for (int k = 0; k < 3; k++) cnt[k] += (uint64_t)__shfl_xor((long long)cnt[k], o, 64);
    big += (uint64_t)__shfl_xor((long long)big, o, 64);
  }
  // workgroup totals, one atomic per counter per workgroup
  __shared__ unsigned long long wsum[4][4];
  if (lane_id() == 0) {
    for (int k = 0; k < 3; k++) wsum[threadIdx.x >> 6][k] = cnt[k];
    wsum[threadIdx.x >> 6][3] = big;
  }
  __syncthreads();
  if (totals && threadIdx.x < 4) {
    const unsigned long long v =
        wsum[0][threadIdx.x] + wsum[1][threadIdx.x] + wsum[2][threadIdx.x] + wsum[3][threadIdx.x];
    if (v) atomicAdd(&totals[threadIdx.x], v);
  }
}

__global__ __launch_bounds__(256) void k_dec_fill(const uint8_t* __restrict__ raw, const DecCtr* __restrict__ q,
                                                  const uint16_t* __restrict__ qkey, const uint32_t* __restrict__ perm,
                                                  const uint64_t* __restrict__ slot, uint64_t C,
                                                  CDesc* __restrict__ desc, uint16_t* __restrict__ keys,
                                                  uint32_t* __restrict__ bm, uint8_t* __restrict__ payload,
                                                  uint64_t* __restrict__ bm_card, int packed) {
  const int lane = lane_id();
  const uint64_t nw = (uint64_t)gridDim.x * 4;
  for (uint64_t p = (uint64_t)blockIdx.x * 4 + (threadIdx.x >> 6); p < C; p += nw) {
    const uint64_t src = perm ? perm[p] : p;
    const DecCtr c = q[src];
    const uint16_t key = qkey[src];
    const uint64_t off = slot[p];
    uint8_t* dst = payload + off + (c.kind == DK_R ? 2 : 0);
    group_copy<64>(dst, raw + c.src, c.len, lane);
    if (c.kind == DK_A && !packed) {  // pad the slot to 16 B with the last value
      const uint16_t last = (uint16_t)rd16b(raw + c.src + c.len - 2);
      uint16_t* d16 = reinterpret_cast<uint16_t*>(payload + off);
      for (uint32_t v = c.len / 2 + lane; v < ((c.len + 15) & ~15u) / 2; v += 64) d16[v] = last;
    }
    uint32_t card = c.card;
    if (c.kind == DK_R) {
      // The deserializer builds the RunContainer from its runs and ignores the header
      // cardinality (RB/RoaringArray.java:583-597, RunContainer.getCardinality
      // RB/RunContainer.java:1003-1009): derive it from the runs.
      const uint32_t nr = (c.len - 2) / 4;
      uint32_t s = 0;
      for (uint32_t j = lane; j < nr; j += 64) s += rd16b(raw + c.src + 2 + 4 * j + 2) + 1;
      card = (uint32_t)wave_sum_i((int)s);
      if (lane == 0 && card != c.card)
        atomicAdd(reinterpret_cast<unsigned long long*>(&bm_card[c.bm]),
                  (unsigned long long)((int64_t)card - (int64_t)c.card));
    }
    if (lane == 0) {
      desc[p] = CDesc{off, card, key, (uint8_t)c.kind, 0};
      keys[p] = key;
      bm[p] = c.bm;
    }
  }
}

__global__ __launch_bounds__(256) void k_iota(uint32_t* __restrict__ v, uint64_t n) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x)
    v[i] = (uint32_t)i;
}

static unsigned grid_of(uint64_t n, uint64_t per, uint64_t cap) {
  return (unsigned)std::max<uint64_t>(1, std::min<uint64_t>((n + per - 1) / per, cap));
}

void launch_dec_head(hipStream_t s, const uint8_t* raw, const uint64_t* in_off, const uint64_t* in_len, uint64_t n,
                     DecHead* hd, uint64_t* nctr, uint64_t* nch, uint32_t* err, uint32_t* any_err) {
  if (!n) return;
  hipLaunchKernelGGL(k_dec_head, dim3(grid_of(n, 256, 1u << 30)), dim3(256), 0, s, raw, in_off, in_len, n, hd, nctr,
                     nch, err, any_err);
}

void launch_dec_ctrs(hipStream_t s, const uint8_t* raw, const uint64_t* in_off, const uint64_t* in_len, uint64_t n,
                     const DecHead* hd, const uint64_t* ctr_base, const uint64_t* nch, const uint64_t* ch_base,
                     const uint64_t* n_chunks, uint64_t max_chunks, uint32_t* map, DecCtr* q, uint16_t* qkey,
                     uint64_t* bm_card, uint32_t* bm_flag, uint64_t* consumed, uint32_t* err, uint32_t* any_err) {
  if (!n) return;
  hipLaunchKernelGGL(k_dec_chunk_map, dim3(grid_of(n, 256, 1u << 30)), dim3(256), 0, s, nch, ch_base, n, map);
  if (max_chunks)
    hipLaunchKernelGGL(k_dec_ctrs, dim3(grid_of(max_chunks, 4, 8192)), dim3(256), 0, s, raw, in_off, in_len,
                       (const uint32_t*)map, ch_base, n_chunks, hd, ctr_base, q, qkey, bm_card, bm_flag, consumed);
  hipLaunchKernelGGL(k_dec_finish, dim3(grid_of(n, 256, 1u << 30)), dim3(256), 0, s, raw, in_off, in_len, n, hd,
                     ctr_base, (const uint32_t*)bm_flag, q, consumed, err, any_err);
}

size_t dec_sort_temp_bytes(uint64_t C) {
  size_t t = 0;
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, t, (const uint16_t*)nullptr, (uint16_t*)nullptr,
                                           (const uint32_t*)nullptr, (uint32_t*)nullptr, (int)C, 0, 16);
  return t;
}

int launch_dec_sort(hipStream_t s, void* temp, size_t temp_bytes, const uint16_t* qkey, uint16_t* skey,
                    uint32_t* iota, uint32_t* perm, uint64_t C) {
  hipLaunchKernelGGL(k_iota, dim3(grid_of(C, 256, 4096)), dim3(256), 0, s, iota, C);
  return (int)hipcub::DeviceRadixSort::SortPairs(temp, temp_bytes, qkey, skey, (const uint32_t*)iota, perm, (int)C, 0,
                                                 16, s);
}

void launch_dec_key_off(hipStream_t s, const uint16_t* skey, uint64_t C, uint32_t* key_off) {
  hipLaunchKernelGGL(k_dec_key_off, dim3(257), dim3(256), 0, s, skey, C, key_off);
}

void launch_dec_sizes(hipStream_t s, const DecCtr* q, const uint32_t* perm, uint64_t C, uint64_t* size,
                      unsigned long long* totals, bool packed) {
  if (!C) return;
  hipLaunchKernelGGL(k_dec_sizes, dim3(grid_of(C, 256, 1024)), dim3(256), 0, s, q, perm, C, size, totals,
                     packed ? 1 : 0);
}

void launch_dec_fill(hipStream_t s, const uint8_t* raw, const DecCtr* q, const uint16_t* qkey, const uint32_t* perm,
                     const uint64_t* slot, uint64_t C, CDesc* desc, uint16_t* keys, uint32_t* bm, uint8_t* payload,
                     uint64_t* bm_card, bool packed) {
  if (!C) return;
  hipLaunchKernelGGL(k_dec_fill, dim3(grid_of(C, 4, 8192)), dim3(256), 0, s, raw, q, qkey, perm, slot, C, desc, keys,
                     bm, payload, bm_card, packed ? 1 : 0);
}

}  // namespace rbg
