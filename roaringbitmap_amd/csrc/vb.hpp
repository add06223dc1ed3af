// A container of one key held across a 256-thread workgroup (4 words per thread, the
// owned-word layout of device.hpp), with the reference's pairwise result-type rule:
// the BSI circuit (bsi.hip), the buffer package's pairwise ops and orNot (ornot.hip).
#pragma once
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

// z = x OP y with the reference's result-type rule; x / y may alias z.  BUF: the buffer
// package's ImmutableRoaringBitmap.and / andNot (RB/buffer/ImmutableRoaringBitmap.java:299-325,
// 441-471), whose run AND / ANDNOT run keep the merged run container, no toEfficientContainer
// (RB/buffer/MappeableRunContainer.java:474-536, 600-663); every other pair types like the heap's.
template <int OP, bool BUF = false>
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
  const bool raw_run = BUF && (OP == OPR_AND || OP == OPR_ANDNOT) && x.kind == DK_R && y.kind == DK_R;
  const bool use_eff = !raw_run && pairwise_needs_runs(OP, x.kind, x.card, y.kind, y.card);
  const int kind = raw_run ? DK_R : use_eff ? eff(c, count_runs(r, lds, sh)) : pairwise_kind(OP, x.kind, y.kind, c);
#pragma unroll
  for (int i = 0; i < 4; i++) z.r[i] = r[i];
  z.present = 1;
  z.kind = kind;
  z.card = c;
  z.src = -1;
}

// an operand container of a pairwise task (absent: kind kAbsent)
__device__ __forceinline__ void pb_load(uint64_t slot, uint32_t card, uint16_t key, uint8_t kind, int src,
                                        const uint8_t* payload, uint32_t* tmp, int* q, VB& z) {
  if (kind == kAbsent) {
    vb_absent(z);
    return;
  }
  materialize(CDesc{slot, card, key, kind, 0}, payload, tmp, q, z.r);
  z.present = 1;
  z.kind = kind;
  z.card = (int)card;
  z.src = src;
}

}  // namespace rbg
