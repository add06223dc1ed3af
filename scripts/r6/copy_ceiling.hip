// Copy-shape ceilings on one MI355X (round 6): a 1:1 copy of 0.27 GB (the size of the C2 AND result) in the
// forms a serializer could take, to find which shape reaches the guide's ~6.3 TB/s (MI355X_MICROARCH.md: float4
// copy) and which ones stop near 5 TB/s (scripts/r6/bb_ceiling.hip's grid-stride copy).  TB/s of read + write bytes.
// Standalone: hipcc -O3 --offload-arch=gfx950 copy_ceiling.hip -o copy_ceiling
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

// one float4 per thread, grid = n / 256 workgroups
__global__ __launch_bounds__(256) void k_flat(const v4u* __restrict__ a, v4u* __restrict__ c, size_t n) {
  const size_t i = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i < n) c[i] = a[i];
}
// U float4 per thread in flight, grid-stride over a resident grid
template <int U, bool NTL, bool NTS>
__global__ __launch_bounds__(256) void k_unroll(const v4u* __restrict__ a, v4u* __restrict__ c, size_t n) {
  const size_t stride = (size_t)gridDim.x * 256 * U;
  for (size_t i0 = (size_t)blockIdx.x * 256 * U + threadIdx.x; i0 < n; i0 += stride) {
    v4u v[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const size_t i = i0 + (size_t)u * 256;
      v[u] = i < n ? (NTL ? __builtin_nontemporal_load(a + i) : a[i]) : v4u{0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      const size_t i = i0 + (size_t)u * 256;
      if (i < n) {
        if (NTS) __builtin_nontemporal_store(v[u], c + i);
        else c[i] = v[u];
      }
    }
  }
}
// one wave per 8 KiB record (the serializer's shape): 8 float4 per lane in flight; records in order
template <bool NTS>
__global__ __launch_bounds__(256) void k_rec(const v4u* __restrict__ a, v4u* __restrict__ c, size_t nrec) {
  const size_t nw = (size_t)gridDim.x * 4;
  for (size_t r = (size_t)blockIdx.x * 4 + (threadIdx.x >> 6); r < nrec; r += nw) {
    const v4u* s = a + r * 512 + (threadIdx.x & 63);
    v4u* d = c + r * 512 + (threadIdx.x & 63);
    v4u v[8];
#pragma unroll
    for (int u = 0; u < 8; u++) v[u] = __builtin_nontemporal_load(s + 64 * u);
#pragma unroll
    for (int u = 0; u < 8; u++) {
      if (NTS) __builtin_nontemporal_store(v[u], d + 64 * u);
      else d[64 * u] = v[u];
    }
  }
}

// the fused serializer's shape: one workgroup of W waves per chunk of R consecutive 8 KiB records, every chunk's
// workgroup resident at once (the whole range in flight), wave w copying records w, w + W, ... of its chunk
template <int W, bool NTS>
__global__ __launch_bounds__(64 * W) void k_chunk(const v4u* __restrict__ a, v4u* __restrict__ c, size_t nrec, int R) {
  const int w = threadIdx.x >> 6, l = threadIdx.x & 63;
  for (size_t r = (size_t)blockIdx.x * R + w; r < (size_t)(blockIdx.x + 1) * R && r < nrec; r += W) {
    const v4u* s = a + r * 512 + l;
    v4u* d = c + r * 512 + l;
    v4u v[8];
#pragma unroll
    for (int u = 0; u < 8; u++) v[u] = __builtin_nontemporal_load(s + 64 * u);
#pragma unroll
    for (int u = 0; u < 8; u++) {
      if (NTS) __builtin_nontemporal_store(v[u], d + 64 * u);
      else d[64 * u] = v[u];
    }
  }
}

template <class F>
static float timeit(F f, int reps) {
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  f();
  hipDeviceSynchronize();
  hipEventRecord(e0);
  for (int i = 0; i < reps; i++) f();
  hipEventRecord(e1);
  hipEventSynchronize(e1);
  float ms = 0;
  hipEventElapsedTime(&ms, e0, e1);
  return ms / reps;
}

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  const size_t nrec = 32768;  // 0.27 GB = 32,768 x 8 KiB
  const size_t n = nrec * 512;  // float4s
  v4u *a, *c;
  if (hipMalloc(&a, n * 16) != hipSuccess || hipMalloc(&c, n * 16) != hipSuccess) return 1;
  hipMemset(a, 1, n * 16);
  hipMemset(c, 0, n * 16);
  // a 2 GB stream between repetitions would evict the Infinity Cache; these numbers are warm-cache-free only
  // because 2 x 0.27 GB exceeds its 256 MiB
  auto line = [&](const char* what, float ms) { printf("%-52s %8.4f ms  %6.3f TB/s\n", what, ms, 2.0 * n * 16 / (ms * 1e-3) / 1e12); };
  line("flat: one float4 per thread, n/256 WGs",
       timeit([&] { hipLaunchKernelGGL(k_flat, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, a, c, n); }, 20));
  for (int wpc : {8, 16, 32}) {
    char b[96];
    snprintf(b, sizeof b, "unroll 4, plain, %d WGs/CU", wpc);
    line(b, timeit([&] { hipLaunchKernelGGL((k_unroll<4, false, false>), dim3(cus * wpc), dim3(256), 0, 0, a, c, n); }, 20));
    snprintf(b, sizeof b, "unroll 4, nt load, %d WGs/CU", wpc);
    line(b, timeit([&] { hipLaunchKernelGGL((k_unroll<4, true, false>), dim3(cus * wpc), dim3(256), 0, 0, a, c, n); }, 20));
    snprintf(b, sizeof b, "unroll 4, nt load + nt store, %d WGs/CU", wpc);
    line(b, timeit([&] { hipLaunchKernelGGL((k_unroll<4, true, true>), dim3(cus * wpc), dim3(256), 0, 0, a, c, n); }, 20));
    snprintf(b, sizeof b, "unroll 8, nt load, %d WGs/CU", wpc);
    line(b, timeit([&] { hipLaunchKernelGGL((k_unroll<8, true, false>), dim3(cus * wpc), dim3(256), 0, 0, a, c, n); }, 20));
  }
  for (int wpc : {4, 8}) {
    char b[96];
    snprintf(b, sizeof b, "record per wave (8 KiB), plain store, %d WGs/CU", wpc);
    line(b, timeit([&] { hipLaunchKernelGGL(k_rec<false>, dim3(cus * wpc), dim3(256), 0, 0, a, c, nrec); }, 20));
    snprintf(b, sizeof b, "record per wave (8 KiB), nt store, %d WGs/CU", wpc);
    line(b, timeit([&] { hipLaunchKernelGGL(k_rec<true>, dim3(cus * wpc), dim3(256), 0, 0, a, c, nrec); }, 20));
  }
  {
    // 32,768 records in 1,024 chunks of 32 (the fused serializer: 1,024 tiles of ~32 KiB... here 256 KiB each)
    line("chunk per WG (8 waves, 1024 x 32 records), nt store",
         timeit([&] { hipLaunchKernelGGL((k_chunk<8, true>), dim3(1024), dim3(512), 0, 0, a, c, nrec, 32); }, 20));
    line("chunk per WG (8 waves, 1024 x 32 records), plain store",
         timeit([&] { hipLaunchKernelGGL((k_chunk<8, false>), dim3(1024), dim3(512), 0, 0, a, c, nrec, 32); }, 20));
    line("chunk per WG (8 waves, 4096 x 8 records), nt store",
         timeit([&] { hipLaunchKernelGGL((k_chunk<8, true>), dim3(4096), dim3(512), 0, 0, a, c, nrec, 8); }, 20));
    line("chunk per WG (4 waves, 2048 x 16 records), nt store",
         timeit([&] { hipLaunchKernelGGL((k_chunk<4, true>), dim3(2048), dim3(256), 0, 0, a, c, nrec, 16); }, 20));
  }
  return 0;
}
