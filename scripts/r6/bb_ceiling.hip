// Ceiling of the B AND B access pattern on this box (round 6): per task, two 8 KiB operands read and one
// 8 KiB result written (C2's B∧B family: 65,536 tasks, 1.61 GB), by one wave per task over a resident grid,
// against a plain 1:1 copy and a read-only stream of the same bytes.  Standalone (hipcc), prints one line
// per variant: ms and TB/s of (read + write) bytes.  Not product code.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("hip error %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)

typedef unsigned int v4u __attribute__((ext_vector_type(4)));

template <int NT_LOAD, int NT_STORE, int WAVES_PER_WG, int STRIDE = 520>
__global__ __launch_bounds__(64 * WAVES_PER_WG) void k_bb(const v4u* __restrict__ a, const v4u* __restrict__ b,
                                                          v4u* __restrict__ c, uint32_t ntask, uint32_t* __restrict__ cards) {
  const uint32_t w = threadIdx.x >> 6, l = threadIdx.x & 63;
  const uint32_t nw = gridDim.x * WAVES_PER_WG;
  for (uint32_t t = blockIdx.x * WAVES_PER_WG + w; t < ntask; t += nw) {
    const v4u* pa = a + (size_t)t * 512 + l;
    const v4u* pb = b + (size_t)t * 512 + l;
    v4u x[8], y[8];
#pragma unroll
    for (int i = 0; i < 8; i++) {
      x[i] = NT_LOAD ? __builtin_nontemporal_load(pa + 64 * i) : pa[64 * i];
      y[i] = NT_LOAD ? __builtin_nontemporal_load(pb + 64 * i) : pb[64 * i];
    }
    uint32_t cnt = 0;
#pragma unroll
    for (int i = 0; i < 8; i++) {
      x[i] &= y[i];
      cnt += __popc(x[i].x) + __popc(x[i].y) + __popc(x[i].z) + __popc(x[i].w);
    }
    for (int o = 32; o > 0; o >>= 1) cnt += __shfl_xor(cnt, o, 64);
    v4u* pc = c + (size_t)t * STRIDE + l;  // slot stride 8320 B (520 vectors) as the engine's scratch slots, or 8192
#pragma unroll
    for (int i = 0; i < 8; i++) {
      if (NT_STORE) __builtin_nontemporal_store(x[i], pc + 64 * i);
      else pc[64 * i] = x[i];
    }
    if (l == 0) cards[t] = cnt;
  }
}

// the same bytes as a flat stream: c[i] = a[i] & b[i], U float4 per thread in flight, grid-stride (no task structure)
template <int U, int NTS>
__global__ __launch_bounds__(256) void k_and_flat(const v4u* __restrict__ a, const v4u* __restrict__ b, v4u* __restrict__ c,
                                                  size_t n) {
  const size_t stride = (size_t)gridDim.x * 256 * U;
  for (size_t i0 = (size_t)blockIdx.x * 256 * U + threadIdx.x; i0 < n; i0 += stride) {
    v4u x[U], y[U];
#pragma unroll
    for (int u = 0; u < U; u++) {
      const size_t i = i0 + (size_t)u * 256;
      x[u] = i < n ? __builtin_nontemporal_load(a + i) : v4u{0, 0, 0, 0};
      y[u] = i < n ? __builtin_nontemporal_load(b + i) : v4u{0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < U; u++) {
      const size_t i = i0 + (size_t)u * 256;
      if (i < n) {
        if (NTS) __builtin_nontemporal_store(x[u] & y[u], c + i);
        else c[i] = x[u] & y[u];
      }
    }
  }
}

__global__ __launch_bounds__(256) void k_copy(const v4u* __restrict__ a, v4u* __restrict__ c, size_t n) {
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) c[i] = a[i];
}
__global__ __launch_bounds__(256) void k_read(const v4u* __restrict__ a, size_t n, uint32_t* out) {
  uint32_t s = 0;
  for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    const v4u v = __builtin_nontemporal_load(a + i);
    s ^= v.x ^ v.y ^ v.z ^ v.w;
  }
  if (s == 0x12345678u) out[0] = s;
}

template <class F>
static float timeit(F f, int reps) {
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  f();
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(e0, 0);
  for (int r = 0; r < reps; r++) f();
  (void)hipEventRecord(e1, 0);
  (void)hipEventSynchronize(e1);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, e0, e1);
  return ms / reps;
}

int main() {
  const uint32_t nt = 65536;
  const size_t bytes = (size_t)nt * 8192;
  v4u *a, *b, *c;
  uint32_t* cards;
  CK(hipMalloc(&a, bytes));
  CK(hipMalloc(&b, bytes));
  CK(hipMalloc(&c, (size_t)nt * 16384));
  CK(hipMalloc(&cards, 4 * nt));
  CK(hipMemset(a, 0x5A, bytes));
  CK(hipMemset(b, 0x3C, bytes));
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const double rw = 3.0 * bytes;  // two operands read, one result written
  auto bb = [&](auto kern, int wpg, int wgs_per_cu, const char* name) {
    const int grid = cus * wgs_per_cu;
    const float ms = timeit([&] { hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * wpg), 0, 0, a, b, c, nt, cards); }, 20);
    printf("%-44s %8.4f ms  %6.3f TB/s\n", name, ms, rw / (ms * 1e-3) / 1e12);
  };
  bb(k_bb<1, 0, 16>, 16, 1, "bb nt-load plain-store 16 waves/CU (1 WG)");
  bb(k_bb<1, 0, 4>, 4, 4, "bb nt-load plain-store 4 WG x 4 waves");
  bb(k_bb<1, 0, 4>, 4, 8, "bb nt-load plain-store 8 WG x 4 waves");
  bb(k_bb<0, 0, 4>, 4, 4, "bb plain-load plain-store 4x4");
  bb(k_bb<1, 1, 4>, 4, 4, "bb nt-load nt-store 4x4");
  bb(k_bb<1, 1, 4>, 4, 8, "bb nt-load nt-store 8x4");
  bb(k_bb<1, 0, 16, 512>, 16, 1, "bb nt-load plain-store 16x1, stride 8192");
  bb(k_bb<1, 0, 4, 512>, 4, 4, "bb nt-load plain-store 4x4, stride 8192");
  bb(k_bb<1, 1, 4, 512>, 4, 4, "bb nt-load nt-store 4x4, stride 8192");
  bb(k_bb<1, 0, 4, 1024>, 4, 4, "bb nt-load plain-store 4x4, stride 16384");
  for (int wpc : {8, 16}) {
    const size_t n = bytes / 16;
    char nm[64];
    snprintf(nm, sizeof nm, "flat a&b, unroll 4, plain store, %d WG/CU", wpc);
    float ms = timeit([&] { hipLaunchKernelGGL((k_and_flat<4, 0>), dim3(cus * wpc), dim3(256), 0, 0, a, b, c, n); }, 20);
    printf("%-44s %8.4f ms  %6.3f TB/s\n", nm, ms, rw / (ms * 1e-3) / 1e12);
    snprintf(nm, sizeof nm, "flat a&b, unroll 4, nt store, %d WG/CU", wpc);
    ms = timeit([&] { hipLaunchKernelGGL((k_and_flat<4, 1>), dim3(cus * wpc), dim3(256), 0, 0, a, b, c, n); }, 20);
    printf("%-44s %8.4f ms  %6.3f TB/s\n", nm, ms, rw / (ms * 1e-3) / 1e12);
  }
  {
    const size_t n = 2 * bytes / 16 / 2;  // 1.07 GB copied: read + write = the bb bytes x 4/3
    const float ms = timeit([&] { hipLaunchKernelGGL(k_copy, dim3(cus * 8), dim3(256), 0, 0, a, c, n); }, 20);
    printf("%-44s %8.4f ms  %6.3f TB/s\n", "copy 0.54 GB (read + write)", ms, 2.0 * n * 16 / (ms * 1e-3) / 1e12);
  }
  {
    const size_t n = 2 * bytes / 16;
    const float ms = timeit([&] { hipLaunchKernelGGL(k_read, dim3(cus * 8), dim3(256), 0, 0, a, n / 2, cards); }, 20);
    printf("%-44s %8.4f ms  %6.3f TB/s\n", "read-only 0.54 GB", ms, (double)n / 2 * 16 / (ms * 1e-3) / 1e12);
  }
  return 0;
}
