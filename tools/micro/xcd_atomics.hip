// Cost of accumulating the W&D gradient with integer atomics in each XCD's L2 instead of writing a per-workgroup slab
// (same launch shape as the chained kernel: 256 workgroups x 512 threads, 140 KB dynamic LDS = one per CU).
// Each scenario is a kernel sequence launched back to back `iters` times; printed: us per sequence.
//   E    empty launch
//   S    every workgroup writes its own 82 KB fp32 slab row (21 MB), plain stores (today's fused-kernel output)
//   W64  every workgroup atomically adds its 20608 values as int64 into acc[xcc][20608] (its XCD's accumulator),
//        workgroup-scope atomics (no sc bits: executed in the XCD's L2)
//   A64  the same with agent-scope atomics
//   W32  int32 atomics, workgroup scope
//   W64+O  W64, then a 93 x 256 reader that sums acc[0..15][col] in int64 and zeroes them (the optimizer's read)
// Correctness (printed): after the W64 runs the 16 accumulators must hold exactly iters * sum_b (b + 1) per column.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/micro/xcd_atomics tools/micro/xcd_atomics.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

constexpr int G = 256, NT = 512, LDSB = 140 * 1024, SLAB = 20608, XM = 16;

__device__ __forceinline__ int xcc() {
  int v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
  return v & 15;
}

__global__ __launch_bounds__(NT, 1) void k_empty(float* p) {
  extern __shared__ float lds[];
  if (threadIdx.x == 9999) p[0] = lds[0];
}
__global__ __launch_bounds__(NT, 1) void k_slab(float* slab) {
  extern __shared__ float lds[];
  float* row = slab + (size_t)blockIdx.x * SLAB;
  for (int i = threadIdx.x; i < SLAB; i += NT) row[i] = (float)(i + blockIdx.x);
  if (threadIdx.x == 9999) row[0] = lds[0];
}
template <int SCOPE, bool W64>
__global__ __launch_bounds__(NT, 1) void k_atom(void* acc) {
  extern __shared__ float lds[];
  const int x = xcc();
  const unsigned long long v = blockIdx.x + 1;
  for (int i = threadIdx.x; i < SLAB; i += NT) {
    if (W64) __hip_atomic_fetch_add((unsigned long long*)acc + (size_t)x * SLAB + i, v, __ATOMIC_RELAXED, SCOPE);
    else __hip_atomic_fetch_add((unsigned int*)acc + (size_t)x * SLAB + i, (unsigned int)v, __ATOMIC_RELAXED, SCOPE);
  }
  if (threadIdx.x == 9999) ((float*)acc)[0] = lds[0];
}
__global__ __launch_bounds__(256) void k_read(unsigned long long* acc, unsigned long long* out) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= SLAB) return;
  unsigned long long v[XM];
#pragma unroll
  for (int x = 0; x < XM; ++x) v[x] = acc[(size_t)x * SLAB + c];
  unsigned long long s = 0;
#pragma unroll
  for (int x = 0; x < XM; ++x) {
    s += v[x];
    acc[(size_t)x * SLAB + c] = 0;
  }
  out[c] += s;
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 200;
  float* slab;
  unsigned long long *acc, *out;
  CK(hipMalloc(&slab, (size_t)G * SLAB * 4));
  CK(hipMalloc(&acc, (size_t)XM * SLAB * 8));
  CK(hipMalloc(&out, (size_t)SLAB * 8));
  CK(hipMemset(acc, 0, (size_t)XM * SLAB * 8));
  CK(hipMemset(out, 0, (size_t)SLAB * 8));
  for (auto f : {(const void*)k_empty, (const void*)k_slab, (const void*)k_atom<__HIP_MEMORY_SCOPE_WORKGROUP, true>,
                 (const void*)k_atom<__HIP_MEMORY_SCOPE_AGENT, true>, (const void*)k_atom<__HIP_MEMORY_SCOPE_WORKGROUP, false>})
    CK(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, LDSB));
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto run = [&](const char* name, auto&& seq) -> int {
    for (int i = 0; i < 5; ++i) seq();
    CK(hipDeviceSynchronize());
    CK(hipEventRecord(e0));
    for (int i = 0; i < iters; ++i) seq();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    printf("{\"sequence\": \"%s\", \"us\": %.2f}\n", name, 1e3 * ms / iters);
    return 0;
  };
  run("E", [&] { hipLaunchKernelGGL(k_empty, dim3(G), dim3(NT), LDSB, 0, slab); });
  run("S", [&] { hipLaunchKernelGGL(k_slab, dim3(G), dim3(NT), LDSB, 0, slab); });
  run("W32", [&] { hipLaunchKernelGGL((k_atom<__HIP_MEMORY_SCOPE_WORKGROUP, false>), dim3(G), dim3(NT), LDSB, 0, (void*)acc); });
  run("A64", [&] { hipLaunchKernelGGL((k_atom<__HIP_MEMORY_SCOPE_AGENT, true>), dim3(G), dim3(NT), LDSB, 0, (void*)acc); });
  CK(hipMemset(acc, 0, (size_t)XM * SLAB * 8));
  CK(hipDeviceSynchronize());
  run("W64", [&] { hipLaunchKernelGGL((k_atom<__HIP_MEMORY_SCOPE_WORKGROUP, true>), dim3(G), dim3(NT), LDSB, 0, (void*)acc); });
  // correctness: (5 + iters) launches of W64 since the memset
  {
    static unsigned long long h[XM * SLAB];
    CK(hipMemcpy(h, acc, sizeof(h), hipMemcpyDeviceToHost));
    const unsigned long long want = (unsigned long long)(5 + iters) * (G * (G + 1) / 2);
    int bad = 0, used = 0;
    for (int x = 0; x < XM; ++x) used += h[(size_t)x * SLAB] != 0;
    for (int c = 0; c < SLAB; ++c) {
      unsigned long long s = 0;
      for (int x = 0; x < XM; ++x) s += h[(size_t)x * SLAB + c];
      bad += s != want;
    }
    printf("{\"check\": \"W64 exact sums\", \"bad_columns\": %d, \"xcds_used\": %d}\n", bad, used);
  }
  CK(hipMemset(acc, 0, (size_t)XM * SLAB * 8));
  CK(hipMemset(out, 0, (size_t)SLAB * 8));
  run("W64+O", [&] {
    hipLaunchKernelGGL((k_atom<__HIP_MEMORY_SCOPE_WORKGROUP, true>), dim3(G), dim3(NT), LDSB, 0, (void*)acc);
    hipLaunchKernelGGL(k_read, dim3((SLAB + 255) / 256), dim3(256), 0, 0, acc, out);
  });
  {
    static unsigned long long h[SLAB];
    CK(hipMemcpy(h, out, sizeof(h), hipMemcpyDeviceToHost));
    const unsigned long long want = (unsigned long long)(5 + iters) * (G * (G + 1) / 2);
    int bad = 0;
    for (int c = 0; c < SLAB; ++c) bad += h[c] != want;
    printf("{\"check\": \"W64+O exact sums across kernel boundaries (zeroed by the reader)\", \"bad_columns\": %d}\n", bad);
  }
  run("O", [&] { hipLaunchKernelGGL(k_read, dim3((SLAB + 255) / 256), dim3(256), 0, 0, acc, out); });
  run("S+O", [&] {
    hipLaunchKernelGGL(k_slab, dim3(G), dim3(NT), LDSB, 0, slab);
    hipLaunchKernelGGL(k_read, dim3((SLAB + 255) / 256), dim3(256), 0, 0, acc, out);
  });
  return 0;
}
