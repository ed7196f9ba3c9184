// Fixed-cost floor of the W&D step on MI355X, same launch shape as the chained kernel (256 workgroups x 512
// threads, 140 KB dynamic LDS). Each scenario is a sequence of kernels launched back to back `iters` times;
// printed: us per sequence.
//   E  empty launch            P  every workgroup copies the same 67 KB weight image into LDS
//   S  every workgroup writes its own 82 KB fp32 slab row (21 MB total), plain stores
//   N  same with nontemporal stores        Y  same with system-scope (write-through) stores
//   R  322 workgroups sum the slab column-wise (the reduce), plain loads
//   Q  same with nontemporal loads          Z  same with system-scope loads
//   X  XCD-local two-level reduce: 8 x 322 workgroups; each sums, for its column chunk, only the slab rows written
//      by workgroups that ran on its own XCD (HW_REG_XCC_ID recorded by S), into per-XCD partials [8][SLAB]
//      (assumes round-robin placement blockIdx % 8 == XCD for the output slot: timing only, not a correct sum
//      when the assumption fails); then 8 -> 1 by a 322-workgroup pass
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/micro/launch_floor tools/micro/launch_floor.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <string.h>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

constexpr int G = 256, NT = 512, LDSB = 140 * 1024, IMG = 33536 * 2, SLAB = 20608;

template <int ST>
__device__ __forceinline__ void store(float* p, float v) {
  if (ST == 0) *p = v;
  else if (ST == 1) __builtin_nontemporal_store(v, p);
  else __hip_atomic_store((unsigned int*)p, __float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
template <int LD>
__device__ __forceinline__ float4 load4(const float4* p) {
  if (LD == 0) return *p;
  if (LD == 1) {
    const float* f = (const float*)p;
    return make_float4(__builtin_nontemporal_load(f), __builtin_nontemporal_load(f + 1),
                       __builtin_nontemporal_load(f + 2), __builtin_nontemporal_load(f + 3));
  }
  const unsigned int* u = (const unsigned int*)p;
  float4 r;
  r.x = __uint_as_float(__hip_atomic_load(u + 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
  r.y = __uint_as_float(__hip_atomic_load(u + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
  r.z = __uint_as_float(__hip_atomic_load(u + 2, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
  r.w = __uint_as_float(__hip_atomic_load(u + 3, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
  return r;
}

__device__ __forceinline__ int xcc_id() {
  int v;
  asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(v));
  return v & 15;
}

__device__ int g_xcd_of[G];

template <int ST>
__global__ __launch_bounds__(512, 1) void k_main(const uint4* img, float* slab, int mode) {
  extern __shared__ __attribute__((aligned(16))) uint4 lds[];
  if (threadIdx.x == 0) g_xcd_of[blockIdx.x] = xcc_id();
  if (mode & 1) {
    constexpr int N = IMG / 16, PER = (N + NT - 1) / NT;
    uint4 v[PER];
#pragma unroll
    for (int i = 0; i < PER; ++i) v[i] = img[min((int)threadIdx.x + i * NT, N - 1)];
#pragma unroll
    for (int i = 0; i < PER; ++i)
      if (threadIdx.x + i * NT < N) lds[threadIdx.x + i * NT] = v[i];
    __syncthreads();
  }
  if (mode & 2) {
    float* my = slab + (size_t)blockIdx.x * SLAB;
    const float x = (float)(threadIdx.x + blockIdx.x) + (mode & 1 ? __uint_as_float(lds[threadIdx.x].x) : 0.f);
    for (int c = threadIdx.x; c < SLAB; c += NT) store<ST>(my + c, x + c);
  }
}

template <int LD>
__global__ __launch_bounds__(256) void k_reduce(const float4* slab, float4* out) {
  __shared__ float4 part[16][16];
  const int lq = threadIdx.x % 16, r = threadIdx.x / 16, S4 = SLAB / 4, q = blockIdx.x * 16 + lq;
  float4 a = make_float4(0, 0, 0, 0);
  if (q < S4)
    for (int g = r; g < G; g += 16) {
      const float4 v = load4<LD>(slab + (size_t)g * S4 + q);
      a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
    }
  part[r][lq] = a;
  __syncthreads();
  if (threadIdx.x < 16 && q < S4) {
    float4 s = part[0][lq];
    for (int k = 1; k < 16; ++k) { s.x += part[k][lq].x; s.y += part[k][lq].y; s.z += part[k][lq].z; s.w += part[k][lq].w; }
    out[q] = s;
  }
}

// level 1: workgroup (chunk c = blockIdx.x / 8) sums the rows written on its own XCD
__global__ __launch_bounds__(256) void k_rx1(const float4* slab, float4* part8, int* placed) {
  __shared__ float4 part[16][16];
  __shared__ int rows[G];
  __shared__ int nrows;
  const int x = xcc_id();
  if (threadIdx.x == 0) {
    nrows = 0;
    placed[blockIdx.x] = x;
  }
  __syncthreads();
  for (int g = threadIdx.x; g < G; g += 256)
    if (g_xcd_of[g] == x) rows[atomicAdd(&nrows, 1)] = g;
  __syncthreads();
  const int c = blockIdx.x / 8;
  const int lq = threadIdx.x % 16, r = threadIdx.x / 16, S4 = SLAB / 4, q = c * 16 + lq;
  float4 a = make_float4(0, 0, 0, 0);
  if (q < S4)
    for (int i = r; i < nrows; i += 16) {
      const float4 v = slab[(size_t)rows[i] * S4 + q];
      a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
    }
  part[r][lq] = a;
  __syncthreads();
  if (threadIdx.x < 16 && q < S4) {
    float4 s = part[0][lq];
    for (int k = 1; k < 16; ++k) { s.x += part[k][lq].x; s.y += part[k][lq].y; s.z += part[k][lq].z; s.w += part[k][lq].w; }
    part8[(size_t)x * S4 + q] = s;
  }
}

__global__ __launch_bounds__(64) void k_rx2(const float4* part8, float4* out) {
  const int S4 = SLAB / 4, q = blockIdx.x * 64 + threadIdx.x;
  if (q >= S4) return;
  float4 s = part8[q];
  for (int x = 1; x < 8; ++x) { const float4 v = part8[(size_t)x * S4 + q]; s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w; }
  out[q] = s;
}

int main(int argc, char** argv) {
  uint4* img; float* slab; float4* out; float4* part8; int* placed;
  CK(hipMalloc(&img, IMG)); CK(hipMalloc(&slab, (size_t)G * SLAB * 4)); CK(hipMalloc(&out, SLAB * 4));
  CK(hipMalloc(&part8, 8 * SLAB * 4)); CK(hipMalloc(&placed, 8 * (SLAB / 64) * 4));
  CK(hipMemset(img, 0, IMG)); CK(hipMemset(slab, 0, (size_t)G * SLAB * 4));
  CK(hipFuncSetAttribute((const void*)k_main<0>, hipFuncAttributeMaxDynamicSharedMemorySize, LDSB));
  CK(hipFuncSetAttribute((const void*)k_main<1>, hipFuncAttributeMaxDynamicSharedMemorySize, LDSB));
  CK(hipFuncSetAttribute((const void*)k_main<2>, hipFuncAttributeMaxDynamicSharedMemorySize, LDSB));
  hipStream_t s; CK(hipStreamCreate(&s));
  hipEvent_t a, b; CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  const char* dflt[] = {"E", "S", "R", "SR", "X", "SX", "SR", "SX"};
  const int nsc = argc > 1 ? argc - 1 : (int)(sizeof(dflt) / sizeof(dflt[0]));
  const int iters = 300;
  for (int i = 0; i < nsc; ++i) {
    const char* sc = argc > 1 ? argv[i + 1] : dflt[i];
    auto seq = [&]() {
      for (const char* c = sc; *c; ++c) {
        switch (*c) {
          case 'E': hipLaunchKernelGGL(k_main<0>, dim3(G), dim3(NT), LDSB, s, img, slab, 0); break;
          case 'P': hipLaunchKernelGGL(k_main<0>, dim3(G), dim3(NT), LDSB, s, img, slab, 1); break;
          case 'S': hipLaunchKernelGGL(k_main<0>, dim3(G), dim3(NT), LDSB, s, img, slab, (c > sc && c[-1] == 'P') ? 3 : 2); break;
          case 'N': hipLaunchKernelGGL(k_main<1>, dim3(G), dim3(NT), LDSB, s, img, slab, 2); break;
          case 'Y': hipLaunchKernelGGL(k_main<2>, dim3(G), dim3(NT), LDSB, s, img, slab, 2); break;
          case 'R': hipLaunchKernelGGL(k_reduce<0>, dim3(SLAB / 64), dim3(256), 0, s, (const float4*)slab, out); break;
          case 'Q': hipLaunchKernelGGL(k_reduce<1>, dim3(SLAB / 64), dim3(256), 0, s, (const float4*)slab, out); break;
          case 'Z': hipLaunchKernelGGL(k_reduce<2>, dim3(SLAB / 64), dim3(256), 0, s, (const float4*)slab, out); break;
          case 'X':
            hipLaunchKernelGGL(k_rx1, dim3(8 * (SLAB / 64)), dim3(256), 0, s, (const float4*)slab, part8, placed);
            hipLaunchKernelGGL(k_rx2, dim3((SLAB / 4 + 63) / 64), dim3(64), 0, s, (const float4*)part8, out);
            break;
        }
      }
    };
    for (int w = 0; w < 20; ++w) seq();
    CK(hipEventRecord(a, s));
    for (int it = 0; it < iters; ++it) seq();
    CK(hipEventRecord(b, s));
    CK(hipEventSynchronize(b));
    float ms;
    CK(hipEventElapsedTime(&ms, a, b));
    printf("{\"sequence\": \"%s\", \"us\": %.2f}\n", sc, 1e3 * ms / iters);
    fflush(stdout);
  }
  // placement check: how often did workgroup b of the level-1 kernel run on XCD b % 8
  int hp[8 * (SLAB / 64)], xo[G];
  CK(hipMemcpy(hp, placed, sizeof(hp), hipMemcpyDeviceToHost));
  CK(hipMemcpyFromSymbol(xo, HIP_SYMBOL(g_xcd_of), sizeof(xo), 0, hipMemcpyDeviceToHost));
  int rr = 0, rr2 = 0, cnt[16] = {0};
  for (int b = 0; b < 8 * (SLAB / 64); ++b) rr += hp[b] == b % 8;
  for (int b = 0; b < G; ++b) { rr2 += xo[b] == b % 8; cnt[xo[b] & 15]++; }
  printf("{\"rx1_round_robin\": %d, \"of\": %d, \"main_round_robin\": %d, \"of_main\": %d, \"main_per_xcd\": [%d,%d,%d,%d,%d,%d,%d,%d]}\n",
         rr, 8 * (SLAB / 64), rr2, G, cnt[0], cnt[1], cnt[2], cnt[3], cnt[4], cnt[5], cnt[6], cnt[7]);
  CK(hipGetLastError());
  return 0;
}
