// Fused transformer epilogues for gfx950: residual-add + LayerNorm and bias + GELU(erf), fwd + bwd.
//
// BASELINE config 4 (BERT-base TP=8). Between the hipBLASLt GEMMs of a BERT layer the remaining
// work is memory-bound elementwise / row-reduction: unfused, `x + attn_out` -> LayerNorm reads and
// writes the [tokens, 768] activation 3x, and `bias + gelu` 2x. Here each is one pass.
//
//  * add_ln_fwd: one wave64 per row (H <= 64*kMaxPer), lane owns H/64 contiguous-strided elements in
//    registers; mean and variance by shuffle reductions (two-pass in registers, fp32); writes y and
//    per-row (mean, rstd). 4 rows per 256-thread workgroup, grid-stride over rows.
//  * add_ln_bwd: recomputes x_hat from (a + r); dx = rstd (g - mean(g) - x_hat mean(g x_hat)), g = dy w;
//    dw / db accumulated per lane across the workgroup's rows, written as per-block partials
//    [nblocks, H] (deterministic; summed by the caller).
//  * bias_gelu_fwd / bwd: column-per-thread over row chunks (no per-element index math); the
//    backward also produces the bias-gradient column partials, reduced by col_reduce2.
// Activations are bf16 or fp32 (template T); LayerNorm gamma/beta, the GELU bias and the parameter
// gradients dw/db are bf16 or fp32 (template P: a bf16 model's parameters are read and their gradients
// written in bf16 directly, no cast kernels around each call); statistics and reductions are fp32.
#include <hip/hip_bf16.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

constexpr int kThreads = 256;
constexpr int kMaxPer = 64;  // H <= 4096

template <typename T>
__device__ __forceinline__ float ld(const T* p) {
  return (float)*p;
}
template <>
__device__ __forceinline__ float ld<__hip_bfloat16>(const __hip_bfloat16* p) {
  return __bfloat162float(*p);
}
template <typename T>
__device__ __forceinline__ void st(T* p, float v) {
  *p = (T)v;
}
template <>
__device__ __forceinline__ void st<__hip_bfloat16>(__hip_bfloat16* p, float v) {
  *p = __float2bfloat16(v);
}

template <typename T>
__device__ __forceinline__ float cvt_round(float v) {
  return (float)(T)v;
}
template <>
__device__ __forceinline__ float cvt_round<__hip_bfloat16>(float v) {
  return __bfloat162float(__float2bfloat16(v));
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// one global access of N contiguous elements (8 or 16 bytes) converted to / from fp32
template <typename T, int N>
struct alignas(sizeof(T) * N) Pack {
  T v[N];
};
template <typename T, int N>
__device__ __forceinline__ void ldv(const T* p, float* o) {
  const Pack<T, N> pk = *(const Pack<T, N>*)p;
#pragma unroll
  for (int i = 0; i < N; ++i) o[i] = ld(&pk.v[i]);
}
template <typename T, int N>
__device__ __forceinline__ void stv(T* p, const float* v) {
  Pack<T, N> pk;
#pragma unroll
  for (int i = 0; i < N; ++i) st(&pk.v[i], v[i]);
  *(Pack<T, N>*)p = pk;
}

// ---- vectorised LayerNorm (H % 256 == 0): lane owns NC chunks of 4 contiguous columns,
// chunk j of lane l = columns [4 (64 j + l), +4) -> every access is one 8/16-byte load per lane
template <typename T, typename P, int NC>
__global__ __launch_bounds__(kThreads) void add_ln_fwd_v(const T* __restrict__ a, const T* __restrict__ r,
                                                        const P* __restrict__ w, const P* __restrict__ b,
                                                        int R, float eps, T* __restrict__ y,
                                                        float* __restrict__ mean_out, float* __restrict__ rstd_out) {
  constexpr int H = NC * 256;
  const int lane = threadIdx.x & 63;
  const int wpb = kThreads / 64;
  for (int row = blockIdx.x * wpb + (threadIdx.x >> 6); row < R; row += gridDim.x * wpb) {
    const size_t base = (size_t)row * H;
    float v[NC][4];
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < NC; ++j) {
      const int c = 4 * (64 * j + lane);
      float t[4];
      ldv<T, 4>(a + base + c, v[j]);
      ldv<T, 4>(r + base + c, t);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[j][e] += t[e];
        s += v[j][e];
      }
    }
    const float mean = wave_sum(s) * (1.f / H);
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < NC; ++j)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float d = v[j][e] - mean;
        q += d * d;
      }
    const float rstd = rsqrtf(wave_sum(q) * (1.f / H) + eps);
#pragma unroll
    for (int j = 0; j < NC; ++j) {
      const int c = 4 * (64 * j + lane);
      float wv[4], bv[4];
      ldv<P, 4>(w + c, wv);
      ldv<P, 4>(b + c, bv);
      float o[4] = {(v[j][0] - mean) * rstd * wv[0] + bv[0], (v[j][1] - mean) * rstd * wv[1] + bv[1],
                    (v[j][2] - mean) * rstd * wv[2] + bv[2], (v[j][3] - mean) * rstd * wv[3] + bv[3]};
      stv<T, 4>(y + base + c, o);
    }
    if (lane == 0) {
      mean_out[row] = mean;
      rstd_out[row] = rstd;
    }
  }
}

template <typename T, typename P, int NC>
__global__ __launch_bounds__(kThreads) void add_ln_bwd_v(const T* __restrict__ dy, const T* __restrict__ a,
                                                        const T* __restrict__ r, const P* __restrict__ w,
                                                        const float* __restrict__ mean_in,
                                                        const float* __restrict__ rstd_in, int R,
                                                        T* __restrict__ dx, float* __restrict__ dw_part,
                                                        float* __restrict__ db_part) {
  constexpr int H = NC * 256;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int wpb = kThreads / 64;
  float dw[NC][4], db[NC][4], wreg[NC][4];
#pragma unroll
  for (int j = 0; j < NC; ++j) {
    ldv<P, 4>(w + 4 * (64 * j + lane), wreg[j]);
#pragma unroll
    for (int e = 0; e < 4; ++e) dw[j][e] = db[j][e] = 0.f;
  }
  for (int row = blockIdx.x * wpb + wv; row < R; row += gridDim.x * wpb) {
    const size_t base = (size_t)row * H;
    const float mean = mean_in[row], rstd = rstd_in[row];
    float xh[NC][4], g[NC][4];
    float sg = 0.f, sgx = 0.f;
#pragma unroll
    for (int j = 0; j < NC; ++j) {
      const int c = 4 * (64 * j + lane);
      float d[4], av[4], rv[4];
      ldv<T, 4>(dy + base + c, d);
      ldv<T, 4>(a + base + c, av);
      ldv<T, 4>(r + base + c, rv);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        xh[j][e] = (av[e] + rv[e] - mean) * rstd;
        g[j][e] = d[e] * wreg[j][e];
        dw[j][e] += d[e] * xh[j][e];
        db[j][e] += d[e];
        sg += g[j][e];
        sgx += g[j][e] * xh[j][e];
      }
    }
    const float mg = wave_sum(sg) * (1.f / H), mgx = wave_sum(sgx) * (1.f / H);
#pragma unroll
    for (int j = 0; j < NC; ++j) {
      float o[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) o[e] = rstd * (g[j][e] - mg - xh[j][e] * mgx);
      stv<T, 4>(dx + base + 4 * (64 * j + lane), o);
    }
  }
  // combine the 4 waves' column partials: LDS image [wave][H] x2, then each thread sums its
  // H/256 columns over the waves in a fixed order -> one partial row per block
  __shared__ float sdw[kThreads / 64][H];
  __shared__ float sdb[kThreads / 64][H];
#pragma unroll
  for (int j = 0; j < NC; ++j) {
    const int c = 4 * (64 * j + lane);
    *(float4*)&sdw[wv][c] = make_float4(dw[j][0], dw[j][1], dw[j][2], dw[j][3]);
    *(float4*)&sdb[wv][c] = make_float4(db[j][0], db[j][1], db[j][2], db[j][3]);
  }
  __syncthreads();
  for (int c = threadIdx.x; c < H; c += kThreads) {
    float tw = 0.f, tb = 0.f;
#pragma unroll
    for (int i = 0; i < wpb; ++i) {
      tw += sdw[i][c];
      tb += sdb[i][c];
    }
    dw_part[(size_t)blockIdx.x * H + c] = tw;
    db_part[(size_t)blockIdx.x * H + c] = tb;
  }
}

template <typename T, typename P, int PER>
__global__ __launch_bounds__(kThreads) void add_ln_fwd(const T* __restrict__ a, const T* __restrict__ r,
                                                      const P* __restrict__ w, const P* __restrict__ b, int R,
                                                      int H, float eps, T* __restrict__ y, float* __restrict__ mean_out,
                                                      float* __restrict__ rstd_out) {
  const int lane = threadIdx.x & 63;
  const int wpb = kThreads / 64;
  for (int row = blockIdx.x * wpb + (threadIdx.x >> 6); row < R; row += gridDim.x * wpb) {
    const size_t base = (size_t)row * H;
    float v[PER];
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int c = lane + k * 64;
      v[k] = c < H ? ld(a + base + c) + ld(r + base + c) : 0.f;
      s += v[k];
    }
    const float mean = wave_sum(s) / H;
    float q = 0.f;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int c = lane + k * 64;
      const float d = c < H ? v[k] - mean : 0.f;
      q += d * d;
    }
    const float rstd = rsqrtf(wave_sum(q) / H + eps);
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int c = lane + k * 64;
      if (c < H) st(y + base + c, (v[k] - mean) * rstd * ld(w + c) + ld(b + c));
    }
    if (lane == 0) {
      mean_out[row] = mean;
      rstd_out[row] = rstd;
    }
  }
}

template <typename T, typename P, int PER>
__global__ __launch_bounds__(kThreads) void add_ln_bwd(const T* __restrict__ dy, const T* __restrict__ a,
                                                      const T* __restrict__ r, const P* __restrict__ w,
                                                      const float* __restrict__ mean_in,
                                                      const float* __restrict__ rstd_in, int R, int H,
                                                      T* __restrict__ dx, float* __restrict__ dw_part,
                                                      float* __restrict__ db_part) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int wpb = kThreads / 64;
  float dw[PER], db[PER];
#pragma unroll
  for (int k = 0; k < PER; ++k) dw[k] = db[k] = 0.f;
  for (int row = blockIdx.x * wpb + wv; row < R; row += gridDim.x * wpb) {
    const size_t base = (size_t)row * H;
    const float mean = mean_in[row], rstd = rstd_in[row];
    float xh[PER], g[PER];
    float sg = 0.f, sgx = 0.f;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int c = lane + k * 64;
      if (c < H) {
        const float d = ld(dy + base + c);
        xh[k] = (ld(a + base + c) + ld(r + base + c) - mean) * rstd;
        g[k] = d * ld(w + c);
        dw[k] += d * xh[k];
        db[k] += d;
      } else {
        xh[k] = g[k] = 0.f;
      }
      sg += g[k];
      sgx += g[k] * xh[k];
    }
    const float mg = wave_sum(sg) / H, mgx = wave_sum(sgx) / H;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int c = lane + k * 64;
      if (c < H) st(dx + base + c, rstd * (g[k] - mg - xh[k] * mgx));
    }
  }
  // combine the 4 waves' column partials in LDS, one row of partials per block
  __shared__ float sdw[kThreads / 64][64];
  __shared__ float sdb[kThreads / 64][64];
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    sdw[wv][lane] = dw[k];
    sdb[wv][lane] = db[k];
    __syncthreads();
    if (wv == 0) {
      const int c = lane + k * 64;
      float tw = 0.f, tb = 0.f;
      for (int i = 0; i < wpb; ++i) {
        tw += sdw[i][lane];
        tb += sdb[i][lane];
      }
      if (c < H) {
        dw_part[(size_t)blockIdx.x * H + c] = tw;
        db_part[(size_t)blockIdx.x * H + c] = tb;
      }
    }
    __syncthreads();
  }
}

__device__ __forceinline__ float gelu_f(float x) { return 0.5f * x * (1.f + erff(x * 0.70710678118654752f)); }
__device__ __forceinline__ float gelu_grad(float x) {
  return 0.5f * (1.f + erff(x * 0.70710678118654752f)) + x * 0.3989422804014327f * expf(-0.5f * x * x);
}

// grid (ceil(N / kThreads), row chunks): thread owns one column, walks its chunk of rows —
// no per-element 64-bit div/mod, coalesced across the wave, and the bias-gradient column
// partial falls out of the same loop (written to db_part[chunk][col]).
template <typename T, typename P>
__global__ __launch_bounds__(kThreads) void bias_gelu_fwd(const T* __restrict__ x, const P* __restrict__ bias,
                                                         int M, int N, T* __restrict__ y) {
  const int col = blockIdx.x * kThreads + threadIdx.x;
  if (col >= N) return;
  const int r0 = (int)((long long)M * blockIdx.y / gridDim.y), r1 = (int)((long long)M * (blockIdx.y + 1) / gridDim.y);
  const float bb = ld(bias + col);
  for (int r = r0; r < r1; ++r) {
    const size_t i = (size_t)r * N + col;
    st(y + i, gelu_f(ld(x + i) + bb));
  }
}

template <typename T, typename P>
__global__ __launch_bounds__(kThreads) void bias_gelu_bwd(const T* __restrict__ dy, const T* __restrict__ x,
                                                         const P* __restrict__ bias, int M, int N,
                                                         T* __restrict__ dx, float* __restrict__ db_part) {
  const int col = blockIdx.x * kThreads + threadIdx.x;
  if (col >= N) return;
  const int r0 = (int)((long long)M * blockIdx.y / gridDim.y), r1 = (int)((long long)M * (blockIdx.y + 1) / gridDim.y);
  const float bb = ld(bias + col);
  float acc = 0.f;
  int r = r0;
  for (; r + 4 <= r1; r += 4) {  // 8 independent loads in flight per thread
    float d[4], v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const size_t i = (size_t)(r + u) * N + col;
      d[u] = ld(dy + i);
      v[u] = ld(x + i);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const float g = d[u] * gelu_grad(v[u] + bb);
      st(dx + (size_t)(r + u) * N + col, g);
      acc += cvt_round<T>(g);  // bias grad of the value actually stored
    }
  }
  for (; r < r1; ++r) {
    const size_t i = (size_t)r * N + col;
    const float g = ld(dy + i) * gelu_grad(ld(x + i) + bb);
    st(dx + i, g);
    acc += cvt_round<T>(g);
  }
  db_part[(size_t)blockIdx.y * N + col] = acc;
}

// ---- vectorised bias+GELU (N % VW == 0, VW = 16 B / sizeof(T)): block = 64 column groups of VW
// contiguous columns x 4 row slices; grid (ceil(N / (64 VW)), row chunks). 16-byte accesses per
// lane; the backward combines its 4 slices' bias-grad partials in LDS (fixed order) and writes one
// partial row per chunk.
constexpr int kGCols = 64, kGSlices = kThreads / kGCols;

template <typename T, typename P, int VW>
__global__ __launch_bounds__(kThreads) void bias_gelu_fwd_v(const T* __restrict__ x, const P* __restrict__ bias,
                                                           int M, int N, T* __restrict__ y) {
  const int cg = threadIdx.x % kGCols, sl = threadIdx.x / kGCols;
  const int col = (blockIdx.x * kGCols + cg) * VW;
  if (col >= N) return;
  const int r0 = (int)((long long)M * blockIdx.y / gridDim.y), r1 = (int)((long long)M * (blockIdx.y + 1) / gridDim.y);
  float bb[VW];
#pragma unroll
  for (int e = 0; e < VW; ++e) bb[e] = ld(bias + col + e);
  for (int r = r0 + sl; r < r1; r += kGSlices) {
    const size_t i = (size_t)r * N + col;
    float v[VW];
    ldv<T, VW>(x + i, v);
#pragma unroll
    for (int e = 0; e < VW; ++e) v[e] = gelu_f(v[e] + bb[e]);
    stv<T, VW>(y + i, v);
  }
}

template <typename T, typename P, int VW>
__global__ __launch_bounds__(kThreads) void bias_gelu_bwd_v(const T* __restrict__ dy, const T* __restrict__ x,
                                                           const P* __restrict__ bias, int M, int N,
                                                           T* __restrict__ dx, float* __restrict__ db_part) {
  __shared__ float sdb[kGSlices][kGCols * VW];
  const int cg = threadIdx.x % kGCols, sl = threadIdx.x / kGCols;
  const int col = (blockIdx.x * kGCols + cg) * VW;
  const bool ok = col < N;
  const int r0 = (int)((long long)M * blockIdx.y / gridDim.y), r1 = (int)((long long)M * (blockIdx.y + 1) / gridDim.y);
  float bb[VW], acc[VW];
#pragma unroll
  for (int e = 0; e < VW; ++e) {
    bb[e] = ok ? ld(bias + col + e) : 0.f;
    acc[e] = 0.f;
  }
  if (ok) {
    for (int r = r0 + sl; r < r1; r += kGSlices) {
      const size_t i = (size_t)r * N + col;
      float d[VW], v[VW];
      ldv<T, VW>(dy + i, d);
      ldv<T, VW>(x + i, v);
#pragma unroll
      for (int e = 0; e < VW; ++e) d[e] *= gelu_grad(v[e] + bb[e]);
      stv<T, VW>(dx + i, d);
#pragma unroll
      for (int e = 0; e < VW; ++e) acc[e] += cvt_round<T>(d[e]);  // bias grad of the value actually stored
    }
  }
#pragma unroll
  for (int e = 0; e < VW; ++e) sdb[sl][cg * VW + e] = acc[e];
  __syncthreads();
  for (int c = threadIdx.x; c < kGCols * VW; c += kThreads) {
    const int gc = blockIdx.x * kGCols * VW + c;
    if (gc >= N) continue;
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < kGSlices; ++i) t += sdb[i][c];
    db_part[(size_t)blockIdx.y * N + gc] = t;
  }
}

// Column sums of an activation gradient [M, N] (the bias gradient of a Linear / bias-add): same block
// shape as bias_gelu_bwd_v (64 column groups of VW contiguous columns x 4 row slices, 16-B loads), one
// partial row per row chunk, reduced by col_reduce2 -> deterministic, replaces a generic reduce kernel.
template <typename T, int VW>
__global__ __launch_bounds__(kThreads) void col_sum_v(const T* __restrict__ x, int M, int N, float* __restrict__ part) {
  __shared__ float sp[kGSlices][kGCols * VW];
  const int cg = threadIdx.x % kGCols, sl = threadIdx.x / kGCols;
  const int col = (blockIdx.x * kGCols + cg) * VW;
  const int r0 = (int)((long long)M * blockIdx.y / gridDim.y), r1 = (int)((long long)M * (blockIdx.y + 1) / gridDim.y);
  float acc[VW];
#pragma unroll
  for (int e = 0; e < VW; ++e) acc[e] = 0.f;
  if (col < N) {
    int r = r0 + sl;
    for (; r + kGSlices < r1; r += 2 * kGSlices) {  // 2 rows in flight per thread
      float v0[VW], v1[VW];
      ldv<T, VW>(x + (size_t)r * N + col, v0);
      ldv<T, VW>(x + (size_t)(r + kGSlices) * N + col, v1);
#pragma unroll
      for (int e = 0; e < VW; ++e) acc[e] += v0[e] + v1[e];
    }
    for (; r < r1; r += kGSlices) {
      float v0[VW];
      ldv<T, VW>(x + (size_t)r * N + col, v0);
#pragma unroll
      for (int e = 0; e < VW; ++e) acc[e] += v0[e];
    }
  }
#pragma unroll
  for (int e = 0; e < VW; ++e) sp[sl][cg * VW + e] = acc[e];
  __syncthreads();
  for (int c = threadIdx.x; c < kGCols * VW; c += kThreads) {
    const int gc = blockIdx.x * kGCols * VW + c;
    if (gc >= N) continue;
    float t = 0.f;
#pragma unroll
    for (int i = 0; i < kGSlices; ++i) t += sp[i][c];
    part[(size_t)blockIdx.y * N + gc] = t;
  }
}

template <typename T>
__global__ __launch_bounds__(kThreads) void col_sum(const T* __restrict__ x, int M, int N, float* __restrict__ part) {
  const int col = blockIdx.x * kThreads + threadIdx.x;
  if (col >= N) return;
  const int r0 = (int)((long long)M * blockIdx.y / gridDim.y), r1 = (int)((long long)M * (blockIdx.y + 1) / gridDim.y);
  float acc = 0.f;
  for (int r = r0; r < r1; ++r) acc += ld(x + (size_t)r * N + col);
  part[(size_t)blockIdx.y * N + col] = acc;
}

// sum `rows` partial rows of width N (fixed order) for up to two buffers in one launch
// block = kRedCols columns x kRedSlices row slices; each slice strides the rows with 8 loads per buffer in
// flight (the partials are L2-resident: the kernel is latency-, not bandwidth-bound), slices combined in
// LDS in a fixed order -> deterministic, N/16 workgroups
constexpr int kRedCols = 16, kRedSlices = kThreads / kRedCols, kRedU = 8;

template <typename PO>
__global__ __launch_bounds__(kThreads) void col_reduce2(const float* __restrict__ p0, const float* __restrict__ p1,
                                                       int rows, int N, PO* __restrict__ o0,
                                                       PO* __restrict__ o1) {
  __shared__ float sa[kRedSlices][kRedCols];
  __shared__ float sb[kRedSlices][kRedCols];
  const int cx = threadIdx.x % kRedCols, sl = threadIdx.x / kRedCols;
  const int col = blockIdx.x * kRedCols + cx;
  float a = 0.f, b = 0.f;
  if (col < N) {
    int r = sl;
    for (; r + (kRedU - 1) * kRedSlices < rows; r += kRedU * kRedSlices) {
      float va[kRedU], vb[kRedU];
#pragma unroll
      for (int u = 0; u < kRedU; ++u) va[u] = p0[(size_t)(r + u * kRedSlices) * N + col];
      if (p1 != nullptr) {
#pragma unroll
        for (int u = 0; u < kRedU; ++u) vb[u] = p1[(size_t)(r + u * kRedSlices) * N + col];
      }
#pragma unroll
      for (int u = 0; u < kRedU; ++u) {
        a += va[u];
        if (p1 != nullptr) b += vb[u];
      }
    }
    for (; r < rows; r += kRedSlices) {
      a += p0[(size_t)r * N + col];
      if (p1 != nullptr) b += p1[(size_t)r * N + col];
    }
  }
  sa[sl][cx] = a;
  sb[sl][cx] = b;
  __syncthreads();
  if (sl != 0 || col >= N) return;
  a = 0.f;
  b = 0.f;
  for (int i = 0; i < kRedSlices; ++i) {
    a += sa[i][cx];
    b += sb[i][cx];
  }
  st(o0 + col, a);
  if (o1 != nullptr) st(o1 + col, b);
}

template <typename T, typename P, int PER>
int launch_add_ln(int fwd, const void* dy, const void* a, const void* r, const void* w, const void* b, int R, int H,
                  float eps, void* out, float* mean, float* rstd, float* dw_part, float* db_part, int blocks,
                  hipStream_t st) {
  if (fwd)
    hipLaunchKernelGGL((add_ln_fwd<T, P, PER>), dim3(blocks), dim3(kThreads), 0, st, (const T*)a, (const T*)r,
                       (const P*)w, (const P*)b, R, H, eps, (T*)out, mean, rstd);
  else
    hipLaunchKernelGGL((add_ln_bwd<T, P, PER>), dim3(blocks), dim3(kThreads), 0, st, (const T*)dy, (const T*)a,
                       (const T*)r, (const P*)w, mean, rstd, R, H, (T*)out, dw_part, db_part);
  return (int)hipGetLastError();
}

template <typename T, typename P, int NC>
int launch_add_ln_v(int fwd, const void* dy, const void* a, const void* r, const void* w, const void* b, int R,
                    float eps, void* out, float* mean, float* rstd, float* dw_part, float* db_part, int blocks,
                    hipStream_t st) {
  if (fwd)
    hipLaunchKernelGGL((add_ln_fwd_v<T, P, NC>), dim3(blocks), dim3(kThreads), 0, st, (const T*)a, (const T*)r,
                       (const P*)w, (const P*)b, R, eps, (T*)out, mean, rstd);
  else
    hipLaunchKernelGGL((add_ln_bwd_v<T, P, NC>), dim3(blocks), dim3(kThreads), 0, st, (const T*)dy, (const T*)a,
                       (const T*)r, (const P*)w, mean, rstd, R, (T*)out, dw_part, db_part);
  return (int)hipGetLastError();
}

template <typename T, typename P>
int dispatch_add_ln(int fwd, const void* dy, const void* a, const void* r, const void* w, const void* b, int R,
                    int H, float eps, void* out, float* mean, float* rstd, float* dw_part, float* db_part, int blocks,
                    hipStream_t st) {
  const uintptr_t al = (uintptr_t)dy | (uintptr_t)a | (uintptr_t)r | (uintptr_t)w | (uintptr_t)b | (uintptr_t)out;
  switch (H % 256 == 0 && al % 16 == 0 ? H / 256 : 0) {  // vectorised paths (BERT-base 768 -> NC 3, large 1024 -> 4)
    case 1: return launch_add_ln_v<T, P, 1>(fwd, dy, a, r, w, b, R, eps, out, mean, rstd, dw_part, db_part, blocks, st);
    case 2: return launch_add_ln_v<T, P, 2>(fwd, dy, a, r, w, b, R, eps, out, mean, rstd, dw_part, db_part, blocks, st);
    case 3: return launch_add_ln_v<T, P, 3>(fwd, dy, a, r, w, b, R, eps, out, mean, rstd, dw_part, db_part, blocks, st);
    case 4: return launch_add_ln_v<T, P, 4>(fwd, dy, a, r, w, b, R, eps, out, mean, rstd, dw_part, db_part, blocks, st);
    default: break;
  }
  const int per = (H + 63) / 64;
  if (per <= 4)
    return launch_add_ln<T, P, 4>(fwd, dy, a, r, w, b, R, H, eps, out, mean, rstd, dw_part, db_part, blocks, st);
  if (per <= 12)
    return launch_add_ln<T, P, 12>(fwd, dy, a, r, w, b, R, H, eps, out, mean, rstd, dw_part, db_part, blocks, st);
  if (per <= 16)
    return launch_add_ln<T, P, 16>(fwd, dy, a, r, w, b, R, H, eps, out, mean, rstd, dw_part, db_part, blocks, st);
  return launch_add_ln<T, P, kMaxPer>(fwd, dy, a, r, w, b, R, H, eps, out, mean, rstd, dw_part, db_part, blocks, st);
}

// (activation dtype, parameter dtype) -> dispatch_add_ln<T, P>; dtype / pdt: 0 fp32, 1 bf16
int dispatch_add_ln_any(int dtype, int pdt, int fwd, const void* dy, const void* a, const void* r, const void* w,
                        const void* b, int R, int H, float eps, void* out, float* mean, float* rstd, float* dw_part,
                        float* db_part, int blocks, hipStream_t st) {
  typedef __hip_bfloat16 bf;
  if (dtype && pdt)
    return dispatch_add_ln<bf, bf>(fwd, dy, a, r, w, b, R, H, eps, out, mean, rstd, dw_part, db_part, blocks, st);
  if (dtype)
    return dispatch_add_ln<bf, float>(fwd, dy, a, r, w, b, R, H, eps, out, mean, rstd, dw_part, db_part, blocks, st);
  if (pdt)
    return dispatch_add_ln<float, bf>(fwd, dy, a, r, w, b, R, H, eps, out, mean, rstd, dw_part, db_part, blocks, st);
  return dispatch_add_ln<float, float>(fwd, dy, a, r, w, b, R, H, eps, out, mean, rstd, dw_part, db_part, blocks, st);
}

template <typename T, typename P>
int launch_gelu(int fwd, const void* dy, const void* x, const void* bias, int M, int N, void* out, float* db_part,
                void* db, int chunks, hipStream_t st) {
  constexpr int VW = 16 / sizeof(T);
  if (N % VW == 0 && ((uintptr_t)dy | (uintptr_t)x | (uintptr_t)out) % 16 == 0) {
    const dim3 vgrid((N / VW + kGCols - 1) / kGCols, chunks);
    if (fwd)
      hipLaunchKernelGGL((bias_gelu_fwd_v<T, P, VW>), vgrid, dim3(kThreads), 0, st, (const T*)x, (const P*)bias, M, N,
                         (T*)out);
    else
      hipLaunchKernelGGL((bias_gelu_bwd_v<T, P, VW>), vgrid, dim3(kThreads), 0, st, (const T*)dy, (const T*)x,
                         (const P*)bias, M, N, (T*)out, db_part);
  } else {
    const dim3 grid((N + kThreads - 1) / kThreads, chunks);
    if (fwd)
      hipLaunchKernelGGL((bias_gelu_fwd<T, P>), grid, dim3(kThreads), 0, st, (const T*)x, (const P*)bias, M, N,
                         (T*)out);
    else
      hipLaunchKernelGGL((bias_gelu_bwd<T, P>), grid, dim3(kThreads), 0, st, (const T*)dy, (const T*)x,
                         (const P*)bias, M, N, (T*)out, db_part);
  }
  if (!fwd)
    hipLaunchKernelGGL(col_reduce2<P>, dim3((N + kRedCols - 1) / kRedCols), dim3(kThreads), 0, st, db_part, nullptr,
                       chunks, N, (P*)db, (P*)nullptr);
  return (int)hipGetLastError();
}

template <typename T, typename P>
int launch_col_sum(const void* x, int M, int N, float* part, void* out, int chunks, hipStream_t st) {
  constexpr int VW = 16 / sizeof(T);
  if (N % VW == 0 && (uintptr_t)x % 16 == 0)
    hipLaunchKernelGGL((col_sum_v<T, VW>), dim3((N / VW + kGCols - 1) / kGCols, chunks), dim3(kThreads), 0, st,
                       (const T*)x, M, N, part);
  else
    hipLaunchKernelGGL(col_sum<T>, dim3((N + kThreads - 1) / kThreads, chunks), dim3(kThreads), 0, st, (const T*)x, M,
                       N, part);
  hipLaunchKernelGGL(col_reduce2<P>, dim3((N + kRedCols - 1) / kRedCols), dim3(kThreads), 0, st, part, nullptr, chunks,
                     N, (P*)out, (P*)nullptr);
  return (int)hipGetLastError();
}

}  // namespace

extern "C" {

// partial-row count used by add_ln_bwd (fewer, fatter blocks: each wave walks many rows)
int mifx_bert_ln_blocks(int R) {
  const int need = (R + 7) / 8;  // 2 rows per wave
  return need < 1024 ? (need > 0 ? need : 1) : 1024;
}

// rows of partials for bias_gelu_bwd
int mifx_bert_gelu_chunks(int M) { return M < 16 ? 1 : (M / 16 < 512 ? M / 16 : 512); }

// dtype: activations, pdt: gamma/beta (and dw/db): 0 fp32, 1 bf16
int mifx_bert_add_ln_fwd(int dtype, int pdt, const void* a, const void* r, const void* w, const void* b, int R, int H,
                         float eps, void* y, float* mean, float* rstd, hipStream_t st) {
  if (H <= 0 || H > 64 * kMaxPer || R <= 0) return -1;
  const int need = (R + 3) / 4;
  const int blocks = need < 4096 ? need : 4096;
  return dispatch_add_ln_any(dtype, pdt, 1, nullptr, a, r, w, b, R, H, eps, y, mean, rstd, nullptr, nullptr, blocks,
                             st);
}

// scratch: dw_part / db_part [mifx_bert_ln_blocks(R), H]; outputs dw, db [H] in the parameter dtype
int mifx_bert_add_ln_bwd(int dtype, int pdt, const void* dy, const void* a, const void* r, const void* w,
                         const float* mean, const float* rstd, int R, int H, void* dx, float* dw_part, float* db_part,
                         void* dw, void* db, hipStream_t st) {
  if (H <= 0 || H > 64 * kMaxPer || R <= 0) return -1;
  const int blocks = mifx_bert_ln_blocks(R);
  const int rc = dispatch_add_ln_any(dtype, pdt, 0, dy, a, r, w, nullptr, R, H, 0.f, dx, (float*)mean, (float*)rstd,
                                     dw_part, db_part, blocks, st);
  if (rc) return rc;
  const dim3 g((H + kRedCols - 1) / kRedCols);
  if (pdt)
    hipLaunchKernelGGL(col_reduce2<__hip_bfloat16>, g, dim3(kThreads), 0, st, dw_part, db_part, blocks, H,
                       (__hip_bfloat16*)dw, (__hip_bfloat16*)db);
  else
    hipLaunchKernelGGL(col_reduce2<float>, g, dim3(kThreads), 0, st, dw_part, db_part, blocks, H, (float*)dw,
                       (float*)db);
  return (int)hipGetLastError();
}

// x: [M, N]; fwd -> out = gelu(x + bias); bwd -> out = dx, db [N] in the bias dtype
// (scratch db_part [gelu_chunks(M), N])
int mifx_bert_bias_gelu(int dtype, int pdt, int fwd, const void* dy, const void* x, const void* bias, int M, int N,
                        void* out, float* db_part, void* db, hipStream_t st) {
  if (M <= 0 || N <= 0) return -1;
  const int chunks = fwd ? (M < 1024 ? M : 1024) : mifx_bert_gelu_chunks(M);
  typedef __hip_bfloat16 bf;
  if (dtype && pdt) return launch_gelu<bf, bf>(fwd, dy, x, bias, M, N, out, db_part, db, chunks, st);
  if (dtype) return launch_gelu<bf, float>(fwd, dy, x, bias, M, N, out, db_part, db, chunks, st);
  if (pdt) return launch_gelu<float, bf>(fwd, dy, x, bias, M, N, out, db_part, db, chunks, st);
  return launch_gelu<float, float>(fwd, dy, x, bias, M, N, out, db_part, db, chunks, st);
}

// out[N] (dtype pdt) = column sums of x [M, N] (dtype); scratch part [gelu_chunks(M), N] fp32
int mifx_bert_col_sum(int dtype, int pdt, const void* x, int M, int N, float* part, void* out, hipStream_t st) {
  if (M <= 0 || N <= 0) return -1;
  const int chunks = mifx_bert_gelu_chunks(M);
  typedef __hip_bfloat16 bf;
  if (dtype && pdt) return launch_col_sum<bf, bf>(x, M, N, part, out, chunks, st);
  if (dtype) return launch_col_sum<bf, float>(x, M, N, part, out, chunks, st);
  if (pdt) return launch_col_sum<float, bf>(x, M, N, part, out, chunks, st);
  return launch_col_sum<float, float>(x, M, N, part, out, chunks, st);
}

}  // extern "C"
