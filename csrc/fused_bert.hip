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
// Activations are bf16 or fp32 (template), LayerNorm params and statistics fp32.
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

template <typename T, int PER>
__global__ __launch_bounds__(kThreads) void add_ln_fwd(const T* __restrict__ a, const T* __restrict__ r,
                                                      const float* __restrict__ w, const float* __restrict__ b, int R,
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
      if (c < H) st(y + base + c, (v[k] - mean) * rstd * w[c] + b[c]);
    }
    if (lane == 0) {
      mean_out[row] = mean;
      rstd_out[row] = rstd;
    }
  }
}

template <typename T, int PER>
__global__ __launch_bounds__(kThreads) void add_ln_bwd(const T* __restrict__ dy, const T* __restrict__ a,
                                                      const T* __restrict__ r, const float* __restrict__ w,
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
        g[k] = d * w[c];
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
template <typename T>
__global__ __launch_bounds__(kThreads) void bias_gelu_fwd(const T* __restrict__ x, const float* __restrict__ bias,
                                                         int M, int N, T* __restrict__ y) {
  const int col = blockIdx.x * kThreads + threadIdx.x;
  if (col >= N) return;
  const int r0 = (int)((long long)M * blockIdx.y / gridDim.y), r1 = (int)((long long)M * (blockIdx.y + 1) / gridDim.y);
  const float bb = bias[col];
  for (int r = r0; r < r1; ++r) {
    const size_t i = (size_t)r * N + col;
    st(y + i, gelu_f(ld(x + i) + bb));
  }
}

template <typename T>
__global__ __launch_bounds__(kThreads) void bias_gelu_bwd(const T* __restrict__ dy, const T* __restrict__ x,
                                                         const float* __restrict__ bias, int M, int N,
                                                         T* __restrict__ dx, float* __restrict__ db_part) {
  const int col = blockIdx.x * kThreads + threadIdx.x;
  if (col >= N) return;
  const int r0 = (int)((long long)M * blockIdx.y / gridDim.y), r1 = (int)((long long)M * (blockIdx.y + 1) / gridDim.y);
  const float bb = bias[col];
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

// sum `rows` partial rows of width N (fixed order) for up to two buffers in one launch
// block = kRedCols columns x kRedSlices row slices (each slice strides the rows, 4 loads in
// flight), slices combined in LDS in a fixed order -> deterministic, ~N/32 workgroups
constexpr int kRedCols = 32, kRedSlices = kThreads / kRedCols;

__global__ __launch_bounds__(kThreads) void col_reduce2(const float* __restrict__ p0, const float* __restrict__ p1,
                                                       int rows, int N, float* __restrict__ o0,
                                                       float* __restrict__ o1) {
  __shared__ float sa[kRedSlices][kRedCols];
  __shared__ float sb[kRedSlices][kRedCols];
  const int cx = threadIdx.x % kRedCols, sl = threadIdx.x / kRedCols;
  const int col = blockIdx.x * kRedCols + cx;
  float a = 0.f, b = 0.f;
  if (col < N) {
    int r = sl;
    for (; r + 3 * kRedSlices < rows; r += 4 * kRedSlices) {
      const float a0 = p0[(size_t)r * N + col], a1 = p0[(size_t)(r + kRedSlices) * N + col];
      const float a2 = p0[(size_t)(r + 2 * kRedSlices) * N + col], a3 = p0[(size_t)(r + 3 * kRedSlices) * N + col];
      a += (a0 + a1) + (a2 + a3);
      if (p1 != nullptr) {
        const float b0 = p1[(size_t)r * N + col], b1 = p1[(size_t)(r + kRedSlices) * N + col];
        const float b2 = p1[(size_t)(r + 2 * kRedSlices) * N + col], b3 = p1[(size_t)(r + 3 * kRedSlices) * N + col];
        b += (b0 + b1) + (b2 + b3);
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
  o0[col] = a;
  if (o1 != nullptr) o1[col] = b;
}

template <typename T, int PER>
int launch_add_ln(int fwd, const void* dy, const void* a, const void* r, const float* w, const float* b, int R, int H,
                  float eps, void* out, float* mean, float* rstd, float* dw_part, float* db_part, int blocks,
                  hipStream_t st) {
  if (fwd)
    hipLaunchKernelGGL((add_ln_fwd<T, PER>), dim3(blocks), dim3(kThreads), 0, st, (const T*)a, (const T*)r, w, b, R,
                       H, eps, (T*)out, mean, rstd);
  else
    hipLaunchKernelGGL((add_ln_bwd<T, PER>), dim3(blocks), dim3(kThreads), 0, st, (const T*)dy, (const T*)a,
                       (const T*)r, w, mean, rstd, R, H, (T*)out, dw_part, db_part);
  return (int)hipGetLastError();
}

template <typename T>
int dispatch_add_ln(int fwd, const void* dy, const void* a, const void* r, const float* w, const float* b, int R,
                    int H, float eps, void* out, float* mean, float* rstd, float* dw_part, float* db_part, int blocks,
                    hipStream_t st) {
  const int per = (H + 63) / 64;
  if (per <= 4) return launch_add_ln<T, 4>(fwd, dy, a, r, w, b, R, H, eps, out, mean, rstd, dw_part, db_part, blocks, st);
  if (per <= 12) return launch_add_ln<T, 12>(fwd, dy, a, r, w, b, R, H, eps, out, mean, rstd, dw_part, db_part, blocks, st);
  if (per <= 16) return launch_add_ln<T, 16>(fwd, dy, a, r, w, b, R, H, eps, out, mean, rstd, dw_part, db_part, blocks, st);
  return launch_add_ln<T, kMaxPer>(fwd, dy, a, r, w, b, R, H, eps, out, mean, rstd, dw_part, db_part, blocks, st);
}

}  // namespace

extern "C" {

// partial-row count used by add_ln_bwd (fewer, fatter blocks: each wave walks many rows)
int mifx_bert_ln_blocks(int R) {
  const int need = (R + 3) / 4;
  return need < 256 ? (need > 0 ? need : 1) : 256;
}

// rows of partials for bias_gelu_bwd
int mifx_bert_gelu_chunks(int M) { return M < 64 ? 1 : (M / 64 < 128 ? M / 64 : 128); }

// dtype: 0 fp32, 1 bf16
int mifx_bert_add_ln_fwd(int dtype, const void* a, const void* r, const float* w, const float* b, int R, int H,
                         float eps, void* y, float* mean, float* rstd, hipStream_t st) {
  if (H <= 0 || H > 64 * kMaxPer || R <= 0) return -1;
  const int need = (R + 3) / 4;
  const int blocks = need < 4096 ? need : 4096;
  return dtype ? dispatch_add_ln<__hip_bfloat16>(1, nullptr, a, r, w, b, R, H, eps, y, mean, rstd, nullptr, nullptr,
                                                 blocks, st)
               : dispatch_add_ln<float>(1, nullptr, a, r, w, b, R, H, eps, y, mean, rstd, nullptr, nullptr, blocks, st);
}

// scratch: dw_part / db_part [mifx_bert_ln_blocks(R), H]; outputs dw, db [H] (fp32)
int mifx_bert_add_ln_bwd(int dtype, const void* dy, const void* a, const void* r, const float* w, const float* mean,
                         const float* rstd, int R, int H, void* dx, float* dw_part, float* db_part, float* dw,
                         float* db, hipStream_t st) {
  if (H <= 0 || H > 64 * kMaxPer || R <= 0) return -1;
  const int blocks = mifx_bert_ln_blocks(R);
  const int rc = dtype ? dispatch_add_ln<__hip_bfloat16>(0, dy, a, r, w, nullptr, R, H, 0.f, dx, (float*)mean,
                                                         (float*)rstd, dw_part, db_part, blocks, st)
                       : dispatch_add_ln<float>(0, dy, a, r, w, nullptr, R, H, 0.f, dx, (float*)mean, (float*)rstd,
                                                dw_part, db_part, blocks, st);
  if (rc) return rc;
  hipLaunchKernelGGL(col_reduce2, dim3((H + kRedCols - 1) / kRedCols), dim3(kThreads), 0, st, dw_part, db_part, blocks,
                     H, dw, db);
  return (int)hipGetLastError();
}

// x: [M, N]; fwd -> out = gelu(x + bias); bwd -> out = dx, db [N] (scratch db_part [gelu_chunks(M), N])
int mifx_bert_bias_gelu(int dtype, int fwd, const void* dy, const void* x, const float* bias, int M, int N, void* out,
                        float* db_part, float* db, hipStream_t st) {
  if (M <= 0 || N <= 0) return -1;
  const int chunks = fwd ? (M < 1024 ? M : 1024) : mifx_bert_gelu_chunks(M);
  const dim3 grid((N + kThreads - 1) / kThreads, chunks);
  if (dtype) {
    if (fwd)
      hipLaunchKernelGGL(bias_gelu_fwd<__hip_bfloat16>, grid, dim3(kThreads), 0, st, (const __hip_bfloat16*)x, bias, M,
                         N, (__hip_bfloat16*)out);
    else
      hipLaunchKernelGGL(bias_gelu_bwd<__hip_bfloat16>, grid, dim3(kThreads), 0, st, (const __hip_bfloat16*)dy,
                         (const __hip_bfloat16*)x, bias, M, N, (__hip_bfloat16*)out, db_part);
  } else {
    if (fwd)
      hipLaunchKernelGGL(bias_gelu_fwd<float>, grid, dim3(kThreads), 0, st, (const float*)x, bias, M, N, (float*)out);
    else
      hipLaunchKernelGGL(bias_gelu_bwd<float>, grid, dim3(kThreads), 0, st, (const float*)dy, (const float*)x, bias, M,
                         N, (float*)out, db_part);
  }
  if (!fwd)
    hipLaunchKernelGGL(col_reduce2, dim3((N + kRedCols - 1) / kRedCols), dim3(kThreads), 0, st, db_part, nullptr,
                       chunks, N, db, nullptr);
  return (int)hipGetLastError();
}

}  // extern "C"
