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
#include <stdlib.h>
#include <stdint.h>

#include "counter_rng.h"

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

// ---- dropout mask: counter-based, recomputed in the backward (nothing stored), hipGraph-replay safe; identical
// on every TP rank for a replicated activation (same seed). Definition: csrc/counter_rng.h.
using mifx_rng::drop_key;
using mifx_rng::keep4;

// Drop: the optional (bias, dropout) prologue of the fused LayerNorm: s = keep ? (a + bias) * scale : 0, + r.
// thr == 0 disables dropout (no hashing); bias == nullptr disables the bias.
// eoff: the flat element index of row 0 in the full activation (sequence parallelism: a rank's token shard draws the
// mask bits the whole tensor would, so the masks do not depend on the TP split; 0 otherwise; a multiple of 4)
template <typename P>
struct Drop {
  const P* bias;
  const int64_t* rng;
  int site;
  uint32_t thr;
  float scale;
  unsigned long long eoff;
};

// ---- vectorised fused [bias +] [dropout +] residual-add + LayerNorm (H % 256 == 0): lane owns NC chunks of
// 4 contiguous columns, chunk j of lane l = columns [4 (64 j + l), +4) -> every access is one 8/16-byte load
template <typename T, typename P, int NC>
__global__ __launch_bounds__(kThreads) void add_ln_fwd_v(const T* __restrict__ a, const T* __restrict__ r,
                                                        const P* __restrict__ w, const P* __restrict__ b,
                                                        Drop<P> dp, int R, float eps, T* __restrict__ y,
                                                        float* __restrict__ mean_out, float* __restrict__ rstd_out) {
  constexpr int H = NC * 256;
  const int lane = threadIdx.x & 63;
  const int wpb = kThreads / 64;
  // gamma / beta / bias loaded once, beside the first row's activations (loading gamma and beta after the row's
  // two reductions put one more dependent L2 round trip on every row)
  float bias[NC][4], wreg[NC][4], breg[NC][4];
#pragma unroll
  for (int j = 0; j < NC; ++j) {
    ldv<P, 4>(w + 4 * (64 * j + lane), wreg[j]);
    ldv<P, 4>(b + 4 * (64 * j + lane), breg[j]);
    if (dp.bias != nullptr)
      ldv<P, 4>(dp.bias + 4 * (64 * j + lane), bias[j]);
    else
      bias[j][0] = bias[j][1] = bias[j][2] = bias[j][3] = 0.f;
  }
  const uint64_t key = dp.thr ? drop_key(dp.rng, dp.site) : 0;
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
      const uint32_t k = dp.thr ? keep4(key, (dp.eoff + base + c) >> 2, dp.thr) : 0xf;
      const float sc = dp.thr ? dp.scale : 1.f;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[j][e] = ((k >> e) & 1 ? (v[j][e] + bias[j][e]) * sc : 0.f) + t[e];
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
      const float* wv = wreg[j];
      const float* bv = breg[j];
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

// backward: recomputes s (bias, mask, residual) and x_hat; ds = rstd (g - mean(g) - x_hat mean(g x_hat)),
// g = dy w. dr = ds; da = keep ? ds * scale : 0 (only written when da != dr, i.e. bias or dropout present).
// Column partials (LayerNorm dw, db and the bias gradient = column sums of da) per block, fixed order.
template <typename T, typename P, int NC>
__global__ __launch_bounds__(kThreads) void add_ln_bwd_v(const T* __restrict__ dy, const T* __restrict__ a,
                                                        const T* __restrict__ r, const P* __restrict__ w,
                                                        Drop<P> dp, const float* __restrict__ mean_in,
                                                        const float* __restrict__ rstd_in, int R,
                                                        T* __restrict__ dr, T* __restrict__ da,
                                                        float* __restrict__ dw_part, float* __restrict__ db_part,
                                                        float* __restrict__ dbias_part) {
  constexpr int H = NC * 256;
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int wpb = kThreads / 64;
  float dw[NC][4], db[NC][4], dbi[NC][4], wreg[NC][4], bias[NC][4];
#pragma unroll
  for (int j = 0; j < NC; ++j) {
    ldv<P, 4>(w + 4 * (64 * j + lane), wreg[j]);
    if (dp.bias != nullptr)
      ldv<P, 4>(dp.bias + 4 * (64 * j + lane), bias[j]);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      dw[j][e] = db[j][e] = dbi[j][e] = 0.f;
      if (dp.bias == nullptr) bias[j][e] = 0.f;
    }
  }
  const uint64_t key = dp.thr ? drop_key(dp.rng, dp.site) : 0;
  const float sc = dp.thr ? dp.scale : 1.f;
  for (int row = blockIdx.x * wpb + wv; row < R; row += gridDim.x * wpb) {
    const size_t base = (size_t)row * H;
    const float mean = mean_in[row], rstd = rstd_in[row];
    float xh[NC][4], g[NC][4];
    uint32_t kp[NC];
    float sg = 0.f, sgx = 0.f;
#pragma unroll
    for (int j = 0; j < NC; ++j) {
      const int c = 4 * (64 * j + lane);
      float d[4], av[4], rv[4];
      ldv<T, 4>(dy + base + c, d);
      ldv<T, 4>(a + base + c, av);
      ldv<T, 4>(r + base + c, rv);
      kp[j] = dp.thr ? keep4(key, (dp.eoff + base + c) >> 2, dp.thr) : 0xf;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float sv = ((kp[j] >> e) & 1 ? (av[e] + bias[j][e]) * sc : 0.f) + rv[e];
        xh[j][e] = (sv - mean) * rstd;
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
      const int c = 4 * (64 * j + lane);
      float o[4], oa[4];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        o[e] = rstd * (g[j][e] - mg - xh[j][e] * mgx);
        oa[e] = (kp[j] >> e) & 1 ? o[e] * sc : 0.f;
        dbi[j][e] += cvt_round<T>(oa[e]);  // bias grad of the value actually stored
      }
      stv<T, 4>(dr + base + c, o);
      if (da != dr) stv<T, 4>(da + base + c, oa);
    }
  }
  // combine the 4 waves' column partials: LDS image [wave][H] x3, then each thread sums its
  // H/256 columns over the waves in a fixed order -> one partial row per block
  __shared__ float sdw[kThreads / 64][H];
  __shared__ float sdb[kThreads / 64][H];
  __shared__ float sdi[kThreads / 64][H];
#pragma unroll
  for (int j = 0; j < NC; ++j) {
    const int c = 4 * (64 * j + lane);
    *(float4*)&sdw[wv][c] = make_float4(dw[j][0], dw[j][1], dw[j][2], dw[j][3]);
    *(float4*)&sdb[wv][c] = make_float4(db[j][0], db[j][1], db[j][2], db[j][3]);
    *(float4*)&sdi[wv][c] = make_float4(dbi[j][0], dbi[j][1], dbi[j][2], dbi[j][3]);
  }
  __syncthreads();
  for (int c = threadIdx.x; c < H; c += kThreads) {
    float tw = 0.f, tb = 0.f, ti = 0.f;
#pragma unroll
    for (int i = 0; i < wpb; ++i) {
      tw += sdw[i][c];
      tb += sdb[i][c];
      ti += sdi[i][c];
    }
    dw_part[(size_t)blockIdx.x * H + c] = tw;
    db_part[(size_t)blockIdx.x * H + c] = tb;
    if (dbias_part != nullptr) dbias_part[(size_t)blockIdx.x * H + c] = ti;
  }
}

// scalar-path mask bit of flat element idx
__device__ __forceinline__ bool keep1(uint64_t key, uint64_t idx, uint32_t thr) {
  return (keep4(key, idx >> 2, thr) >> (idx & 3)) & 1;
}

template <typename T, typename P, int PER>
__global__ __launch_bounds__(kThreads) void add_ln_fwd(const T* __restrict__ a, const T* __restrict__ r,
                                                      const P* __restrict__ w, const P* __restrict__ b, Drop<P> dp,
                                                      int R, int H, float eps, T* __restrict__ y,
                                                      float* __restrict__ mean_out, float* __restrict__ rstd_out) {
  const int lane = threadIdx.x & 63;
  const int wpb = kThreads / 64;
  const uint64_t key = dp.thr ? drop_key(dp.rng, dp.site) : 0;
  for (int row = blockIdx.x * wpb + (threadIdx.x >> 6); row < R; row += gridDim.x * wpb) {
    const size_t base = (size_t)row * H;
    float v[PER];
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int c = lane + k * 64;
      if (c < H) {
        float x = ld(a + base + c) + (dp.bias != nullptr ? ld(dp.bias + c) : 0.f);
        if (dp.thr) x = keep1(key, dp.eoff + base + c, dp.thr) ? x * dp.scale : 0.f;
        v[k] = x + ld(r + base + c);
      } else {
        v[k] = 0.f;
      }
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
                                                      const T* __restrict__ r, const P* __restrict__ w, Drop<P> dp,
                                                      const float* __restrict__ mean_in,
                                                      const float* __restrict__ rstd_in, int R, int H,
                                                      T* __restrict__ dr, T* __restrict__ da,
                                                      float* __restrict__ dw_part, float* __restrict__ db_part,
                                                      float* __restrict__ dbias_part) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int wpb = kThreads / 64;
  const uint64_t key = dp.thr ? drop_key(dp.rng, dp.site) : 0;
  const float sc = dp.thr ? dp.scale : 1.f;
  float dw[PER], db[PER], dbi[PER];
#pragma unroll
  for (int k = 0; k < PER; ++k) dw[k] = db[k] = dbi[k] = 0.f;
  for (int row = blockIdx.x * wpb + wv; row < R; row += gridDim.x * wpb) {
    const size_t base = (size_t)row * H;
    const float mean = mean_in[row], rstd = rstd_in[row];
    float xh[PER], g[PER];
    bool kp[PER];
    float sg = 0.f, sgx = 0.f;
#pragma unroll
    for (int k = 0; k < PER; ++k) {
      const int c = lane + k * 64;
      kp[k] = true;
      if (c < H) {
        const float d = ld(dy + base + c);
        float x = ld(a + base + c) + (dp.bias != nullptr ? ld(dp.bias + c) : 0.f);
        if (dp.thr) {
          kp[k] = keep1(key, dp.eoff + base + c, dp.thr);
          x = kp[k] ? x * sc : 0.f;
        }
        xh[k] = (x + ld(r + base + c) - mean) * rstd;
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
      if (c < H) {
        const float o = rstd * (g[k] - mg - xh[k] * mgx);
        const float oa = kp[k] ? o * sc : 0.f;
        dbi[k] += cvt_round<T>(oa);
        st(dr + base + c, o);
        if (da != dr) st(da + base + c, oa);
      }
    }
  }
  // combine the 4 waves' column partials in LDS, one row of partials per block
  __shared__ float sdw[kThreads / 64][64];
  __shared__ float sdb[kThreads / 64][64];
  __shared__ float sdi[kThreads / 64][64];
#pragma unroll
  for (int k = 0; k < PER; ++k) {
    sdw[wv][lane] = dw[k];
    sdb[wv][lane] = db[k];
    sdi[wv][lane] = dbi[k];
    __syncthreads();
    if (wv == 0) {
      const int c = lane + k * 64;
      float tw = 0.f, tb = 0.f, ti = 0.f;
      for (int i = 0; i < wpb; ++i) {
        tw += sdw[i][lane];
        tb += sdb[i][lane];
        ti += sdi[i][lane];
      }
      if (c < H) {
        dw_part[(size_t)blockIdx.x * H + c] = tw;
        db_part[(size_t)blockIdx.x * H + c] = tb;
        if (dbias_part != nullptr) dbias_part[(size_t)blockIdx.x * H + c] = ti;
      }
    }
    __syncthreads();
  }
}

// standalone dropout (the embedding-LayerNorm output and the pooled output): y = keep ? x * scale : 0 with the
// same mask function; the backward is the same kernel applied to dy. One group of 4 elements per thread.
template <typename T>
__global__ __launch_bounds__(kThreads) void dropout_k(const T* __restrict__ x, long long n, const int64_t* rng,
                                                     int site, uint32_t thr, float scale, T* __restrict__ y) {
  const uint64_t key = drop_key(rng, site);
  const long long groups = (n + 3) >> 2;
  for (long long g = (long long)blockIdx.x * kThreads + threadIdx.x; g < groups; g += (long long)gridDim.x * kThreads) {
    const uint32_t k = keep4(key, (uint64_t)g, thr);
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const long long i = 4 * g + e;
      if (i < n) st(y + i, (k >> e) & 1 ? ld(x + i) * scale : 0.f);
    }
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
// LDS in a fixed order -> deterministic, N/16 workgroups (8 columns x 32 slices -- twice the workgroups, half the
// dependent load batches, but 32-byte row segments -- measured slower on the BERT step: 5137-5146 vs 5228-5234
// seq/s, profiles/bert_redcols8_rejected_r4.txt; 32 columns x 8 slices: 5162-5172, bert_redcols32_rejected_r4.txt)
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

// the same reduction for up to three (partials, output) pairs in ONE launch: blockIdx.y picks the pair (the
// LayerNorm backward's dw, db and bias-gradient partials; one launch instead of two per LayerNorm backward, and
// three times the workgroups of the two-buffer form)
template <typename PO>
__global__ __launch_bounds__(kThreads) void col_reduce_y(const float* __restrict__ p0, const float* __restrict__ p1,
                                                        const float* __restrict__ p2, int rows, int N,
                                                        PO* __restrict__ o0, PO* __restrict__ o1,
                                                        PO* __restrict__ o2) {
  __shared__ float sa[kRedSlices][kRedCols];
  const float* __restrict__ p = blockIdx.y == 0 ? p0 : (blockIdx.y == 1 ? p1 : p2);
  PO* __restrict__ o = blockIdx.y == 0 ? o0 : (blockIdx.y == 1 ? o1 : o2);
  const int cx = threadIdx.x % kRedCols, sl = threadIdx.x / kRedCols;
  const int col = blockIdx.x * kRedCols + cx;
  float a = 0.f;
  if (col < N) {
    int r = sl;
    for (; r + (kRedU - 1) * kRedSlices < rows; r += kRedU * kRedSlices) {
      float va[kRedU];
#pragma unroll
      for (int u = 0; u < kRedU; ++u) va[u] = p[(size_t)(r + u * kRedSlices) * N + col];
#pragma unroll
      for (int u = 0; u < kRedU; ++u) a += va[u];
    }
    for (; r < rows; r += kRedSlices) a += p[(size_t)r * N + col];
  }
  sa[sl][cx] = a;
  __syncthreads();
  if (sl != 0 || col >= N) return;
  a = 0.f;
  for (int i = 0; i < kRedSlices; ++i) a += sa[i][cx];
  st(o + col, a);
}

// one launch description for the fused [bias +] [dropout +] residual-add + LayerNorm, forward or backward
struct LnArgs {
  int fwd;
  const void *dy, *a, *r, *w, *b, *bias;
  const int64_t* rng;
  int site;
  uint32_t thr;
  float scale;
  unsigned long long eoff;
  int R, H;
  float eps;
  void *out, *da;  // fwd: y; bwd: dr (out) and da
  float *mean, *rstd, *dw_part, *db_part, *dbias_part;
  int blocks;
  hipStream_t st;
};

template <typename T, typename P, int PER>
int launch_add_ln(const LnArgs& x) {
  const Drop<P> dp{(const P*)x.bias, x.rng, x.site, x.thr, x.scale, x.eoff};
  if (x.fwd)
    hipLaunchKernelGGL((add_ln_fwd<T, P, PER>), dim3(x.blocks), dim3(kThreads), 0, x.st, (const T*)x.a, (const T*)x.r,
                       (const P*)x.w, (const P*)x.b, dp, x.R, x.H, x.eps, (T*)x.out, x.mean, x.rstd);
  else
    hipLaunchKernelGGL((add_ln_bwd<T, P, PER>), dim3(x.blocks), dim3(kThreads), 0, x.st, (const T*)x.dy, (const T*)x.a,
                       (const T*)x.r, (const P*)x.w, dp, x.mean, x.rstd, x.R, x.H, (T*)x.out, (T*)x.da, x.dw_part,
                       x.db_part, x.dbias_part);
  return (int)hipGetLastError();
}

template <typename T, typename P, int NC>
int launch_add_ln_v(const LnArgs& x) {
  const Drop<P> dp{(const P*)x.bias, x.rng, x.site, x.thr, x.scale, x.eoff};
  if (x.fwd)
    hipLaunchKernelGGL((add_ln_fwd_v<T, P, NC>), dim3(x.blocks), dim3(kThreads), 0, x.st, (const T*)x.a,
                       (const T*)x.r, (const P*)x.w, (const P*)x.b, dp, x.R, x.eps, (T*)x.out, x.mean, x.rstd);
  else
    hipLaunchKernelGGL((add_ln_bwd_v<T, P, NC>), dim3(x.blocks), dim3(kThreads), 0, x.st, (const T*)x.dy,
                       (const T*)x.a, (const T*)x.r, (const P*)x.w, dp, x.mean, x.rstd, x.R, (T*)x.out, (T*)x.da,
                       x.dw_part, x.db_part, x.dbias_part);
  return (int)hipGetLastError();
}

template <typename T, typename P>
int dispatch_add_ln(const LnArgs& x) {
  const uintptr_t al = (uintptr_t)x.dy | (uintptr_t)x.a | (uintptr_t)x.r | (uintptr_t)x.w | (uintptr_t)x.b |
                       (uintptr_t)x.bias | (uintptr_t)x.out | (uintptr_t)x.da;
  switch (x.H % 256 == 0 && al % 16 == 0 ? x.H / 256 : 0) {  // vectorised paths (BERT-base 768 -> NC 3, large 1024 -> 4)
    case 1: return launch_add_ln_v<T, P, 1>(x);
    case 2: return launch_add_ln_v<T, P, 2>(x);
    case 3: return launch_add_ln_v<T, P, 3>(x);
    case 4: return launch_add_ln_v<T, P, 4>(x);
    default: break;
  }
  const int per = (x.H + 63) / 64;
  if (per <= 4) return launch_add_ln<T, P, 4>(x);
  if (per <= 12) return launch_add_ln<T, P, 12>(x);
  if (per <= 16) return launch_add_ln<T, P, 16>(x);
  return launch_add_ln<T, P, kMaxPer>(x);
}

// (activation dtype, parameter dtype) -> dispatch_add_ln<T, P>; dtype / pdt: 0 fp32, 1 bf16
int dispatch_add_ln_any(int dtype, int pdt, const LnArgs& x) {
  typedef __hip_bfloat16 bf;
  if (dtype && pdt) return dispatch_add_ln<bf, bf>(x);
  if (dtype) return dispatch_add_ln<bf, float>(x);
  if (pdt) return dispatch_add_ln<float, bf>(x);
  return dispatch_add_ln<float, float>(x);
}

uint32_t drop_threshold(float p) {
  if (!(p > 0.f)) return 0;
  const float t = p * 65536.f + 0.5f;
  return t >= 65536.f ? 65536u : (uint32_t)t;
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

// few rows (e.g. the per-tile bias-gradient partials of the fused FFN backward, 32 rows): ONE pass, one thread per
// VW columns summing every row in order (the two-pass partial + reduce launch pair cost ~8 us for ~0.4 MB)
template <typename T, typename P, int VW>
__global__ __launch_bounds__(kThreads) void col_sum_small(const T* __restrict__ x, int M, int N, P* __restrict__ out) {
  const int c0 = (blockIdx.x * kThreads + threadIdx.x) * VW;
  if (c0 >= N) return;
  float a[VW] = {};
  constexpr int U = 8;
  for (int r0 = 0; r0 < M; r0 += U) {
    Pack<T, VW> v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (r0 + u < M) v[u] = *(const Pack<T, VW>*)(x + (size_t)(r0 + u) * N + c0);
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (r0 + u < M)
#pragma unroll
        for (int e = 0; e < VW; ++e) a[e] += ld(&v[u].v[e]);
  }
#pragma unroll
  for (int e = 0; e < VW; ++e) st(out + c0 + e, a[e]);
}

template <typename T, typename P>
int launch_col_sum(const void* x, int M, int N, float* part, void* out, int chunks, hipStream_t st) {
  constexpr int VW = 16 / sizeof(T);
  if (M <= 64 && N % VW == 0 && (uintptr_t)x % 16 == 0) {
    hipLaunchKernelGGL((col_sum_small<T, P, VW>), dim3((N / VW + kThreads - 1) / kThreads), dim3(kThreads), 0, st,
                       (const T*)x, M, N, (P*)out);
    return (int)hipGetLastError();
  }
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

// Deterministic embedding gradient g[V, H] (fp32, zero-filled by the caller) += dy[N, H] scattered by ids[N]. No
// atomics (a captured training step stays bit-reproducible) and no sort (PyTorch's sort + unique-by-key backward
// faults under hipGraph replay on ROCm, see mifx.ops.fused_bert._Embedding). An id's occurrences, in token order, are
// cut into chunks of kEmbCh; the token at rank r % kEmbCh == 0 of its id leads a chunk and sums the chunk's rows in
// order. An id with one chunk is written directly; a heavier one (e.g. the token-type ids: 2048 occurrences each)
// leaves its chunk sums in `part` [N, H] (slot = the leader's token index) and emb_bwd_combine adds them in chunk
// order -- a heavy row is spread over many workgroups instead of one CU walking thousands of rows (which cost ~0.5 ms
// per BERT step).
constexpr int kEmbCh = 64;

// block-wide sum of an int (every thread gets the total)
__device__ __forceinline__ int block_sum_i(int v, int* sred) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sred[w] = v;
  __syncthreads();
  return sred[0] + sred[1] + sred[2] + sred[3];
}

// compact, in token order, the occurrences of id at j >= j0 (ranks rank0, rank0 + 1, ... in that order) whose rank
// satisfies keep(rank), at most cap of them, into list; returns how many (every thread of the block)
template <typename Keep>
__device__ int compact_occ(const long long* __restrict__ ids, int N, long long id, int j0, int rank0, int cap,
                           Keep keep, int* list, int* wc) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  int seen = 0, kept = 0;  // block-uniform
  for (int jb = j0; jb < N && kept < cap; jb += 256) {
    const int j = jb + tid;
    const bool m = j < N && ids[j] == id;
    const unsigned long long b = __ballot(m);
    if (lane == 0) wc[w] = __popcll(b);
    __syncthreads();
    int before = 0;
    for (int i = 0; i < w; ++i) before += wc[i];
    const int tot = wc[0] + wc[1] + wc[2] + wc[3];
    const bool k = m && keep(rank0 + seen + before + __popcll(b & ((1ull << lane) - 1)));
    const unsigned long long bk = __ballot(k);
    __syncthreads();
    if (lane == 0) wc[w] = __popcll(bk);
    __syncthreads();
    int kb = 0;
    for (int i = 0; i < w; ++i) kb += wc[i];
    const int nk = wc[0] + wc[1] + wc[2] + wc[3];
    const int slot = kept + kb + __popcll(bk & ((1ull << lane) - 1));
    if (k && slot < cap) list[slot] = j;
    __syncthreads();
    kept += nk;
    seen += tot;
  }
  return kept < cap ? kept : cap;
}

// rows list[0..m) of dy summed in list order for every column, fp32 -> out (H floats, global)
template <typename T, typename O>
__device__ void sum_rows(const T* __restrict__ dy, int H, const int* list, int m, O* __restrict__ out,
                         float* sacc) {
  constexpr int VEC = 16 / sizeof(T);
  const int tid = threadIdx.x;
  const int NG = H / VEC;
  if (H % VEC == 0 && NG <= 256) {
    // thread -> (column group cg, row slice sl): slice sl sums rows sl, sl + S, ... in order, 8 loads in flight;
    // slices are then added in slice order
    const int S = 256 / NG, cg = tid % NG, sl = tid / NG;
    float a[VEC] = {};
    if (sl < S) {
      for (int k0 = sl; k0 < m; k0 += 8 * S) {
        Pack<T, VEC> v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) {
          const int k = k0 + u * S;
          if (k < m) v[u] = *(const Pack<T, VEC>*)(dy + (size_t)list[k] * H + (size_t)cg * VEC);
        }
#pragma unroll
        for (int u = 0; u < 8; ++u)
          if (k0 + u * S < m)
#pragma unroll
            for (int e = 0; e < VEC; ++e) a[e] += ld(&v[u].v[e]);
      }
    }
    // slice partials through LDS [S][H], summed in slice order by slice 0
    for (int sl2 = 1; sl2 < S; ++sl2) {
      __syncthreads();
      if (sl == sl2)
#pragma unroll
        for (int e = 0; e < VEC; ++e) sacc[cg * VEC + e] = a[e];
      __syncthreads();
      if (sl == 0)
#pragma unroll
        for (int e = 0; e < VEC; ++e) a[e] += sacc[cg * VEC + e];
    }
    if (sl == 0)
#pragma unroll
      for (int e = 0; e < VEC; ++e) st(out + cg * VEC + e, a[e]);
  } else {
    for (int h = tid; h < H; h += 256) {
      float a = 0.f;
      for (int k = 0; k < m; ++k) a += ld(dy + (size_t)list[k] * H + h);
      st(out + h, a);
    }
  }
}

template <typename T, typename G>
__global__ __launch_bounds__(256) void emb_bwd_chunks(const long long* __restrict__ ids, int N, const T* __restrict__ dy,
                                                      int H, long long V, G* __restrict__ g,
                                                      float* __restrict__ part, int* __restrict__ heavy) {
  __shared__ int list[kEmbCh];
  __shared__ int sred[4], wc[4];
  __shared__ float sacc[2048];
  const int n = blockIdx.x, tid = threadIdx.x;
  const long long id = ids[n];
  if (id < 0 || id >= V) {  // (uniform) out-of-range ids contribute nothing
    if (tid == 0) heavy[n] = 0;
    return;
  }
  // rank (earlier occurrences) and count of this id, 8 id loads in flight per thread
  int rl = 0, cl = 0;
  for (int j0 = tid; j0 < N; j0 += 8 * 256) {
    long long v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = j0 + u * 256 < N ? ids[j0 + u * 256] : -1;
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (v[u] == id) {
        ++cl;
        rl += j0 + u * 256 < n ? 1 : 0;
      }
  }
  const int r = block_sum_i(rl, sred);
  const int c = block_sum_i(cl, sred);
  if (tid == 0) heavy[n] = (r == 0 && c > kEmbCh) ? 1 : 0;
  if (r % kEmbCh != 0) return;  // (uniform) not a chunk leader
  const int m = min(kEmbCh, c - r);
  const int got = compact_occ(ids, N, id, n, r, m, [](int) { return true; }, list, wc);
  __syncthreads();
  if (c <= kEmbCh)
    sum_rows<T, G>(dy, H, list, got, g + (size_t)id * H, sacc);
  else
    sum_rows<T, float>(dy, H, list, got, part + (size_t)n * H, sacc);
}

// heavy ids (more than one chunk): the id's first token sums its chunks' partials in chunk order
template <typename G>
__global__ __launch_bounds__(256) void emb_bwd_combine(const long long* __restrict__ ids, int N, int H,
                                                       const float* __restrict__ part, const int* __restrict__ heavy,
                                                       G* __restrict__ g) {
  __shared__ int leaders[32768 / kEmbCh + 1];
  __shared__ int wc[4];
  const int n = blockIdx.x, tid = threadIdx.x;
  if (!heavy[n]) return;  // (uniform)
  const long long id = ids[n];
  const int K = compact_occ(ids, N, id, n, 0, N / kEmbCh + 1, [](int rank) { return rank % kEmbCh == 0; }, leaders,
                            wc);
  __syncthreads();
  for (int h = tid; h < H; h += 256) {
    float a = 0.f;
    for (int k = 0; k < K; ++k) a += part[(size_t)leaders[k] * H + h];
    st(g + (size_t)id * H + h, a);
  }
}

template <typename T, typename G>
void launch_emb(const long long* ids, int N, const void* dy, int H, long long V, void* g, float* part, int* heavy,
                hipStream_t st) {
  hipLaunchKernelGGL((emb_bwd_chunks<T, G>), dim3(N), dim3(256), 0, st, ids, N, (const T*)dy, H, V, (G*)g, part,
                     heavy);
  hipLaunchKernelGGL(emb_bwd_combine<G>, dim3(N), dim3(256), 0, st, ids, N, H, (const float*)part, (const int*)heavy,
                     (G*)g);
}

}  // namespace

extern "C" {

// partial-row count used by add_ln_bwd (fewer, fatter blocks: each wave walks many rows). Rows per wave:
// MIFX_BERT_LN_RPW, default 2 -- measured on the BERT-base step: 5199-5208 seq/s against 5139-5149 at 1 (twice the
// partial rows for the column reduction) and 5192-5195 at 4 (profiles/bert_ln_rpw_ab_r4.txt)
int mifx_bert_ln_blocks(int R) {
  static const int rpw = [] {
    const char* e = getenv("MIFX_BERT_LN_RPW");
    const int v = e ? atoi(e) : 2;
    return v < 1 ? 1 : (v > 16 ? 16 : v);
  }();
  const int need = (R + 4 * rpw - 1) / (4 * rpw);
  return need < 1024 ? (need > 0 ? need : 1) : 1024;
}

// rows of partials for bias_gelu_bwd
int mifx_bert_gelu_chunks(int M) { return M < 16 ? 1 : (M / 16 < 512 ? M / 16 : 512); }

// Fused y = LayerNorm(dropout_p(a [+ bias]) + r) * w + b, and its backward.
// dtype: activations, pdt: gamma/beta/bias (and their gradients): 0 fp32, 1 bf16. bias may be null; p == 0
// disables dropout (rng unused). rng: device int64 [seed, counter]; site distinguishes the call sites of a step.
int mifx_bert_bdaln_fwd2(int dtype, int pdt, const void* a, const void* bias, const void* r, const void* w,
                         const void* b, int R, int H, float eps, float p, const int64_t* rng, int site, long long eoff,
                         void* y, float* mean, float* rstd, hipStream_t st);
int mifx_bert_bdaln_fwd(int dtype, int pdt, const void* a, const void* bias, const void* r, const void* w,
                        const void* b, int R, int H, float eps, float p, const int64_t* rng, int site, void* y,
                        float* mean, float* rstd, hipStream_t st) {
  return mifx_bert_bdaln_fwd2(dtype, pdt, a, bias, r, w, b, R, H, eps, p, rng, site, 0, y, mean, rstd, st);
}
// ... with the dropout mask's element offset eoff (sequence-parallel token shards; % 4 == 0)
int mifx_bert_bdaln_fwd2(int dtype, int pdt, const void* a, const void* bias, const void* r, const void* w,
                         const void* b, int R, int H, float eps, float p, const int64_t* rng, int site, long long eoff,
                         void* y, float* mean, float* rstd, hipStream_t st) {
  if (H <= 0 || H > 64 * kMaxPer || R <= 0 || p < 0.f || p >= 1.f || eoff < 0 || eoff % 4 != 0) return -1;
  if (p > 0.f && rng == nullptr) return -1;
  const int need = (R + 3) / 4;
  LnArgs x{};
  x.fwd = 1;
  x.a = a;
  x.r = r;
  x.w = w;
  x.b = b;
  x.bias = bias;
  x.rng = rng;
  x.site = site;
  x.thr = drop_threshold(p);
  x.scale = 1.f / (1.f - p);
  x.eoff = (unsigned long long)eoff;
  x.R = R;
  x.H = H;
  x.eps = eps;
  x.out = y;
  x.mean = mean;
  x.rstd = rstd;
  x.blocks = need < 4096 ? need : 4096;
  x.st = st;
  return dispatch_add_ln_any(dtype, pdt, x);
}

// backward: dr = dL/dr, da = dL/da (da may alias dr when there is neither bias nor dropout), dw, db and dbias
// ([H], parameter dtype; dbias only with a bias). scratch: part [3, mifx_bert_ln_blocks(R), H] fp32.
int mifx_bert_bdaln_bwd2(int dtype, int pdt, const void* dy, const void* a, const void* bias, const void* r,
                         const void* w, const float* mean, const float* rstd, int R, int H, float p,
                         const int64_t* rng, int site, long long eoff, void* dr, void* da, float* part, void* dw,
                         void* db, void* dbias, hipStream_t st);
int mifx_bert_bdaln_bwd(int dtype, int pdt, const void* dy, const void* a, const void* bias, const void* r,
                        const void* w, const float* mean, const float* rstd, int R, int H, float p, const int64_t* rng,
                        int site, void* dr, void* da, float* part, void* dw, void* db, void* dbias, hipStream_t st) {
  return mifx_bert_bdaln_bwd2(dtype, pdt, dy, a, bias, r, w, mean, rstd, R, H, p, rng, site, 0, dr, da, part, dw, db,
                              dbias, st);
}
int mifx_bert_bdaln_bwd2(int dtype, int pdt, const void* dy, const void* a, const void* bias, const void* r,
                         const void* w, const float* mean, const float* rstd, int R, int H, float p,
                         const int64_t* rng, int site, long long eoff, void* dr, void* da, float* part, void* dw,
                         void* db, void* dbias, hipStream_t st) {
  if (H <= 0 || H > 64 * kMaxPer || R <= 0 || p < 0.f || p >= 1.f || eoff < 0 || eoff % 4 != 0) return -1;
  if (p > 0.f && rng == nullptr) return -1;
  if ((p > 0.f || bias != nullptr) && da == dr) return -1;
  const int blocks = mifx_bert_ln_blocks(R);
  LnArgs x{};
  x.fwd = 0;
  x.dy = dy;
  x.a = a;
  x.r = r;
  x.w = w;
  x.bias = bias;
  x.rng = rng;
  x.site = site;
  x.thr = drop_threshold(p);
  x.scale = 1.f / (1.f - p);
  x.eoff = (unsigned long long)eoff;
  x.R = R;
  x.H = H;
  x.out = dr;
  x.da = da;
  x.mean = (float*)mean;
  x.rstd = (float*)rstd;
  x.dw_part = part;
  x.db_part = part + (size_t)blocks * H;
  x.dbias_part = bias != nullptr ? part + 2 * (size_t)blocks * H : nullptr;
  x.blocks = blocks;
  x.st = st;
  const int rc = dispatch_add_ln_any(dtype, pdt, x);
  if (rc) return rc;
  const dim3 g((H + kRedCols - 1) / kRedCols, bias != nullptr ? 3 : 2);
  typedef __hip_bfloat16 bf;
  if (pdt)
    hipLaunchKernelGGL(col_reduce_y<bf>, g, dim3(kThreads), 0, st, x.dw_part, x.db_part, x.dbias_part, blocks, H,
                       (bf*)dw, (bf*)db, (bf*)dbias);
  else
    hipLaunchKernelGGL(col_reduce_y<float>, g, dim3(kThreads), 0, st, x.dw_part, x.db_part, x.dbias_part, blocks, H,
                       (float*)dw, (float*)db, (float*)dbias);
  return (int)hipGetLastError();
}

// y = keep ? x * 1/(1-p) : 0 over n elements (dtype 0 fp32, 1 bf16); the backward is the same call on dy
int mifx_bert_dropout(int dtype, const void* x, long long n, float p, const int64_t* rng, int site, void* y,
                      hipStream_t st) {
  if (n <= 0 || p <= 0.f || p >= 1.f || rng == nullptr) return -1;
  const long long groups = (n + 3) / 4;
  const long long need = (groups + kThreads - 1) / kThreads;
  const int blocks = (int)(need < 2048 ? need : 2048);
  const uint32_t thr = drop_threshold(p);
  const float scale = 1.f / (1.f - p);
  if (dtype)
    hipLaunchKernelGGL(dropout_k<__hip_bfloat16>, dim3(blocks), dim3(kThreads), 0, st, (const __hip_bfloat16*)x, n,
                       rng, site, thr, scale, (__hip_bfloat16*)y);
  else
    hipLaunchKernelGGL(dropout_k<float>, dim3(blocks), dim3(kThreads), 0, st, (const float*)x, n, rng, site, thr, scale,
                       (float*)y);
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
// g [V, H] (gdtype 0 fp32, 1 bf16; zero-filled by the caller) = the embedding gradient of dy [N, H] (dtype 0 fp32,
// 1 bf16) at int64 ids [N], deterministic (emb_bwd_chunks + emb_bwd_combine; written straight in the weight's dtype,
// no fp32 image + cast). N <= 32768. Scratch: part [N, H] fp32, heavy [N] int.
int mifx_bert_emb_bwd(int dtype, const long long* ids, int N, const void* dy, int H, long long V, void* g, int gdtype,
                      float* part, int* heavy, hipStream_t st) {
  if (N <= 0 || N > 32768 || H <= 0 || V <= 0 || ids == nullptr || dy == nullptr || g == nullptr || part == nullptr ||
      heavy == nullptr)
    return -1;
  typedef __hip_bfloat16 bf;
  if (dtype == 1 && gdtype == 1)
    launch_emb<bf, bf>(ids, N, dy, H, V, g, part, heavy, st);
  else if (dtype == 1)
    launch_emb<bf, float>(ids, N, dy, H, V, g, part, heavy, st);
  else if (gdtype == 1)
    launch_emb<float, bf>(ids, N, dy, H, V, g, part, heavy, st);
  else
    launch_emb<float, float>(ids, N, dy, H, V, g, part, heavy, st);
  return (int)hipGetLastError();
}

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
