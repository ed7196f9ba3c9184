// Differential-privacy kernels for gfx950 (DP-SGD aggregation, PATE noisy-max aggregation).
//
// Reference ops: the DP optimizer's per-microbatch loop
// (`privacy/optimizers/dp_optimizer.py:85-96`: clip each microbatch gradient to global L2 norm C,
// sum, add N(0, (C*sigma)^2), divide by the number of microbatches — `gaussian_query.py:91-111`)
// and PATE's vote aggregation (`research/pate_2017/aggregation.py:60-91`: per-sample bincount of
// teacher labels + Laplace noise + argmax). The reference runs the first as a sequential
// tf.while_loop and the second as a Python double loop; here both are single HBM-streaming passes.
//
//  * dp_row_sumsq: grid (chunks, M) — each block reduces a CH-wide slice of one microbatch row of
//    G[M, ld] (float4 loads, wave64 shuffle tree) into partial[m][chunk]. Deterministic (no atomics).
//  * dp_clip_sum_noise: each block first turns the partials into per-row clip scales
//    min(1, C / ||g_m||) in LDS, then every thread owns 4 consecutive columns: acc = sum_m s_m G[m, p]
//    (M-loop unrolled x4 for memory-level parallelism), plus stddev * N(0,1) from an in-kernel
//    Philox4x32-10 stream keyed by (seed, offset) and indexed by column, divided by `denom`.
//    HBM traffic = 2 reads of G + 1 write of the result: the memory-bound floor for global-norm clipping.
//  * pate_noisy_max: one thread per query sample, votes for C<=kMaxC classes counted in registers,
//    Laplace (mode 0) or Gaussian (mode 1, GNMax) noise from Philox, argmax; optional clean votes.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

constexpr int kThreads = 256;
constexpr int kChunk = 8192;  // columns per dp_row_sumsq block (256 threads x 4 floats x 8 iters)
constexpr int kMaxRows = 4096;
constexpr int kMaxC = 64;

// ---- Philox4x32-10 counter-based RNG --------------------------------------------------------
struct U4 {
  uint32_t x, y, z, w;
};

__device__ __forceinline__ U4 philox(U4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c.x;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c.z;
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    c = U4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

// uniform in (0, 1]: never 0, so log() is finite
__device__ __forceinline__ float u01(uint32_t v) { return ((float)(v >> 8) + 1.0f) * (1.0f / 16777216.0f); }

__device__ __forceinline__ void box_muller(uint32_t a, uint32_t b, float& z0, float& z1) {
  const float r = sqrtf(-2.0f * logf(u01(a)));
  float s, c;
  sincosf(6.283185307179586f * u01(b), &s, &c);
  z0 = r * c;
  z1 = r * s;
}

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

__global__ __launch_bounds__(kThreads) void dp_row_sumsq(const float* __restrict__ G, int ld, int P,
                                                        float* __restrict__ partial, int nchunk) {
  const int m = blockIdx.y, c = blockIdx.x;
  const float* row = G + (size_t)m * ld;
  const int c0 = c * kChunk;
  float acc = 0.f;
  // ld % 4 == 0 (host pads), columns in [P, ld) are zero
  for (int j = c0 + threadIdx.x * 4; j < c0 + kChunk && j < ld; j += kThreads * 4) {
    const float4 v = *reinterpret_cast<const float4*>(row + j);
    acc += v.x * v.x + v.y * v.y + v.z * v.z + v.w * v.w;
  }
  acc = wave_sum(acc);
  __shared__ float ws[kThreads / 64];
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int i = 0; i < kThreads / 64; ++i) t += ws[i];
    partial[(size_t)m * nchunk + c] = t;
  }
  (void)P;
}

__global__ __launch_bounds__(kThreads) void dp_clip_sum_noise(const float* __restrict__ G, int M, int ld, int P,
                                                             const float* __restrict__ partial, int nchunk,
                                                             float clip, float stddev, float inv_denom,
                                                             uint32_t seed_lo, uint32_t seed_hi, uint32_t off_lo,
                                                             uint32_t off_hi, float* __restrict__ out,
                                                             float* __restrict__ norms_out) {
  __shared__ float scale[kMaxRows];
  for (int m = threadIdx.x; m < M; m += kThreads) {
    float s = 0.f;
    for (int c = 0; c < nchunk; ++c) s += partial[(size_t)m * nchunk + c];
    const float nrm = sqrtf(s);
    scale[m] = nrm > clip ? clip / nrm : 1.0f;  // tf.clip_by_global_norm semantics
    if (norms_out != nullptr && blockIdx.x == 0) norms_out[m] = nrm;
  }
  __syncthreads();
  const int q = blockIdx.x * kThreads + threadIdx.x;  // float4 column group
  const int p = q * 4;
  if (p >= ld) return;
  float4 acc = {0.f, 0.f, 0.f, 0.f};
  int m = 0;
  for (; m + 4 <= M; m += 4) {
    float4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = *reinterpret_cast<const float4*>(G + (size_t)(m + u) * ld + p);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const float s = scale[m + u];
      acc.x += s * v[u].x;
      acc.y += s * v[u].y;
      acc.z += s * v[u].z;
      acc.w += s * v[u].w;
    }
  }
  for (; m < M; ++m) {
    const float4 v = *reinterpret_cast<const float4*>(G + (size_t)m * ld + p);
    const float s = scale[m];
    acc.x += s * v.x;
    acc.y += s * v.y;
    acc.z += s * v.z;
    acc.w += s * v.w;
  }
  if (stddev != 0.f) {
    const U4 r = philox(U4{(uint32_t)q, 0u, off_lo, off_hi}, seed_lo, seed_hi);
    float z0, z1, z2, z3;
    box_muller(r.x, r.y, z0, z1);
    box_muller(r.z, r.w, z2, z3);
    acc.x += stddev * z0;
    acc.y += stddev * z1;
    acc.z += stddev * z2;
    acc.w += stddev * z3;
  }
  float vals[4] = {acc.x * inv_denom, acc.y * inv_denom, acc.z * inv_denom, acc.w * inv_denom};
#pragma unroll
  for (int u = 0; u < 4; ++u)
    if (p + u < P) out[p + u] = vals[u];
}

__global__ __launch_bounds__(kThreads) void pate_noisy_max(const int* __restrict__ labels, int T, int N, int C,
                                                          float noise_scale, int mode, uint32_t seed_lo,
                                                          uint32_t seed_hi, uint32_t off_lo, uint32_t off_hi,
                                                          int* __restrict__ out, int* __restrict__ clean) {
  const int i = blockIdx.x * kThreads + threadIdx.x;
  if (i >= N) return;
  int votes[kMaxC];
#pragma unroll
  for (int c = 0; c < kMaxC; ++c) votes[c] = 0;
  for (int t = 0; t < T; ++t) {
    const int l = labels[(size_t)t * N + i];  // coalesced across the wave
#pragma unroll
    for (int c = 0; c < kMaxC; ++c) votes[c] += (c == l);  // register-resident bincount
  }
  float best = -INFINITY;
  int arg = 0;
  for (int c0 = 0; c0 < C; c0 += 4) {
    const U4 r = philox(U4{(uint32_t)i, (uint32_t)c0, off_lo, off_hi}, seed_lo, seed_hi);
    float n[4];
    if (mode == 0) {  // Laplace(0, b): -b sgn(u) ln(1 - 2|u|), u in (-1/2, 1/2]
      const uint32_t rr[4] = {r.x, r.y, r.z, r.w};
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float u = u01(rr[k]) - 0.5f;
        n[k] = -noise_scale * copysignf(1.0f, u) * logf(fmaxf(1.0f - 2.0f * fabsf(u), 1e-30f));
      }
    } else {
      box_muller(r.x, r.y, n[0], n[1]);
      box_muller(r.z, r.w, n[2], n[3]);
#pragma unroll
      for (int k = 0; k < 4; ++k) n[k] *= noise_scale;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int c = c0 + k;
      if (c < C) {
        int v = 0;
#pragma unroll
        for (int cc = 0; cc < kMaxC; ++cc) v = (cc == c) ? votes[cc] : v;
        const float s = (float)v + n[k];
        if (s > best) {
          best = s;
          arg = c;
        }
        if (clean != nullptr) clean[(size_t)i * C + c] = v;
      }
    }
  }
  out[i] = arg;
}

}  // namespace

extern "C" {

int mifx_dp_max_rows() { return kMaxRows; }
int mifx_dp_chunk() { return kChunk; }
int mifx_pate_max_classes() { return kMaxC; }

// G: [M, ld] fp32 (ld % 4 == 0, padding columns zero); partial: [M * ceil(ld / kChunk)] fp32 scratch;
// out: [P]; norms_out (optional): [M] per-row L2 norms before clipping
int mifx_dp_clip_sum_noise(const float* G, int M, int ld, int P, float clip, float stddev, float denom,
                           unsigned long long seed, unsigned long long offset, float* partial, float* out,
                           float* norms_out, hipStream_t st) {
  if (M <= 0 || M > kMaxRows || ld % 4 != 0 || P > ld || P <= 0 || denom == 0.f) return -1;
  const int nchunk = (ld + kChunk - 1) / kChunk;
  hipLaunchKernelGGL(dp_row_sumsq, dim3(nchunk, M), dim3(kThreads), 0, st, G, ld, P, partial, nchunk);
  const int groups = ld / 4;
  const int blocks = (groups + kThreads - 1) / kThreads;
  hipLaunchKernelGGL(dp_clip_sum_noise, dim3(blocks), dim3(kThreads), 0, st, G, M, ld, P, partial, nchunk, clip,
                     stddev, 1.0f / denom, (uint32_t)seed, (uint32_t)(seed >> 32), (uint32_t)offset,
                     (uint32_t)(offset >> 32), out, norms_out);
  return (int)hipGetLastError();
}

// labels: [T, N] int32 teacher predictions; out: [N]; clean (optional): [N, C] vote counts
int mifx_pate_noisy_max(const int* labels, int T, int N, int C, float noise_scale, int mode,
                        unsigned long long seed, unsigned long long offset, int* out, int* clean, hipStream_t st) {
  if (C <= 0 || C > kMaxC || T <= 0 || N <= 0 || (mode != 0 && mode != 1)) return -1;
  hipLaunchKernelGGL(pate_noisy_max, dim3((N + kThreads - 1) / kThreads), dim3(kThreads), 0, st, labels, T, N, C,
                     noise_scale, mode, (uint32_t)seed, (uint32_t)(seed >> 32), (uint32_t)offset,
                     (uint32_t)(offset >> 32), out, clean);
  return (int)hipGetLastError();
}

}  // extern "C"
