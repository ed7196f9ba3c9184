// Fused BatchNorm(train) + ReLU for NHWC activations on gfx950 (ResNet-50 v2, BASELINE config 5).
//
// Profile that motivated it (profiles/archive/resnet50_steady_kernels_r1.md, B=256 bf16 channels_last):
// MIOpen BatchNorm fwd/bwd kernels + the separate ReLU clamp / threshold-backward kernels were
// ~16.5 ms of the 37.4 ms step — more than all convolutions. Pre-activation ResNet applies ReLU
// right after every BatchNorm, so both directions fuse:
//
//   forward : stats pass (per-channel sum / sum of squares)  -> finalize (mean, rstd, running
//             stats, scale = w*rstd, shift = b - mean*scale)  -> apply y = relu(x*scale + shift)
//   backward: reduce pass (g = dy * [x*scale + shift > 0];  sum g, sum g*xhat) -> finalize
//             (dgamma, dbeta, per-channel coefficients) -> apply dx = k1 (g - k2 - xhat k3)
//
// 3 + 5 activation passes instead of MIOpen's 5 + 8 with the unfused ReLU. The activation is
// viewed as [M = N*H*W, C] (channels_last memory): a thread owns 8 consecutive channels (one
// 16-byte bf16 load), C/8 threads cover a row, 256/(C/8) rows are in flight per block. Partial
// sums of the shifted values x - K_c (K_c = the channel's row-0 value, so large means do not cancel)
// are per block (fp32, fixed order) and combined in fp64 in a fixed order by the finalize
// kernels -> bitwise deterministic, no atomics. The ReLU mask is recomputed in backward with the
// same fused multiply-add as forward, so it matches the forward output exactly.
#include <hip/hip_bf16.h>
#include <hip/hip_runtime.h>
#include <stdlib.h>
#include <stdint.h>

namespace {

constexpr int kThreads = 256;
constexpr int kVec = 8;  // channels per thread

template <typename T>
__device__ __forceinline__ float ld(const T* p) {
  return (float)*p;
}
template <>
__device__ __forceinline__ float ld<__hip_bfloat16>(const __hip_bfloat16* p) {
  return __bfloat162float(*p);
}
template <typename T>
__device__ __forceinline__ T cvt(float v) {
  return (T)v;
}
template <>
__device__ __forceinline__ __hip_bfloat16 cvt<__hip_bfloat16>(float v) {
  return __float2bfloat16(v);
}

template <typename T>
struct alignas(sizeof(T) * kVec) Pack {
  T v[kVec];
};
template <typename T>
__device__ __forceinline__ void ldv(const T* p, float* o) {
  const Pack<T> pk = *(const Pack<T>*)p;
#pragma unroll
  for (int i = 0; i < kVec; ++i) o[i] = ld(&pk.v[i]);
}
template <typename T>
__device__ __forceinline__ void stv(T* p, const float* v) {
  Pack<T> pk;
#pragma unroll
  for (int i = 0; i < kVec; ++i) pk.v[i] = cvt<T>(v[i]);
  *(Pack<T>*)p = pk;
}
__device__ __forceinline__ void ld8f(const float* p, float* o) {
  const float4 a = *(const float4*)p, b = *(const float4*)(p + 4);
  o[0] = a.x, o[1] = a.y, o[2] = a.z, o[3] = a.w, o[4] = b.x, o[5] = b.y, o[6] = b.z, o[7] = b.w;
}

// rows [r0, r1) of block b
__device__ __forceinline__ void block_rows(long long M, int& r0, int& r1) {
  r0 = (int)(M * blockIdx.x / gridDim.x);
  r1 = (int)(M * (blockIdx.x + 1) / gridDim.x);
}

// x2 != null: the activation is the residual sum s = x + x2, rounded to T, written to s_out and
// reduced as stored (so the apply pass, which reads s_out, normalises exactly what was measured)
template <typename T>
__device__ __forceinline__ void load_sum(const T* x, const T* x2, T* s_out, size_t off, float* u) {
  ldv(x + off, u);
  if (x2 != nullptr) {
    float v[kVec];
    ldv(x2 + off, v);
    Pack<T> pk;
#pragma unroll
    for (int e = 0; e < kVec; ++e) {
      pk.v[e] = cvt<T>(u[e] + v[e]);
      u[e] = ld(&pk.v[e]);
    }
    *(Pack<T>*)(s_out + off) = pk;
  }
}

template <typename T>
__global__ __launch_bounds__(kThreads) void bn_stats(const T* __restrict__ x, const T* __restrict__ x2,
                                                    T* __restrict__ s_out, long long M, int C,
                                                    float* __restrict__ psum, float* __restrict__ psq,
                                                    float* __restrict__ kout) {
  __shared__ float s1[kThreads * kVec];
  __shared__ float s2[kThreads * kVec];
  const int tpr = C / kVec, rpb = kThreads / tpr;
  const int slice = threadIdx.x / tpr, cg = threadIdx.x % tpr;
  int r0, r1;
  block_rows(M, r0, r1);
  float a[kVec] = {}, q[kVec] = {};
  if (slice < rpb) {
    const size_t c0 = (size_t)cg * kVec;
    // Shifted sums: accumulate d = x - K_c with K_c = row 0's (stored) value of the channel, the same for every
    // block. |mean - K| is of the order of the channel's std, so sum d^2 stays well conditioned in fp32 even
    // when the mean dwarfs the std (e.g. residual sums); finalize recovers mean = K + S/M, var = Q/M - (S/M)^2
    // in fp64. Block 0 hands K to finalize through the mean slot of the stats output.
    float ks[kVec];
    {
      ldv(x + c0, ks);
      if (x2 != nullptr) {
        float v[kVec];
        ldv(x2 + c0, v);
#pragma unroll
        for (int e = 0; e < kVec; ++e) {
          const T t = cvt<T>(ks[e] + v[e]);
          ks[e] = ld(&t);
        }
      }
    }
    if (blockIdx.x == 0 && slice == 0) {
#pragma unroll
      for (int e = 0; e < kVec; ++e) kout[c0 + e] = ks[e];
    }
    int r = r0 + slice;
    // four rows in flight per thread: at 512 workgroups x 256 threads that is ~8 MB of loads in flight,
    // enough to cover HBM latency (two rows ran at ~half the bandwidth of the apply pass)
    for (; r + 3 * rpb < r1; r += 4 * rpb) {
      float u[4][kVec];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        load_sum(x, x2, s_out, (size_t)(r + k * rpb) * C + c0, u[k]);
#pragma unroll
        for (int e = 0; e < kVec; ++e) u[k][e] -= ks[e];
      }
#pragma unroll
      for (int e = 0; e < kVec; ++e) {
        a[e] += (u[0][e] + u[1][e]) + (u[2][e] + u[3][e]);
        q[e] += (u[0][e] * u[0][e] + u[1][e] * u[1][e]) + (u[2][e] * u[2][e] + u[3][e] * u[3][e]);
      }
    }
    for (; r < r1; r += rpb) {
      float u[kVec];
      load_sum(x, x2, s_out, (size_t)r * C + c0, u);
#pragma unroll
      for (int e = 0; e < kVec; ++e) {
        u[e] -= ks[e];
        a[e] += u[e];
        q[e] += u[e] * u[e];
      }
    }
  }
  // LDS image [slice][C] (slice < rpb); every thread of the block owns kVec entries
#pragma unroll
  for (int e = 0; e < kVec; ++e) {
    s1[threadIdx.x * kVec + e] = a[e];
    s2[threadIdx.x * kVec + e] = q[e];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += kThreads) {
    float t1 = 0.f, t2 = 0.f;
    const int g = c / kVec, e = c % kVec;
    for (int s = 0; s < rpb; ++s) {
      t1 += s1[(s * tpr + g) * kVec + e];
      t2 += s2[(s * tpr + g) * kVec + e];
    }
    psum[(size_t)blockIdx.x * C + c] = t1;
    psq[(size_t)blockIdx.x * C + c] = t2;
  }
}

// Partial-sum combine: block = 8 channels x 32 slices; slice s sums partial rows s, s+32, ... in
// fp64, then the 32 slices are added in slice order (fixed order -> deterministic). grid = C / 8.
// The combine is latency-bound (a few hundred partial rows, ~1 MB): 32 slices with four loads in flight
// keep each thread's dependent chain short (was 32 x 8: ~11 us per call, 98 calls per ResNet-50 step).
constexpr int kFinCols = 8, kFinSlices = kThreads / kFinCols;

__device__ __forceinline__ void combine2(const float* __restrict__ p0, const float* __restrict__ p1, int nb, int C,
                                         int c, int sl, double& s0, double& s1) {
  __shared__ double l0[kFinSlices][kFinCols];
  __shared__ double l1[kFinSlices][kFinCols];
  double a = 0.0, b = 0.0;
  if (c < C) {
    int i = sl;
    for (; i + 3 * kFinSlices < nb; i += 4 * kFinSlices) {
      const float* q0 = p0 + (size_t)i * C + c;
      const float* q1 = p1 + (size_t)i * C + c;
      const size_t d = (size_t)kFinSlices * C;
      a += ((double)q0[0] + (double)q0[d]) + ((double)q0[2 * d] + (double)q0[3 * d]);
      b += ((double)q1[0] + (double)q1[d]) + ((double)q1[2 * d] + (double)q1[3 * d]);
    }
    for (; i < nb; i += kFinSlices) {
      a += p0[(size_t)i * C + c];
      b += p1[(size_t)i * C + c];
    }
  }
  l0[sl][threadIdx.x % kFinCols] = a;
  l1[sl][threadIdx.x % kFinCols] = b;
  __syncthreads();
  s0 = s1 = 0.0;
  for (int k = 0; k < kFinSlices; ++k) {
    s0 += l0[k][threadIdx.x % kFinCols];
    s1 += l1[k][threadIdx.x % kFinCols];
  }
}

__global__ __launch_bounds__(kThreads) void bn_finalize_fwd(const float* __restrict__ psum,
                                                           const float* __restrict__ psq, int nb, long long M, int C,
                                                           const float* __restrict__ w, const float* __restrict__ b,
                                                           float eps, float momentum, float* __restrict__ run_mean,
                                                           float* __restrict__ run_var, float* __restrict__ mean_out,
                                                           float* __restrict__ rstd_out, float* __restrict__ scale,
                                                           float* __restrict__ shift) {
  const int sl = threadIdx.x / kFinCols, c = blockIdx.x * kFinCols + threadIdx.x % kFinCols;
  double s, q;
  combine2(psum, psq, nb, C, c, sl, s, q);
  if (sl != 0 || c >= C) return;
  const double dm = s / (double)M;  // mean of the shifted values x - K
  const double mean = (double)mean_out[c] + dm;  // bn_stats left K in mean_out
  double var = q / (double)M - dm * dm;
  var = var > 0.0 ? var : 0.0;
  const float rstd = (float)(1.0 / sqrt(var + (double)eps));
  mean_out[c] = (float)mean;
  rstd_out[c] = rstd;
  const float sc = w[c] * rstd;
  scale[c] = sc;
  shift[c] = b[c] - (float)mean * sc;
  if (run_mean != nullptr) {
    const double unbiased = M > 1 ? var * (double)M / (double)(M - 1) : var;
    run_mean[c] = (1.f - momentum) * run_mean[c] + momentum * (float)mean;
    run_var[c] = (1.f - momentum) * run_var[c] + momentum * (float)unbiased;
  }
}

// Finalize from per-TILE statistics produced by the GEMM that wrote x (csrc/gemm8.hip EPI_STATS / EPI_ADD_STATS: the
// BatchNorm statistics of a 1x1 convolution's output folded into its epilogue, so no statistics pass re-reads x):
// pmean / pm2 [T][C] = each tile's column mean and sum of squared deviations over its rows (nt rows each, M = T nt).
// Two launches: (1) grid (C / 64, G), 1024 threads = 64 channels x 16 tile slices: each thread combines its slice of
// equal-count tiles in fp64 (mean of the means, then M2 = sum M2_t + nt sum (mean_t - mean_s)^2), thread 0 of each
// channel merges the 16 slices by Chan's formula into ws[g] = (count, mean, M2); (2) one thread per channel merges the
// G group results (Chan) and writes the same outputs as bn_finalize_fwd ([mean, rstd, scale, shift], running stats).
__device__ __forceinline__ void chan_merge(double& n, double& mean, double& M2, double nk, double mk, double m2k) {
  if (nk <= 0.0) return;
  const double delta = mk - mean, nn = n + nk;
  mean += delta * nk / nn;
  M2 += m2k + delta * delta * n * nk / nn;
  n = nn;
}

// per-channel merge of the G group records + the outputs of bn_finalize_fwd (shared by both finalize forms)
__device__ __forceinline__ void tiles_final_channel(int c, const double* __restrict__ ws, int G, int C,
                                                    const float* __restrict__ w, const float* __restrict__ b, float eps,
                                                    float momentum, float* __restrict__ run_mean,
                                                    float* __restrict__ run_var, float* __restrict__ mean_out,
                                                    float* __restrict__ rstd_out, float* __restrict__ scale,
                                                    float* __restrict__ shift) {
  double n = 0.0, mean = 0.0, M2 = 0.0;
  int g = 0;
  for (; g + 4 <= G; g += 4) {  // four groups' records loaded before the (ordered) merges
    double r[4][3];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const double* o = ws + ((size_t)(g + u) * C + c) * 3;
      r[u][0] = o[0];
      r[u][1] = o[1];
      r[u][2] = o[2];
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) chan_merge(n, mean, M2, r[u][0], r[u][1], r[u][2]);
  }
  for (; g < G; ++g) {
    const double* o = ws + ((size_t)g * C + c) * 3;
    chan_merge(n, mean, M2, o[0], o[1], o[2]);
  }
  double var = M2 / n;
  var = var > 0.0 ? var : 0.0;
  const float rstd = (float)(1.0 / sqrt(var + (double)eps));
  mean_out[c] = (float)mean;
  rstd_out[c] = rstd;
  const float sc = w[c] * rstd;
  scale[c] = sc;
  shift[c] = b[c] - (float)mean * sc;
  if (run_mean != nullptr) {
    const double unbiased = n > 1 ? M2 / (n - 1) : var;
    run_mean[c] = (1.f - momentum) * run_mean[c] + momentum * (float)mean;
    run_var[c] = (1.f - momentum) * run_var[c] + momentum * (float)unbiased;
  }
}

struct TilesFinal {
  const float* w;
  const float* b;
  float eps, momentum;
  float* run_mean;
  float* run_var;
  float* stats;  // [mean, rstd, scale, shift][C]
};

// LAST = true (opt-in, measured slower: see mifx_bn_relu_fwd_tiles): the group workgroup that arrives last for its
// 64-channel block (an agent-scope ticket per block, reset by that workgroup for the next call) also merges the G
// records of its channels -- the second launch folded into the first (same fixed merge order, same bits); the records
// are published with a device-scope fence first.
template <bool LAST>
__global__ __launch_bounds__(1024) void bn_tiles_partial(const float* __restrict__ pmean, const float* __restrict__ pm2,
                                                        int T, int nt, int C, double* __restrict__ ws, TilesFinal fin,
                                                        unsigned int* __restrict__ ticket) {
  __shared__ double sm[16][64], sq[16][64];
  __shared__ int sk[16];
  __shared__ int s_last;
  const int G = gridDim.y, g = blockIdx.y;
  const int cl = threadIdx.x & 63, sl = threadIdx.x >> 6, c = blockIdx.x * 64 + cl;
  const int gb = (int)((long long)T * g / G), ge = (int)((long long)T * (g + 1) / G);
  const int t0 = gb + (int)((long long)(ge - gb) * sl / 16), t1 = gb + (int)((long long)(ge - gb) * (sl + 1) / 16);
  double mu = 0.0, m2 = 0.0;
  if (c < C && t1 > t0) {
    // one pass, shifted by the first tile's mean (fp64: no cancellation at these sizes), 8 tiles' loads in flight
    // at a time -- the two dependent passes of one load per tile were latency-bound (~12 us per BatchNorm,
    // profiles/resnet_steady_r5m.md)
    const double K0 = (double)pmean[(size_t)t0 * C + c];
    double sd = 0.0, sd2 = 0.0;
    int t = t0;
    for (; t + 8 <= t1; t += 8) {
      float a[8], q[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        a[u] = pmean[(size_t)(t + u) * C + c];
        q[u] = pm2[(size_t)(t + u) * C + c];
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const double d = (double)a[u] - K0;
        sd += d;
        sd2 += d * d;
        m2 += (double)q[u];
      }
    }
    for (; t < t1; ++t) {
      const double d = (double)pmean[(size_t)t * C + c] - K0;
      sd += d;
      sd2 += d * d;
      m2 += (double)pm2[(size_t)t * C + c];
    }
    const double k = (double)(t1 - t0);
    mu = K0 + sd / k;
    const double d2 = sd2 - sd * sd / k;
    m2 += (double)nt * (d2 > 0.0 ? d2 : 0.0);
  }
  sm[sl][cl] = mu;
  sq[sl][cl] = m2;
  if (cl == 0) sk[sl] = t1 - t0;
  __syncthreads();
  if (sl == 0 && c < C) {
    double n = 0.0, mean = 0.0, M2 = 0.0;
    for (int k = 0; k < 16; ++k) chan_merge(n, mean, M2, (double)sk[k] * nt, sm[k][cl], sq[k][cl]);
    double* o = ws + ((size_t)g * C + c) * 3;
    o[0] = n;
    o[1] = mean;
    o[2] = M2;
  }
  if constexpr (LAST) {
    __threadfence();  // this group's records visible to the workgroup of any XCD that merges them
    __syncthreads();
    if (threadIdx.x == 0) {
      const unsigned int old =
          __hip_atomic_fetch_add(ticket + blockIdx.x, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
      s_last = old == (unsigned int)G - 1;
      if (s_last) __hip_atomic_store(ticket + blockIdx.x, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    __syncthreads();
    if (!s_last) return;
    __threadfence();  // the other groups' records, published before their tickets
    if (sl == 0 && c < C)
      tiles_final_channel(c, ws, G, C, fin.w, fin.b, fin.eps, fin.momentum, fin.run_mean, fin.run_var, fin.stats,
                          fin.stats + C, fin.stats + 2 * C, fin.stats + 3 * C);
  }
}

__global__ __launch_bounds__(256) void bn_tiles_final(const double* __restrict__ ws, int G, int C,
                                                     const float* __restrict__ w, const float* __restrict__ b,
                                                     float eps, float momentum, float* __restrict__ run_mean,
                                                     float* __restrict__ run_var, float* __restrict__ mean_out,
                                                     float* __restrict__ rstd_out, float* __restrict__ scale,
                                                     float* __restrict__ shift) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  if (c >= C) return;
  tiles_final_channel(c, ws, G, C, w, b, eps, momentum, run_mean, run_var, mean_out, rstd_out, scale, shift);
}

// per-64-channel-block arrival tickets of the one-launch finalize (zero at load; each call's last arriver resets its
// block's ticket; calls on one stream are ordered, and a process issues them on one stream)
__device__ unsigned int g_tiles_ticket[64];

// groups of tiles of the first finalize launch: ~12 tiles per thread (16 slices per group)
int tile_groups(int T) { return T / 192 < 1 ? 1 : (T / 192 > 32 ? 32 : T / 192); }

// y = relu(x * scale + shift) (relu optional). Same [row slice x channel group] layout as the
// reductions: a thread keeps its 8 channels' scale/shift in registers across all its rows.
// x2 != null (inference over a residual sum): s = x + x2 rounded to T is written to s_out and normalised, as the
// training forward's load_sum does
template <typename T>
__global__ __launch_bounds__(kThreads) void bn_apply(const T* __restrict__ x, const T* __restrict__ x2,
                                                    T* __restrict__ s_out, long long M, int C,
                                                    const float* __restrict__ scale, const float* __restrict__ shift,
                                                    int relu, T* __restrict__ y) {
  const int tpr = C / kVec, rpb = kThreads / tpr;
  const int slice = threadIdx.x / tpr, cg = threadIdx.x % tpr;
  if (slice >= rpb) return;
  int r0, r1;
  block_rows(M, r0, r1);
  const int c0 = cg * kVec;
  float sc[kVec], sh[kVec];
  ld8f(scale + c0, sc);
  ld8f(shift + c0, sh);
  int r = r0 + slice;
  if (x2 == nullptr) {  // four rows' 16-byte loads in flight per thread before any store (the pass is latency-bound
                        // at one load per thread: ~5 TB/s)
    for (; r + 3 * rpb < r1; r += 4 * rpb) {
      float u[4][kVec];
#pragma unroll
      for (int k = 0; k < 4; ++k) ldv(x + (size_t)(r + k * rpb) * C + c0, u[k]);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
#pragma unroll
        for (int e = 0; e < kVec; ++e) {
          const float t = fmaf(u[k][e], sc[e], sh[e]);
          u[k][e] = relu ? fmaxf(t, 0.f) : t;
        }
        stv(y + (size_t)(r + k * rpb) * C + c0, u[k]);
      }
    }
  }
  for (; r < r1; r += rpb) {
    float u[kVec];
    load_sum(x, x2, s_out, (size_t)r * C + c0, u);
#pragma unroll
    for (int e = 0; e < kVec; ++e) {
      const float t = fmaf(u[e], sc[e], sh[e]);
      u[e] = relu ? fmaxf(t, 0.f) : t;
    }
    stv(y + (size_t)r * C + c0, u);
  }
}

// backward reduction: g = dy * mask; sums of g and g * xhat per channel
template <typename T>
__global__ __launch_bounds__(kThreads) void bn_bwd_reduce(const T* __restrict__ dy, const T* __restrict__ x, long long M,
                                                         int C, const float* __restrict__ scale,
                                                         const float* __restrict__ shift,
                                                         const float* __restrict__ mean,
                                                         const float* __restrict__ rstd, int relu,
                                                         float* __restrict__ pg, float* __restrict__ pgx) {
  __shared__ float s1[kThreads * kVec];
  __shared__ float s2[kThreads * kVec];
  const int tpr = C / kVec, rpb = kThreads / tpr;
  const int slice = threadIdx.x / tpr, cg = threadIdx.x % tpr;
  int r0, r1;
  block_rows(M, r0, r1);
  float a[kVec] = {}, q[kVec] = {};
  if (slice < rpb) {
    const int c0 = cg * kVec;
    float sc[kVec], sh[kVec], mu[kVec], rs[kVec];
    ld8f(scale + c0, sc);
    ld8f(shift + c0, sh);
    ld8f(mean + c0, mu);
    ld8f(rstd + c0, rs);
    int r = r0 + slice;
    for (; r + 3 * rpb < r1; r += 4 * rpb) {  // four rows (eight 16-B loads) in flight per thread
      float d[4][kVec], u[4][kVec];
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        ldv(dy + (size_t)(r + k * rpb) * C + c0, d[k]);
        ldv(x + (size_t)(r + k * rpb) * C + c0, u[k]);
      }
#pragma unroll
      for (int k = 0; k < 4; ++k)
#pragma unroll
        for (int e = 0; e < kVec; ++e) {
          const float g = (relu && fmaf(u[k][e], sc[e], sh[e]) <= 0.f) ? 0.f : d[k][e];
          a[e] += g;
          q[e] += g * ((u[k][e] - mu[e]) * rs[e]);
        }
    }
    for (; r < r1; r += rpb) {
      float d[kVec], u[kVec];
      ldv(dy + (size_t)r * C + c0, d);
      ldv(x + (size_t)r * C + c0, u);
#pragma unroll
      for (int e = 0; e < kVec; ++e) {
        const float g = (relu && fmaf(u[e], sc[e], sh[e]) <= 0.f) ? 0.f : d[e];
        a[e] += g;
        q[e] += g * ((u[e] - mu[e]) * rs[e]);
      }
    }
  }
#pragma unroll
  for (int e = 0; e < kVec; ++e) {
    s1[threadIdx.x * kVec + e] = a[e];
    s2[threadIdx.x * kVec + e] = q[e];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += kThreads) {
    float t1 = 0.f, t2 = 0.f;
    const int g = c / kVec, e = c % kVec;
    for (int s = 0; s < rpb; ++s) {
      t1 += s1[(s * tpr + g) * kVec + e];
      t2 += s2[(s * tpr + g) * kVec + e];
    }
    pg[(size_t)blockIdx.x * C + c] = t1;
    pgx[(size_t)blockIdx.x * C + c] = t2;
  }
}

// dbeta = sum g, dgamma = sum g xhat. dx = w rstd (g - dbeta/M - xhat dgamma/M) is folded into
// dx = A g + B x + Cc per channel (A = w rstd, B = -A rstd dgamma/M, Cc = -A dbeta/M - B mean).
__global__ __launch_bounds__(kThreads) void bn_finalize_bwd(const float* __restrict__ pg, const float* __restrict__ pgx,
                                                           int nb, long long M, int C, const float* __restrict__ w,
                                                           const float* __restrict__ mean,
                                                           const float* __restrict__ rstd,
                                                           float* __restrict__ dgamma, float* __restrict__ dbeta,
                                                           float* __restrict__ k) {
  const int sl = threadIdx.x / kFinCols, c = blockIdx.x * kFinCols + threadIdx.x % kFinCols;
  double s, q;
  combine2(pg, pgx, nb, C, c, sl, s, q);
  if (sl != 0 || c >= C) return;
  dbeta[c] = (float)s;
  dgamma[c] = (float)q;
  const double A = (double)w[c] * rstd[c];
  const double B = -A * rstd[c] * (q / (double)M);
  k[c] = (float)A;
  k[C + c] = (float)B;
  k[2 * C + c] = (float)(-A * (s / (double)M) - B * mean[c]);
}

template <typename T>
__global__ __launch_bounds__(kThreads) void bn_bwd_apply(const T* __restrict__ dy, const T* __restrict__ x,
                                                        long long M, int C, const float* __restrict__ scale,
                                                        const float* __restrict__ shift, const float* __restrict__ k,
                                                        int relu, const T* __restrict__ dres, T* __restrict__ dx,
                                                        T* __restrict__ act) {
  const int tpr = C / kVec, rpb = kThreads / tpr;
  const int slice = threadIdx.x / tpr, cg = threadIdx.x % tpr;
  if (slice >= rpb) return;
  int r0, r1;
  block_rows(M, r0, r1);
  const int c0 = cg * kVec;
  float sc[kVec], sh[kVec], A[kVec], B[kVec], Cc[kVec];
  ld8f(scale + c0, sc);
  ld8f(shift + c0, sh);
  ld8f(k + c0, A);
  ld8f(k + C + c0, B);
  ld8f(k + 2 * C + c0, Cc);
  int r = r0 + slice;
  for (; r + 3 * rpb < r1; r += 4 * rpb) {  // four rows in flight (8-12 16-byte loads per thread)
    float d[4][kVec], u[4][kVec], rr[4][kVec];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      ldv(dy + (size_t)(r + k * rpb) * C + c0, d[k]);
      ldv(x + (size_t)(r + k * rpb) * C + c0, u[k]);
      if (dres != nullptr) ldv(dres + (size_t)(r + k * rpb) * C + c0, rr[k]);
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      float a[kVec];
#pragma unroll
      for (int e = 0; e < kVec; ++e) {
        const float t = fmaf(u[k][e], sc[e], sh[e]);
        a[e] = relu ? fmaxf(t, 0.f) : t;
        const float g = (relu && t <= 0.f) ? 0.f : d[k][e];
        d[k][e] = fmaf(A[e], g, fmaf(B[e], u[k][e], Cc[e]));
        if (dres != nullptr) d[k][e] += rr[k][e];
      }
      stv(dx + (size_t)(r + k * rpb) * C + c0, d[k]);
      if (act != nullptr) stv(act + (size_t)(r + k * rpb) * C + c0, a);  // the forward's activation, re-derived
    }
  }
  for (; r < r1; r += rpb) {
    float d[kVec], u[kVec];
    ldv(dy + (size_t)r * C + c0, d);
    ldv(x + (size_t)r * C + c0, u);
    float a[kVec];
#pragma unroll
    for (int e = 0; e < kVec; ++e) {
      const float t = fmaf(u[e], sc[e], sh[e]);
      a[e] = relu ? fmaxf(t, 0.f) : t;
      const float g = (relu && t <= 0.f) ? 0.f : d[e];
      d[e] = fmaf(A[e], g, fmaf(B[e], u[e], Cc[e]));
    }
    if (dres != nullptr) {  // gradient arriving through the identity shortcut, accumulated here
      float rr[kVec];
      ldv(dres + (size_t)r * C + c0, rr);
#pragma unroll
      for (int e = 0; e < kVec; ++e) d[e] += rr[e];
    }
    stv(dx + (size_t)r * C + c0, d);
    if (act != nullptr) stv(act + (size_t)r * C + c0, a);
  }
}

// workgroups of the statistics / backward-reduction passes (>= 16 rows per thread, at most MIFX_BN_BLOCKS_CAP,
// default 512: 1024 and 2048 measured equal or slower on the ResNet-50 step, profiles/resnet_bn_cap_ab_r4.txt --
// the passes already stream at 4.5-6 TB/s, and more workgroups only add partial rows to combine)
int blocks_cap() {
  static const int cap = [] {
    const char* e = getenv("MIFX_BN_BLOCKS_CAP");
    const int v = e ? atoi(e) : 512;
    return v < 64 ? 64 : (v > 8192 ? 8192 : v);
  }();
  return cap;
}
int blocks_for(long long M, int C) {
  const int rpb = kThreads / (C / kVec);
  long long nb = (M + (long long)rpb * 16 - 1) / ((long long)rpb * 16);  // >= 16 rows per thread
  if (nb > blocks_cap()) nb = blocks_cap();
  return nb < 1 ? 1 : (int)nb;
}

int apply_rows() {  // rows per thread of the apply passes (MIFX_BN_APPLY_ROWS, default 8: A/B)
  static const int v = [] {
    const char* e = getenv("MIFX_BN_APPLY_ROWS");
    const int r = e ? atoi(e) : 8;
    return r < 1 ? 1 : (r > 64 ? 64 : r);
  }();
  return v;
}
int apply_blocks(long long M, int C) {  // ~8 rows per thread, params loaded once per thread
  const int rpb = kThreads / (C / kVec), rpt = apply_rows();
  long long g = (M + (long long)rpb * rpt - 1) / ((long long)rpb * rpt);
  if (g > 16384) g = 16384;
  return g < 1 ? 1 : (int)g;
}

bool shape_ok(long long M, int C) { return M > 0 && C >= kVec && C % kVec == 0 && C / kVec <= kThreads; }

}  // namespace

extern "C" {

// scratch rows (blocks) used by the reductions for [M, C]
int mifx_bn_blocks(long long M, int C) { return shape_ok(M, C) ? blocks_for(M, C) : -1; }

// dtype 1 = bf16, 0 = fp32. stats6 = [mean, rstd, scale, shift] (4*C floats) out;
// part = scratch [2, blocks, C]; run_mean / run_var may be null (no running-stat update).
// x2 / sum_out non-null: normalise s = x + x2 (written to sum_out) -- residual add fused in
int mifx_bn_relu_fwd(int dtype, const void* x, const void* x2, void* sum_out, long long M, int C, const float* w,
                     const float* b, float eps, float momentum, float* run_mean, float* run_var, int relu, float* part,
                     float* stats, void* y, hipStream_t st) {
  if (!shape_ok(M, C)) return -1;
  const int nb = blocks_for(M, C);
  if (dtype)
    hipLaunchKernelGGL(bn_stats<__hip_bfloat16>, dim3(nb), dim3(kThreads), 0, st, (const __hip_bfloat16*)x,
                       (const __hip_bfloat16*)x2, (__hip_bfloat16*)sum_out, M, C, part, part + (size_t)nb * C, stats);
  else
    hipLaunchKernelGGL(bn_stats<float>, dim3(nb), dim3(kThreads), 0, st, (const float*)x, (const float*)x2,
                       (float*)sum_out, M, C, part, part + (size_t)nb * C, stats);
  const void* xa = x2 != nullptr ? (const void*)sum_out : x;  // apply normalises the stored sum
  hipLaunchKernelGGL(bn_finalize_fwd, dim3((C + kFinCols - 1) / kFinCols), dim3(kThreads), 0, st, part,
                     part + (size_t)nb * C, nb, M, C, w, b, eps, momentum, run_mean, run_var, stats, stats + C,
                     stats + 2 * C, stats + 3 * C);
  if (dtype)
    hipLaunchKernelGGL(bn_apply<__hip_bfloat16>, dim3(apply_blocks(M, C)), dim3(kThreads), 0, st,
                       (const __hip_bfloat16*)xa, (const __hip_bfloat16*)nullptr, (__hip_bfloat16*)nullptr, M, C, stats + 2 * C, stats + 3 * C, relu, (__hip_bfloat16*)y);
  else
    hipLaunchKernelGGL(bn_apply<float>, dim3(apply_blocks(M, C)), dim3(kThreads), 0, st, (const float*)xa,
                       (const float*)nullptr, (float*)nullptr, M, C,
                       stats + 2 * C, stats + 3 * C, relu, (float*)y);
  return (int)hipGetLastError();
}

// Training forward from per-tile statistics (see bn_tiles_partial): part = [2][T][C] (tile means, tile M2), nt rows
// per tile, x [M = T nt, C]; ws = fp64 scratch of mifx_bn_tiles_ws(T, C) doubles; writes stats = [mean, rstd, scale,
// shift] and y = relu(x * scale + shift) (y null: the statistics only).
int mifx_bn_tiles_ws(int T, int C) { return tile_groups(T) * C * 3; }

int mifx_bn_relu_fwd_tiles(int dtype, const void* x, long long M, int C, const float* part, int T, int nt,
                           const float* w, const float* b, float eps, float momentum, float* run_mean, float* run_var,
                           int relu, float* stats, double* ws, void* y, hipStream_t st) {
  if (!shape_ok(M, C) || T <= 0 || nt <= 0 || (long long)T * nt != M || part == nullptr || ws == nullptr) return -1;
  const int G = tile_groups(T);
  const TilesFinal fin{w, b, eps, momentum, run_mean, run_var, stats};
  // MIFX_BN_TILES_ONE_LAUNCH=1: the finalize folded into the partial kernel (last-arriving group merges) -- measured
  // SLOWER in the ResNet-50 step (20.97 vs 20.61 ms, profiles/resnet_bn_one_launch_ab_r6.jsonl): its device-scope
  // fences write back and invalidate the XCD's L2, which the BatchNorm apply pass right after then re-reads from HBM
  static const bool one = getenv("MIFX_BN_TILES_ONE_LAUNCH") != nullptr;
  if (!one || (C + 63) / 64 > 64) {
    hipLaunchKernelGGL(bn_tiles_partial<false>, dim3((C + 63) / 64, G), dim3(1024), 0, st, part, part + (size_t)T * C,
                       T, nt, C, ws, fin, (unsigned int*)nullptr);
    hipLaunchKernelGGL(bn_tiles_final, dim3((C + 255) / 256), dim3(256), 0, st, ws, G, C, w, b, eps, momentum,
                       run_mean, run_var, stats, stats + C, stats + 2 * C, stats + 3 * C);
  } else {
    static unsigned int* ticket = nullptr;
    if (ticket == nullptr && hipGetSymbolAddress((void**)&ticket, HIP_SYMBOL(g_tiles_ticket)) != hipSuccess) return -1;
    hipLaunchKernelGGL(bn_tiles_partial<true>, dim3((C + 63) / 64, G), dim3(1024), 0, st, part, part + (size_t)T * C,
                       T, nt, C, ws, fin, ticket);
  }
  if (y == nullptr) return (int)hipGetLastError();  // statistics only: the consumer GEMM applies (gemm8 AX operands)
  if (dtype)
    hipLaunchKernelGGL(bn_apply<__hip_bfloat16>, dim3(apply_blocks(M, C)), dim3(kThreads), 0, st,
                       (const __hip_bfloat16*)x, (const __hip_bfloat16*)nullptr, (__hip_bfloat16*)nullptr, M, C,
                       stats + 2 * C, stats + 3 * C, relu, (__hip_bfloat16*)y);
  else
    hipLaunchKernelGGL(bn_apply<float>, dim3(apply_blocks(M, C)), dim3(kThreads), 0, st, (const float*)x,
                       (const float*)nullptr, (float*)nullptr, M, C, stats + 2 * C, stats + 3 * C, relu, (float*)y);
  return (int)hipGetLastError();
}

// Backward from per-tile reductions computed by the GEMM that produced dy (csrc/gemm8.hip EPI_BNBWD): pg / pgx [T][C]
// = per-tile sum g and sum g xhat; then the same finalize and apply as mifx_bn_relu_bwd (no reduction pass over dy, x).
// act non-null: also writes the forward's activation relu(x scale + shift) (for a consumer convolution whose forward
// applied the BatchNorm in its GEMM and whose weight gradient needs the activation: mifx.ops.conv1x1.bn_conv1x1)
int mifx_bn_relu_bwd_tiles(int dtype, const void* dy, const void* x, const void* dres, long long M, int C,
                           const float* w, const float* stats, int relu, const float* pg, const float* pgx, int T,
                           float* kbuf, void* dx, float* dgamma, float* dbeta, void* act, hipStream_t st) {
  if (!shape_ok(M, C) || T <= 0 || pg == nullptr || pgx == nullptr) return -1;
  const float *mean = stats, *rstd = stats + C, *scale = stats + 2 * C, *shift = stats + 3 * C;
  hipLaunchKernelGGL(bn_finalize_bwd, dim3((C + kFinCols - 1) / kFinCols), dim3(kThreads), 0, st, pg, pgx, T, M, C, w,
                     mean, rstd, dgamma, dbeta, kbuf);
  if (dtype)
    hipLaunchKernelGGL(bn_bwd_apply<__hip_bfloat16>, dim3(apply_blocks(M, C)), dim3(kThreads), 0, st,
                       (const __hip_bfloat16*)dy, (const __hip_bfloat16*)x, M, C, scale, shift, kbuf, relu,
                       (const __hip_bfloat16*)dres, (__hip_bfloat16*)dx, (__hip_bfloat16*)act);
  else
    hipLaunchKernelGGL(bn_bwd_apply<float>, dim3(apply_blocks(M, C)), dim3(kThreads), 0, st, (const float*)dy,
                       (const float*)x, M, C, scale, shift, kbuf, relu, (const float*)dres, (float*)dx, (float*)act);
  return (int)hipGetLastError();
}

// eval / inference: y = relu(x * scale + shift) with precomputed per-channel scale / shift
// inference BatchNorm (+ ReLU) with precomputed per-channel scale / shift; x2 / s_out non-null: over the residual
// sum s = x + x2, also written to s_out (the identity shortcut of the next block reads it)
int mifx_bn_add_relu_apply(int dtype, const void* x, const void* x2, void* s_out, long long M, int C,
                           const float* scale, const float* shift, int relu, void* y, hipStream_t st) {
  if (!shape_ok(M, C) || (x2 != nullptr) != (s_out != nullptr)) return -1;
  if (dtype)
    hipLaunchKernelGGL(bn_apply<__hip_bfloat16>, dim3(apply_blocks(M, C)), dim3(kThreads), 0, st,
                       (const __hip_bfloat16*)x, (const __hip_bfloat16*)x2, (__hip_bfloat16*)s_out, M, C, scale, shift,
                       relu, (__hip_bfloat16*)y);
  else
    hipLaunchKernelGGL(bn_apply<float>, dim3(apply_blocks(M, C)), dim3(kThreads), 0, st, (const float*)x,
                       (const float*)x2, (float*)s_out, M, C, scale, shift, relu, (float*)y);
  return (int)hipGetLastError();
}

int mifx_bn_relu_apply(int dtype, const void* x, long long M, int C, const float* scale, const float* shift, int relu,
                       void* y, hipStream_t st) {
  return mifx_bn_add_relu_apply(dtype, x, nullptr, nullptr, M, C, scale, shift, relu, y, st);
}

// backward: stats = forward's [mean, rstd, scale, shift]; part = scratch [2, blocks, C];
// kbuf = scratch [3, C]; outputs dx, dgamma, dbeta
// dres non-null: dx += dres (gradient of the residual sum through its identity-shortcut use)
int mifx_bn_relu_bwd(int dtype, const void* dy, const void* x, const void* dres, long long M, int C, const float* w,
                     const float* stats, int relu, float* part, float* kbuf, void* dx, float* dgamma, float* dbeta,
                     hipStream_t st) {
  if (!shape_ok(M, C)) return -1;
  const int nb = blocks_for(M, C);
  const float *mean = stats, *rstd = stats + C, *scale = stats + 2 * C, *shift = stats + 3 * C;
  if (dtype)
    hipLaunchKernelGGL(bn_bwd_reduce<__hip_bfloat16>, dim3(nb), dim3(kThreads), 0, st, (const __hip_bfloat16*)dy,
                       (const __hip_bfloat16*)x, M, C, scale, shift, mean, rstd, relu, part, part + (size_t)nb * C);
  else
    hipLaunchKernelGGL(bn_bwd_reduce<float>, dim3(nb), dim3(kThreads), 0, st, (const float*)dy, (const float*)x, M, C,
                       scale, shift, mean, rstd, relu, part, part + (size_t)nb * C);
  hipLaunchKernelGGL(bn_finalize_bwd, dim3((C + kFinCols - 1) / kFinCols), dim3(kThreads), 0, st, part,
                     part + (size_t)nb * C, nb, M, C, w, mean, rstd, dgamma, dbeta, kbuf);
  if (dtype)
    hipLaunchKernelGGL(bn_bwd_apply<__hip_bfloat16>, dim3(apply_blocks(M, C)), dim3(kThreads), 0, st,
                       (const __hip_bfloat16*)dy, (const __hip_bfloat16*)x, M, C, scale, shift, kbuf, relu,
                       (const __hip_bfloat16*)dres, (__hip_bfloat16*)dx, (__hip_bfloat16*)nullptr);
  else
    hipLaunchKernelGGL(bn_bwd_apply<float>, dim3(apply_blocks(M, C)), dim3(kThreads), 0, st, (const float*)dy,
                       (const float*)x, M, C, scale, shift, kbuf, relu, (const float*)dres, (float*)dx,
                       (float*)nullptr);
  return (int)hipGetLastError();
}

}  // extern "C"
