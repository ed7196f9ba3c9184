// Small-CNN training kernels for gfx950: the PATE / DP-SGD / Fashion-MNIST model family.
//
// Reference ops:
//  * softmax cross-entropy head (`research/pate_2017/deep_cnn.py:343-348`,
//    `tutorials/mnist_dpsgd_tutorial.py:63-66`): one pass produces the per-row loss AND dlogits
//    (softmax - onehot), so the backward of the head is free;
//  * tf.nn.lrn(depth_radius=4, bias=1, alpha=0.001/9, beta=0.75) of PATE `deep_cnn.inference`
//    (`deep_cnn.py:115,141`) on NHWC activations: the 9-channel window is summed from an LDS image of
//    the row, forward saves the normaliser N so backward needs one LDS pass as well;
//  * SGD + exponential-moving-average shadow update (`deep_cnn.py:397-422`, decay 0.9999 with TF's
//    num_updates rule) fused into one multi-tensor sweep: w -= lr*g; s += (1-decay)*(w - s).
//
// Row-parallel layout: the head uses a 16-lane (C <= 256) or 64-lane group per row with
// shuffle reductions (C=10 classes -> 4 rows per wave); LRN stages whole NHWC rows (C channels
// contiguous) in LDS, 256 threads per block, ceil(1024/C) rows per block.
#include <hip/hip_bf16.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

template <typename T>
__device__ __forceinline__ float ldf(const T* p) {
  return (float)*p;
}
template <>
__device__ __forceinline__ float ldf<__hip_bfloat16>(const __hip_bfloat16* p) {
  return __bfloat162float(*p);
}
template <typename T>
__device__ __forceinline__ T stf(float v) {
  return (T)v;
}
template <>
__device__ __forceinline__ __hip_bfloat16 stf<__hip_bfloat16>(float v) {
  return __float2bfloat16(v);
}

// ------------------------------------------------------------------ softmax cross-entropy
// labels outside [0, C) (e.g. ignore_index -100) contribute loss 0 and gradient 0.
template <typename T, int G>
__global__ __launch_bounds__(256) void softmax_xent(const T* __restrict__ logits, const long long* __restrict__ labels,
                                                    int B, int C, float* __restrict__ loss, T* __restrict__ dlogits) {
  const int lane = threadIdx.x % G;
  const int row = (blockIdx.x * 256 + threadIdx.x) / G;
  const bool live = row < B;  // every lane stays for the shuffles
  const T* x = logits + (size_t)(live ? row : 0) * C;
  float mx = -INFINITY;
  for (int c = lane; c < C; c += G) mx = fmaxf(mx, ldf(x + c));
#pragma unroll
  for (int o = G / 2; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o, G));
  float se = 0.f;
  for (int c = lane; c < C; c += G) se += __expf(ldf(x + c) - mx);
#pragma unroll
  for (int o = G / 2; o > 0; o >>= 1) se += __shfl_xor(se, o, G);
  if (!live) return;
  const long long y = labels[row];
  const bool valid = y >= 0 && y < C;
  const float inv = 1.f / se;
  T* d = dlogits + (size_t)row * C;
  for (int c = lane; c < C; c += G) {
    const float p = __expf(ldf(x + c) - mx) * inv;
    d[c] = stf<T>(valid ? p - (c == y ? 1.f : 0.f) : 0.f);
  }
  if (lane == 0) loss[row] = valid ? (logf(se) + mx - ldf(x + y)) : 0.f;
}

// ------------------------------------------------------------------------------------ LRN
// y = x * N^-beta,  N = bias + alpha * sum_{|j-c|<=r} x_j^2   (zero outside [0, C))
template <typename T>
__global__ __launch_bounds__(256) void lrn_fwd(const T* __restrict__ x, long long M, int C, int r, float bias,
                                               float alpha, float beta, T* __restrict__ y, float* __restrict__ nrm) {
  extern __shared__ float sq[];
  const int R = (1024 + C - 1) / C;
  const long long m0 = (long long)blockIdx.x * R;
  const int rows = (int)min((long long)R, M - m0);
  const int n = rows * C;
  const T* xb = x + m0 * C;
  for (int i = threadIdx.x; i < n; i += 256) {
    const float v = ldf(xb + i);
    sq[i] = v * v;
  }
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += 256) {
    const int c = i % C, base = i - c;
    const int lo = max(c - r, 0), hi = min(c + r, C - 1);
    float s = 0.f;
    for (int j = lo; j <= hi; ++j) s += sq[base + j];
    const float N = bias + alpha * s;
    nrm[m0 * C + i] = N;
    y[m0 * C + i] = stf<T>(ldf(xb + i) * __powf(N, -beta));
  }
}

// dx = dy * N^-beta - 2*alpha*beta * x * sum_{|j-c|<=r} dy_j x_j N_j^(-beta-1)
template <typename T>
__global__ __launch_bounds__(256) void lrn_bwd(const T* __restrict__ x, const T* __restrict__ dy,
                                               const float* __restrict__ nrm, long long M, int C, int r, float alpha,
                                               float beta, T* __restrict__ dx) {
  extern __shared__ float t[];
  const int R = (1024 + C - 1) / C;
  const long long m0 = (long long)blockIdx.x * R;
  const int rows = (int)min((long long)R, M - m0);
  const int n = rows * C;
  const size_t o = (size_t)m0 * C;
  for (int i = threadIdx.x; i < n; i += 256) {
    const float N = nrm[o + i];
    t[i] = ldf(dy + o + i) * ldf(x + o + i) * __powf(N, -beta - 1.f);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < n; i += 256) {
    const int c = i % C, base = i - c;
    const int lo = max(c - r, 0), hi = min(c + r, C - 1);
    float s = 0.f;
    for (int j = lo; j <= hi; ++j) s += t[base + j];
    const float N = nrm[o + i];
    dx[o + i] = stf<T>(ldf(dy + o + i) * __powf(N, -beta) - 2.f * alpha * beta * ldf(x + o + i) * s);
  }
}

// ---- bf16 rows of C = 8 * LPR channels, radius 4: LPR lanes per row, 8 channels (one 16-byte load) per lane.
// The 9-channel window needs the 4 nearest channels of each neighbouring lane (8 shuffles); the backward pass
// recomputes the normaliser from x instead of reading a stored fp32 copy, so forward moves 4 B per element
// and backward 6 B (the generic kernels above: 8 and 10 B).
typedef unsigned int u4v __attribute__((ext_vector_type(4)));

__device__ __forceinline__ void unpack8(u4v p, float (&v)[8]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    v[2 * i] = __uint_as_float(p[i] << 16);
    v[2 * i + 1] = __uint_as_float(p[i] & 0xffff0000u);
  }
}
__device__ __forceinline__ unsigned int bf16_bits(float f) {  // round to nearest even (finite inputs)
  const unsigned int u = __float_as_uint(f);
  return (u + 0x7fffu + ((u >> 16) & 1u)) >> 16;
}
__device__ __forceinline__ u4v pack8(const float (&v)[8]) {
  u4v p;
#pragma unroll
  for (int i = 0; i < 4; ++i) p[i] = bf16_bits(v[2 * i]) | (bf16_bits(v[2 * i + 1]) << 16);
  return p;
}

// window sums over [c-4, c+4] of a per-channel quantity q (8 per lane), neighbours' values by shuffle
template <int LPR>
__device__ __forceinline__ void window9(const float (&q)[8], int j, float (&out)[8]) {
  const int lane = threadIdx.x & 63;
  float ext[16];  // channels 8j-4 .. 8j+11
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float l = __shfl(q[4 + i], lane - 1 < 0 ? 0 : lane - 1);
    const float r = __shfl(q[i], lane + 1 > 63 ? 63 : lane + 1);
    ext[i] = j > 0 ? l : 0.f;
    ext[12 + i] = j < LPR - 1 ? r : 0.f;
  }
#pragma unroll
  for (int i = 0; i < 8; ++i) ext[4 + i] = q[i];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    float a = 0.f;
#pragma unroll
    for (int k = 0; k < 9; ++k) a += ext[i + k];
    out[i] = a;
  }
}

// N^-beta with the native v_log_f32 / v_exp_f32 (N >= bias > 0); __powf lowers to the full-precision
// library pow here (~1600 instructions per 8 channels), which made these kernels instruction-bound
__device__ __forceinline__ float npow(float N, float nb) { return __builtin_amdgcn_exp2f(nb * __builtin_amdgcn_logf(N)); }

template <int LPR>
__global__ __launch_bounds__(256) void lrn_fwd_v8(const u4v* __restrict__ x, long long M, float bias, float alpha,
                                                  float beta, u4v* __restrict__ y) {
  const long long gl = (long long)blockIdx.x * 256 + threadIdx.x;
  const long long row = gl / LPR;
  const int j = (int)(gl % LPR);
  const bool live = row < M;
  float v[8], sq[8], w[8];
  unpack8(live ? x[gl] : u4v{0, 0, 0, 0}, v);
#pragma unroll
  for (int i = 0; i < 8; ++i) sq[i] = v[i] * v[i];
  window9<LPR>(sq, j, w);
  float o[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) o[i] = v[i] * npow(bias + alpha * w[i], -beta);
  if (live) y[gl] = pack8(o);
}

// dx_c = dy_c N_c^-beta - 2 alpha beta x_c sum_{|j-c|<=4} dy_j x_j N_j^(-beta-1)
template <int LPR>
__global__ __launch_bounds__(256) void lrn_bwd_v8(const u4v* __restrict__ x, const u4v* __restrict__ dy, long long M,
                                                  float bias, float alpha, float beta, u4v* __restrict__ dx) {
  const long long gl = (long long)blockIdx.x * 256 + threadIdx.x;
  const long long row = gl / LPR;
  const int j = (int)(gl % LPR);
  const bool live = row < M;
  float v[8], g[8], sq[8], w[8], p[8], t[8], ts[8];
  unpack8(live ? x[gl] : u4v{0, 0, 0, 0}, v);
  unpack8(live ? dy[gl] : u4v{0, 0, 0, 0}, g);
#pragma unroll
  for (int i = 0; i < 8; ++i) sq[i] = v[i] * v[i];
  window9<LPR>(sq, j, w);
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const float N = bias + alpha * w[i];
    p[i] = npow(N, -beta);
    t[i] = g[i] * v[i] * p[i] * __builtin_amdgcn_rcpf(N);
  }
  window9<LPR>(t, j, ts);
  float o[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) o[i] = g[i] * p[i] - 2.f * alpha * beta * v[i] * ts[i];
  if (live) dx[gl] = pack8(o);
}

// ------------------------------------------------------------------------- SGD + EMA
struct TensorRef {
  float* w;
  const float* g;
  float* s;
  long long n;
};

constexpr int kChunk = 8192;

// grid = total chunks; chunk k belongs to tensor tix[k] and starts at element cst[k]
__global__ __launch_bounds__(256) void sgd_ema(const TensorRef* __restrict__ tabs, const int* __restrict__ tix,
                                               const long long* __restrict__ cst, float lr, float one_minus_decay,
                                               float weight_decay) {
  const TensorRef tr = tabs[tix[blockIdx.x]];
  const long long b = cst[blockIdx.x];
  const long long e = min(b + kChunk, tr.n);
  for (long long i = b + threadIdx.x; i < e; i += 256) {
    float w = tr.w[i];
    w -= lr * (tr.g[i] + weight_decay * w);
    tr.w[i] = w;
    if (tr.s != nullptr) {
      const float s = tr.s[i];
      tr.s[i] = s + one_minus_decay * (w - s);
    }
  }
}

int blocks_for(long long n, int per) { return (int)((n + per - 1) / per); }

}  // namespace

extern "C" {

// dtype: 0 fp32, 1 bf16. loss fp32 [B]; dlogits same dtype as logits, unscaled (softmax - onehot).
int mifx_cnn_softmax_xent(int dtype, const void* logits, const long long* labels, int B, int C, float* loss,
                          void* dlogits, hipStream_t st) {
  if (B < 0 || C <= 0) return -1;
  if (B == 0) return 0;
  if (C <= 256) {
    const int grid = blocks_for((long long)B * 16, 256);
    if (dtype)
      hipLaunchKernelGGL((softmax_xent<__hip_bfloat16, 16>), dim3(grid), dim3(256), 0, st,
                         (const __hip_bfloat16*)logits, labels, B, C, loss, (__hip_bfloat16*)dlogits);
    else
      hipLaunchKernelGGL((softmax_xent<float, 16>), dim3(grid), dim3(256), 0, st, (const float*)logits, labels, B, C,
                         loss, (float*)dlogits);
  } else {
    const int grid = blocks_for((long long)B * 64, 256);
    if (dtype)
      hipLaunchKernelGGL((softmax_xent<__hip_bfloat16, 64>), dim3(grid), dim3(256), 0, st,
                         (const __hip_bfloat16*)logits, labels, B, C, loss, (__hip_bfloat16*)dlogits);
    else
      hipLaunchKernelGGL((softmax_xent<float, 64>), dim3(grid), dim3(256), 0, st, (const float*)logits, labels, B, C,
                         loss, (float*)dlogits);
  }
  return (int)hipGetLastError();
}

int mifx_cnn_lrn_fwd(int dtype, const void* x, long long M, int C, int r, float bias, float alpha, float beta,
                     void* y, float* nrm, hipStream_t st) {
  if (M < 0 || C <= 0 || C > 4096 || r < 0) return -1;
  if (M == 0) return 0;
  const int R = (1024 + C - 1) / C;
  const int grid = blocks_for(M, R);
  const size_t lds = (size_t)R * C * sizeof(float);
  if (dtype)
    hipLaunchKernelGGL(lrn_fwd<__hip_bfloat16>, dim3(grid), dim3(256), lds, st, (const __hip_bfloat16*)x, M, C, r, bias,
                       alpha, beta, (__hip_bfloat16*)y, nrm);
  else
    hipLaunchKernelGGL(lrn_fwd<float>, dim3(grid), dim3(256), lds, st, (const float*)x, M, C, r, bias, alpha, beta,
                       (float*)y, nrm);
  return (int)hipGetLastError();
}

int mifx_cnn_lrn_bwd(int dtype, const void* x, const void* dy, const float* nrm, long long M, int C, int r,
                     float alpha, float beta, void* dx, hipStream_t st) {
  if (M < 0 || C <= 0 || C > 4096 || r < 0) return -1;
  if (M == 0) return 0;
  const int R = (1024 + C - 1) / C;
  const int grid = blocks_for(M, R);
  const size_t lds = (size_t)R * C * sizeof(float);
  if (dtype)
    hipLaunchKernelGGL(lrn_bwd<__hip_bfloat16>, dim3(grid), dim3(256), lds, st, (const __hip_bfloat16*)x,
                       (const __hip_bfloat16*)dy, nrm, M, C, r, alpha, beta, (__hip_bfloat16*)dx);
  else
    hipLaunchKernelGGL(lrn_bwd<float>, dim3(grid), dim3(256), lds, st, (const float*)x, (const float*)dy, nrm, M, C, r,
                       alpha, beta, (float*)dx);
  return (int)hipGetLastError();
}

// bf16, depth radius 4, C in {64, 128}, 16-byte aligned rows: vectorised kernels without a stored normaliser
int mifx_cnn_lrn_v8_ok(int C, int r) { return (r == 4 && (C == 64 || C == 128)) ? 1 : 0; }

int mifx_cnn_lrn_fwd_v8(const void* x, long long M, int C, float bias, float alpha, float beta, void* y,
                        hipStream_t st) {
  if (M < 0 || !mifx_cnn_lrn_v8_ok(C, 4)) return -1;
  if (M == 0) return 0;
  const int grid = blocks_for(M * (C / 8), 256);
  if (C == 64)
    hipLaunchKernelGGL(lrn_fwd_v8<8>, dim3(grid), dim3(256), 0, st, (const u4v*)x, M, bias, alpha, beta, (u4v*)y);
  else
    hipLaunchKernelGGL(lrn_fwd_v8<16>, dim3(grid), dim3(256), 0, st, (const u4v*)x, M, bias, alpha, beta, (u4v*)y);
  return (int)hipGetLastError();
}

int mifx_cnn_lrn_bwd_v8(const void* x, const void* dy, long long M, int C, float bias, float alpha, float beta,
                        void* dx, hipStream_t st) {
  if (M < 0 || !mifx_cnn_lrn_v8_ok(C, 4)) return -1;
  if (M == 0) return 0;
  const int grid = blocks_for(M * (C / 8), 256);
  if (C == 64)
    hipLaunchKernelGGL(lrn_bwd_v8<8>, dim3(grid), dim3(256), 0, st, (const u4v*)x, (const u4v*)dy, M, bias, alpha,
                       beta, (u4v*)dx);
  else
    hipLaunchKernelGGL(lrn_bwd_v8<16>, dim3(grid), dim3(256), 0, st, (const u4v*)x, (const u4v*)dy, M, bias, alpha,
                       beta, (u4v*)dx);
  return (int)hipGetLastError();
}

int mifx_cnn_chunk_elems() { return kChunk; }

// tables are device arrays built once by the host (see mifx/ops/cnn_ops.py: SGDEMA)
int mifx_cnn_sgd_ema(const void* tabs, const int* tix, const long long* cst, int nchunks, float lr,
                     float one_minus_decay, float weight_decay, hipStream_t st) {
  if (nchunks < 0) return -1;
  if (nchunks == 0) return 0;
  hipLaunchKernelGGL(sgd_ema, dim3(nchunks), dim3(256), 0, st, (const TensorRef*)tabs, tix, cst, lr, one_minus_decay,
                     weight_decay);
  return (int)hipGetLastError();
}

int mifx_cnn_tensor_ref_bytes() { return (int)sizeof(TensorRef); }

}  // extern "C"
