// Direct fp32 convolutions for the small image CNNs of the reference notebooks (MIOpen-free), gfx950.
//
// Parity targets: `serving/Predict_Fashion_MNIST.ipynb` (Conv2D(8, 3x3, stride 2)), `tpu/Keras_MNIST_TPU.ipynb`
// (Conv2D 32 / 64 / 64, 3x3 valid), `privacy/tutorials/mnist_dpsgd_tutorial.py:42-58` (Conv16 8x8 s2 SAME,
// Conv32 4x4 s2 valid), PATE `deep_cnn.py` first layers (1 or 3 input channels, 5x5). These have 1-64 channels on
// 28x28 images: too few channels for an MFMA implicit GEMM tile (csrc/gconv.hip needs C, K % 32), so they run as
// register-blocked direct convolutions on the VALU in fp32 (the models train in fp32), NCHW:
//  * forward: one wave per (image, 64 output pixels, KB output channels); each lane keeps KB accumulators, every
//    input value it loads feeds KB FMAs, and the weights are wave-uniform (scalar loads);
//  * input gradient: the same shape over input pixels and CB input channels (taps whose output position is
//    off-grid or out of range skipped; any stride);
//  * weight gradient: 256-thread workgroups per (k, c, split of the image x output-pixel range) computing all R x S
//    taps: each thread accumulates its strided share in registers, wave shuffles + a fixed-order sum of the 4 waves,
//    then a second kernel adds the splits in order -> deterministic.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

constexpr int KB = 8;      // output channels per forward lane
constexpr int CB = 4;      // input channels per input-gradient lane
constexpr int MAXRS = 64;  // R * S <= 64 (8x8 kernels)

struct Geo {
  int N, C, H, W, K, R, S, stride, pad_h, pad_w, Ho, Wo;
};

__global__ __launch_bounds__(64) void conv_fwd(const float* __restrict__ x, const float* __restrict__ w,
                                               const float* __restrict__ bias, float* __restrict__ y, Geo g) {
  const int P = g.Ho * g.Wo, ptiles = (P + 63) / 64, kblocks = (g.K + KB - 1) / KB;
  int b = blockIdx.x;
  const int kb = b % kblocks;
  b /= kblocks;
  const int pt = b % ptiles, n = b / ptiles;
  const int p = pt * 64 + threadIdx.x;
  const bool live = p < P;
  const int oh = live ? p / g.Wo : 0, ow = live ? p % g.Wo : 0;
  const int k0 = kb * KB;
  float acc[KB];
#pragma unroll
  for (int j = 0; j < KB; ++j) acc[j] = (bias != nullptr && k0 + j < g.K) ? bias[k0 + j] : 0.f;
  const int ih0 = oh * g.stride - g.pad_h, iw0 = ow * g.stride - g.pad_w;
  for (int c = 0; c < g.C; ++c) {
    const float* xc = x + ((size_t)n * g.C + c) * g.H * g.W;
    for (int r = 0; r < g.R; ++r) {
      const int ih = ih0 + r;
      const bool hin = ih >= 0 && ih < g.H;
      for (int s = 0; s < g.S; ++s) {
        const int iw = iw0 + s;
        const float xv = (live && hin && iw >= 0 && iw < g.W) ? xc[ih * g.W + iw] : 0.f;
        const float* wp = w + (((size_t)k0 * g.C + c) * g.R + r) * g.S + s;
        const size_t wk = (size_t)g.C * g.R * g.S;
#pragma unroll
        for (int j = 0; j < KB; ++j)
          if (k0 + j < g.K) acc[j] = fmaf(xv, wp[j * wk], acc[j]);
      }
    }
  }
  if (!live) return;
#pragma unroll
  for (int j = 0; j < KB; ++j)
    if (k0 + j < g.K) y[(((size_t)n * g.K + k0 + j) * g.Ho + oh) * g.Wo + ow] = acc[j];
}

__global__ __launch_bounds__(64) void conv_dgrad(const float* __restrict__ dy, const float* __restrict__ w,
                                                 float* __restrict__ dx, Geo g) {
  const int P = g.H * g.W, ptiles = (P + 63) / 64, cblocks = (g.C + CB - 1) / CB;
  int b = blockIdx.x;
  const int cb = b % cblocks;
  b /= cblocks;
  const int pt = b % ptiles, n = b / ptiles;
  const int p = pt * 64 + threadIdx.x;
  const bool live = p < P;
  const int ih = live ? p / g.W : 0, iw = live ? p % g.W : 0;
  const int c0 = cb * CB;
  float acc[CB] = {0.f, 0.f, 0.f, 0.f};
  for (int k = 0; k < g.K; ++k) {
    const float* dyk = dy + ((size_t)n * g.K + k) * g.Ho * g.Wo;
    for (int r = 0; r < g.R; ++r) {
      const int th = ih + g.pad_h - r;  // = oh * stride
      const int oh = th / g.stride;
      const bool hok = th >= 0 && oh * g.stride == th && oh < g.Ho;
      for (int s = 0; s < g.S; ++s) {
        const int tw = iw + g.pad_w - s;
        const int ow = tw / g.stride;
        const bool ok = live && hok && tw >= 0 && ow * g.stride == tw && ow < g.Wo;
        const float gv = ok ? dyk[oh * g.Wo + ow] : 0.f;
        const float* wp = w + (((size_t)k * g.C + c0) * g.R + r) * g.S + s;
#pragma unroll
        for (int j = 0; j < CB; ++j)
          if (c0 + j < g.C) acc[j] = fmaf(gv, wp[(size_t)j * g.R * g.S], acc[j]);
      }
    }
  }
  if (!live) return;
#pragma unroll
  for (int j = 0; j < CB; ++j)
    if (c0 + j < g.C) dx[(((size_t)n * g.C + c0 + j) * g.H + ih) * g.W + iw] = acc[j];
}

// weight gradient, split over the (image, output pixel) positions: workgroup (k, c, split) sums its contiguous
// range into part[split][k][c][tap]; wgrad_sum adds the splits in order (deterministic)
template <int RS>
__global__ __launch_bounds__(256) void conv_wgrad(const float* __restrict__ x, const float* __restrict__ dy,
                                                  float* __restrict__ part, Geo g, int splits) {
  __shared__ float red[256];
  const int kc = blockIdx.x / splits, sp = blockIdx.x % splits;
  const int k = kc / g.C, c = kc % g.C;
  const int P = g.Ho * g.Wo;
  const long long tot = (long long)g.N * P;
  const long long i0 = tot * sp / splits, i1 = tot * (sp + 1) / splits;
  float acc[RS];
#pragma unroll
  for (int t = 0; t < RS; ++t) acc[t] = 0.f;
  for (long long i = i0 + threadIdx.x; i < i1; i += 256) {
    const int n = (int)(i / P), p = (int)(i % P);
    const int oh = p / g.Wo, ow = p % g.Wo;
    const float gv = dy[((size_t)n * g.K + k) * P + p];
    const float* xc = x + ((size_t)n * g.C + c) * g.H * g.W;
    const int ih0 = oh * g.stride - g.pad_h, iw0 = ow * g.stride - g.pad_w;
#pragma unroll
    for (int t = 0; t < RS; ++t) {
      if (t >= g.R * g.S) break;
      const int r = t / g.S, s = t % g.S, ih = ih0 + r, iw = iw0 + s;
      if (ih >= 0 && ih < g.H && iw >= 0 && iw < g.W) acc[t] = fmaf(gv, xc[ih * g.W + iw], acc[t]);
    }
  }
  const int RSn = g.R * g.S;
  for (int t = 0; t < RSn && t < RS; ++t) {
    float v = acc[t];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);  // wave sums, then the 4 waves in order
    if ((threadIdx.x & 63) == 0) red[(threadIdx.x >> 6) * RS + t] = v;
  }
  __syncthreads();
  if (threadIdx.x < RSn)
    part[((size_t)sp * g.K * g.C + kc) * RSn + threadIdx.x] =
        ((red[threadIdx.x] + red[RS + threadIdx.x]) + red[2 * RS + threadIdx.x]) + red[3 * RS + threadIdx.x];
}

__global__ __launch_bounds__(256) void wgrad_sum(const float* __restrict__ part, float* __restrict__ dw, int n,
                                                 int splits) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  float v = 0.f;
  for (int sp = 0; sp < splits; ++sp) v += part[(size_t)sp * n + i];
  dw[i] = v;
}

bool geo_ok(const Geo& g) {
  return g.N > 0 && g.C > 0 && g.H > 0 && g.W > 0 && g.K > 0 && g.R > 0 && g.S > 0 && g.R * g.S <= MAXRS &&
         g.stride > 0 && g.pad_h >= 0 && g.pad_w >= 0 && g.Ho > 0 && g.Wo > 0 &&
         (g.Ho - 1) * g.stride + g.R <= g.H + 2 * g.pad_h && (g.Wo - 1) * g.stride + g.S <= g.W + 2 * g.pad_w;
}

}  // namespace

extern "C" {

// x [N, C, H, W], w [K, C, R, S], bias [K] or null, y [N, K, Ho, Wo]; fp32 contiguous NCHW. Symmetric padding
// (pad_h, pad_w); TF SAME's asymmetric padding is applied by the caller as an explicit pad.
int mifx_convs_fwd(const float* x, const float* w, const float* bias, float* y, int N, int C, int H, int W, int K,
                   int R, int S, int stride, int pad_h, int pad_w, int Ho, int Wo, hipStream_t st) {
  const Geo g{N, C, H, W, K, R, S, stride, pad_h, pad_w, Ho, Wo};
  if (!geo_ok(g) || x == nullptr || w == nullptr || y == nullptr) return -1;
  const long long blocks = (long long)N * ((Ho * Wo + 63) / 64) * ((K + KB - 1) / KB);
  if (blocks >= (1ll << 31)) return -1;
  hipLaunchKernelGGL(conv_fwd, dim3((unsigned)blocks), dim3(64), 0, st, x, w, bias, y, g);
  return (int)hipGetLastError();
}

int mifx_convs_dgrad(const float* dy, const float* w, float* dx, int N, int C, int H, int W, int K, int R, int S,
                     int stride, int pad_h, int pad_w, int Ho, int Wo, hipStream_t st) {
  const Geo g{N, C, H, W, K, R, S, stride, pad_h, pad_w, Ho, Wo};
  if (!geo_ok(g) || dy == nullptr || w == nullptr || dx == nullptr) return -1;
  const long long blocks = (long long)N * ((H * W + 63) / 64) * ((C + CB - 1) / CB);
  if (blocks >= (1ll << 31)) return -1;
  hipLaunchKernelGGL(conv_dgrad, dim3((unsigned)blocks), dim3(64), 0, st, dy, w, dx, g);
  return (int)hipGetLastError();
}

// splits of the (image, output pixel) range per (k, c) so the launch has >= ~1024 workgroups; part: scratch of
// mifx_convs_wgrad_splits(...) * K * C * R * S floats
int mifx_convs_wgrad_splits(int N, int K, int C, int Ho, int Wo) {
  const long long tot = (long long)N * Ho * Wo;
  long long sp = (1024 + (long long)K * C - 1) / ((long long)K * C);
  sp = sp < 1 ? 1 : sp;
  const long long maxsp = (tot + 1023) / 1024;  // >= ~1024 positions per workgroup
  if (sp > maxsp) sp = maxsp;
  return (int)(sp < 1 ? 1 : (sp > 4096 ? 4096 : sp));
}

int mifx_convs_wgrad(const float* x, const float* dy, float* dw, float* part, int N, int C, int H, int W, int K, int R,
                     int S, int stride, int pad_h, int pad_w, int Ho, int Wo, hipStream_t st) {
  const Geo g{N, C, H, W, K, R, S, stride, pad_h, pad_w, Ho, Wo};
  if (!geo_ok(g) || x == nullptr || dy == nullptr || dw == nullptr || part == nullptr) return -1;
  const int splits = mifx_convs_wgrad_splits(N, K, C, Ho, Wo);
  if ((long long)K * C * splits >= (1ll << 31)) return -1;
  const dim3 grid((unsigned)(K * C * splits));
  // (RS template: the LDS red[] holds 4 waves x RS taps <= 256 floats)
  if (R * S <= 9)
    hipLaunchKernelGGL(conv_wgrad<9>, grid, dim3(256), 0, st, x, dy, part, g, splits);
  else if (R * S <= 25)
    hipLaunchKernelGGL(conv_wgrad<25>, grid, dim3(256), 0, st, x, dy, part, g, splits);
  else
    hipLaunchKernelGGL(conv_wgrad<MAXRS>, grid, dim3(256), 0, st, x, dy, part, g, splits);
  const int n = K * C * R * S;
  hipLaunchKernelGGL(wgrad_sum, dim3((n + 255) / 256), dim3(256), 0, st, part, dw, n, splits);
  return (int)hipGetLastError();
}

}  // extern "C"
