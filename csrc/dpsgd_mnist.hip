// DP-SGD MNIST tutorial CNN: per-microbatch gradients of the whole network in ONE kernel.
//
// Reference: `privacy/tutorials/mnist_dpsgd_tutorial.py:43-64` (Conv16 8x8 s2 SAME ->
// MaxPool2 s1 -> Conv32 4x4 s2 VALID -> MaxPool2 s1 -> Dense32 -> Dense10, no activations, sparse softmax CE)
// trained by `dp_optimizer.py:59-90`, which runs one backward per microbatch in a tf.while_loop. Here one
// workgroup owns one microbatch: for each of its examples it runs the forward and the full backward with
// every activation, the padded image, the conv weights and the pool argmaxes resident in LDS (~120 KB,
// one workgroup per CU), and accumulates the example's parameter gradient into its row of
// G[M, ld] (the same thread owns the same G elements for every example, so the accumulation needs no
// fence or atomics). G then feeds the fused clip/sum/noise kernel of csrc/dp.hip. All math is fp32 with
// the PyTorch reference's semantics (first-max pooling, ignore-index labels), so G matches a
// torch.func.vmap(grad) of `mifx.models.cnn.MnistDPCNN` to fp32 rounding.
//
// Layouts: activations are HWC (channel fastest) in LDS; parameters are PyTorch's (conv [co][ci][kh][kw],
// linear [out][in]) and G's columns follow `MnistDPCNN.named_parameters()` order. The conv weight images
// are padded (w1 rows 65 floats, w2 rows 257) and conv2 has a second [kh][kw][co][ci] image for the
// input-gradient pass, so the wave's LDS reads are conflict-free or broadcasts.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

constexpr int kThreads = 512;
constexpr int H0 = 28, XP = 34, PAD1 = 3;  // input 28x28, SAME-padded (3 top/left, 3 bottom/right) to 34x34
constexpr int C1 = 16, K1 = 8, O1 = 14;    // conv1: 16 x 8x8 stride 2 -> 14x14x16
constexpr int P1 = 13;                     // max-pool 2x2 stride 1 -> 13x13x16
constexpr int C2 = 32, K2 = 4, O2 = 5;     // conv2: 32 x 4x4 stride 2 VALID -> 5x5x32
constexpr int P2 = 4, NF = 512;            // max-pool 2x2 stride 1 -> 4x4x32, flattened NCHW (c*16+h*4+w)
constexpr int F1 = 32, NC = 10;
constexpr int W1S = 65, W2S = 257;
// G column offsets (named_parameters order)
constexpr int OW1 = 0, OB1 = 1024, OW2 = 1040, OB2 = 9232, OW3 = 9264, OB3 = 25648, OW4 = 25680, OB4 = 26000;
constexpr int NP = 26010;

struct Smem {
  float xp[XP * XP];
  float w1[C1 * W1S];
  float w2[C2 * W2S];
  float w2t[K2 * K2 * C2 * C1];  // [kh*4+kw][co][ci]
  float b1[C1], b2[C2];
  float y1[O1 * O1 * C1];   // conv1 output, then its gradient
  float p1[P1 * P1 * C1];
  float dp1[P1 * P1 * C1];
  float y2[O2 * O2 * C2];   // conv2 output, then its gradient
  float p2[NF], dp2[NF];
  float h3[F1], dh3[F1];
  float dl[16];
  uint8_t am1[P1 * P1 * C1];
  uint8_t am2[NF];
};

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// the four taps of a 2x2 window in PyTorch's scan order; first strict maximum wins, NaN propagates
__device__ __forceinline__ float pool4(float a, float b, float c, float d, uint8_t& idx) {
  float m = a;
  int k = 0;
  if (b > m || b != b) { m = b; k = 1; }
  if (c > m || c != c) { m = c; k = 2; }
  if (d > m || d != d) { m = d; k = 3; }
  idx = (uint8_t)k;
  return m;
}

__global__ __launch_bounds__(kThreads) void dpmnist_grads(const float* __restrict__ x, const long long* __restrict__ y,
                                                          int per, const float* __restrict__ gw1,
                                                          const float* __restrict__ gb1, const float* __restrict__ gw2,
                                                          const float* __restrict__ gb2, const float* __restrict__ W3,
                                                          const float* __restrict__ b3, const float* __restrict__ W4,
                                                          const float* __restrict__ b4, float* __restrict__ G, int ld,
                                                          float* __restrict__ loss_out) {
  __shared__ Smem s;
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int m = blockIdx.x;
  float* g = G + (size_t)m * ld;

  for (int i = t; i < C1 * K1 * K1; i += kThreads) s.w1[(i >> 6) * W1S + (i & 63)] = gw1[i];
  for (int i = t; i < C2 * C1 * K2 * K2; i += kThreads) {
    const float v = gw2[i];
    const int co = i >> 8, r = i & 255, ci = r >> 4, k = r & 15;
    s.w2[co * W2S + r] = v;
    s.w2t[(k * C2 + co) * C1 + ci] = v;
  }
  if (t < C1) s.b1[t] = gb1[t];
  if (t < C2) s.b2[t] = gb2[t];
  for (int i = NP + t; i < ld; i += kThreads) g[i] = 0.f;  // row padding

  for (int ex = 0; ex < per; ++ex) {
    const long long e = (long long)m * per + ex;
    const bool first = ex == 0;
    // G[m, c] (+)= v; thread-owned columns, see the header
#define GPUT(col, val)                       \
  do {                                       \
    const int c_ = (col);                    \
    const float v_ = (val);                  \
    g[c_] = first ? v_ : g[c_] + v_;         \
  } while (0)

    const float* xe = x + e * (H0 * H0);
    for (int i = t; i < XP * XP; i += kThreads) {
      const int r = i / XP - PAD1, c = i % XP - PAD1;
      s.xp[i] = (r >= 0 && r < H0 && c >= 0 && c < H0) ? xe[r * H0 + c] : 0.f;
    }
    __syncthreads();

    // conv1 forward: thread owns one output channel (64 weights in registers) and a strided set of positions
    {
      const int co = t & (C1 - 1);
      float w[K1 * K1];
#pragma unroll
      for (int k = 0; k < K1 * K1; ++k) w[k] = s.w1[co * W1S + k];
      for (int p = t >> 4; p < O1 * O1; p += kThreads / C1) {
        const int oh = p / O1, ow = p % O1;
        const float* xr = s.xp + (2 * oh) * XP + 2 * ow;
        float acc = s.b1[co];
#pragma unroll
        for (int kh = 0; kh < K1; ++kh)
#pragma unroll
          for (int kw = 0; kw < K1; ++kw) acc += w[kh * K1 + kw] * xr[kh * XP + kw];
        s.y1[p * C1 + co] = acc;
      }
    }
    __syncthreads();
    for (int o = t; o < P1 * P1 * C1; o += kThreads) {
      const int c = o & (C1 - 1), p = o >> 4, h = p / P1, w = p % P1;
      const float* r0 = s.y1 + (h * O1 + w) * C1 + c;
      uint8_t k;
      s.p1[o] = pool4(r0[0], r0[C1], r0[O1 * C1], r0[O1 * C1 + C1], k);
      s.am1[o] = k;
    }
    __syncthreads();

    // conv2 forward: 4 lanes per output (ci = 4j + q), shuffle-reduced
    for (int i0 = 0; i0 < O2 * O2 * C2 * 4; i0 += kThreads) {
      const int i = i0 + t;
      const int o = i >> 2, q = i & 3;
      float acc = 0.f;
      if (o < O2 * O2 * C2) {
        const int co = o & (C2 - 1), p = o >> 5, oh = p / O2, ow = p % O2;
        const float* wr = s.w2 + co * W2S;
        for (int j = 0; j < C1 / 4; ++j) {
          const int ci = 4 * j + q;
#pragma unroll 2
          for (int kh = 0; kh < K2; ++kh)
#pragma unroll
            for (int kw = 0; kw < K2; ++kw)
              acc += wr[ci * 16 + kh * 4 + kw] * s.p1[((2 * oh + kh) * P1 + 2 * ow + kw) * C1 + ci];
        }
      }
      acc += __shfl_xor(acc, 1);
      acc += __shfl_xor(acc, 2);
      if (o < O2 * O2 * C2 && q == 0) s.y2[o] = acc + s.b2[o & (C2 - 1)];
    }
    __syncthreads();
    for (int o = t; o < NF; o += kThreads) {
      const int c = o >> 4, h = (o >> 2) & 3, w = o & 3;
      const float* r0 = s.y2 + (h * O2 + w) * C2 + c;
      uint8_t k;
      s.p2[o] = pool4(r0[0], r0[C2], r0[O2 * C2], r0[O2 * C2 + C2], k);
      s.am2[o] = k;
    }
    __syncthreads();

    // dense 512 -> 32: wave wv computes outputs wv, wv+8, wv+16, wv+24
    for (int j = wv; j < F1; j += kThreads / 64) {
      float a = 0.f;
#pragma unroll
      for (int i = lane; i < NF; i += 64) a += W3[j * NF + i] * s.p2[i];
      a = wave_sum(a);
      if (lane == 0) s.h3[j] = a + b3[j];
    }
    __syncthreads();
    // dense 32 -> 10, softmax cross-entropy, dlogits (wave 0)
    if (wv == 0) {
      float lg = -INFINITY;
      if (lane < NC) {
        lg = b4[lane];
#pragma unroll 8
        for (int j = 0; j < F1; ++j) lg += W4[lane * F1 + j] * s.h3[j];
      }
      float mx = lg;
#pragma unroll
      for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
      const float ex_ = lane < NC ? expf(lg - mx) : 0.f;
      const float se = wave_sum(ex_);
      const long long lab = y[e];
      const bool valid = lab >= 0 && lab < NC;
      const float lgy = __shfl(lg, valid ? (int)lab : 0);
      if (lane < NC) s.dl[lane] = valid ? ex_ / se - (lane == lab ? 1.f : 0.f) : 0.f;
      if (lane == 0) loss_out[e] = valid ? logf(se) + mx - lgy : 0.f;
    }
    __syncthreads();

    // dense 32 -> 10 gradients; dh3
    for (int i = t; i < NC * F1; i += kThreads) GPUT(OW4 + i, s.dl[i / F1] * s.h3[i % F1]);
    if (t < NC) GPUT(OB4 + t, s.dl[t]);
    if (t < F1) {
      float a = 0.f;
#pragma unroll
      for (int k = 0; k < NC; ++k) a += W4[k * F1 + t] * s.dl[k];
      s.dh3[t] = a;
    }
    __syncthreads();
    // dense 512 -> 32 gradients; dp2
    for (int i = t; i < F1 * NF; i += kThreads) GPUT(OW3 + i, s.dh3[i / NF] * s.p2[i % NF]);
    if (t < F1) GPUT(OB3 + t, s.dh3[t]);
    for (int i = t; i < NF; i += kThreads) {
      float a = 0.f;
#pragma unroll 8
      for (int j = 0; j < F1; ++j) a += W3[j * NF + i] * s.dh3[j];
      s.dp2[i] = a;
    }
    __syncthreads();
    // max-pool 2 backward (gather over the <= 4 windows covering each conv2 output), into y2
    for (int o = t; o < O2 * O2 * C2; o += kThreads) {
      const int c = o & (C2 - 1), p = o >> 5, h = p / O2, w = p % O2;
      float a = 0.f;
#pragma unroll
      for (int dh = 1; dh >= 0; --dh)
#pragma unroll
        for (int dw = 1; dw >= 0; --dw) {
          const int ph = h - dh, pw = w - dw;
          if (ph >= 0 && ph < P2 && pw >= 0 && pw < P2) {
            const int q = c * 16 + ph * 4 + pw;
            if (s.am2[q] == dh * 2 + dw) a += s.dp2[q];
          }
        }
      s.y2[o] = a;
    }
    __syncthreads();
    // conv2 bias / weight gradients and input gradient (independent, one barrier)
    if (t < C2) {
      float a = 0.f;
      for (int p = 0; p < O2 * O2; ++p) a += s.y2[p * C2 + t];
      GPUT(OB2 + t, a);
    }
    for (int i = t; i < C2 * C1 * K2 * K2; i += kThreads) {
      const int co = i >> 8, ci = (i >> 4) & 15, kh = (i >> 2) & 3, kw = i & 3;
      float a = 0.f;
      for (int oh = 0; oh < O2; ++oh)
#pragma unroll
        for (int ow = 0; ow < O2; ++ow)
          a += s.y2[(oh * O2 + ow) * C2 + co] * s.p1[((2 * oh + kh) * P1 + 2 * ow + kw) * C1 + ci];
      GPUT(OW2 + i, a);
    }
    for (int o = t; o < P1 * P1 * C1; o += kThreads) {
      const int ci = o & (C1 - 1), p = o >> 4, h = p / P1, w = p % P1;
      float a = 0.f;
#pragma unroll
      for (int a_ = 0; a_ < 2; ++a_) {
        const int kh = (h & 1) + 2 * a_, oh = (h - kh) >> 1;
        if (h - kh < 0 || oh >= O2) continue;
#pragma unroll
        for (int b_ = 0; b_ < 2; ++b_) {
          const int kw = (w & 1) + 2 * b_, ow = (w - kw) >> 1;
          if (w - kw < 0 || ow >= O2) continue;
          const float* wt = s.w2t + (kh * K2 + kw) * C2 * C1 + ci;
          const float* dy = s.y2 + (oh * O2 + ow) * C2;
#pragma unroll 8
          for (int co = 0; co < C2; ++co) a += wt[co * C1] * dy[co];
        }
      }
      s.dp1[o] = a;
    }
    __syncthreads();
    // max-pool 1 backward into y1
    for (int o = t; o < O1 * O1 * C1; o += kThreads) {
      const int c = o & (C1 - 1), p = o >> 4, h = p / O1, w = p % O1;
      float a = 0.f;
#pragma unroll
      for (int dh = 1; dh >= 0; --dh)
#pragma unroll
        for (int dw = 1; dw >= 0; --dw) {
          const int ph = h - dh, pw = w - dw;
          if (ph >= 0 && ph < P1 && pw >= 0 && pw < P1) {
            const int q = (ph * P1 + pw) * C1 + c;
            if (s.am1[q] == dh * 2 + dw) a += s.dp1[q];
          }
        }
      s.y1[o] = a;
    }
    __syncthreads();
    // conv1 bias / weight gradients
    if (t < C1) {
      float a = 0.f;
      for (int p = 0; p < O1 * O1; ++p) a += s.y1[p * C1 + t];
      GPUT(OB1 + t, a);
    }
    for (int i = t; i < C1 * K1 * K1; i += kThreads) {
      const int co = i >> 6, kh = (i >> 3) & 7, kw = i & 7;
      float a = 0.f;
      for (int oh = 0; oh < O1; ++oh) {
        const float* xr = s.xp + (2 * oh + kh) * XP + kw;
        const float* dy = s.y1 + oh * O1 * C1 + co;
#pragma unroll
        for (int ow = 0; ow < O1; ++ow) a += dy[ow * C1] * xr[2 * ow];
      }
      GPUT(OW1 + i, a);
    }
    __syncthreads();  // the next example overwrites xp / y1 / ...
#undef GPUT
  }
}

}  // namespace

extern "C" {

int mifx_dpmnist_num_params() { return NP; }

// x [B, 28, 28] fp32, y [B] int64; params in PyTorch layout; G [M, ld] fp32 (ld >= NP, pad columns zeroed),
// loss [B] per-example softmax cross-entropy. Microbatch m = examples [m*B/M, (m+1)*B/M).
int mifx_dpmnist_grads(const float* x, const long long* y, int B, int M, const float* w1, const float* b1,
                       const float* w2, const float* b2, const float* w3, const float* b3, const float* w4,
                       const float* b4, float* G, int ld, float* loss, hipStream_t st) {
  if (B <= 0 || M <= 0 || B % M != 0 || ld < NP) return -1;
  hipLaunchKernelGGL(dpmnist_grads, dim3(M), dim3(kThreads), 0, st, x, y, B / M, w1, b1, w2, b2, w3, b3, w4, b4, G,
                     ld, loss);
  return (int)hipGetLastError();
}

}  // extern "C"
