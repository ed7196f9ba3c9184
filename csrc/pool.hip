// 3x3 / stride 2 max pooling for NHWC bf16 activations: the ResNet-50 stem (pad 1, BASELINE config 5) and the
// PATE CNN's TF-SAME pooling (`deep_cnn.py:123,151`: top/left pad = total // 2, the rest at the bottom/right).
//
// PyTorch's NHWC max-pool saves an int64 argmax per OUTPUT element and scatters the backward through it
// (profiles/archive/resnet50_steady_kernels_s3.md: 252 us fwd + 620 us bwd per step at B=256, 112x112x64). Here:
//  * forward: one thread per (n, oh, ow, 8 channels): nine 16-byte window loads, per-channel max, and a
//    1-byte window position (0..8) per channel -> the index traffic is 1/8 of int64 indices;
//  * backward in gather form: one thread per (n, ih, iw, 8 channels) visits the (at most 2x2) output
//    windows that contain its input position and adds dout where the stored position points at it.
//    Every input gradient is written exactly once (no zero-fill, no atomics: deterministic). For the stem's
//    even-sized image a thread owns a 2 x 2 input block and loads its four windows once (maxpool_bwd_even:
//    278 -> 145 us at B=256, bit-identical, profiles/resnet_pool_bwd_ab_r5.txt).
// Semantics follow PyTorch: padding never wins, ties keep the first position in window order, NaN wins.
#include <hip/hip_bf16.h>
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

namespace {

constexpr int kThreads = 256;
constexpr int kVec = 8;  // channels per thread (16 bytes of bf16)
constexpr uint8_t kNone = 255;  // window position of a window that passes no gradient (fused ReLU)

struct alignas(16) Bf8 {
  __hip_bfloat16 v[kVec];
};
struct alignas(8) U8x8 {
  uint8_t v[kVec];
};

// I: the flat thread-index type -- 32-bit whenever the element count allows (the ResNet stem's 25.7 M work items:
// three 64-bit divisions per item are emulated in ~100 VALU instructions each, so the int64 build is ALU-bound)
template <typename I>
__global__ __launch_bounds__(kThreads) void maxpool_fwd(const __hip_bfloat16* __restrict__ x, int N, int H, int W, int C,
                                                       int OH, int OW, int pt, int pl, int relu,
                                                       __hip_bfloat16* __restrict__ y, uint8_t* __restrict__ idx) {
  const int cg = C / kVec;
  const I total = (I)N * OH * OW * cg;
  for (I t = (I)blockIdx.x * kThreads + threadIdx.x; t < total; t += (I)gridDim.x * kThreads) {
    const int g = (int)(t % cg);
    I p = t / cg;
    const int ow = (int)(p % OW);
    p /= OW;
    const int oh = (int)(p % OH);
    const int n = (int)(p / OH);
    float m[kVec];
    U8x8 k8;
#pragma unroll
    for (int e = 0; e < kVec; ++e) {
      m[e] = -INFINITY;
      k8.v[e] = 0;
    }
    bool first = true;
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
      const int ih = 2 * oh - pt + kh;
      if (ih < 0 || ih >= H) continue;
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int iw = 2 * ow - pl + kw;
        if (iw < 0 || iw >= W) continue;
        const Bf8 v8 = *(const Bf8*)(x + (((size_t)n * H + ih) * W + iw) * C + g * kVec);
#pragma unroll
        for (int e = 0; e < kVec; ++e) {
          const float v = __bfloat162float(v8.v[e]);
          if (first || v > m[e] || v != v) {  // first valid tap, strictly greater, or NaN (PyTorch: last NaN wins)
            m[e] = v;
            k8.v[e] = (uint8_t)(kh * 3 + kw);
          }
        }
        first = false;
      }
    }
    if (relu) {  // relu(max) == max(relu): windows whose max is <= 0 (or NaN) pass no gradient (idx kNone)
#pragma unroll
      for (int e = 0; e < kVec; ++e) {
        if (!(m[e] > 0.f)) {
          k8.v[e] = kNone;
          if (m[e] == m[e]) m[e] = 0.f;
        }
      }
    }
    Bf8 o;
#pragma unroll
    for (int e = 0; e < kVec; ++e) o.v[e] = __float2bfloat16(m[e]);
    const size_t off = (((size_t)n * OH + oh) * OW + ow) * C + g * kVec;
    *(Bf8*)(y + off) = o;
    *(U8x8*)(idx + off) = k8;
  }
}

// Forward over PAIRS of horizontally adjacent windows (ow = 2q, 2q + 1): their 3 x 5 input patch shares one column,
// so a thread issues 15 loads for two outputs instead of 18, all before the first compare (clamped addresses, so
// every load is unconditional; out-of-image taps are masked at the compare). Per-window tap order, tie and NaN
// rules are those of maxpool_fwd (bit-identical outputs and positions).
template <typename I>
__global__ __launch_bounds__(kThreads) void maxpool_fwd2(const __hip_bfloat16* __restrict__ x, int N, int H, int W,
                                                        int C, int OH, int OW, int pt, int pl, int relu,
                                                        __hip_bfloat16* __restrict__ y, uint8_t* __restrict__ idx) {
  const int cg = C / kVec, OQ = (OW + 1) >> 1;
  const I total = (I)N * OH * OQ * cg;
  for (I t = (I)blockIdx.x * kThreads + threadIdx.x; t < total; t += (I)gridDim.x * kThreads) {
    const int g = (int)(t % cg);
    I p = t / cg;
    const int q = (int)(p % OQ);
    p /= OQ;
    const int oh = (int)(p % OH);
    const int n = (int)(p / OH);
    const bool two = 2 * q + 1 < OW;
    Bf8 v[3][5];
    bool ok[3][5];
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
      const int ih = 2 * oh - pt + kh;
      const bool rok = ih >= 0 && ih < H;
      const int ihc = min(max(ih, 0), H - 1);
#pragma unroll
      for (int c = 0; c < 5; ++c) {
        const int iw = 4 * q - pl + c;
        ok[kh][c] = rok && iw >= 0 && iw < W && (c < 3 || two);
        const int iwc = min(max(iw, 0), W - 1);
        v[kh][c] = *(const Bf8*)(x + (((size_t)n * H + ihc) * W + iwc) * C + g * kVec);
      }
    }
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      if (s2 == 1 && !two) break;
      float m[kVec];
      U8x8 k8;
#pragma unroll
      for (int e = 0; e < kVec; ++e) {
        m[e] = -INFINITY;
        k8.v[e] = 0;
      }
      bool first = true;
#pragma unroll
      for (int kh = 0; kh < 3; ++kh)
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) {
          if (!ok[kh][2 * s2 + kw]) continue;
          const Bf8& v8 = v[kh][2 * s2 + kw];
#pragma unroll
          for (int e = 0; e < kVec; ++e) {
            const float f = __bfloat162float(v8.v[e]);
            if (first || f > m[e] || f != f) {
              m[e] = f;
              k8.v[e] = (uint8_t)(kh * 3 + kw);
            }
          }
          first = false;
        }
      if (relu) {
#pragma unroll
        for (int e = 0; e < kVec; ++e) {
          if (!(m[e] > 0.f)) {
            k8.v[e] = kNone;
            if (m[e] == m[e]) m[e] = 0.f;
          }
        }
      }
      Bf8 o;
#pragma unroll
      for (int e = 0; e < kVec; ++e) o.v[e] = __float2bfloat16(m[e]);
      const size_t off = (((size_t)n * OH + oh) * OW + 2 * q + s2) * C + g * kVec;
      *(Bf8*)(y + off) = o;
      *(U8x8*)(idx + off) = k8;
    }
  }
}

template <typename I>
__global__ __launch_bounds__(kThreads) void maxpool_bwd(const __hip_bfloat16* __restrict__ dy,
                                                       const uint8_t* __restrict__ idx, int N, int H, int W, int C,
                                                       int OH, int OW, int pt, int pl, __hip_bfloat16* __restrict__ dx) {
  const int cg = C / kVec;
  const I total = (I)N * H * W * cg;
  for (I t = (I)blockIdx.x * kThreads + threadIdx.x; t < total; t += (I)gridDim.x * kThreads) {
    const int g = (int)(t % cg);
    I p = t / cg;
    const int iw = (int)(p % W);
    p /= W;
    const int ih = (int)(p % H);
    const int n = (int)(p / H);
    // output windows containing ih: 2 oh - pt <= ih <= 2 oh - pt + 2, i.e. oh in [ceil((u - 2) / 2), u / 2], u = ih + pt
    const int uh = ih + pt, uw = iw + pl;
    const int oh1 = uh >> 1, oh0 = max(0, (uh - 1) >> 1);
    const int ow1 = uw >> 1, ow0 = max(0, (uw - 1) >> 1);
    float acc[kVec];
#pragma unroll
    for (int e = 0; e < kVec; ++e) acc[e] = 0.f;
#pragma unroll
    for (int a = 0; a < 2; ++a) {
      const int oh = a ? oh1 : oh0;
      if ((a && oh1 == oh0) || oh >= OH) continue;
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int ow = b ? ow1 : ow0;
        if ((b && ow1 == ow0) || ow >= OW) continue;
        const uint8_t k = (uint8_t)((ih - (2 * oh - pt)) * 3 + (iw - (2 * ow - pl)));
        const size_t off = (((size_t)n * OH + oh) * OW + ow) * C + g * kVec;
        const U8x8 k8 = *(const U8x8*)(idx + off);
        const Bf8 d8 = *(const Bf8*)(dy + off);
#pragma unroll
        for (int e = 0; e < kVec; ++e)
          if (k8.v[e] == k) acc[e] += __bfloat162float(d8.v[e]);
      }
    }
    Bf8 o;
#pragma unroll
    for (int e = 0; e < kVec; ++e) o.v[e] = __float2bfloat16(acc[e]);
    *(Bf8*)(dx + (((size_t)n * H + ih) * W + iw) * C + g * kVec) = o;
  }
}

// Backward of the pad-1 pool over an even-sized image (H = 2 OH, W = 2 OW: the ResNet stem), one thread per
// (n, a, b, 8 channels) owning the 2 x 2 input block rows 2a, 2a + 1 x columns 2b, 2b + 1: row 2a lies only in window
// row a (tap row 1), row 2a + 1 in window rows a (tap row 2) and a + 1 (tap row 0); columns likewise. The four windows
// (a | a + 1) x (b | b + 1) are loaded once for the four input pixels instead of once per input pixel, and the
// per-pixel sums run in the general kernel's window order (bit-identical results).
template <typename I>
__global__ __launch_bounds__(kThreads) void maxpool_bwd_even(const __hip_bfloat16* __restrict__ dy,
                                                            const uint8_t* __restrict__ idx, int N, int C, int OH,
                                                            int OW, __hip_bfloat16* __restrict__ dx) {
  const int cg = C / kVec, H = 2 * OH, W = 2 * OW;
  const I total = (I)N * OH * OW * cg;
  for (I t = (I)blockIdx.x * kThreads + threadIdx.x; t < total; t += (I)gridDim.x * kThreads) {
    const int g = (int)(t % cg);
    I p = t / cg;
    const int b = (int)(p % OW);
    p /= OW;
    const int a = (int)(p % OH);
    const int n = (int)(p / OH);
    // windows [wa][wb] = (a + wa, b + wb); absent ones (past the last row / column) route nothing
    U8x8 k8[2][2];
    Bf8 d8[2][2];
#pragma unroll
    for (int wa = 0; wa < 2; ++wa)
#pragma unroll
      for (int wb = 0; wb < 2; ++wb) {
        if (a + wa < OH && b + wb < OW) {
          const size_t off = (((size_t)n * OH + a + wa) * OW + b + wb) * C + g * kVec;
          k8[wa][wb] = *(const U8x8*)(idx + off);
          d8[wa][wb] = *(const Bf8*)(dy + off);
        } else {
#pragma unroll
          for (int e = 0; e < kVec; ++e) k8[wa][wb].v[e] = kNone;
        }
      }
    // input pixel (2a + sh, 2b + sw): window (a + wa, b + wb) contributes when it contains it -- wa = 0 always,
    // wa = 1 only for sh = 1 (likewise columns) -- at tap (sh ? (wa ? 0 : 2) : 1, sw ? (wb ? 0 : 2) : 1)
#pragma unroll
    for (int sh = 0; sh < 2; ++sh)
#pragma unroll
      for (int sw = 0; sw < 2; ++sw) {
        float acc[kVec];
#pragma unroll
        for (int e = 0; e < kVec; ++e) acc[e] = 0.f;
#pragma unroll
        for (int wa = 0; wa <= sh; ++wa)
#pragma unroll
          for (int wb = 0; wb <= sw; ++wb) {
            const uint8_t k = (uint8_t)((sh ? (wa ? 0 : 2) : 1) * 3 + (sw ? (wb ? 0 : 2) : 1));
#pragma unroll
            for (int e = 0; e < kVec; ++e)
              if (k8[wa][wb].v[e] == k) acc[e] += __bfloat162float(d8[wa][wb].v[e]);
          }
        Bf8 o;
#pragma unroll
        for (int e = 0; e < kVec; ++e) o.v[e] = __float2bfloat16(acc[e]);
        *(Bf8*)(dx + (((size_t)n * H + 2 * a + sh) * W + 2 * b + sw) * C + g * kVec) = o;
      }
  }
}

int grid_for(long long total) {
  long long g = (total + kThreads - 1) / kThreads;
  if (g > 65536) g = 65536;
  return g < 1 ? 1 : (int)g;
}

// 32-bit indices when total + one grid stride stays below 2^32 (the grid-stride loop's last increment)
bool pair_off() {  // MIFX_POOL_PAIR=0: one window per thread in the forward (A/B)
  static const bool off = getenv("MIFX_POOL_PAIR") && getenv("MIFX_POOL_PAIR")[0] == '0';
  return off;
}
bool even_off() {  // MIFX_POOL_EVEN=0: the general gather kernel for the stem too (A/B)
  static const bool off = getenv("MIFX_POOL_EVEN") && getenv("MIFX_POOL_EVEN")[0] == '0';
  return off;
}
bool small_index(long long total) { return total + 65536LL * kThreads < (1LL << 32); }

}  // namespace

extern "C" {

// x, y, dx: NHWC bf16 (channels_last), C % 8 == 0, 16-byte aligned; idx: [N, OH, OW, C] uint8. relu != 0: the pool
// of relu(x) (y = max(window max, 0); a window whose max is <= 0 routes no gradient). Window (oh, ow)
// covers rows 2 oh - pt .. 2 oh - pt + 2 (columns likewise with pl); taps outside the image never win, and every
// window must hold at least one tap of the image.
int mifx_maxpool3s2p_fwd(const void* x, int N, int H, int W, int C, int pt, int pl, int OH, int OW, int relu, void* y,
                         void* idx, hipStream_t st) {
  if (N <= 0 || H <= 0 || W <= 0 || C <= 0 || C % kVec || pt < 0 || pt > 2 || pl < 0 || pl > 2 || OH <= 0 ||
      OW <= 0 || 2 * (OH - 1) - pt >= H || 2 * (OW - 1) - pl >= W)
    return -1;
  if (!pair_off()) {
    const long long tp = (long long)N * OH * ((OW + 1) / 2) * (C / kVec);
    if (small_index(tp))
      hipLaunchKernelGGL(maxpool_fwd2<uint32_t>, dim3(grid_for(tp)), dim3(kThreads), 0, st, (const __hip_bfloat16*)x, N,
                         H, W, C, OH, OW, pt, pl, relu, (__hip_bfloat16*)y, (uint8_t*)idx);
    else
      hipLaunchKernelGGL(maxpool_fwd2<long long>, dim3(grid_for(tp)), dim3(kThreads), 0, st, (const __hip_bfloat16*)x,
                         N, H, W, C, OH, OW, pt, pl, relu, (__hip_bfloat16*)y, (uint8_t*)idx);
    return (int)hipGetLastError();
  }
  const long long total = (long long)N * OH * OW * (C / kVec);
  if (small_index(total))
    hipLaunchKernelGGL(maxpool_fwd<uint32_t>, dim3(grid_for(total)), dim3(kThreads), 0, st, (const __hip_bfloat16*)x, N,
                       H, W, C, OH, OW, pt, pl, relu, (__hip_bfloat16*)y, (uint8_t*)idx);
  else
    hipLaunchKernelGGL(maxpool_fwd<long long>, dim3(grid_for(total)), dim3(kThreads), 0, st, (const __hip_bfloat16*)x,
                       N, H, W, C, OH, OW, pt, pl, relu, (__hip_bfloat16*)y, (uint8_t*)idx);
  return (int)hipGetLastError();
}

int mifx_maxpool3s2p_bwd(const void* dy, const void* idx, int N, int H, int W, int C, int pt, int pl, int OH, int OW,
                         void* dx, hipStream_t st) {
  if (N <= 0 || H <= 0 || W <= 0 || C <= 0 || C % kVec || pt < 0 || pt > 2 || pl < 0 || pl > 2 || OH <= 0 ||
      OW <= 0)
    return -1;
  if (pt == 1 && pl == 1 && H == 2 * OH && W == 2 * OW && !even_off()) {
    const long long te = (long long)N * OH * OW * (C / kVec);
    if (small_index(te))
      hipLaunchKernelGGL(maxpool_bwd_even<uint32_t>, dim3(grid_for(te)), dim3(kThreads), 0, st,
                         (const __hip_bfloat16*)dy, (const uint8_t*)idx, N, C, OH, OW, (__hip_bfloat16*)dx);
    else
      hipLaunchKernelGGL(maxpool_bwd_even<long long>, dim3(grid_for(te)), dim3(kThreads), 0, st,
                         (const __hip_bfloat16*)dy, (const uint8_t*)idx, N, C, OH, OW, (__hip_bfloat16*)dx);
    return (int)hipGetLastError();
  }
  const long long total = (long long)N * H * W * (C / kVec);
  if (small_index(total))
    hipLaunchKernelGGL(maxpool_bwd<uint32_t>, dim3(grid_for(total)), dim3(kThreads), 0, st, (const __hip_bfloat16*)dy,
                       (const uint8_t*)idx, N, H, W, C, OH, OW, pt, pl, (__hip_bfloat16*)dx);
  else
    hipLaunchKernelGGL(maxpool_bwd<long long>, dim3(grid_for(total)), dim3(kThreads), 0, st, (const __hip_bfloat16*)dy,
                       (const uint8_t*)idx, N, H, W, C, OH, OW, pt, pl, (__hip_bfloat16*)dx);
  return (int)hipGetLastError();
}

// ResNet stem: pad 1, OH = (H - 1) / 2 + 1
int mifx_maxpool3s2_fwd(const void* x, int N, int H, int W, int C, void* y, void* idx, hipStream_t st) {
  return mifx_maxpool3s2p_fwd(x, N, H, W, C, 1, 1, (H - 1) / 2 + 1, (W - 1) / 2 + 1, 0, y, idx, st);
}

int mifx_maxpool3s2_bwd(const void* dy, const void* idx, int N, int H, int W, int C, void* dx, hipStream_t st) {
  return mifx_maxpool3s2p_bwd(dy, idx, N, H, W, C, 1, 1, (H - 1) / 2 + 1, (W - 1) / 2 + 1, dx, st);
}

}  // extern "C"
