// Image input pipeline kernel for gfx950: random-crop + horizontal flip + normalize, uint8 NHWC -> bf16 NHWC.
//
// BASELINE config 5 (ResNet-50 image pipeline, DP=8): the dataset lives in HBM as uint8 NHWC
// (288 GB per GPU holds ~1.9M 256x256x3 images), so the per-step input work is a gather of the
// batch's images fused with augmentation and normalisation into the bf16 channels_last tensor
// the first convolution consumes — one read of B*256*256*3 bytes and one write of B*224*224*3*2.
//
// grid (ceil(W_out*C / (kThreads*kVec)), H_out, B): block row = one output row of one image;
// each thread writes kVec consecutive channel-interleaved elements (16-byte bf16 stores).
// Per-image crop offsets and the flip bit come from an in-kernel Philox4x32-10 keyed by
// (seed) with counter (image slot, step), so augmentation is reproducible and needs no host RNG.
#include <hip/hip_bf16.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

constexpr int kThreads = 128;
constexpr int kVec = 8;

struct U4 {
  uint32_t x, y, z, w;
};

__device__ __forceinline__ U4 philox(U4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c.x;
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c.z;
    c = U4{(uint32_t)(p1 >> 32) ^ c.y ^ k0, (uint32_t)p1, (uint32_t)(p0 >> 32) ^ c.w ^ k1, (uint32_t)p0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

template <typename TOut>
__device__ __forceinline__ TOut cvt(float v);
template <>
__device__ __forceinline__ float cvt<float>(float v) {
  return v;
}
template <>
__device__ __forceinline__ __hip_bfloat16 cvt<__hip_bfloat16>(float v) {
  return __float2bfloat16(v);
}

template <typename TOut>
__global__ __launch_bounds__(kThreads) void crop_flip_norm(const uint8_t* __restrict__ src, const int* __restrict__ idx,
                                                          int Hin, int Win, int C, int Hout, int Wout, int train,
                                                          uint32_t seed_lo, uint32_t seed_hi, uint32_t step,
                                                          const long long* __restrict__ step_dev,
                                                          const float* __restrict__ mean,
                                                          const float* __restrict__ inv_std,
                                                          TOut* __restrict__ out) {
  const int b = blockIdx.z, y = blockIdx.y;
  int oy, ox, flip;
  if (train) {
    if (step_dev) step = (uint32_t)step_dev[0];  // device step counter (captured hipGraph steps)
    const U4 r = philox(U4{(uint32_t)b, step, 0x1234u, 0u}, seed_lo, seed_hi);
    oy = (int)(r.x % (uint32_t)(Hin - Hout + 1));
    ox = (int)(r.y % (uint32_t)(Win - Wout + 1));
    flip = (int)(r.z & 1u);
  } else {
    oy = (Hin - Hout) / 2;
    ox = (Win - Wout) / 2;
    flip = 0;
  }
  const uint8_t* row = src + ((size_t)idx[b] * Hin + (oy + y)) * (size_t)Win * C;
  TOut* orow = out + ((size_t)b * Hout + y) * (size_t)Wout * C;
  const int rowlen = Wout * C;
  const int e0 = (blockIdx.x * kThreads + threadIdx.x) * kVec;
#pragma unroll
  for (int k = 0; k < kVec; ++k) {
    const int e = e0 + k;
    if (e < rowlen) {
      const int x = e / C, c = e - x * C;
      const int sx = ox + (flip ? (Wout - 1 - x) : x);
      const float v = (float)row[sx * C + c] * (1.0f / 255.0f);
      orow[e] = cvt<TOut>((v - mean[c]) * inv_std[c]);
    }
  }
}

}  // namespace

extern "C" {

// src: [N, Hin, Win, C] uint8; idx: [B] int32 image ids; out: [B, Hout, Wout, C] (dtype 0 fp32, 1 bf16).
// step_dev (optional): device int64 read by the kernel in place of `step` (a graph replayed every step)
int mifx_img_crop_flip_norm(const uint8_t* src, const int* idx, int B, int Hin, int Win, int C, int Hout, int Wout,
                            int train, unsigned long long seed, unsigned int step, const long long* step_dev,
                            const float* mean,
                            const float* inv_std, int dtype, void* out, hipStream_t st) {
  if (B <= 0 || Hout > Hin || Wout > Win || C <= 0 || C > 4) return -1;
  const dim3 grid((Wout * C + kThreads * kVec - 1) / (kThreads * kVec), Hout, B);
  if (dtype)
    hipLaunchKernelGGL(crop_flip_norm<__hip_bfloat16>, grid, dim3(kThreads), 0, st, src, idx, Hin, Win, C, Hout, Wout,
                       train, (uint32_t)seed, (uint32_t)(seed >> 32), step, step_dev, mean, inv_std, (__hip_bfloat16*)out);
  else
    hipLaunchKernelGGL(crop_flip_norm<float>, grid, dim3(kThreads), 0, st, src, idx, Hin, Win, C, Hout, Wout, train,
                       (uint32_t)seed, (uint32_t)(seed >> 32), step, step_dev, mean, inv_std, (float*)out);
  return (int)hipGetLastError();
}

}  // extern "C"
