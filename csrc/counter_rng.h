// Counter-based dropout masks shared by the BERT kernels (csrc/fused_bert.hip, csrc/attention.hip).
// rng points at device int64 [seed, step counter]; the counter is advanced by an in-graph op once per step, so
// captured hipGraphs draw fresh masks on every replay without host state. A 64-bit finaliser (murmur3 fmix64) of
// (seed, counter, site) gives the per-call key; each group of 4 consecutive elements (flat index 4g..4g+3) takes
// the four 16-bit lanes of mix64(key + g * golden) and keeps element e iff lane_e >= thr (thr = round(p * 65536)).
// mifx.ops.fused_bert.keep_mask is the host twin (bit-identical).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mifx_rng {

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z ^= z >> 33;
  z *= 0xff51afd7ed558ccdULL;
  z ^= z >> 33;
  z *= 0xc4ceb9fe1a85ec53ULL;
  z ^= z >> 33;
  return z;
}
constexpr uint64_t kGolden = 0x9E3779B97F4A7C15ULL;

__device__ __forceinline__ uint64_t drop_key(const int64_t* rng, int site) {
  return mix64((uint64_t)rng[0] ^ mix64((uint64_t)rng[1] * kGolden + (uint64_t)site));
}
__device__ __forceinline__ uint32_t keep4(uint64_t key, uint64_t g, uint32_t thr) {
  const uint64_t h = mix64(key + g * kGolden);
  return (uint32_t)((h & 0xffff) >= thr) | ((uint32_t)(((h >> 16) & 0xffff) >= thr) << 1) |
         ((uint32_t)(((h >> 32) & 0xffff) >= thr) << 2) | ((uint32_t)((h >> 48) >= thr) << 3);
}

}  // namespace mifx_rng
