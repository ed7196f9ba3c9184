// Per-step weight preparation for the GEMM-shaped convolutions of ResNet-50 (BASELINE config 5), in ONE launch.
//
// The implicit-GEMM convolutions (csrc/gemm8.hip) read bf16 weights in two layouts each step: the forward operand
// (1x1: [Cout][C]; 3x3: the channels_last [Cout][3][3][C]) and the input-gradient operand (1x1: W^T [C][Cout]; 3x3:
// flipped and transposed [C][3][3][Cout]). Casting and transposing them per convolution cost ~100 small launches per
// step (profiles/resnet_steady_r5l.md: 56 casts, 24 permute / flip copies, transposes). Here a job table (built once,
// device-resident) lists every (source fp32, destination bf16, geometry) and one kernel walks it:
//   * copy jobs: dst[i] = bf16(src[i]) over n elements, 2048 per workgroup (8 per thread, 16-byte loads);
//   * transpose jobs: dst[c * dld + r] = bf16(src[r * sld + c]) for r < R, c < C, 64 x 64 tiles through LDS
//     (coalesced 256-byte row reads, 128-byte row writes). A 3x3 flip-transpose is 9 such jobs, one per tap.
// Workgroups find their job by binary search over the jobs' first work-item indices.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

typedef __bf16 bf16;

struct Job {
  const float* src;
  bf16* dst;
  long long n;     // copy: element count
  int R, C;        // transpose: source rows / columns
  int sld, dld;    // row strides (elements)
  int first;       // first work item of this job
  int kind;        // 0 copy, 1 transpose
};

constexpr int COPY_ITEM = 2048;

__global__ __launch_bounds__(256) void weight_prep(const Job* __restrict__ jobs, int njobs) {
  const int item = blockIdx.x;
  int lo = 0, hi = njobs - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (jobs[mid].first <= item) lo = mid; else hi = mid - 1;
  }
  const Job j = jobs[lo];
  const int local = item - j.first;
  if (j.kind == 0) {
    const long long base = (long long)local * COPY_ITEM + threadIdx.x * 8;
    if (base + 8 <= j.n) {
      const float4 a = *(const float4*)(j.src + base), b = *(const float4*)(j.src + base + 4);
      bf16 o[8] = {(bf16)a.x, (bf16)a.y, (bf16)a.z, (bf16)a.w, (bf16)b.x, (bf16)b.y, (bf16)b.z, (bf16)b.w};
      *(uint4*)(j.dst + base) = *(const uint4*)o;
    } else {
      for (long long q = base; q < j.n && q < base + 8; ++q) j.dst[q] = (bf16)j.src[q];
    }
    return;
  }
  __shared__ float tile[64][65];
  const int tc = j.C / 64, r0 = (local / tc) * 64, c0 = (local % tc) * 64;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;  // 4 rows per pass
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int r = ty + 4 * k;
    tile[r][tx] = j.src[(size_t)(r0 + r) * j.sld + c0 + tx];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < 16; ++k) {
    const int c = ty + 4 * k;
    j.dst[(size_t)(c0 + c) * j.dld + r0 + tx] = (bf16)tile[tx][c];
  }
}

}  // namespace

extern "C" {

int mifx_weight_prep_job_bytes() { return (int)sizeof(Job); }

// Fill a host job record (the caller packs them into a device table). kind 0: copy n elements; kind 1: transpose
// R x C (both % 64) with row strides sld / dld. Returns the job's work-item count, < 0 on bad arguments.
int mifx_weight_prep_job(void* out, int kind, const void* src, void* dst, long long n, int R, int C, int sld, int dld,
                         int first) {
  if (out == nullptr || src == nullptr || dst == nullptr || first < 0) return -1;
  Job j{(const float*)src, (bf16*)dst, n, R, C, sld, dld, first, kind};
  int items;
  if (kind == 0) {
    if (n <= 0 || (uintptr_t)src % 16 || (uintptr_t)dst % 16) return -1;
    items = (int)((n + COPY_ITEM - 1) / COPY_ITEM);
  } else if (kind == 1) {
    if (R <= 0 || C <= 0 || R % 64 || C % 64 || sld < C || dld < R) return -1;
    items = (R / 64) * (C / 64);
  } else {
    return -1;
  }
  __builtin_memcpy(out, &j, sizeof(Job));
  return items;
}

int mifx_weight_prep(const void* jobs, int njobs, int items, hipStream_t st) {
  if (jobs == nullptr || njobs <= 0 || items <= 0) return -1;
  hipLaunchKernelGGL(weight_prep, dim3(items), dim3(256), 0, st, (const Job*)jobs, njobs);
  return (int)hipGetLastError();
}

}  // extern "C"
