// Flat mixed-precision AdamW for gfx950: bf16 model weights + bf16 gradients in two flat buffers,
// fp32 master weights and moments. One launch updates every parameter of the model.
//
// Why (profiles/archive/bert_base_steady_kernels_r1.md, BERT-base B=32 S=128): with fp32 parameters under
// bf16 autocast every step re-casts each weight to bf16 for the forward (103 copy kernels) and casts
// each bf16 weight-gradient back to fp32 (91 kernels), ~0.8 ms, and torch's fused AdamW runs as 6
// multi-tensor launches (~0.77 ms). Keeping the model itself in bf16 (views into one flat buffer)
// and the fp32 master state here removes the casts; the update reads g (2 B) + master/m/v (12 B)
// and writes master/m/v (12 B) + the bf16 weight (2 B) = 28 B/param, one pass, 16-byte accesses.
//
// Graph-capturable: the step counter lives on the device (bias corrections are computed from it
// in-kernel; a 1-thread kernel advances it after the update), so a captured step replays correctly.
#include <hip/hip_bf16.h>
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

constexpr int kThreads = 256;
constexpr int kVec = 8;

struct alignas(16) Bf8 {
  __hip_bfloat16 v[kVec];
};

__global__ __launch_bounds__(kThreads) void adamw_flat(__hip_bfloat16* __restrict__ param,
                                                      const __hip_bfloat16* __restrict__ grad,
                                                      float* __restrict__ master, float* __restrict__ m,
                                                      float* __restrict__ v, long long n, const int* __restrict__ step,
                                                      float lr, float beta1, float beta2, float eps, float wd,
                                                      float grad_scale) {
  const int t = *step + 1;
  const float bc1 = 1.f - powf(beta1, (float)t), bc2 = 1.f - powf(beta2, (float)t);
  const float step_size = lr / bc1, inv_sqrt_bc2 = rsqrtf(bc2);
  const long long nvec = n / kVec;
  for (long long i = (long long)blockIdx.x * kThreads + threadIdx.x; i < nvec; i += (long long)gridDim.x * kThreads) {
    const long long o = i * kVec;
    const Bf8 g8 = *(const Bf8*)(grad + o);
    float w[kVec], mm[kVec], vv[kVec];
    *(float4*)&w[0] = *(const float4*)(master + o);
    *(float4*)&w[4] = *(const float4*)(master + o + 4);
    *(float4*)&mm[0] = *(const float4*)(m + o);
    *(float4*)&mm[4] = *(const float4*)(m + o + 4);
    *(float4*)&vv[0] = *(const float4*)(v + o);
    *(float4*)&vv[4] = *(const float4*)(v + o + 4);
    Bf8 p8;
#pragma unroll
    for (int e = 0; e < kVec; ++e) {
      const float g = __bfloat162float(g8.v[e]) * grad_scale;
      mm[e] = fmaf(beta1, mm[e], (1.f - beta1) * g);
      vv[e] = fmaf(beta2, vv[e], (1.f - beta2) * g * g);
      const float denom = sqrtf(vv[e]) * inv_sqrt_bc2 + eps;
      w[e] = w[e] * (1.f - lr * wd) - step_size * mm[e] / denom;  // decoupled weight decay (AdamW)
      p8.v[e] = __float2bfloat16(w[e]);
    }
    *(float4*)(master + o) = *(float4*)&w[0];
    *(float4*)(master + o + 4) = *(float4*)&w[4];
    *(float4*)(m + o) = *(float4*)&mm[0];
    *(float4*)(m + o + 4) = *(float4*)&mm[4];
    *(float4*)(v + o) = *(float4*)&vv[0];
    *(float4*)(v + o + 4) = *(float4*)&vv[4];
    *(Bf8*)(param + o) = p8;
  }
  // scalar tail (n % 8), handled by block 0
  if (blockIdx.x == 0) {
    for (long long i = nvec * kVec + threadIdx.x; i < n; i += kThreads) {
      const float g = __bfloat162float(grad[i]) * grad_scale;
      m[i] = fmaf(beta1, m[i], (1.f - beta1) * g);
      v[i] = fmaf(beta2, v[i], (1.f - beta2) * g * g);
      master[i] = master[i] * (1.f - lr * wd) - step_size * m[i] / (sqrtf(v[i]) * inv_sqrt_bc2 + eps);
      param[i] = __float2bfloat16(master[i]);
    }
  }
}

// Same update, but each parameter's gradient is read from its OWN tensor (the one autograd produced),
// so the step needs neither a zero-fill of a flat gradient buffer nor the per-parameter in-place
// accumulate (`grad += new`) autograd runs when .grad is a pre-existing view: on BERT-base that was
// 201 add kernels (~1.0 ms) + a 220 MB fill per step (profiles/archive/bert_base_steady_kernels_s3.md).
// Workgroup b updates chunk b: parameter bp[b], elements [bo[b], bo[b] + bn[b]) of it; gptr[param] is the
// gradient's device address this step (0 = no gradient: the parameter is left untouched, as torch's
// AdamW skips params whose .grad is None), poff[param] its (8-aligned) offset in the flat buffers.
// (Non-temporal loads / stores of master / m / v measured slower on the BERT-base step: 5049-5070 vs 5193-5208
// seq/s, profiles/bert_adamw_nt_ab_r4.txt.)
constexpr int kChunk = kThreads * kVec;  // 2048 elements per workgroup: one 16-B vector per thread,
                                          // all loads in flight at once

__global__ __launch_bounds__(kThreads) void adamw_chunks(
    __hip_bfloat16* __restrict__ param, const unsigned long long* __restrict__ gptr,
    const long long* __restrict__ poff, const int* __restrict__ bp, const int* __restrict__ bo,
    const int* __restrict__ bn, float* __restrict__ master, float* __restrict__ m, float* __restrict__ v,
    const int* __restrict__ step, float lr, float beta1, float beta2, float eps, float wd, float grad_scale) {
  const int pi = bp[blockIdx.x];
  const __hip_bfloat16* grad = (const __hip_bfloat16*)gptr[pi];
  if (grad == nullptr) return;
  const int t = *step + 1;
  const float bc1 = 1.f - powf(beta1, (float)t), bc2 = 1.f - powf(beta2, (float)t);
  const float step_size = lr / bc1, inv_sqrt_bc2 = rsqrtf(bc2);
  const int o0 = bo[blockIdx.x], n = bn[blockIdx.x];
  const long long f0 = poff[pi] + o0;  // flat index of the chunk's first element (multiple of 8)
  grad += o0;
  const bool vec_ok = ((o0 | (int)((unsigned long long)grad & 15)) & 7) == 0;  // 16-B aligned gradient
  const int nvec = vec_ok ? n / kVec : 0;
  for (int i = threadIdx.x; i < nvec; i += kThreads) {
    const long long o = f0 + (long long)i * kVec;
    const Bf8 g8 = *(const Bf8*)(grad + i * kVec);
    float w[kVec], mm[kVec], vv[kVec];
    *(float4*)&w[0] = *(const float4*)(master + o);
    *(float4*)&w[4] = *(const float4*)(master + o + 4);
    *(float4*)&mm[0] = *(const float4*)(m + o);
    *(float4*)&mm[4] = *(const float4*)(m + o + 4);
    *(float4*)&vv[0] = *(const float4*)(v + o);
    *(float4*)&vv[4] = *(const float4*)(v + o + 4);
    Bf8 p8;
#pragma unroll
    for (int e = 0; e < kVec; ++e) {
      const float g = __bfloat162float(g8.v[e]) * grad_scale;
      mm[e] = fmaf(beta1, mm[e], (1.f - beta1) * g);
      vv[e] = fmaf(beta2, vv[e], (1.f - beta2) * g * g);
      const float denom = sqrtf(vv[e]) * inv_sqrt_bc2 + eps;
      w[e] = w[e] * (1.f - lr * wd) - step_size * mm[e] / denom;
      p8.v[e] = __float2bfloat16(w[e]);
    }
    *(float4*)(master + o) = *(float4*)&w[0];
    *(float4*)(master + o + 4) = *(float4*)&w[4];
    *(float4*)(m + o) = *(float4*)&mm[0];
    *(float4*)(m + o + 4) = *(float4*)&mm[4];
    *(float4*)(v + o) = *(float4*)&vv[0];
    *(float4*)(v + o + 4) = *(float4*)&vv[4];
    *(Bf8*)(param + o) = p8;
  }
  for (int i = nvec * kVec + threadIdx.x; i < n; i += kThreads) {  // tail / unaligned gradient
    const long long o = f0 + i;
    const float g = __bfloat162float(grad[i]) * grad_scale;
    m[o] = fmaf(beta1, m[o], (1.f - beta1) * g);
    v[o] = fmaf(beta2, v[o], (1.f - beta2) * g * g);
    master[o] = master[o] * (1.f - lr * wd) - step_size * m[o] / (sqrtf(v[o]) * inv_sqrt_bc2 + eps);
    param[o] = __float2bfloat16(master[o]);
  }
}

__global__ void advance_step(int* step) { *step += 1; }

}  // namespace

extern "C" {

int mifx_adamw_flat(void* param, const void* grad, float* master, float* m, float* v, long long n, int* step, float lr,
                    float beta1, float beta2, float eps, float wd, float grad_scale, hipStream_t st) {
  if (n <= 0) return -1;
  long long g = (n / kVec + kThreads - 1) / kThreads;
  if (g > 4096) g = 4096;
  if (g < 1) g = 1;
  hipLaunchKernelGGL(adamw_flat, dim3((unsigned)g), dim3(kThreads), 0, st, (__hip_bfloat16*)param,
                     (const __hip_bfloat16*)grad, master, m, v, n, step, lr, beta1, beta2, eps, wd, grad_scale);
  hipLaunchKernelGGL(advance_step, dim3(1), dim3(1), 0, st, step);
  return (int)hipGetLastError();
}

int mifx_adamw_chunk_size() { return kChunk; }

int mifx_adamw_chunks(void* param, const unsigned long long* gptr, const long long* poff, const int* bp, const int* bo,
                      const int* bn, int nblocks, float* master, float* m, float* v, int* step, float lr, float beta1,
                      float beta2, float eps, float wd, float grad_scale, hipStream_t st) {
  if (nblocks <= 0) return -1;
  hipLaunchKernelGGL(adamw_chunks, dim3((unsigned)nblocks), dim3(kThreads), 0, st, (__hip_bfloat16*)param, gptr, poff,
                     bp, bo, bn, master, m, v, step, lr, beta1, beta2, eps, wd, grad_scale);
  hipLaunchKernelGGL(advance_step, dim3(1), dim3(1), 0, st, step);
  return (int)hipGetLastError();
}

// the chunk kernel WITHOUT the step advance (a step split into several launches, e.g. per gradient bucket overlapped
// with the backward: every launch reads the same step, mifx_adamw_advance runs once after all of them)
int mifx_adamw_chunks_noadv(void* param, const unsigned long long* gptr, const long long* poff, const int* bp,
                            const int* bo, const int* bn, int nblocks, float* master, float* m, float* v, int* step,
                            float lr, float beta1, float beta2, float eps, float wd, float grad_scale,
                            hipStream_t st) {
  if (nblocks <= 0) return -1;
  hipLaunchKernelGGL(adamw_chunks, dim3((unsigned)nblocks), dim3(kThreads), 0, st, (__hip_bfloat16*)param, gptr, poff,
                     bp, bo, bn, master, m, v, step, lr, beta1, beta2, eps, wd, grad_scale);
  return (int)hipGetLastError();
}

int mifx_adamw_advance(int* step, hipStream_t st) {
  hipLaunchKernelGGL(advance_step, dim3(1), dim3(1), 0, st, step);
  return (int)hipGetLastError();
}

}  // extern "C"
