// Multi-tensor SGD (weight decay, momentum, dampening, Nesterov) for gfx950: one launch updates every fp32 parameter
// of a model in place from its own gradient and momentum tensors.
//
// Why (profiles/archive/resnet_steady_r5za.md, ResNet-50 B=256): torch.optim.SGD's captured update is six _foreach
// passes per parameter group (wd add, momentum mul, momentum add, Nesterov add, lr mul, param add) -- 14
// multi_tensor_apply launches, ~280 us per step -- each re-reading and re-writing the 25.6 M fp32 values. Here each
// element is read once (param, grad, momentum: 12 B) and written once (param, momentum: 8 B), in one launch.
//
// Semantics (torch.optim.SGD, foreach path): g' = g + wd p; buf = mom buf + (1 - damp) g';
// u = nesterov ? g' + mom buf : buf; p += neg_lr u, with neg_lr = -lr read from device memory (a replayed graph
// follows the learning-rate schedule). fp32 throughout; results match the foreach reference to fp32 rounding (FMA
// contraction may differ), not bit for bit.
//
// Workgroup b updates chunk b: tensor tp[b], elements [to[b], to[b] + tn[b]); per tensor: param / grad / momentum
// device addresses and its weight decay.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

constexpr int kThreads = 256;
constexpr int kChunk = kThreads * 8;  // 2048 fp32 per workgroup: two float4 per thread

struct SgdArgs {
  const unsigned long long *pp, *gp, *bp;  // [P] param / grad / momentum addresses
  const float* wd;                         // [P]
  const int *tp, *to, *tn;                 // [nblocks] chunk -> (tensor, offset, length)
  const float* neg_lr;                     // device scalar: -lr
  float mom, damp;
  int nesterov;
};

__device__ __forceinline__ void sgd1(float& p, float g, float& b, float wd, float mom, float damp, bool nest,
                                     float nlr) {
  const float gg = g + wd * p;
  b = mom * b + (1.f - damp) * gg;
  const float u = nest ? gg + mom * b : b;
  p = p + nlr * u;
}

__global__ __launch_bounds__(kThreads) void sgd_chunks(const SgdArgs a) {
  const int ti = a.tp[blockIdx.x];
  float* p = (float*)a.pp[ti];
  const float* g = (const float*)a.gp[ti];
  float* b = (float*)a.bp[ti];
  const int o0 = a.to[blockIdx.x], n = a.tn[blockIdx.x];
  p += o0;
  g += o0;
  b += o0;
  const float wd = a.wd[ti], nlr = *a.neg_lr, mom = a.mom, damp = a.damp;
  const bool nest = a.nesterov != 0;
  const bool vec = (((unsigned long long)p | (unsigned long long)g | (unsigned long long)b) & 15) == 0;
  const int nv = vec ? n / 4 : 0;
  float4 pv[2], gv[2], bv[2];
#pragma unroll
  for (int u = 0; u < 2; ++u) {  // both vectors' loads in flight before the first update
    const int i = threadIdx.x + u * kThreads;
    if (i < nv) {
      pv[u] = ((const float4*)p)[i];
      gv[u] = ((const float4*)g)[i];
      bv[u] = ((const float4*)b)[i];
    }
  }
#pragma unroll
  for (int u = 0; u < 2; ++u) {
    const int i = threadIdx.x + u * kThreads;
    if (i >= nv) break;
    sgd1(pv[u].x, gv[u].x, bv[u].x, wd, mom, damp, nest, nlr);
    sgd1(pv[u].y, gv[u].y, bv[u].y, wd, mom, damp, nest, nlr);
    sgd1(pv[u].z, gv[u].z, bv[u].z, wd, mom, damp, nest, nlr);
    sgd1(pv[u].w, gv[u].w, bv[u].w, wd, mom, damp, nest, nlr);
    ((float4*)p)[i] = pv[u];
    ((float4*)b)[i] = bv[u];
  }
  for (int i = nv * 4 + threadIdx.x; i < n; i += kThreads) {  // tail / unaligned tensor
    float pp = p[i], bb = b[i];
    sgd1(pp, g[i], bb, wd, mom, damp, nest, nlr);
    p[i] = pp;
    b[i] = bb;
  }
}

}  // namespace

extern "C" {

int mifx_sgd_chunk_size() { return kChunk; }

int mifx_sgd_chunks(const unsigned long long* pp, const unsigned long long* gp, const unsigned long long* bp,
                    const float* wd, const int* tp, const int* to, const int* tn, int nblocks, const float* neg_lr,
                    float mom, float damp, int nesterov, hipStream_t st) {
  if (nblocks <= 0 || pp == nullptr || gp == nullptr || bp == nullptr || wd == nullptr || neg_lr == nullptr) return -1;
  const SgdArgs a{pp, gp, bp, wd, tp, to, tn, neg_lr, mom, damp, nesterov};
  hipLaunchKernelGGL(sgd_chunks, dim3((unsigned)nblocks), dim3(kThreads), 0, st, a);
  return (int)hipGetLastError();
}

}  // extern "C"
