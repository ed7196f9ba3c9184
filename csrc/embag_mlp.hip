// KFP taxi DNN (one-hot indicator columns -> hidden 1500 -> 1 logit) as gather / scatter kernels.
//
// Reference: `kubeflow-pipelines/taxi/preprocessing.py:104-124` builds a
// 6,170-wide one-hot input (13 indicator columns + 3 numeric) that TF multiplies by a dense
// 6170x1500 W1 (`hidden_layer_size='1500'`, Adagrad lr 0.1, 3,000 steps). A one-hot row times W1
// is a row gather, so:
//   forward  z_b = b1 + sum_f W1[row_bf] + sum_d x_bd W1[dense_d];  a_b = relu(z_b);
//            logit_b = a_b . w2 + b2;  loss_b = BCE(logit_b, y_b)
//   backward dz_b = (sigmoid(logit_b) - y_b) * w2 * [z_b > 0]
// and, because Adagrad leaves rows with zero gradient untouched (acc += 0, w -= 0), the optimizer
// only needs to visit the <= B*13 distinct gathered rows plus the dense parameters — exactly the
// TF result at a fraction of the 9.26M-parameter dense update.
//
//  * tdnn_fwd + tdnn_head_bwd: grid (B, H/256) — each thread gathers its hidden unit from the 16
//    rows (coalesced across the wave), partial logits per block, then logit/BCE/dz per example.
//  * tdnn_sparse_adagrad: one workgroup per (example, field) pair; the pair that holds the FIRST
//    occurrence of its row in the batch (fields own disjoint row ranges, so only the same field can
//    repeat a row) lists every example that touched the row, sums their dz in ascending example order
//    (deterministic, no atomics, no sort) and applies acc += g^2; w -= lr * g * rsqrt(acc); the other
//    pairs exit. No host-side sort/unique (whose dynamic output size forced a device->host sync per
//    step), so the whole step is hipGraph-capturable.
//  * Batch selection on the device: example b of a step is the record the feed of csrc/feed.h gives for stream
//    position step_ctr[0] * stride + offset + b of the resident dataset (optionally shuffled per epoch; or a fixed
//    start, stored order), and tdnn_dense_apply advances step_ctr at the end of the step -- replayed graphs walk
//    through the data with no host work.
//  * tdnn_dense_partial + tdnn_dense_apply: batch-chunked reductions for the dense W1 rows, b1, w2
//    (grid H/256 x chunks), then a fixed-order combine and the same update; block 0 updates b2. Up to
//    64 examples tdnn_head_bwd writes one chunk per example itself (no tdnn_dense_partial launch).
#include <hip/hip_runtime.h>
#include "feed.h"
#include <stdint.h>

namespace {

constexpr int kThreads = 256;
constexpr int kMaxH = 4096;
constexpr int kMaxFields = 32;
constexpr int kMaxDense = 8;

__device__ __forceinline__ float block_sum(float v, float* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) red[w] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < kThreads / 64; ++i) t += red[i];
  __syncthreads();
  return t;
}

// record of example b of this step (see the header): the record feed of csrc/feed.h at step step_ctr[0] (global
// stream stride / offset, optional per-epoch shuffle), or records start_fixed.. in stored order
struct BatchSel {
  long long n;
  const long long* ctr;
  long long start_fixed;
  int B;
  MifxFeed feed;
  long long* rec_out;  // nullable: tdnn_head_bwd records which record each example of the step was
  __device__ __forceinline__ MifxFeedStep start() const {
    if (ctr) return mifx_feed_step(feed, ctr[0], n);
    MifxFeedStep s;
    s.e0 = 0;
    s.i0 = start_fixed;
    s.h = 1;
    return s;
  }
  __device__ __forceinline__ long long rec(const MifxFeedStep& st, int b) const {
    if (!ctr) {
      const long long e = st.i0 + b;
      return e >= n ? e - n : e;  // host guarantees B <= n
    }
    return mifx_feed_record(feed, st, b, n);
  }
};

// grid (B, nh): block (b, c) owns hidden units [256c, 256c + 256) of example b — B x ceil(H/256)
// workgroups so even the B=32 reference batch puts ~200 WGs in flight; each thread issues its
// 16 independent row loads back to back. Writes a = relu(z) and this block's partial logit.
__global__ __launch_bounds__(kThreads) void tdnn_fwd(const float* __restrict__ W1, const float* __restrict__ b1,
                                                    const float* __restrict__ w2, const int* __restrict__ rows, int F,
                                                    const float* __restrict__ xd, int D, int dense_row0, int H,
                                                    BatchSel sel, float* __restrict__ a_out,
                                                    float* __restrict__ part_out) {
  __shared__ int srow[kMaxFields];
  __shared__ float sx[kMaxDense];
  __shared__ float red[kThreads / 64];
  const int b = blockIdx.x, nh = gridDim.y;
  const long long e = sel.rec(sel.start(), b);
  if (threadIdx.x < F) srow[threadIdx.x] = rows[(size_t)e * F + threadIdx.x];
  if (threadIdx.x < D) sx[threadIdx.x] = xd[(size_t)e * D + threadIdx.x];
  __syncthreads();
  const int h = blockIdx.y * kThreads + threadIdx.x;
  float p = 0.f;
  if (h < H) {
    float acc = b1[h];
#pragma unroll 4
    for (int f = 0; f < F; ++f) acc += W1[(size_t)srow[f] * H + h];
    for (int d = 0; d < D; ++d) acc += sx[d] * W1[(size_t)(dense_row0 + d) * H + h];
    const float a = fmaxf(acc, 0.f);
    a_out[(size_t)b * H + h] = a;
    p = a * w2[h];
  }
  const float t = block_sum(p, red);
  if (threadIdx.x == 0) part_out[(size_t)b * nh + blockIdx.y] = t;
}

// grid (B, nh): logit from the partials (fixed order), BCE loss, dlogit, dz = dlogit * w2 * [a > 0]
__global__ __launch_bounds__(kThreads) void tdnn_head_bwd(const float* __restrict__ w2, const float* __restrict__ b2,
                                                         const float* __restrict__ y, BatchSel sel,
                                                         const float* __restrict__ part,
                                                         const float* __restrict__ a, int H, float grad_scale,
                                                         int train, float* __restrict__ dz_out,
                                                         float* __restrict__ logit_out, float* __restrict__ dlogit_out,
                                                         float* __restrict__ loss_out, const float* __restrict__ xd,
                                                         int D, float* __restrict__ dense_part) {
  const int b = blockIdx.x, nh = gridDim.y;
  float logit = b2[0];
  for (int c = 0; c < nh; ++c) logit += part[(size_t)b * nh + c];
  if (blockIdx.y == 0 && threadIdx.x == 0) logit_out[b] = logit;
  if (!train) return;
  const long long rec = sel.rec(sel.start(), b);
  if (sel.rec_out != nullptr && blockIdx.y == 0 && threadIdx.x == 0) sel.rec_out[b] = rec;
  const float yy = y[rec];
  const float dl = (1.f / (1.f + expf(-logit)) - yy) * grad_scale;
  if (blockIdx.y == 0 && threadIdx.x == 0) {
    // stable BCE with logits: max(l,0) - l*y + log1p(exp(-|l|))
    loss_out[b] = fmaxf(logit, 0.f) - logit * yy + log1pf(expf(-fabsf(logit)));
    dlogit_out[b] = dl;
  }
  const int h = blockIdx.y * kThreads + threadIdx.x;
  if (h >= H) return;
  const float av = a[(size_t)b * H + h];
  const float g = av > 0.f ? dl * w2[h] : 0.f;
  dz_out[(size_t)b * H + h] = g;
  if (dense_part) {  // small batch: one "chunk" per example -- this example's dense-parameter gradients, so no
                     // separate batch-reduction launch (tdnn_dense_apply sums the B chunks in example order)
    float* out = dense_part + (size_t)b * (D + 2) * H;
    const long long e = sel.rec(sel.start(), b);
    for (int d = 0; d < D; ++d) out[(size_t)d * H + h] = xd[(size_t)e * D + d] * g;
    out[(size_t)D * H + h] = g;
    out[(size_t)(D + 1) * H + h] = dl * av;
  }
}

// grid (B * F): workgroup p = (b, f). Row r = rows[rec(b)][f]; fields own disjoint row ranges, so the
// examples that touched r are the b' with rows[rec(b')][f] == r. The pair with the smallest such b' owns
// the row: it lists them (ascending, in LDS) and sums their dz in that order; every other pair exits.
constexpr int kMaxList = 8192;  // batch bound of this kernel (LDS list of one row's examples)
__global__ __launch_bounds__(kThreads) void tdnn_sparse_adagrad(float* __restrict__ W1, float* __restrict__ acc1,
                                                               const int* __restrict__ rows, int F, BatchSel sel,
                                                               const float* __restrict__ dz, int H, float lr) {
  __shared__ int list[kMaxList];
  __shared__ int wcnt[kThreads / 64];
  __shared__ int s_n, s_earlier;
  const int B = sel.B;
  const int b = blockIdx.x / F, f = blockIdx.x % F;
  const MifxFeedStep st = sel.start();
  const int r = rows[(size_t)sel.rec(st, b) * F + f];
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  if (t == 0) {
    s_n = 0;
    s_earlier = 0;
  }
  __syncthreads();
  for (int b0 = 0; b0 < B; b0 += kThreads) {  // chunks of 256 examples, compacted in example order
    const int bb = b0 + t;
    const bool hit = bb < B && rows[(size_t)sel.rec(st, bb) * F + f] == r;
    const unsigned long long m = __ballot(hit);
    if (lane == 0) wcnt[w] = __popcll(m);
    __syncthreads();
    int base = s_n;
    for (int i = 0; i < w; ++i) base += wcnt[i];
    if (hit) {
      if (bb < b) s_earlier = 1;  // every writer stores 1
      list[base + __popcll(m & ((1ull << lane) - 1))] = bb;
    }
    __syncthreads();
    if (t == 0)
      for (int i = 0; i < kThreads / 64; ++i) s_n += wcnt[i];
    __syncthreads();
    if (s_earlier) return;  // uniform: an earlier example's pair owns the row
  }
  const int cnt = s_n;
  // (an unrolled variant with 4 columns' loads in flight per thread measured 2.2x slower at B=1024: 163 vs 76 us)
  for (int h = t; h < H; h += kThreads) {
    float g = 0.f;
    for (int k = 0; k < cnt; ++k) g += dz[(size_t)list[k] * H + h];
    const size_t i = (size_t)r * H + h;
    const float a = acc1[i] + g * g;
    acc1[i] = a;
    W1[i] -= lr * g * rsqrtf(a);
  }
}

// grid (ceil(H/256), nchunk): per-chunk batch reductions for the dense params, into
// part[chunk][k][h] with k = 0..D-1 dense W1 rows, D = b1, D+1 = w2
__global__ __launch_bounds__(kThreads) void tdnn_dense_partial(const float* __restrict__ xd, int D, BatchSel sel,
                                                              const float* __restrict__ a,
                                                              const float* __restrict__ dz,
                                                              const float* __restrict__ dlogit, int B, int H,
                                                              float* __restrict__ part) {
  const int h = blockIdx.x * kThreads + threadIdx.x;
  if (h >= H) return;
  const MifxFeedStep st = sel.start();
  const int nchunk = gridDim.y, c = blockIdx.y;
  const int b0 = (int)((long long)B * c / nchunk), b1e = (int)((long long)B * (c + 1) / nchunk);
  float gd[kMaxDense];
#pragma unroll
  for (int d = 0; d < kMaxDense; ++d) gd[d] = 0.f;
  float gb1 = 0.f, gw2 = 0.f;
  for (int b = b0; b < b1e; ++b) {
    const float g = dz[(size_t)b * H + h];
    gb1 += g;
    gw2 += dlogit[b] * a[(size_t)b * H + h];
#pragma unroll
    for (int d = 0; d < kMaxDense; ++d)
      if (d < D) gd[d] += xd[(size_t)sel.rec(st, b) * D + d] * g;
  }
  float* out = part + (size_t)c * (D + 2) * H;
  for (int d = 0; d < D; ++d) out[(size_t)d * H + h] = gd[d];
  out[(size_t)D * H + h] = gb1;
  out[(size_t)(D + 1) * H + h] = gw2;
}

__device__ __forceinline__ void adagrad_one(float* w, float* acc, float g, float lr) {
  const float s = *acc + g * g;
  *acc = s;
  *w -= lr * g * rsqrtf(s);
}

// grid (ceil(H/256), D + 3): blockIdx.y = k < D + 2 sums row k of the chunk partials (dense W1 row k, b1 at
// k = D, w2 at k = D + 1) in chunk order -- 8 loads in flight per thread -- and updates it; the (0, D + 2) block
// updates b2 and advances the step counter.
__global__ __launch_bounds__(kThreads) void tdnn_dense_apply(float* __restrict__ W1, float* __restrict__ acc1,
                                                            float* __restrict__ b1, float* __restrict__ accb1,
                                                            float* __restrict__ w2, float* __restrict__ accw2,
                                                            float* __restrict__ b2, float* __restrict__ accb2,
                                                            int D, int dense_row0, const float* __restrict__ part,
                                                            int nchunk, const float* __restrict__ dlogit, int B,
                                                            int H, float lr, long long* __restrict__ step_ctr) {
  const int k = blockIdx.y;
  if (k == D + 2) {
    if (blockIdx.x != 0) return;
    __shared__ float red[kThreads / 64];
    float p = 0.f;
    for (int b = threadIdx.x; b < B; b += kThreads) p += dlogit[b];
    const float g = block_sum(p, red);
    if (threadIdx.x == 0) {
      adagrad_one(b2, accb2, g, lr);
      // every reader of step_ctr in this step ran in an earlier launch: advance to the next batch
      if (step_ctr) step_ctr[0] += 1;
    }
    return;
  }
  const int h = blockIdx.x * kThreads + threadIdx.x;
  if (h >= H) return;
  const size_t cstride = (size_t)(D + 2) * H;
  const float* src = part + (size_t)k * H + h;
  float g = 0.f;
  constexpr int U = 8;
  for (int c0 = 0; c0 < nchunk; c0 += U) {
    float v[U];
#pragma unroll
    for (int u = 0; u < U; ++u) v[u] = c0 + u < nchunk ? src[(size_t)(c0 + u) * cstride] : 0.f;
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (c0 + u < nchunk) g += v[u];  // fixed chunk order
  }
  if (k < D) {
    const size_t i = (size_t)(dense_row0 + k) * H + h;
    adagrad_one(W1 + i, acc1 + i, g, lr);
  } else if (k == D) {
    adagrad_one(b1 + h, accb1 + h, g, lr);
  } else {
    adagrad_one(w2 + h, accw2 + h, g, lr);
  }
}

}  // namespace

extern "C" {

int mifx_tdnn_limits(int* out) {
  out[0] = kMaxH;
  out[1] = kMaxFields;
  out[2] = kMaxDense;
  return 0;
}

// batch chunks of the dense-parameter reduction: one per example up to 64 (written by tdnn_head_bwd itself),
// else chunks of >= 32 examples (tdnn_dense_partial), at most 64
constexpr int kDirectChunks = 64;
int mifx_tdnn_chunks(int B) { return B <= kDirectChunks ? B : (B / 32 < 64 ? B / 32 : 64); }

// rows [n, F] int32 global W1 rows, xd [n, D], y [n]: the resident dataset (or one batch with n = B). Example b
// of the step is the feed's record (csrc/feed.h) when step_ctr is set, else record (start_fixed + b) % n.
// rec_out (nullable, int64 [B]): receives the record index of every example.
// scratch: part_logit [B * ceil(H/256)]
int mifx_tdnn_fwd_bwd(const float* W1, const float* b1, const float* w2, const float* b2, const int* rows, int F,
                      const float* xd, int D, int dense_row0, const float* y, long long n, const long long* step_ctr,
                      long long start_fixed, int B, int H, float grad_scale, int train, float* a_out,
                      float* part_logit, float* dz_out, float* logit_out, float* dlogit_out, float* loss_out,
                      float* dense_part, long long feed_stride, long long feed_offset, unsigned long long shuffle_key,
                      long long* rec_out, hipStream_t st) {
  if (H <= 0 || H > kMaxH || F > kMaxFields || D > kMaxDense || B <= 0 || n < B || start_fixed < 0 ||
      start_fixed >= n || feed_stride < B || feed_offset < 0 || feed_offset + B > feed_stride)
    return -1;
  const BatchSel sel{n, step_ctr, start_fixed, B, MifxFeed{feed_stride, feed_offset, shuffle_key}, rec_out};
  const dim3 grid(B, (H + kThreads - 1) / kThreads);
  hipLaunchKernelGGL(tdnn_fwd, grid, dim3(kThreads), 0, st, W1, b1, w2, rows, F, xd, D, dense_row0, H, sel, a_out,
                     part_logit);
  float* direct = train && B <= kDirectChunks ? dense_part : nullptr;
  if (train && B <= kDirectChunks && dense_part == nullptr) return -1;
  hipLaunchKernelGGL(tdnn_head_bwd, grid, dim3(kThreads), 0, st, w2, b2, y, sel, part_logit, a_out, H, grad_scale,
                     train, dz_out, logit_out, dlogit_out, loss_out, xd, D, direct);
  return (int)hipGetLastError();
}

int mifx_tdnn_max_batch() { return kMaxList; }

// scratch: dense_part [mifx_tdnn_chunks(B) * (D + 2) * H]; advances step_ctr (when set) after the update
int mifx_tdnn_adagrad(float* W1, float* acc1, float* b1, float* accb1, float* w2, float* accw2, float* b2,
                      float* accb2, const int* rows, int F, const float* xd, int D, int dense_row0, long long n,
                      long long* step_ctr, long long start_fixed, const float* a, const float* dz,
                      const float* dlogit, int B, int H, float lr, float* dense_part, long long feed_stride,
                      long long feed_offset, unsigned long long shuffle_key, hipStream_t st) {
  if (H <= 0 || H > kMaxH || D > kMaxDense || F > kMaxFields || B <= 0 || B > kMaxList || n < B ||
      start_fixed < 0 || start_fixed >= n || feed_stride < B || feed_offset < 0 || feed_offset + B > feed_stride)
    return -1;
  const BatchSel sel{n, step_ctr, start_fixed, B, MifxFeed{feed_stride, feed_offset, shuffle_key}, nullptr};
  hipLaunchKernelGGL(tdnn_sparse_adagrad, dim3(B * F), dim3(kThreads), 0, st, W1, acc1, rows, F, sel, dz, H, lr);
  const int nchunk = mifx_tdnn_chunks(B);
  const int hb = (H + kThreads - 1) / kThreads;
  if (B > kDirectChunks)  // (small batches: tdnn_head_bwd wrote the per-example chunks)
    hipLaunchKernelGGL(tdnn_dense_partial, dim3(hb, nchunk), dim3(kThreads), 0, st, xd, D, sel, a, dz, dlogit, B, H,
                       dense_part);
  hipLaunchKernelGGL(tdnn_dense_apply, dim3(hb, D + 3), dim3(kThreads), 0, st, W1, acc1, b1, accb1, w2, accw2, b2,
                     accb2, D,
                     dense_row0, dense_part, nchunk, dlogit, B, H, lr, step_ctr);
  return (int)hipGetLastError();
}

}  // extern "C"
