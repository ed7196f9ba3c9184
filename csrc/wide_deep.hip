// Fused Wide&Deep (Chicago-Taxi DNNLinearCombinedClassifier) training step for gfx950.
//
// Parity target: reference `airflow-dags/taxi_utils.py:148-191` (_build_estimator) with the
// hidden sizes of `trainer_fn` (`taxi_utils.py:300-345`: [100, 70, 48, 34], batch 40),
// wide part = 9 categorical identity columns (`taxi_utils.py:168-185`), sigmoid CE head.
//
// Design (MI355X-first, not a translation of TF's graph):
//  * One kernel does forward + loss + backward for a 64-example tile per workgroup
//    iteration. 4 waves; wave w owns examples [16w, 16w+16) of the tile for the whole
//    forward and the activation-gradient chain (wave-local, no block barriers), using
//    v_mfma_f32_16x16x32_bf16 in the transposed form Z^T = W^T . A^T so that each
//    lane's accumulator (4 consecutive features of one example) is stored with one 8-B
//    ds_write into the row-major activation image.
//  * Weight gradients dW^T = dZ^T . A (reduction over the 64 examples of the tile) are
//    computed cooperatively: every wave owns 27 of the 108 16x16 dW tiles and keeps them
//    in accumulator registers across ALL tiles the workgroup processes (MFMA K-accumulation
//    == batch reduction). Operands with examples along K come from the row-major images
//    through ds_read_b64_tr_b16 (hardware transpose), so no second image is written.
//  * Biases live in the weight matrices: each layer input carries a constant-1 column,
//    so bias-add, bias-grad and the dense GEMM are one MFMA chain.
//  * The wide (linear) part is an embedding-bag gather of 9 fp32 weights per example from
//    the L2-resident table; its gradient is a ds_add_f32 histogram in LDS.
//  * Each workgroup writes one fp32 gradient slab (tile-native order, fully coalesced);
//    wd_reduce sums slabs, wd_optimizer applies Adagrad (DNN) / FTRL (wide) / Adam / SGD and
//    re-emits the bf16 weight image. A device-side step counter drives the data offset so
//    the whole step is hipGraph-capturable.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

typedef __bf16 bf16;
typedef __bf16 v8bf __attribute__((ext_vector_type(8)));
typedef __bf16 v4bf __attribute__((ext_vector_type(4)));
typedef short v4s __attribute__((ext_vector_type(4)));
typedef short v8s __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4s lds_v4s;

constexpr int T = 64;       // examples per tile
constexpr int PAD = 8;      // bf16 elements of row padding (2-way max bank conflicts)
constexpr int NTHR = 256;

// padded layer dims: layer l maps K_l -> N_l ; real: 3->100->70->48->34->1
constexpr int K1 = 32, N1 = 128;
constexpr int K2 = 128, N2 = 96;
constexpr int K3 = 96, N3 = 64;
constexpr int K4 = 64, N4 = 64;
constexpr int K5 = 64, N5 = 16;

// canonical bf16/fp32 weight offsets (W^T row-major [N][K] per layer)
constexpr int OFF1 = 0;
constexpr int OFF2 = OFF1 + N1 * K1;
constexpr int OFF3 = OFF2 + N2 * K2;
constexpr int OFF4 = OFF3 + N3 * K3;
constexpr int OFF5 = OFF4 + N4 * K4;
constexpr int WTOT = OFF5 + N5 * K5;  // 27648

// LDS layout (bf16 element offsets)
constexpr int LW1 = 0;
constexpr int LW2 = LW1 + N1 * (K1 + PAD);
constexpr int LW3 = LW2 + N2 * (K2 + PAD);
constexpr int LW4 = LW3 + N3 * (K3 + PAD);
constexpr int LW5 = LW4 + N4 * (K4 + PAD);
constexpr int LWEND = LW5 + N5 * (K5 + PAD);
constexpr int LA0 = LWEND;
constexpr int LA1 = LA0 + T * (K1 + PAD);
constexpr int LA2 = LA1 + T * (K2 + PAD);
constexpr int LA3 = LA2 + T * (K3 + PAD);
constexpr int LA4 = LA3 + T * (K4 + PAD);
constexpr int LD5 = LA4 + T * (K5 + PAD);
constexpr int LP = LD5 + T * (N5 + PAD);
constexpr int LQ = LP + T * (N2 + PAD);
constexpr int LEND = LQ + T * (N1 + PAD);
static_assert((LEND * 2) % 16 == 0, "fp32 region must be 16B aligned");

constexpr int NWIDE = 2128;         // 2127 identity buckets + bias
constexpr int WIDE_BIAS = 2127;
constexpr int WIDE_PAD = 2176;
constexpr int NTILE = 108;          // 16x16 dW tiles
constexpr int STRIDE = NTILE * 256 + WIDE_PAD;   // 29824 floats per slab
constexpr int LDS_BYTES = LEND * 2 + WIDE_PAD * 4 + 64 * 4;
static_assert(LDS_BYTES <= 163840, "LDS budget");

// tile bases in tile-native order
constexpr int TB1 = 0, TB2 = TB1 + (N1 / 16) * (K1 / 16), TB3 = TB2 + (N2 / 16) * (K2 / 16),
              TB4 = TB3 + (N3 / 16) * (K3 / 16), TB5 = TB4 + (N4 / 16) * (K4 / 16);
static_assert(TB5 + (N5 / 16) * (K5 / 16) == NTILE, "tile count");

// wide feature offsets: payment_type_xf, company_xf (1010 each), 4 lat/lon buckets (10 each),
// trip_start_hour (24), trip_start_day (31), trip_start_month (12)
__constant__ int kWideOff[9] = {0, 1010, 2020, 2030, 2040, 2050, 2060, 2084, 2115};
__constant__ int kWideNb[9] = {1010, 1010, 10, 10, 10, 10, 24, 31, 12};

struct __attribute__((packed, aligned(16))) Rec {
  float d[3];
  uint16_t id[9];
  uint16_t label;
};
static_assert(sizeof(Rec) == 32, "record is 32 B");

__device__ __forceinline__ v4s tr_read(const uint16_t* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(p));
}
__device__ __forceinline__ v8bf cat8(v4s a, v4s b) {
  v8s r = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  return __builtin_bit_cast(v8bf, r);
}
__device__ __forceinline__ v8bf ld8(const uint16_t* p) { return *(const v8bf*)p; }
__device__ __forceinline__ v4f mfma(v8bf a, v8bf b, v4f c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// ---------------------------------------------------------------- forward layer (wave-local)
// Z^T[n][t] = sum_k Wt[n][k] * A[t][k]; A rows t in [16w, 16w+16). RELU -> bf16 -> Aout.
template <int K, int N, bool RELU_STORE>
__device__ __forceinline__ void fwd_layer(const uint16_t* W, const uint16_t* A, uint16_t* Aout,
                                          int w, int r, int h, v4f* zlast) {
  constexpr int KS = K / 32;
  v8bf b[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) b[s] = ld8(A + (16 * w + r) * (K + PAD) + 32 * s + 8 * h);
#pragma unroll
  for (int nt = 0; nt < N / 16; ++nt) {
    v4f acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < KS; ++s) acc = mfma(ld8(W + (16 * nt + r) * (K + PAD) + 32 * s + 8 * h), b[s], acc);
    if constexpr (RELU_STORE) {
      v4bf o;
#pragma unroll
      for (int i = 0; i < 4; ++i) o[i] = (bf16)fmaxf(acc[i], 0.f);
      *(v4bf*)(Aout + (16 * w + r) * (N + PAD) + 16 * nt + 4 * h) = o;
    } else {
      *zlast = acc;
    }
  }
}

// ------------------------------------------------------- activation gradient (wave-local)
// dA^T[k][t] = sum_n W[k][n] dZ^T[n][t]   (W = layer with dims K x N, stored as Wt[N][K])
// dZout[t][k] = dA[t][k] * (Aact[t][k] > 0)
template <int K, int N>
__device__ __forceinline__ void bwd_dA(const uint16_t* W, const uint16_t* dZ, const uint16_t* Aact,
                                       uint16_t* dZout, int w, int r, int h) {
  constexpr int NS = (N + 31) / 32;
  const int q = r >> 2, p = r & 3;
  v8bf b[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    v8bf v = ld8(dZ + (16 * w + r) * (N + PAD) + 32 * s + 8 * h);
    if (N % 32 != 0 && 32 * s + 8 * h >= N) v = (v8bf){};
    b[s] = v;
  }
#pragma unroll
  for (int kt = 0; kt < K / 16; ++kt) {
    v4f acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const uint16_t* pa = W + (32 * s + 8 * h + q) * (K + PAD) + 16 * kt + 4 * p;
      v8bf a = cat8(tr_read(pa), tr_read(pa + 4 * (K + PAD)));
      if (N % 32 != 0 && 32 * s + 8 * h >= N) a = (v8bf){};
      acc = mfma(a, b[s], acc);
    }
    const int off = (16 * w + r) * (K + PAD) + 16 * kt + 4 * h;
    const uint2 m = *(const uint2*)(Aact + off);
    const uint16_t mk[4] = {(uint16_t)(m.x & 0xffff), (uint16_t)(m.x >> 16), (uint16_t)(m.y & 0xffff),
                            (uint16_t)(m.y >> 16)};
    v4bf o;
#pragma unroll
    for (int i = 0; i < 4; ++i) o[i] = (bf16)(mk[i] ? acc[i] : 0.f);
    *(v4bf*)(dZout + off) = o;
  }
}

// ------------------------------------------------------------- weight gradient (cooperative)
// dWt[n][k] += sum_t dZ[t][n] * A[t][k] over the 64 tile rows; wave w owns tiles
// [w*CNT, (w+1)*CNT) of this layer (row-major over (nt, kt)).
template <int K, int N, int CNT>
__device__ __forceinline__ void dw_phase(v4f (&acc)[CNT], const uint16_t* dZ, const uint16_t* A,
                                         int w, int r, int h) {
  constexpr int KT = K / 16;
  const int q = r >> 2, p = r & 3;
#pragma unroll
  for (int j = 0; j < CNT; ++j) {
    const int idx = w * CNT + j;
    const int nt = idx / KT, kt = idx % KT;
#pragma unroll
    for (int s = 0; s < T / 32; ++s) {
      const uint16_t* pa = dZ + (32 * s + 8 * h + q) * (N + PAD) + 16 * nt + 4 * p;
      const uint16_t* pb = A + (32 * s + 8 * h + q) * (K + PAD) + 16 * kt + 4 * p;
      v8bf a = cat8(tr_read(pa), tr_read(pa + 4 * (N + PAD)));
      v8bf b = cat8(tr_read(pb), tr_read(pb + 4 * (K + PAD)));
      acc[j] = mfma(a, b, acc[j]);
    }
  }
}

template <int CNT>
__device__ __forceinline__ void store_tiles(float* slab, const v4f (&acc)[CNT], int tbase, int w, int lane) {
#pragma unroll
  for (int j = 0; j < CNT; ++j) {
    float* dst = slab + (size_t)(tbase + w * CNT + j) * 256 + lane;
#pragma unroll
    for (int i = 0; i < 4; ++i) dst[i * 64] = acc[j][i];
  }
}

__device__ __forceinline__ void wt_locate(int e, int& lofs, int& k, int& n, int& K) {
  int base;
  if (e < OFF2) { base = OFF1; K = K1; lofs = LW1; }
  else if (e < OFF3) { base = OFF2; K = K2; lofs = LW2; }
  else if (e < OFF4) { base = OFF3; K = K3; lofs = LW3; }
  else if (e < OFF5) { base = OFF4; K = K4; lofs = LW4; }
  else { base = OFF5; K = K5; lofs = LW5; }
  n = (e - base) / K;
  k = (e - base) % K;
}

template <bool TRAIN>
__global__ __launch_bounds__(NTHR, 1) void wd_fused(
    const Rec* __restrict__ data, long long n_data, long long batch, long long start_fixed,
    const long long* __restrict__ step_ctr, const uint16_t* __restrict__ wt, const float* __restrict__ wide,
    float* __restrict__ slab, float* __restrict__ slab_loss, float* __restrict__ logits_out,
    float grad_scale) {
  extern __shared__ __attribute__((aligned(16))) uint16_t lds[];
  float* wgrad = (float*)(lds + LEND);
  float* red = wgrad + WIDE_PAD;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, r = lane & 15, h = lane >> 4;

  // stage the bf16 weight image (canonical [N][K] per layer) into padded LDS rows
  for (int c = tid; c < WTOT / 8; c += NTHR) {
    int lofs, k, n, K;
    wt_locate(c * 8, lofs, k, n, K);
    *(uint4*)(lds + lofs + n * (K + PAD) + k) = *(const uint4*)(wt + c * 8);
  }
  for (int c = tid; c < T * (K1 + PAD) / 8; c += NTHR) *(uint4*)(lds + LA0 + c * 8) = make_uint4(0, 0, 0, 0);
  if (TRAIN) {
    for (int c = tid; c < WIDE_PAD; c += NTHR) wgrad[c] = 0.f;
    for (int c = tid; c < T * (N5 + PAD) / 8; c += NTHR) *(uint4*)(lds + LD5 + c * 8) = make_uint4(0, 0, 0, 0);
  }
  __syncthreads();

  const long long start = step_ctr ? (step_ctr[0] * batch) % n_data : start_fixed;
  const long long ntiles = (batch + T - 1) / T;

  v4f acc1[4], acc2[12], acc3[6], acc4[4], acc5[1];
#pragma unroll
  for (int j = 0; j < 4; ++j) acc1[j] = acc4[j] = (v4f){0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j < 12; ++j) acc2[j] = (v4f){0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j < 6; ++j) acc3[j] = (v4f){0.f, 0.f, 0.f, 0.f};
  acc5[0] = (v4f){0.f, 0.f, 0.f, 0.f};
  float loss_sum = 0.f, dl_sum = 0.f;

  uint16_t* A0 = lds + LA0;
  uint16_t* A1 = lds + LA1;
  uint16_t* A2 = lds + LA2;
  uint16_t* A3 = lds + LA3;
  uint16_t* A4 = lds + LA4;
  uint16_t* D5 = lds + LD5;
  uint16_t* P = lds + LP;
  uint16_t* Q = lds + LQ;

  for (long long tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
    const long long row = tile * T + 16 * w + r;
    const bool valid = row < batch;
    long long di = start + row;
    di = di % n_data;
    uint4 u0 = make_uint4(0, 0, 0, 0), u1 = make_uint4(0, 0, 0, 0);
    if (valid) {
      const uint4* src = (const uint4*)(data + di);
      u0 = src[0];
      u1 = src[1];
    }
    const float d0 = __uint_as_float(u0.x), d1 = __uint_as_float(u0.y), d2 = __uint_as_float(u0.z);
    const uint32_t idw[5] = {u0.w, u1.x, u1.y, u1.z, u1.w};
    if (h == 0) {
      v8bf x = {(bf16)d0, (bf16)d1, (bf16)d2, (bf16)1.0f, (bf16)0.f, (bf16)0.f, (bf16)0.f, (bf16)0.f};
      *(v8bf*)(A0 + (16 * w + r) * (K1 + PAD)) = x;
    }
    wave_sync();
    v4f z5;
    fwd_layer<K1, N1, true>(lds + LW1, A0, A1, w, r, h, nullptr);
    wave_sync();
    fwd_layer<K2, N2, true>(lds + LW2, A1, A2, w, r, h, nullptr);
    wave_sync();
    fwd_layer<K3, N3, true>(lds + LW3, A2, A3, w, r, h, nullptr);
    wave_sync();
    fwd_layer<K4, N4, true>(lds + LW4, A3, A4, w, r, h, nullptr);
    wave_sync();
    fwd_layer<K5, N5, false>(lds + LW5, A4, nullptr, w, r, h, &z5);

    // ---- wide part + loss (every lane recomputes for example r; lane h==0 owns it)
    const float zd = __shfl(z5[0], r);
    float wl = wide[WIDE_BIAS];
    int ids[9];
#pragma unroll
    for (int f = 0; f < 9; ++f) {
      int id = (f & 1) ? (idw[f >> 1] >> 16) : (idw[f >> 1] & 0xffff);
      id = id < kWideNb[f] ? id : 0;
      ids[f] = kWideOff[f] + id;
      wl += wide[ids[f]];
    }
    const float x = zd + wl;
    const float y = (float)(idw[4] >> 16);
    if (!TRAIN) {
      if (h == 0 && valid) logits_out[row] = x;
      if (h == 0 && valid) loss_sum += fmaxf(x, 0.f) - x * y + log1pf(__expf(-fabsf(x)));
      continue;
    }
    float dl = 0.f;
    if (valid) {
      if (h == 0) loss_sum += fmaxf(x, 0.f) - x * y + log1pf(__expf(-fabsf(x)));
      dl = (1.f / (1.f + __expf(-x)) - y) * grad_scale;
    }
    if (h == 0 && valid) {
#pragma unroll
      for (int f = 0; f < 9; ++f) atomicAdd(&wgrad[ids[f]], dl);
      dl_sum += dl;
    }
    {
      v4bf o = {(bf16)(h == 0 ? dl : 0.f), (bf16)0.f, (bf16)0.f, (bf16)0.f};
      *(v4bf*)(D5 + (16 * w + r) * (N5 + PAD) + 4 * h) = o;
    }
    wave_sync();
    bwd_dA<K5, N5>(lds + LW5, D5, A4, P, w, r, h);   // dz4 -> P
    __syncthreads();                                  // B1
    dw_phase<K5, N5, 1>(acc5, D5, A4, w, r, h);
    dw_phase<K4, N4, 4>(acc4, P, A3, w, r, h);
    bwd_dA<K4, N4>(lds + LW4, P, A3, Q, w, r, h);    // dz3 -> Q
    __syncthreads();                                  // B2
    dw_phase<K3, N3, 6>(acc3, Q, A2, w, r, h);
    bwd_dA<K3, N3>(lds + LW3, Q, A2, P, w, r, h);    // dz2 -> P
    __syncthreads();                                  // B3
    dw_phase<K2, N2, 12>(acc2, P, A1, w, r, h);
    bwd_dA<K2, N2>(lds + LW2, P, A1, Q, w, r, h);    // dz1 -> Q
    __syncthreads();                                  // B4
    dw_phase<K1, N1, 4>(acc1, Q, A0, w, r, h);
    __syncthreads();                                  // B5
  }

  // ---- epilogue: per-workgroup slab
  for (int o = 32; o > 0; o >>= 1) {
    loss_sum += __shfl_xor(loss_sum, o);
    dl_sum += __shfl_xor(dl_sum, o);
  }
  if (lane == 0) { red[w] = loss_sum; red[4 + w] = dl_sum; }
  if (TRAIN) {
    float* my = slab + (size_t)blockIdx.x * STRIDE;
    store_tiles<4>(my, acc1, TB1, w, lane);
    store_tiles<12>(my, acc2, TB2, w, lane);
    store_tiles<6>(my, acc3, TB3, w, lane);
    store_tiles<4>(my, acc4, TB4, w, lane);
    store_tiles<1>(my, acc5, TB5, w, lane);
  }
  __syncthreads();
  if (TRAIN) {
    float* my = slab + (size_t)blockIdx.x * STRIDE + NTILE * 256;
    for (int c = tid; c < WIDE_PAD; c += NTHR) {
      float v = wgrad[c];
      if (c == WIDE_BIAS) v += red[4] + red[5] + red[6] + red[7];
      my[c] = v;
    }
  }
  if (tid == 0 && slab_loss) slab_loss[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}

// partial[sp][e] = sum_{g in split sp} slab[g][e]   (float4 granules)
__global__ __launch_bounds__(256) void wd_reduce(const float4* __restrict__ slab, int G, int gchunk,
                                                 float4* __restrict__ partial) {
  constexpr int S4 = STRIDE / 4;
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= S4) return;
  const int g0 = blockIdx.y * gchunk;
  const int g1 = min(G, g0 + gchunk);
  float4 a = make_float4(0, 0, 0, 0), b = a;
  int g = g0;
  for (; g + 1 < g1; g += 2) {
    float4 u = slab[(size_t)g * S4 + e], v = slab[(size_t)(g + 1) * S4 + e];
    a.x += u.x; a.y += u.y; a.z += u.z; a.w += u.w;
    b.x += v.x; b.y += v.y; b.z += v.z; b.w += v.w;
  }
  if (g < g1) {
    float4 u = slab[(size_t)g * S4 + e];
    a.x += u.x; a.y += u.y; a.z += u.z; a.w += u.w;
  }
  partial[(size_t)blockIdx.y * S4 + e] = make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
}

struct OptHyper {
  int kind;        // 0 sgd, 1 adagrad, 2 ftrl, 3 adam
  float lr, beta1, beta2, eps, l1, l2, lr_power;
};

// One thread per canonical parameter. DNN segment [0, WTOT) then wide segment [WTOT, WTOT+NWIDE).
__global__ __launch_bounds__(256) void wd_optimizer(
    const float* __restrict__ partial, int nparts, const int* __restrict__ gidx, const uint8_t* __restrict__ mask,
    float* __restrict__ param, float* __restrict__ s0, float* __restrict__ s1, uint16_t* __restrict__ wt_out,
    long long* __restrict__ step_ctr, OptHyper hd, OptHyper hw) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  const long long step = step_ctr[0] + 1;
  if (c < WTOT + NWIDE) {
    const bool dnn = c < WTOT;
    const OptHyper& hp = dnn ? hd : hw;
    float w = param[c];
    if (mask[c]) {
      const int gi = gidx[c];
      float g = 0.f;
      for (int pidx = 0; pidx < nparts; ++pidx) g += partial[(size_t)pidx * STRIDE + gi];
      if (hp.kind == 0) {
        w -= hp.lr * g;
      } else if (hp.kind == 1) {
        float a = s0[c] + g * g;
        s0[c] = a;
        w -= hp.lr * g * rsqrtf(a);
      } else if (hp.kind == 2) {
        const float a = s0[c];
        const float an = a + g * g;
        float lin = s1[c];
        float sq_new, sq_old;
        if (hp.lr_power == -0.5f) { sq_new = sqrtf(an); sq_old = sqrtf(a); }
        else { sq_new = powf(an, -hp.lr_power); sq_old = powf(a, -hp.lr_power); }
        lin += g - (sq_new - sq_old) / hp.lr * w;
        const float quad = sq_new / hp.lr + 2.f * hp.l2;
        w = fabsf(lin) > hp.l1 ? (copysignf(hp.l1, lin) - lin) / quad : 0.f;
        s0[c] = an;
        s1[c] = lin;
      } else {
        float m = hp.beta1 * s0[c] + (1.f - hp.beta1) * g;
        float v = hp.beta2 * s1[c] + (1.f - hp.beta2) * g * g;
        s0[c] = m;
        s1[c] = v;
        const float bc1 = 1.f - powf(hp.beta1, (float)step);
        const float bc2 = 1.f - powf(hp.beta2, (float)step);
        w -= hp.lr * (m / bc1) / (sqrtf(v / bc2) + hp.eps);
      }
      param[c] = w;
    }
    if (dnn) wt_out[c] = __builtin_bit_cast(uint16_t, (bf16)w);
  }
  if (c == 0) step_ctr[0] = step;
}

}  // namespace

extern "C" {

int mifx_wd_constants(int* out, int n) {
  const int v[] = {T, WTOT, NWIDE, STRIDE, NTILE, LDS_BYTES, OFF1, OFF2, OFF3, OFF4, OFF5,
                   TB1, TB2, TB3, TB4, TB5};
  const int m = (int)(sizeof(v) / sizeof(int));
  for (int i = 0; i < n && i < m; ++i) out[i] = v[i];
  return m;
}

int mifx_wd_fused(const void* data, long long n_data, long long batch, long long start_fixed,
                  const long long* step_ctr, const void* wt, const float* wide, float* slab, float* slab_loss,
                  float* logits_out, float grad_scale, int grid, int train, hipStream_t stream) {
  static bool attr_done = false;
  if (!attr_done) {
    hipFuncSetAttribute((const void*)wd_fused<true>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
    hipFuncSetAttribute((const void*)wd_fused<false>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
    attr_done = true;
  }
  if (grid <= 0 || n_data <= 0 || batch <= 0) return -1;
  if (train)
    hipLaunchKernelGGL(wd_fused<true>, dim3(grid), dim3(NTHR), LDS_BYTES, stream, (const Rec*)data, n_data, batch,
                       start_fixed, step_ctr, (const uint16_t*)wt, wide, slab, slab_loss, logits_out, grad_scale);
  else
    hipLaunchKernelGGL(wd_fused<false>, dim3(grid), dim3(NTHR), LDS_BYTES, stream, (const Rec*)data, n_data, batch,
                       start_fixed, step_ctr, (const uint16_t*)wt, wide, slab, slab_loss, logits_out, grad_scale);
  return (int)hipGetLastError();
}

int mifx_wd_reduce(const float* slab, int G, int nsplit, float* partial, hipStream_t stream) {
  if (G <= 0 || nsplit <= 0) return -1;
  const int gchunk = (G + nsplit - 1) / nsplit;
  dim3 grid((STRIDE / 4 + 255) / 256, nsplit);
  hipLaunchKernelGGL(wd_reduce, grid, dim3(256), 0, stream, (const float4*)slab, G, gchunk, (float4*)partial);
  return (int)hipGetLastError();
}

int mifx_wd_optimizer(const float* partial, int nparts, const int* gidx, const uint8_t* mask, float* param,
                      float* s0, float* s1, void* wt_out, long long* step_ctr, const float* hyper_dnn,
                      const float* hyper_wide, hipStream_t stream) {
  OptHyper hd{(int)hyper_dnn[0], hyper_dnn[1], hyper_dnn[2], hyper_dnn[3], hyper_dnn[4], hyper_dnn[5], hyper_dnn[6],
              hyper_dnn[7]};
  OptHyper hw{(int)hyper_wide[0], hyper_wide[1], hyper_wide[2], hyper_wide[3], hyper_wide[4], hyper_wide[5],
              hyper_wide[6], hyper_wide[7]};
  const int n = WTOT + NWIDE;
  hipLaunchKernelGGL(wd_optimizer, dim3((n + 255) / 256), dim3(256), 0, stream, partial, nparts, gidx, mask, param, s0,
                     s1, (uint16_t*)wt_out, step_ctr, hd, hw);
  return (int)hipGetLastError();
}

}  // extern "C"
