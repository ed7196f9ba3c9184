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
//    Tile ownership is chosen per layer so each wave re-uses its dZ / activation fragments
//    across the tiles it owns (104 transposed reads per wave per tile instead of 216).
//  * Every phase issues all LDS operand reads of a batch before its MFMAs (and prefetches
//    the next batch), so MFMAs do not each wait out a full LDS round trip.
//  * Biases live in the weight matrices: each layer input carries a constant-1 column,
//    so bias-add, bias-grad and the dense GEMM are one MFMA chain.
//  * The wide (linear) part is an embedding-bag gather of 9 fp32 weights per example from
//    the L2-resident table (issued before the forward so its latency hides under MFMAs);
//    its gradient is a ds_add_f32 histogram in LDS.
//  * Block barriers wait only on LDS (lgkmcnt) so the next tile's record prefetch stays in
//    flight across them.
//  * Each workgroup writes one fp32 gradient slab (tile-native order, fully coalesced);
//    wd_reduce sums slabs, wd_optimizer applies Adagrad (DNN) / FTRL (wide) / Adam / SGD and
//    re-emits the bf16 weight image. A device-side step counter drives the data offset so
//    the whole step is hipGraph-capturable.
//
// MIFX_HIPCC_FLAGS: -fno-honor-nans -fno-honor-infinities -mllvm -amdgpu-mfma-vgpr-form
// (no NaN canonicalisation v_max before every ReLU; MFMA results in VGPRs instead of
//  AGPR->VGPR copies feeding the epilogues)
#include <hip/hip_runtime.h>
#include "feed.h"
#include <stdlib.h>
#include "xcd.h"
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
constexpr int NTHR = 512;   // 8 waves: 4 row groups x 2 halves of every layer's output tiles
constexpr int NWAVE = NTHR / 64;

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

// tile bases in tile-native order (tile id = TB + nt * (K/16) + kt)
constexpr int TB1 = 0, TB2 = TB1 + (N1 / 16) * (K1 / 16), TB3 = TB2 + (N2 / 16) * (K2 / 16),
              TB4 = TB3 + (N3 / 16) * (K3 / 16), TB5 = TB4 + (N4 / 16) * (K4 / 16);
static_assert(TB5 + (N5 / 16) * (K5 / 16) == NTILE, "tile count");

// wide feature offsets: payment_type_xf, company_xf (1010 each), 4 lat/lon buckets (10 each),
// trip_start_hour (24), trip_start_day (31), trip_start_month (12)
__constant__ int kWideOff[9] = {0, 1010, 2020, 2030, 2040, 2050, 2060, 2084, 2115};
__constant__ int kWideNb[9] = {1010, 1010, 10, 10, 10, 10, 24, 31, 12};

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
#ifdef WD_STAMPS  // diagnostic build only: per-wave s_memtime at phase boundaries of block 0
__device__ unsigned long long g_stamps[NWAVE][32];
__device__ unsigned long long g_blk[1024][2];  // per-workgroup (start, end) s_memrealtime (100 MHz)
#define STAMP(i)                                                                       \
  do {                                                                                 \
    __builtin_amdgcn_sched_barrier(0);                                                 \
    if (blockIdx.x == 0 && lane == 0 && stamp_on) g_stamps[w][i] = __builtin_amdgcn_s_memtime(); \
    __builtin_amdgcn_sched_barrier(0);                                                 \
  } while (0)
#else
#define STAMP(i) \
  do {           \
  } while (0)
#endif

// Same-wave LDS write->read ordering: DS ops of one wave execute in order, so only the
// compiler must be kept from reordering (no s_waitcnt, outstanding global loads survive).
__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_wave_barrier();
  asm volatile("" ::: "memory");
}
// Block barrier that waits for LDS traffic only (global prefetches stay in flight).
__device__ __forceinline__ void block_sync_lds() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// ---------------------------------------------------------------- forward layer (wave pair)
// Z^T[n][t] = sum_k Wt[n][k] * A[t][k]; A rows t in [16 wr, 16 wr + 16). The two waves of row group wr
// split the layer's n-tiles (half 0: the first ceil(NT/2), half 1: the rest), so the caller must barrier
// before the next layer reads Aout. RELU -> bf16 -> Aout. Weight fragments are read in batches of NB
// n-tiles, the next batch prefetched.
template <int K, int N, bool LAST>
__device__ __forceinline__ void fwd_layer(const uint16_t* W, const uint16_t* A, uint16_t* Aout, int wr, int half,
                                          int r, int h, v4f* zlast) {
  constexpr int KS = K / 32, NT = N / 16, NTH = (NT + 1) / 2;
  constexpr int NB = KS >= 3 ? 2 : (KS == 2 ? 4 : 8);
  constexpr int NBATCH = (NTH + NB - 1) / NB;
  const int nt0 = half * NTH;
  v8bf b[KS];
#pragma unroll
  for (int s = 0; s < KS; ++s) b[s] = ld8(A + (16 * wr + r) * (K + PAD) + 32 * s + 8 * h);
  v8bf wa[2][NB][KS];
#pragma unroll
  for (int j = 0; j < NB; ++j)
#pragma unroll
    for (int s = 0; s < KS; ++s)
      if (j < NTH && nt0 + j < NT) wa[0][j][s] = ld8(W + (16 * (nt0 + j) + r) * (K + PAD) + 32 * s + 8 * h);
#pragma unroll
  for (int bi = 0; bi < NBATCH; ++bi) {
    if (bi + 1 < NBATCH) {
#pragma unroll
      for (int j = 0; j < NB; ++j)
#pragma unroll
        for (int s = 0; s < KS; ++s) {
          const int jl = (bi + 1) * NB + j;
          if (jl < NTH && nt0 + jl < NT)
            wa[(bi + 1) & 1][j][s] = ld8(W + (16 * (nt0 + jl) + r) * (K + PAD) + 32 * s + 8 * h);
        }
    }
#pragma unroll
    for (int j = 0; j < NB; ++j) {
      const int jl = bi * NB + j, nt = nt0 + jl;
      if (jl >= NTH || nt >= NT) continue;
      v4f acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < KS; ++s) acc = mfma(wa[bi & 1][j][s], b[s], acc);
      if constexpr (!LAST) {
        v4bf o;
#pragma unroll
        for (int i = 0; i < 4; ++i) o[i] = (bf16)fmaxf(acc[i], 0.f);
        *(v4bf*)(Aout + (16 * wr + r) * (N + PAD) + 16 * nt + 4 * h) = o;
      } else {
        *zlast = acc;
      }
    }
  }
}

// ------------------------------------------------------- activation gradient (wave pair)
// dA^T[k][t] = sum_n W[k][n] dZ^T[n][t]   (W = layer with dims K x N, stored as Wt[N][K])
// dZout[t][k] = dA[t][k] * (Aact[t][k] > 0) for the rows of row group wr; the two halves split the
// k-tiles. Weight fragments via transposed reads, batched.
template <int K, int N>
__device__ __forceinline__ void bwd_dA(const uint16_t* W, const uint16_t* dZ, const uint16_t* Aact, uint16_t* dZout,
                                       int wr, int half, int r, int h) {
  constexpr int NS = (N + 31) / 32, KT = K / 16, KTH = KT / 2;
  static_assert(KT % 2 == 0, "k-tiles split evenly between the two halves");
  constexpr int KB = NS >= 3 ? 2 : 4;
  constexpr int NBATCH = (KTH + KB - 1) / KB;
  const int kt0 = half * KTH;
  const int q = r >> 2, p = r & 3;
  const bool live = (N % 32 == 0) || (8 * h < N % 32);  // only the last k-step can be partial
  v8bf b[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    v8bf v = ld8(dZ + (16 * wr + r) * (N + PAD) + 32 * s + 8 * h);
    if (s == NS - 1 && !live) v = (v8bf){};
    b[s] = v;
  }
  v8bf wa[2][KB][NS];
  auto load = [&](int buf, int bi) {
#pragma unroll
    for (int j = 0; j < KB; ++j)
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        const int jl = bi * KB + j, kt = kt0 + jl;
        if (jl < KTH) {
          const uint16_t* pa = W + (32 * s + 8 * h + q) * (K + PAD) + 16 * kt + 4 * p;
          v8bf a = cat8(tr_read(pa), tr_read(pa + 4 * (K + PAD)));
          if (s == NS - 1 && !live) a = (v8bf){};
          wa[buf][j][s] = a;
        }
      }
  };
  load(0, 0);
#pragma unroll
  for (int bi = 0; bi < NBATCH; ++bi) {
    if (bi + 1 < NBATCH) load((bi + 1) & 1, bi + 1);
#pragma unroll
    for (int j = 0; j < KB; ++j) {
      const int jl = bi * KB + j, kt = kt0 + jl;
      if (jl >= KTH) continue;
      v4f acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int s = 0; s < NS; ++s) acc = mfma(wa[bi & 1][j][s], b[s], acc);
      const int off = (16 * wr + r) * (K + PAD) + 16 * kt + 4 * h;
      const uint2 m = *(const uint2*)(Aact + off);
      v4bf o;
      o[0] = (bf16)((m.x & 0xffffu) ? acc[0] : 0.f);
      o[1] = (bf16)((m.x >> 16) ? acc[1] : 0.f);
      o[2] = (bf16)((m.y & 0xffffu) ? acc[2] : 0.f);
      o[3] = (bf16)((m.y >> 16) ? acc[3] : 0.f);
      *(v4bf*)(dZout + off) = o;
    }
  }
}

// ------------------------------------------------------------- weight gradient (cooperative)
// dWt[n][k] += sum_t dZ[t][n] * A[t][k] over the 64 tile rows. The wave owns the NTW x KTW
// tiles nt = nt0 + i*ntS, kt = kt0 + j*ktS; all operand fragments are loaded first (each
// dZ n-block once, each activation k-block once), then 2*NTW*KTW MFMAs.
template <int K, int N, int NTW, int KTW>
__device__ __forceinline__ void dw_phase(v4f (&acc)[NTW * KTW], const uint16_t* dZ, const uint16_t* A, int nt0,
                                         int ntS, int kt0, int ktS, int r, int h) {
  const int q = r >> 2, p = r & 3;
  v8bf fa[NTW][2], fb[KTW][2];
#pragma unroll
  for (int i = 0; i < NTW; ++i)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const uint16_t* pa = dZ + (32 * s + 8 * h + q) * (N + PAD) + 16 * (nt0 + i * ntS) + 4 * p;
      fa[i][s] = cat8(tr_read(pa), tr_read(pa + 4 * (N + PAD)));
    }
#pragma unroll
  for (int j = 0; j < KTW; ++j)
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      const uint16_t* pb = A + (32 * s + 8 * h + q) * (K + PAD) + 16 * (kt0 + j * ktS) + 4 * p;
      fb[j][s] = cat8(tr_read(pb), tr_read(pb + 4 * (K + PAD)));
    }
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int i = 0; i < NTW; ++i)
#pragma unroll
      for (int j = 0; j < KTW; ++j) acc[i * KTW + j] = mfma(fa[i][s], fb[j][s], acc[i * KTW + j]);
}

// tmap: tile -> position in the compact slab (-1: tile holds only padding, never stored/reduced).
// The wave's entries are fetched once at kernel start (load_ct) so the epilogue stores do not wait
// on dependent scalar loads.
template <int K, int NTW, int KTW>
__device__ __forceinline__ void load_ct(int (&ct)[NTW * KTW], int tbase, int nt0, int ntS, int kt0, int ktS,
                                        const int* __restrict__ tmap) {
#pragma unroll
  for (int i = 0; i < NTW; ++i)
#pragma unroll
    for (int j = 0; j < KTW; ++j) ct[i * KTW + j] = tmap[tbase + (nt0 + i * ntS) * (K / 16) + kt0 + j * ktS];
}

template <int NTW, int KTW>
__device__ __forceinline__ void store_tiles(float* slab, const v4f (&acc)[NTW * KTW], const int (&ct)[NTW * KTW],
                                            int lane) {
#pragma unroll
  for (int i = 0; i < NTW; ++i)
#pragma unroll
    for (int j = 0; j < KTW; ++j) {
      if (ct[i * KTW + j] < 0) continue;
      float* dst = slab + (size_t)ct[i * KTW + j] * 256 + lane;
#pragma unroll
      for (int e = 0; e < 4; ++e) dst[e * 64] = acc[i * KTW + j][e];
    }
}

template <int BASE, int K, int LOFS>
__device__ __forceinline__ int wt_off(int e) {  // constant divisor per layer
  return LOFS + ((e - BASE) / K) * (K + PAD) + (e - BASE) % K;
}
__device__ __forceinline__ int wt_lds_offset(int e) {
  if (e < OFF2) return wt_off<OFF1, K1, LW1>(e);
  if (e < OFF3) return wt_off<OFF2, K2, LW2>(e);
  if (e < OFF4) return wt_off<OFF3, K3, LW3>(e);
  if (e < OFF5) return wt_off<OFF4, K4, LW4>(e);
  return wt_off<OFF5, K5, LW5>(e);
}

// live rows / 16-byte granules per row of each layer's weight image (host: models.wide_deep.stage_dims)
struct StageDims {
  int rows[5];
  int gpr[5];
  int total;
};

template <bool TRAIN>
__global__ __launch_bounds__(NTHR, 1) void wd_fused(
    const uint4* __restrict__ data, long long n_data, long long batch, long long start_fixed,
    const long long* __restrict__ step_ctr, const uint16_t* __restrict__ wt, const float* __restrict__ wide,
    float* __restrict__ slab, float* __restrict__ slab_loss, float* __restrict__ logits_out, float grad_scale,
    const int* __restrict__ tmap, int stride, StageDims sd, MifxFeed feed) {
  extern __shared__ __attribute__((aligned(16))) uint16_t lds[];
  float* wgrad = (float*)(lds + LEND);
  float* red = wgrad + WIDE_PAD;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, r = lane & 15, h = lane >> 4;
  const int wr = w & 3, half = w >> 2;  // row group (16 examples of the tile) and half of the layer's tiles
#ifdef WD_STAMPS
  if (blockIdx.x == 0 && lane == 0) g_stamps[w][0] = __builtin_amdgcn_s_memtime();
  if (tid == 0 && blockIdx.x < 1024) g_blk[blockIdx.x][0] = __builtin_amdgcn_s_memrealtime();
#endif

  if (sd.total == WTOT / 8) {
    // stage the whole padded bf16 weight image: issue all global loads, then all LDS stores
    constexpr int NCH = WTOT / 8, PER = (NCH + NTHR - 1) / NTHR;
    uint4 v[PER];
#pragma unroll
    for (int i = 0; i < PER; ++i) v[i] = *(const uint4*)(wt + min(tid + i * NTHR, NCH - 1) * 8);
#pragma unroll
    for (int i = 0; i < PER; ++i) {
      const int c = tid + i * NTHR;
      if (c < NCH) *(uint4*)(lds + wt_lds_offset(c * 8)) = v[i];
    }
  } else {
    // Stage only the LIVE part of the image: per layer the rows that hold real weights (plus the
    // constant-1 producer row) and the 16-byte granules up to the last real column (1715 of the 3456
    // granules for the taxi tower) after zero-filling the weight region. (rocprof: same kernel time as
    // the full image at B=65536 and slower for the single-workgroup B=40 step -- the prologue is
    // latency-, not byte-bound -- so the trainer stages the full image by default.) A plain strided
    // loop: register arrays of the granules were demoted to scratch by the compiler, which made every
    // launch of the kernel (either path) reserve scratch.
    for (int c = tid; c < LWEND / 8; c += NTHR) *(uint4*)(lds + c * 8) = make_uint4(0, 0, 0, 0);
    block_sync_lds();
    for (int c = tid; c < sd.total; c += NTHR) {
      int l = 0, cc = c;
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (l == q && cc >= sd.rows[q] * sd.gpr[q]) {
          cc -= sd.rows[q] * sd.gpr[q];
          l = q + 1;
        }
      // select chain, not sd.gpr[l]: a runtime index into the by-value struct would put it in scratch
      const int gpr = l == 0 ? sd.gpr[0] : l == 1 ? sd.gpr[1] : l == 2 ? sd.gpr[2] : l == 3 ? sd.gpr[3] : sd.gpr[4];
      const int row = cc / gpr, g = cc - row * gpr;
      const int K = l == 0 ? K1 : l == 1 ? K2 : l == 2 ? K3 : l == 3 ? K4 : K5;
      const int off = l == 0 ? OFF1 : l == 1 ? OFF2 : l == 2 ? OFF3 : l == 3 ? OFF4 : OFF5;
      const int lw = l == 0 ? LW1 : l == 1 ? LW2 : l == 2 ? LW3 : l == 3 ? LW4 : LW5;
      *(uint4*)(lds + lw + row * (K + PAD) + g * 8) = *(const uint4*)(wt + off + row * K + g * 8);
    }
  }
  for (int c = tid; c < T * (K1 + PAD) / 8; c += NTHR) *(uint4*)(lds + LA0 + c * 8) = make_uint4(0, 0, 0, 0);
  if (TRAIN) {
    for (int c = tid; c < WIDE_PAD; c += NTHR) wgrad[c] = 0.f;
    for (int c = tid; c < T * (N5 + PAD) / 8; c += NTHR) *(uint4*)(lds + LD5 + c * 8) = make_uint4(0, 0, 0, 0);
  }
  __syncthreads();
  bool stamp_on = true;
  (void)stamp_on;
  STAMP(1);

  // record feed (csrc/feed.h); a fixed start (eval / predict) reads records start_fixed.. in stored order
  MifxFeed fd = feed;
  MifxFeedStep fs;
  if (step_ctr) {
    fs = mifx_feed_step(fd, step_ctr[0], n_data);
  } else {
    fd.key = 0;
    fs.e0 = 0;
    fs.i0 = start_fixed;
    fs.h = 1;
  }
  const int ntiles = (int)((batch + T - 1) / T);
  // Wide-part gradient: LDS histogram in 32-bit fixed point, so the result does not depend on the
  // order in which lanes/waves hit a bucket (integer adds commute; fp32 ds_add_f32 would not).
  // |dl| <= |grad_scale| for labels in {0, 1}; the scale is the largest power of two that keeps
  // this workgroup's whole-bucket sum below 2^30, i.e. ~2^-30 of the bucket bound per unit.
  const int my_tiles = (ntiles - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x;
  const float qbound = fmaxf(fabsf(grad_scale) * (float)(max(my_tiles, 1) * T), 1e-30f);
  const float qscale = exp2f(fminf(floorf(log2f(1073741824.f / qbound)), 100.f));
  const float qinv = 1.f / qscale;  // exact: power of two
  const float qmax = 1073741824.f / (float)(max(my_tiles, 1) * T);
  int* wgi = (int*)wgrad;

  // dW tile ownership (see dw_phase), wave w = 4 half + wr: L1 nt{w} x kt{0,1}; L2 nt{0..5} x kt{w};
  // L3 nt{wr} x kt{3 half..+2}; L4 nt{wr} x kt{2 half, +1}; L5 nt{0} x kt{wr} (half 0 only)
  v4f acc1[2], acc2[6], acc3[3], acc4[2], acc5[1];
#pragma unroll
  for (int j = 0; j < 2; ++j) acc1[j] = acc4[j] = (v4f){0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j < 6; ++j) acc2[j] = (v4f){0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int j = 0; j < 3; ++j) acc3[j] = (v4f){0.f, 0.f, 0.f, 0.f};
  acc5[0] = (v4f){0.f, 0.f, 0.f, 0.f};
  float loss_sum = 0.f, dl_sum = 0.f;
  int ct1[2], ct2[6], ct3[3], ct4[2], ct5[1];  // compact slab positions of this wave's dW tiles
  if (TRAIN) {
    load_ct<K1, 1, 2>(ct1, TB1, w, 0, 0, 1, tmap);
    load_ct<K2, 6, 1>(ct2, TB2, 0, 1, w, 0, tmap);
    load_ct<K3, 1, 3>(ct3, TB3, wr, 0, 3 * half, 1, tmap);
    load_ct<K4, 1, 2>(ct4, TB4, wr, 0, 2 * half, 1, tmap);
    load_ct<K5, 1, 1>(ct5, TB5, 0, 0, wr, 0, tmap);
    if (half) ct5[0] = -1;  // L5 has 4 dW tiles: owned by half 0
  }

  uint16_t* A0 = lds + LA0;
  uint16_t* A1 = lds + LA1;
  uint16_t* A2 = lds + LA2;
  uint16_t* A3 = lds + LA3;
  uint16_t* A4 = lds + LA4;
  uint16_t* D5 = lds + LD5;
  uint16_t* P = lds + LP;
  uint16_t* Q = lds + LQ;

  // Branch-free record fetch (a conditional load makes hipcc drain vmcnt at the join, which
  // would serialise the prefetch). Rows past the batch read a valid record; they carry
  // dl = 0 and are excluded from loss and wide-gradient, so they contribute nothing.
  auto fetch = [&](int tile, uint4& a, uint4& b) {
    const long long row = min((long long)tile * T + 16 * wr + r, batch - 1);
    const long long di = mifx_feed_record(fd, fs, row, n_data);  // host guarantees batch <= n_data
    a = data[2 * di];
    b = data[2 * di + 1];
  };
  uint4 nu0, nu1;
  fetch(blockIdx.x, nu0, nu1);

  for (int tile = blockIdx.x; tile < ntiles; tile += gridDim.x) {
#ifdef WD_STAMPS
    // stamp the second tile of the workgroup when there is one (steady state: records prefetched)
    stamp_on = ntiles > (int)gridDim.x ? tile == (int)(blockIdx.x + gridDim.x) : tile == (int)blockIdx.x;
    STAMP(1);
#endif
    const long long row = (long long)tile * T + 16 * wr + r;
    const bool valid = row < batch;
    const uint4 u0 = nu0, u1 = nu1;
    fetch(tile + gridDim.x, nu0, nu1);  // prefetch the next tile's records

    const uint32_t idw[5] = {u0.w, u1.x, u1.y, u1.z, u1.w};
    int ids[9];
    float wv[9];
#pragma unroll
    for (int f = 0; f < 9; ++f) {
      int id = (f & 1) ? (idw[f >> 1] >> 16) : (idw[f >> 1] & 0xffff);
      id = id < kWideNb[f] ? id : 0;
      ids[f] = kWideOff[f] + id;
      wv[f] = wide[ids[f]];  // issued now, consumed after the forward
    }
    const float wbias = wide[WIDE_BIAS];
    if (h == 0 && half == 0) {
      v8bf x = {(bf16)__uint_as_float(u0.x), (bf16)__uint_as_float(u0.y), (bf16)__uint_as_float(u0.z),
                (bf16)1.0f, (bf16)0.f, (bf16)0.f, (bf16)0.f, (bf16)0.f};
      *(v8bf*)(A0 + (16 * wr + r) * (K1 + PAD)) = x;
    }
    // each layer's output is written by both waves of a row group: barrier before the next layer reads it
    block_sync_lds();
    v4f z5 = {0.f, 0.f, 0.f, 0.f};
    fwd_layer<K1, N1, false>(lds + LW1, A0, A1, wr, half, r, h, nullptr);
    block_sync_lds();
    fwd_layer<K2, N2, false>(lds + LW2, A1, A2, wr, half, r, h, nullptr);
    block_sync_lds();
    fwd_layer<K3, N3, false>(lds + LW3, A2, A3, wr, half, r, h, nullptr);
    block_sync_lds();
    fwd_layer<K4, N4, false>(lds + LW4, A3, A4, wr, half, r, h, nullptr);
    block_sync_lds();
    fwd_layer<K5, N5, true>(lds + LW5, A4, nullptr, wr, half, r, h, &z5);  // 1 n-tile: half 0
    STAMP(2);

    // ---- wide part + loss (every lane recomputes for example r; lane h==0 owns it)
    float wl = wbias;
#pragma unroll
    for (int f = 0; f < 9; ++f) wl += wv[f];
    const float x = __shfl(z5[0], r) + wl;
    const float y = (float)(idw[4] >> 16);
    const float lossv = fmaxf(x, 0.f) - x * y + log1pf(__expf(-fabsf(x)));
    if (!TRAIN) {
      if (h == 0 && half == 0 && valid) {
        logits_out[row] = x;
        loss_sum += lossv;
      }
      continue;
    }
    const float dl = valid ? (1.f / (1.f + __expf(-x)) - y) * grad_scale : 0.f;
    if (h == 0 && half == 0 && valid) {
      loss_sum += lossv;
      const int q = __float2int_rn(fminf(fmaxf(dl * qscale, -qmax), qmax));
#pragma unroll
      for (int f = 0; f < 9; ++f) atomicAdd(&wgi[ids[f]], q);
      dl_sum += dl;
    }
    if (half == 0) {
      v4bf o = {(bf16)(h == 0 ? dl : 0.f), (bf16)0.f, (bf16)0.f, (bf16)0.f};
      *(v4bf*)(D5 + (16 * wr + r) * (N5 + PAD) + 4 * h) = o;
    }
    block_sync_lds();  // D5 rows come from half 0, read by both halves
    STAMP(3);
    bwd_dA<K5, N5>(lds + LW5, D5, A4, P, wr, half, r, h);   // dz4 -> P
    STAMP(4);
    block_sync_lds();                                 // B1
    STAMP(5);
    if (half == 0) dw_phase<K5, N5, 1, 1>(acc5, D5, A4, 0, 0, wr, 0, r, h);
    dw_phase<K4, N4, 1, 2>(acc4, P, A3, wr, 0, 2 * half, 1, r, h);
    STAMP(6);
    bwd_dA<K4, N4>(lds + LW4, P, A3, Q, wr, half, r, h);    // dz3 -> Q
    STAMP(7);
    block_sync_lds();                                 // B2
    STAMP(8);
    dw_phase<K3, N3, 1, 3>(acc3, Q, A2, wr, 0, 3 * half, 1, r, h);
    STAMP(9);
    bwd_dA<K3, N3>(lds + LW3, Q, A2, P, wr, half, r, h);    // dz2 -> P
    STAMP(10);
    block_sync_lds();                                 // B3
    STAMP(11);
    dw_phase<K2, N2, 6, 1>(acc2, P, A1, 0, 1, w, 0, r, h);
    STAMP(12);
    bwd_dA<K2, N2>(lds + LW2, P, A1, Q, wr, half, r, h);    // dz1 -> Q
    STAMP(13);
    block_sync_lds();                                 // B4
    STAMP(14);
    dw_phase<K1, N1, 1, 2>(acc1, Q, A0, w, 0, 0, 1, r, h);
    STAMP(15);
    block_sync_lds();                                 // B5
    STAMP(16);
    stamp_on = false;
  }

  // ---- epilogue: per-workgroup slab
  for (int o = 32; o > 0; o >>= 1) {
    loss_sum += __shfl_xor(loss_sum, o);
    dl_sum += __shfl_xor(dl_sum, o);
  }
  if (lane == 0) {
    red[w] = loss_sum;
    red[NWAVE + w] = dl_sum;
  }
  if (TRAIN) {
    float* my = slab + (size_t)blockIdx.x * stride;
    store_tiles<1, 2>(my, acc1, ct1, lane);
    store_tiles<6, 1>(my, acc2, ct2, lane);
    store_tiles<1, 3>(my, acc3, ct3, lane);
    store_tiles<1, 2>(my, acc4, ct4, lane);
    store_tiles<1, 1>(my, acc5, ct5, lane);
  }
  __syncthreads();
  if (TRAIN) {
    float* my = slab + (size_t)blockIdx.x * stride + (stride - WIDE_PAD);
    for (int c = tid; c < WIDE_PAD; c += NTHR) {
      float v = (float)wgi[c] * qinv;
      if (c == WIDE_BIAS) {
#pragma unroll
        for (int i = 0; i < NWAVE; ++i) v += red[NWAVE + i];
      }
      my[c] = v;
    }
  }
  if (tid == 0 && slab_loss) {
    float l = 0.f;
#pragma unroll
    for (int i = 0; i < NWAVE; ++i) l += red[i];
    slab_loss[blockIdx.x] = l;
  }
  stamp_on = true;
  STAMP(17);
#ifdef WD_STAMPS
  __syncthreads();
  if (tid == 0 && blockIdx.x < 1024) g_blk[blockIdx.x][1] = __builtin_amdgcn_s_memrealtime();
#endif
}

// partial[sp][e] = sum_{g in split sp} slab[g][e]   (float4 granules, 4 loads in flight)
__global__ __launch_bounds__(256) void wd_reduce(const float4* __restrict__ slab, int G, int gchunk,
                                                 float4* __restrict__ partial, int stride) {
  const int S4 = stride / 4;
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= S4) return;
  const int g0 = blockIdx.y * gchunk;
  const int g1 = min(G, g0 + gchunk);
  float4 acc[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) acc[u] = make_float4(0, 0, 0, 0);
  int g = g0;
  for (; g + 3 < g1; g += 4) {
    float4 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) v[u] = slab[(size_t)(g + u) * S4 + e];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      acc[u].x += v[u].x; acc[u].y += v[u].y; acc[u].z += v[u].z; acc[u].w += v[u].w;
    }
  }
  for (; g < g1; ++g) {
    const float4 v = slab[(size_t)g * S4 + e];
    acc[0].x += v.x; acc[0].y += v.y; acc[0].z += v.z; acc[0].w += v.w;
  }
  partial[(size_t)blockIdx.y * S4 + e] =
      make_float4(acc[0].x + acc[1].x + acc[2].x + acc[3].x, acc[0].y + acc[1].y + acc[2].y + acc[3].y,
                  acc[0].z + acc[1].z + acc[2].z + acc[3].z, acc[0].w + acc[1].w + acc[2].w + acc[3].w);
}

#include "wd_opt.h"

// Step counters: the optimizer step is needed by every workgroup (Adam bias correction) and the next fused
// launch derives its data offset from it. A single counter bumped by one workgroup races with the others'
// reads, and a last-workgroup-done atomic costs an agent-scope fence (L2 writeback) per workgroup, so each
// workgroup owns a slot: step_ctr[blockIdx.x] is read and bumped by that workgroup only; slot 0 is the
// canonical step the fused kernel reads. All STEP_SLOTS slots start equal (host set_step).

// One thread per canonical parameter. DNN segment [0, WTOT) then wide segment [WTOT, WTOT+NWIDE).
__global__ __launch_bounds__(256) void wd_optimizer(
    const float* __restrict__ partial, int nparts, const int* __restrict__ gidx, const uint8_t* __restrict__ mask,
    float* __restrict__ param, float* __restrict__ s0, float* __restrict__ s1, uint16_t* __restrict__ wt_out,
    long long* __restrict__ step_ctr, OptHyper hd, OptHyper hw, int stride) {
  const int c = blockIdx.x * 256 + threadIdx.x;
  __shared__ long long s_step;
  if (threadIdx.x == 0) s_step = step_ctr[blockIdx.x] + 1;  // the slot's only reader and writer: thread 0
  __syncthreads();
  const long long step = s_step;
  if (c < WTOT + NWIDE) {
    const bool dnn = c < WTOT;
    float w = param[c];
    if (mask[c]) {
      const int gi = gidx[c];
      float gs[4] = {0.f, 0.f, 0.f, 0.f};
      int pidx = 0;
      for (; pidx + 3 < nparts; pidx += 4) {
#pragma unroll
        for (int u = 0; u < 4; ++u) gs[u] += partial[(size_t)(pidx + u) * stride + gi];
      }
      for (; pidx < nparts; ++pidx) gs[0] += partial[(size_t)pidx * stride + gi];
      const float g = (gs[0] + gs[1]) + (gs[2] + gs[3]);
      float a0 = s0[c], a1 = s1[c];
      w = opt_update(dnn ? hd : hw, w, g, a0, a1, step);
      s0[c] = a0;
      s1[c] = a1;
      param[c] = w;
    }
    if (dnn) wt_out[c] = __builtin_bit_cast(uint16_t, (bf16)w);
  }
  if (threadIdx.x == 0) step_ctr[blockIdx.x] = step;
}

// Fused slab reduction + optimizer: one workgroup owns RQ float4 columns (4*RQ gradient entries) of the
// compact slab and sums ALL G rows of them (row groups of 256/RQ threads, fixed order -> deterministic), so
// the full per-column gradient is available in one workgroup and the optimizer runs right there through
// the inverse map inv[slab column] -> canonical parameter (-1 = padding). Replaces wd_reduce + wd_optimizer
// (two launches, a [nsplit, stride] round trip) on the single-rank step; with OPT=false it is the local
// full reduction feeding the DP all-reduce.
constexpr int RQ = 16;               // float4 columns per workgroup
constexpr int RG = 256 / RQ;         // row groups
constexpr int RU = 8;            // slab rows in flight per thread (G=256: 322 workgroups x 256 threads x
                                     // 8 x 16 B = the whole 21 MB slab requested in two rounds; RU 16, all of
                                     // it in one round, measured 2 us slower per step: profiles/archive/wd_ab_r2s.txt)

// Column sums of the slab: float4 column q = blockIdx.x * RQ + threadIdx.x % RQ over rows [0, G), row groups of
// RG threads, fixed order (deterministic). The full sum is returned to threads threadIdx.x < RQ. (A chunk-major
// slab layout -- this workgroup's columns one contiguous [G][RQ] block -- measured no faster: profiles/archive/wd_ab_r2s.txt)
__device__ __forceinline__ float4 slab_column_sum(const float4* __restrict__ slab, int G, int S4,
                                                  float4 (&part)[RG][RQ]) {
  const int lq = threadIdx.x % RQ, r = threadIdx.x / RQ;
  const int q = blockIdx.x * RQ + lq;
  float4 acc[RU];
#pragma unroll
  for (int u = 0; u < RU; ++u) acc[u] = make_float4(0, 0, 0, 0);
  if (q < S4) {
    const float4* base = slab + q;
    const size_t rs = S4;
    int g = r;
    for (; g + (RU - 1) * RG < G; g += RU * RG) {
      float4 v[RU];
#pragma unroll
      for (int u = 0; u < RU; ++u) v[u] = base[(size_t)(g + u * RG) * rs];
#pragma unroll
      for (int u = 0; u < RU; ++u) {
        acc[u].x += v[u].x; acc[u].y += v[u].y; acc[u].z += v[u].z; acc[u].w += v[u].w;
      }
    }
    for (; g < G; g += RG) {
      const float4 v = base[(size_t)g * rs];
      acc[0].x += v.x; acc[0].y += v.y; acc[0].z += v.z; acc[0].w += v.w;
    }
  }
#pragma unroll
  for (int h = RU / 2; h >= 1; h /= 2)
#pragma unroll
    for (int u = 0; u < h; ++u) {
      acc[u].x += acc[u + h].x; acc[u].y += acc[u + h].y; acc[u].z += acc[u + h].z; acc[u].w += acc[u + h].w;
    }
  part[r][lq] = acc[0];
  __syncthreads();
  float4 s = make_float4(0, 0, 0, 0);
  if (threadIdx.x < RQ) {
    s = part[0][lq];
#pragma unroll
    for (int k = 1; k < RG; ++k) {
      const float4 v = part[k][lq];
      s.x += v.x; s.y += v.y; s.z += v.z; s.w += v.w;
    }
  }
  return s;
}

template <bool OPT>
__global__ __launch_bounds__(256) void wd_reduce_opt(
    const float4* __restrict__ slab, int G, int stride, float4* __restrict__ out, const int* __restrict__ inv,
    float* __restrict__ param, float* __restrict__ s0, float* __restrict__ s1, uint16_t* __restrict__ wt_out,
    const int* __restrict__ wmap, long long* __restrict__ step_ctr, OptHyper hd, OptHyper hw) {
  __shared__ float4 part[RG][RQ];
  __shared__ float gsum[4 * RQ];
  __shared__ long long s_step;
  if (OPT && threadIdx.x == 0) s_step = step_ctr[blockIdx.x] + 1;  // slot read and written by thread 0 only
  const int S4 = stride / 4;
  const int lq = threadIdx.x % RQ;
  const int q = blockIdx.x * RQ + lq;
  const float4 s = slab_column_sum(slab, G, S4, part);
  if (threadIdx.x < RQ) {
    if (!OPT) {
      if (q < S4) out[q] = s;
    } else {
      gsum[4 * lq + 0] = s.x; gsum[4 * lq + 1] = s.y; gsum[4 * lq + 2] = s.z; gsum[4 * lq + 3] = s.w;
    }
  }
  if (!OPT) return;
  __syncthreads();
  const long long step = s_step;
  if (threadIdx.x < 4 * RQ) {
    const int gi = blockIdx.x * 4 * RQ + threadIdx.x;
    const int c = gi < stride ? inv[gi] : -1;
    if (c >= 0) {
      const bool dnn = c < WTOT;
      float a0 = s0[c], a1 = s1[c];
      const float w = opt_update(dnn ? hd : hw, param[c], gsum[threadIdx.x], a0, a1, step);
      s0[c] = a0;
      s1[c] = a1;
      param[c] = w;
      // bf16 weight image: canonical order, or through wmap (canonical -> image offset) for the
      // register-chained kernel's C-ordered LDS image (csrc/wd_chain.hip)
      if (dnn) wt_out[wmap != nullptr ? wmap[c] : c] = __builtin_bit_cast(uint16_t, (bf16)w);
    }
  }
  if (threadIdx.x == 0) step_ctr[blockIdx.x] = step;
}

// Slab-column-order optimizer state (the register-chained trainer): param / s0 / s1 are indexed by slab column and
// wsc[col] says what the column is (-1 padding, -2 wide weight, >= 0 DNN weight with that bf16 weight-image offset).
// No indirection: a thread's state is loaded before the slab reduction starts and is in registers when the summed
// gradient arrives (the canonical-order kernel above must wait for the gradient's inv[] entry, then for param/s0/s1
// at that index, then for wmap).
__global__ __launch_bounds__(256) void wd_reduce_opt_sc(const float4* __restrict__ slab, int G, int stride,
                                                        const int* __restrict__ wsc, float* __restrict__ param,
                                                        float* __restrict__ s0, float* __restrict__ s1,
                                                        uint16_t* __restrict__ wt_out, long long* __restrict__ step_ctr,
                                                        OptHyper hd, OptHyper hw) {
  __shared__ float4 part[RG][RQ];
  __shared__ float gsum[4 * RQ];
  __shared__ long long s_step;
  if (threadIdx.x == 0) s_step = step_ctr[blockIdx.x] + 1;
  const int gi = blockIdx.x * 4 * RQ + threadIdx.x;
  ScState st{-1, 0.f, 0.f, 0.f};
  if (threadIdx.x < 4 * RQ) st = sc_load(gi, stride, wsc, param, s0, s1);  // in flight during the reduction
  const int lq = threadIdx.x % RQ;
  const float4 s = slab_column_sum(slab, G, stride / 4, part);
  if (threadIdx.x < RQ) {
    gsum[4 * lq + 0] = s.x; gsum[4 * lq + 1] = s.y; gsum[4 * lq + 2] = s.z; gsum[4 * lq + 3] = s.w;
  }
  __syncthreads();
  if (threadIdx.x < 4 * RQ) sc_update(gi, st, gsum[threadIdx.x], hd, hw, s_step, param, s0, s1, wt_out);
  if (threadIdx.x == 0) step_ctr[blockIdx.x] = s_step;
}

// One slab row (the reference batch's single fused workgroup, or the data-parallel all-reduced gradient): nothing
// to reduce, so one thread per column and a quarter of wd_reduce_opt_sc's workgroups (93 vs 370). Bit-identical:
// the general kernel's column sum of one row adds only zeros to it. Each workgroup owns step slot blockIdx.x, as
// there; a trainer always takes the same path (its slab height is fixed), so the slots it reads stay in step.
__global__ __launch_bounds__(256) void wd_opt1_sc(const float* __restrict__ slab, int stride,
                                                  const int* __restrict__ wsc, float* __restrict__ param,
                                                  float* __restrict__ s0, float* __restrict__ s1,
                                                  uint16_t* __restrict__ wt_out, long long* __restrict__ step_ctr,
                                                  OptHyper hd, OptHyper hw) {
  __shared__ long long s_step;
  if (threadIdx.x == 0) s_step = step_ctr[blockIdx.x] + 1;
  const int gi = blockIdx.x * 256 + threadIdx.x;
  const ScState st = sc_load(gi, stride, wsc, param, s0, s1);
  const float g = gi < stride ? slab[gi] : 0.f;
  __syncthreads();
  if (gi < stride) sc_update(gi, st, g, hd, hw, s_step, param, s0, s1, wt_out);
  if (threadIdx.x == 0) step_ctr[blockIdx.x] = s_step;
}

// system-scope (write-through / cache-bypassing) 32-bit stores and loads, for data another XCD or GPU reads
__device__ __forceinline__ void st_sys(float* p, float v) {
  __hip_atomic_store((unsigned int*)p, __float_as_uint(v), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ float ld_sys(const float* p) {
  return __uint_as_float(__hip_atomic_load((const unsigned int*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
}

// ---- xGMI exchange synchronisation (release / acquire at system scope; bounded, sticky failure)
// A rank publishes epoch e for a chunk with a RELEASE store of the flag (its partial stores are ordered before it:
// they are write-through system-scope stores, drained by the s_waitcnt before the workgroup barrier, and the
// release orders everything the workgroup did before the barrier), and a waiter re-reads the flag with relaxed
// loads and then issues an ACQUIRE fence before loading the partials. The wait is bounded by WALL-CLOCK time
// (s_memrealtime, 100 MHz): a peer that never arrives sets the rank's sticky err flag instead of hanging the
// GPU; every exchange kernel reads err first and does nothing once it is set (no publish, no parameter update,
// no counter advance) -- the peers then time out too, so every rank stops with its weights untouched by
// garbage and the host raises at its next check (FusedWideDeepTrainer._check_exchange).
constexpr long long XG_TIMEOUT_TICKS = 1000ll * 1000 * 1000;  // 10 s at the 100 MHz real-time clock

__device__ __forceinline__ bool xg_failed(const int* err) {
  return __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0;
}

__device__ __forceinline__ void xg_publish(unsigned int* flag, unsigned int e) {
  __hip_atomic_store(flag, e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}

// wait until *f reaches epoch e (wrapping compare); false on timeout or when another workgroup already failed
__device__ __forceinline__ bool xg_wait(const unsigned int* f, unsigned int e, int* err) {
  const long long t0 = wall_clock64();
  while ((int)(__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - e) < 0) {
    __builtin_amdgcn_s_sleep(2);
    if (xg_failed(err)) return false;
    if (wall_clock64() - t0 > XG_TIMEOUT_TICKS) {
      __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return false;
    }
  }
  return true;
}

// xGMI exchange peers (see the data-parallel section below)
constexpr int XG_MAXW = 8;
constexpr int XB_THR = 64;               // kernel B: one wave, one float4 column per thread
constexpr int XB_CHUNKS = XB_THR / RQ;   // chunks per kernel-B workgroup
struct XgPeers {
  const float* part[XG_MAXW];  // peer p's [2][stride] partial buffer (p == rank: our own)
  unsigned int* sig[XG_MAXW];   // peer p's flag array [chunks][XG_MAXW] (uncached)
};

// ---- XCD-local slab reduction + optimizer (the register-chained trainer's step on one GPU).
// The fused kernel's workgroups write their 82 KB slab rows into the L2 of the XCD they run on (8 XCDs, 4 MB L2
// each; 32 rows per XCD at grid 256). A one-pass reduction reads every row from every XCD: measured, the fused
// kernel then runs 29-30 us instead of 23 us (its slab writes pay for the lines the previous reduction pulled
// across XCDs), whatever cache policy the reduction's loads use (plain, nontemporal or agent-scope:
// profiles/archive/wd_ab_r2s.txt), and a standalone write + read-back of 21 MB costs 12 us against 3.6 us for re-reading
// a clean slab (tools/micro/launch_floor.hip). So:
//   level 1 (wd_reduce_xcd, 8 x 81 workgroups): workgroup (chunk c = blockIdx / 8) sums, for its 256 columns, only
//     the rows written on ITS OWN XCD (the fused kernel records each workgroup's XCD in xcd_of), ascending -- L2
//     hits -- into the per-XCD partial part[xcd], and stamps ok[xcd][c] with the epoch;
//   level 2 (wd_xcd_opt_sc, one thread per column): sums the per-XCD partials and runs the optimizer.
// Determinism: the dispatcher hands out workgroups round-robin over the XCDs but the starting XCD rotates with
// launch history, so level 2 adds the partials in the order of each XCD's FIRST row, not of XCD id: the same
// association for every rotation. Completeness: an XCD holding rows that no level-1 workgroup of a chunk ran on
// (another placement; XCC ids >= 8) is seen through the epoch stamps and summed from the slab by level 2 itself.
// (One kernel with a last-arriver finalizer measured slower, 12.9 us vs 5.0 + 6.0: its chain of write-through
// stores, counter atomic and partial loads is longer than a kernel boundary.)
constexpr int XMAX = 16;  // XCC_ID range
constexpr int X1C = 64;   // float4 columns per level-1 workgroup (1 KB of each slab row): one per lane of a wave
static_assert(X1C == 64, "wd_reduce_xcd maps lane -> float4 column of its chunk");

__global__ __launch_bounds__(256) void wd_reduce_xcd(const float4* __restrict__ slab, int G, int stride,
                                                     const int* __restrict__ xcd_of, float4* __restrict__ part,
                                                     int* __restrict__ ok, const long long* __restrict__ xep) {
  __shared__ int rows[256];
  __shared__ int wcnt[4];
  __shared__ float4 red[4][X1C];
  const int x = mifx_xcc_id();
  const int S4 = stride / 4, nc1 = (S4 + X1C - 1) / X1C;
  const int c = blockIdx.x / 8;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  // ascending list of the rows written on this XCD
  const bool sel = t < G && xcd_of[t] == x;
  const unsigned long long m = __ballot(sel);
  if (lane == 0) wcnt[w] = __popcll(m);
  __syncthreads();
  int base = 0;
  for (int i = 0; i < w; ++i) base += wcnt[i];
  if (sel) rows[base + __popcll(m & ((1ull << lane) - 1))] = t;
  const int n = wcnt[0] + wcnt[1] + wcnt[2] + wcnt[3];
  __syncthreads();
  if (c >= nc1) return;
  const int q = c * X1C + lane;
  float4 a = make_float4(0, 0, 0, 0);
  if (q < S4) {  // rows w, w + 4, ... of the list, 8 loads in flight (32 rows per XCD at grid 256: one round)
    constexpr int U = 8;
    for (int i0 = w; i0 < n; i0 += 4 * U) {
      float4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int i = i0 + 4 * u;
        v[u] = i < n ? slab[(size_t)rows[i] * S4 + q] : make_float4(0, 0, 0, 0);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        a.x += v[u].x; a.y += v[u].y; a.z += v[u].z; a.w += v[u].w;
      }
    }
  }
  red[w][lane] = a;
  __syncthreads();
  if (w == 0 && q < S4) {
    float4 sm = red[0][lane];
#pragma unroll
    for (int k2 = 1; k2 < 4; ++k2) {
      sm.x += red[k2][lane].x; sm.y += red[k2][lane].y; sm.z += red[k2][lane].z; sm.w += red[k2][lane].w;
    }
    part[(size_t)x * S4 + q] = sm;
  }
  if (t == 0) ok[x * nc1 + c] = (int)(xep[0] + 1);
}

// ---- residue-class two-level reduction (the register-chained trainer's default step tail on one GPU).
// Level 1 (wd_reduce_res, 8 x nchunks workgroups): workgroup j sums, for its 256 columns (chunk j / 8), the slab rows
// b == j (mod 8), ascending, into part[j % 8]. Level 2 (wd_res_opt_sc, one thread per column): part[0] + ... +
// part[7] in that order, then the optimizer. Both sums run over fixed row sets in a fixed order whatever the
// placement, so the step is deterministic with no record of where anything ran, and neither kernel has a dependent
// load before its data loads (wd_reduce_xcd first reads xcd_of, wd_xcd_opt_sc orders the XCDs and checks epoch
// stamps). Locality: the dispatcher hands workgroups to the XCDs round-robin from a pointer that carries over between
// launches, and both the fused kernel's grid (256) and this one's (8 x nchunks) are multiples of 8, so fused
// workgroup b and level-1 workgroup j with j == b (mod 8) run on the same XCD and the rows are L2 hits -- as in
// wd_reduce_xcd. A placement that breaks this only costs cross-XCD reads, never a different result.
__global__ __launch_bounds__(256) void wd_reduce_res(const float4* __restrict__ slab, int G, int stride,
                                                     float4* __restrict__ part) {
  __shared__ float4 red[4][X1C];
  const int S4 = stride / 4;
  const int k = blockIdx.x & 7, c = blockIdx.x >> 3;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int q = c * X1C + lane;
  float4 a = make_float4(0, 0, 0, 0);
  if (q < S4) {  // rows k + 8 (w + 4 i): 8 loads in flight per thread (32 rows per residue at G = 256: one round)
    constexpr int U = 8;
    for (int i0 = k + 8 * w; i0 < G; i0 += 32 * U) {
      float4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int r = i0 + 32 * u;
        v[u] = r < G ? slab[(size_t)r * S4 + q] : make_float4(0, 0, 0, 0);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        a.x += v[u].x; a.y += v[u].y; a.z += v[u].z; a.w += v[u].w;
      }
    }
  }
  red[w][lane] = a;
  __syncthreads();
  if (w == 0 && q < S4) {
    float4 sm = red[0][lane];
#pragma unroll
    for (int k2 = 1; k2 < 4; ++k2) {
      sm.x += red[k2][lane].x; sm.y += red[k2][lane].y; sm.z += red[k2][lane].z; sm.w += red[k2][lane].w;
    }
    part[(size_t)k * S4 + q] = sm;
  }
}

// level 2 of the residue-class reduction: MODE 0 plain sum into out, 1 optimizer on slab-order state
template <int MODE>
__global__ __launch_bounds__(256) void wd_res_opt_sc(const float* __restrict__ part, int stride, float* __restrict__ out,
                                                     const int* __restrict__ wsc, float* __restrict__ param,
                                                     float* __restrict__ s0, float* __restrict__ s1,
                                                     uint16_t* __restrict__ wt_out, long long* __restrict__ step_ctr,
                                                     OptHyper hd, OptHyper hw) {
  const int t = threadIdx.x, gi = blockIdx.x * 256 + t;
  const long long step = MODE == 1 ? step_ctr[blockIdx.x] + 1 : 0;
  float pv[8];
#pragma unroll
  for (int x = 0; x < 8; ++x) pv[x] = gi < stride ? part[(size_t)x * stride + gi] : 0.f;
  ScState st{-1, 0.f, 0.f, 0.f};
  if (MODE == 1) st = sc_load(gi, stride, wsc, param, s0, s1);
  if (gi < stride) {
    float g = pv[0];
#pragma unroll
    for (int x = 1; x < 8; ++x) g += pv[x];
    if (MODE == 0) out[gi] = g;
    if (MODE == 1) sc_update(gi, st, g, hd, hw, step, param, s0, s1, wt_out);
  }
  if (MODE == 1) {
    if (t == 0) step_ctr[blockIdx.x] = step;
    if (blockIdx.x == 0)
      for (int i = gridDim.x + t; i < STEP_SLOTS; i += 256) step_ctr[i] = step;
  }
}

// Both levels in ONE launch (opt-in, MIFX_WD_RES_FUSED=1): level 1 exactly as wd_reduce_res; the LAST of a
// chunk's 8 residue workgroups to finish (a per-chunk ticket) then adds the chunk's 8 partials in residue order and
// applies the optimizer to its 256 columns -- wd_res_opt_sc<1>'s sums and state updates, bit for bit, without the
// second launch. The partials are stored and loaded at agent scope (coherent across the XCDs' L2s) and completed
// before the ticket increment; the last arriver resets the ticket. No workgroup ever waits for another.
__global__ __launch_bounds__(256) void wd_reduce_res_fused(const float4* __restrict__ slab, int G, int stride,
                                                           float* __restrict__ part, int* __restrict__ ticket,
                                                           const int* __restrict__ wsc, float* __restrict__ param,
                                                           float* __restrict__ s0, float* __restrict__ s1,
                                                           uint16_t* __restrict__ wt_out,
                                                           long long* __restrict__ step_ctr, OptHyper hd, OptHyper hw) {
  __shared__ float4 red[4][X1C];
  __shared__ int last;
  const int S4 = stride / 4, nc1 = (S4 + X1C - 1) / X1C;
  const int k = blockIdx.x & 7, c = blockIdx.x >> 3;
  const int t = threadIdx.x, lane = t & 63, w = t >> 6;
  const int q = c * X1C + lane;
  float4 a = make_float4(0, 0, 0, 0);
  if (q < S4) {
    constexpr int U = 8;
    for (int i0 = k + 8 * w; i0 < G; i0 += 32 * U) {
      float4 v[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int r = i0 + 32 * u;
        v[u] = r < G ? slab[(size_t)r * S4 + q] : make_float4(0, 0, 0, 0);
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        a.x += v[u].x; a.y += v[u].y; a.z += v[u].z; a.w += v[u].w;
      }
    }
  }
  red[w][lane] = a;
  __syncthreads();
  if (w == 0 && q < S4) {
    float4 sm = red[0][lane];
#pragma unroll
    for (int k2 = 1; k2 < 4; ++k2) {
      sm.x += red[k2][lane].x; sm.y += red[k2][lane].y; sm.z += red[k2][lane].z; sm.w += red[k2][lane].w;
    }
    float* dst = part + (size_t)k * stride + 4 * q;
    __hip_atomic_store(dst + 0, sm.x, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(dst + 1, sm.y, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(dst + 2, sm.z, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(dst + 3, sm.w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (t == 0) {
    // wave 0 made the partial stores; they are agent-scope (coherent across the XCDs' L2s), so completing them
    // (vmcnt 0) before the increment orders them -- a release fence here (an L2 writeback) measured ~5 us slower
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    __builtin_amdgcn_s_waitcnt(0);
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    const int old = __hip_atomic_fetch_add(ticket + c, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    last = old == 7;
  }
  __syncthreads();
  if (!last) return;
  const int gi = c * 256 + t;
  const long long step = step_ctr[c] + 1;
  float pv[8];
#pragma unroll
  for (int x = 0; x < 8; ++x)
    pv[x] = gi < stride ? __hip_atomic_load(part + (size_t)x * stride + gi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                        : 0.f;
  ScState st = sc_load(gi, stride, wsc, param, s0, s1);
  if (gi < stride) {
    float g = pv[0];
#pragma unroll
    for (int x = 1; x < 8; ++x) g += pv[x];
    sc_update(gi, st, g, hd, hw, step, param, s0, s1, wt_out);
  }
  if (t == 0) {
    step_ctr[c] = step;
    __hip_atomic_store(ticket + c, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  if (c == 0)
    for (int i = nc1 + t; i < STEP_SLOTS; i += 256) step_ctr[i] = step;
}

// level 2: one thread per slab column. MODE 0: plain sum into out; 1: optimizer on slab-order state; 2: xGMI data
// parallelism, publish half -- store the local sum into half (epoch & 1) of this rank's IPC buffer and stamp the 4
// RQ-float4 chunks' flags in every peer, no wait (wd_xgmi_gather_opt waits, gathers and applies the optimizer in
// one-wave workgroups); 3: the same with the wait, the gather over xGMI and the optimizer in this kernel (opt-in,
// MIFX_XGMI_FUSED_WAIT=1: one launch fewer, but 256-thread workgroups spin on the peers).
template <int MODE>
__global__ __launch_bounds__(256) void wd_xcd_opt_sc(const float* __restrict__ part, const int* __restrict__ ok,
                                                     const float* __restrict__ slab, int G, int stride,
                                                     const int* __restrict__ xcd_of, long long* __restrict__ xep,
                                                     float* __restrict__ out, const int* __restrict__ wsc,
                                                     float* __restrict__ param, float* __restrict__ s0,
                                                     float* __restrict__ s1, uint16_t* __restrict__ wt_out,
                                                     long long* __restrict__ step_ctr, OptHyper hd, OptHyper hw,
                                                     XgPeers peers, int world, int rank,
                                                     long long* __restrict__ xctr,
                                                     const unsigned int* __restrict__ my_sig,
                                                     int* __restrict__ err) {
  __shared__ int first[XMAX];
  __shared__ int order[XMAX];
  __shared__ int nord;
  __shared__ long long s_e, s_step;
  __shared__ int s_bad;
  const int t = threadIdx.x;
  constexpr bool opt = MODE == 1 || MODE == 3;
  if (MODE >= 2) {  // the exchange already failed on this rank: touch nothing (see xg_wait)
    if (t == 0) s_bad = xg_failed(err) ? 1 : 0;
    __syncthreads();
    if (s_bad) return;
  }
  if (t < XMAX) first[t] = 1 << 30;
  if (t == 0) {
    s_e = xep[blockIdx.x] + 1;
    if (opt) s_step = step_ctr[blockIdx.x] + 1;
  }
  const int gi = blockIdx.x * 256 + t;
  const int S4 = stride / 4, nc1 = (S4 + X1C - 1) / X1C;
  const int c1 = min(gi, stride - 1) / 4 / X1C;
  // everything in flight at once: the row XCDs, the 8 stamps and 8 partials of this column, the optimizer state
  const int xo = t < G ? xcd_of[t] : -1;
  int okv[8];
  float pv[8];
#pragma unroll
  for (int x = 0; x < 8; ++x) {
    okv[x] = ok[x * nc1 + c1];
    pv[x] = gi < stride ? part[(size_t)x * stride + gi] : 0.f;
  }
  ScState st{-1, 0.f, 0.f, 0.f};
  if (opt) st = sc_load(gi, stride, wsc, param, s0, s1);
  __syncthreads();
  if (xo >= 0) atomicMin(&first[xo], t);
  __syncthreads();
  if (t < XMAX) {  // XCDs holding rows, by first row: lane t's rank among the distinct valid first rows (a serial
                   // insertion sort by one lane cost ~1.5 us of dependent LDS round trips per workgroup)
    const int f = first[t];
    const bool valid = f < (1 << 30);
    int rank = 0;
#pragma unroll
    for (int y = 0; y < XMAX; ++y) rank += first[y] < f ? 1 : 0;
    if (valid) order[rank] = t;
    const unsigned long long vm = __ballot(valid);
    if (t == 0) nord = __popcll(vm);
  }
  __syncthreads();
  const int e = (int)s_e;
  float g = 0.f;
  if (gi < stride) {
    for (int k2 = 0; k2 < nord; ++k2) {
      const int xx = order[k2];
      float v = 0.f;
#pragma unroll
      for (int x = 0; x < 8; ++x)
        if (x == xx) v = pv[x];
      if (!(xx < 8 && okv[xx & 7] == e)) {  // no level-1 workgroup ran on XCD xx for this chunk: its rows, here
        v = 0.f;
        for (int r = 0; r < G; ++r)
          if (xcd_of[r] == xx) v += slab[(size_t)r * stride + gi];
      }
      g += v;
    }
    if (MODE == 0) out[gi] = g;
    if (MODE == 1) sc_update(gi, st, g, hd, hw, s_step, param, s0, s1, wt_out);
  }
  if (MODE == 2) {  // publish only: the wait, gather and optimizer run in wd_xgmi_gather_opt (one-wave waiters)
    const long long ex = xctr[blockIdx.x] + 1;  // exchange epoch: slot b is advanced by the gather kernel's block b
    const size_t hoff = (size_t)(ex & 1) * stride;
    if (gi < stride) {
      st_sys((float*)peers.part[rank] + hoff + gi, g);
      __builtin_amdgcn_s_waitcnt(0);  // acknowledged before the chunk flags below
    }
    __syncthreads();
    const int nch = (stride / 4 + RQ - 1) / RQ;
    if (t < 4 * world) {
      const int cc = 4 * blockIdx.x + t / world, p = t % world;
      if (cc < nch) xg_publish(peers.sig[p] + cc * XG_MAXW + rank, (unsigned int)ex);
    }
  }
  if (MODE == 3) {
    const long long ex = xctr[blockIdx.x] + 1;  // exchange epoch (own slot)
    const unsigned int uex = (unsigned int)ex;
    const size_t hoff = (size_t)(ex & 1) * stride;
    if (gi < stride) {
      st_sys((float*)peers.part[rank] + hoff + gi, g);
      __builtin_amdgcn_s_waitcnt(0);  // acknowledged before the chunk flags below
    }
    __syncthreads();
    // the 256 columns are 4 exchange chunks of RQ float4: stamp each in every peer, then wait for every peer's
    const int nch = (stride / 4 + RQ - 1) / RQ;
    if (t < 4 * world) {
      const int cc = 4 * blockIdx.x + t / world, p = t % world;
      if (cc < nch) {
        xg_publish(peers.sig[p] + cc * XG_MAXW + rank, uex);
        if (!xg_wait(my_sig + cc * XG_MAXW + p, uex, err)) s_bad = 1;
      }
    }
    __syncthreads();
    if (s_bad) return;  // a peer never arrived: no update, no counter advance (err is set)
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // the peers' partials published before their flags
    if (gi < stride) {
      float pv2[XG_MAXW];
#pragma unroll
      for (int p = 0; p < XG_MAXW; ++p) pv2[p] = p < world ? ld_sys(peers.part[p] + hoff + gi) : 0.f;
      float gs = pv2[0];
#pragma unroll
      for (int p = 1; p < XG_MAXW; ++p)
        if (p < world) gs += pv2[p];
      sc_update(gi, st, gs, hd, hw, s_step, param, s0, s1, wt_out);
    }
    __syncthreads();
    if (t == 0) xctr[blockIdx.x] = ex;
    if (blockIdx.x == 0)
      for (int i = gridDim.x + t; i < STEP_SLOTS; i += 256) xctr[i] = ex;
  }
  __syncthreads();
  if (t == 0) {
    xep[blockIdx.x] = s_e;
    if (opt) step_ctr[blockIdx.x] = s_step;
  }
  if (blockIdx.x == 0)
    for (int i = gridDim.x + t; i < STEP_SLOTS; i += 256) {
      xep[i] = s_e;
      if (opt) step_ctr[i] = s_step;
    }
}

// ---- data parallelism over xGMI: one-shot cross-GPU exchange of the local gradient, no host collective
// (mifx/parallel/xgmi.py). Two kernels per step after the fused fwd/bwd:
//   A wd_reduce_xgmi_publish (322 workgroups): workgroup c sums its RQ float4 columns ("chunk c") over the G slab
//     rows (as wd_reduce_opt, fixed order), stores the chunk into half (epoch & 1) of this rank's IPC-shared
//     partial buffer with system-scope (write-through) stores, waits for their completion and publishes epoch e
//     for chunk c into every peer's flag array (uncached memory): sig[c][rank] = e. No waiting.
//   B wd_xgmi_gather_opt (81 one-wave workgroups, 4 chunks each): waits until all ranks published e for its
//     chunks (bounded spin: a peer that never arrives sets err, no wave can hang), loads the world partials from
//     the peers' HBM over xGMI with system-scope loads, sums them in rank order -- identical on every rank, so
//     the replicas stay bit-identical -- and runs the optimizer on its columns.
// No cache-wide writeback or invalidate anywhere. The waiting kernel is small on purpose: it never holds the CUs
// another rank's fused kernel needs (ranks sharing a GPU in tests, or anything else running on the node).
// Double buffering by epoch parity makes one flag per epoch enough: rank r rewrites half e & 1 of chunk c only in
// epoch e + 2, after its epoch e + 1 kernel B saw every peer's e + 1 flag for chunk c, which that peer published
// after its epoch-e kernel B (its reads of chunk c) completed. The W&D gradient is one 82 KB bucket: every GPU
// reads 7 x 82 KB over 7 point-to-point xGMI links in one round.


// epoch of the coming exchange: xctr holds the last completed one (per-workgroup slots of kernel B; kernel A
// reads slot 0, written by kernel B's workgroup 0 of the previous step)
__global__ __launch_bounds__(256) void wd_reduce_xgmi_publish(const float4* __restrict__ slab, int G, int stride,
                                                              XgPeers peers, int world, int rank,
                                                              const long long* __restrict__ xctr,
                                                              const int* __restrict__ err) {
  __shared__ float4 part[RG][RQ];
  __shared__ int s_bad;
  if (threadIdx.x == 0) s_bad = xg_failed(err) ? 1 : 0;
  __syncthreads();
  if (s_bad) return;  // failed exchange: publish nothing (the peers time out and stop too)
  const int S4 = stride / 4;
  const int q = blockIdx.x * RQ + threadIdx.x % RQ;
  const long long e = xctr[0] + 1;
  const float4 s = slab_column_sum(slab, G, S4, part);
  if (threadIdx.x < RQ && q < S4) {
    float* dst = (float*)peers.part[rank] + (size_t)(e & 1) * stride + 4 * q;
    st_sys(dst + 0, s.x);
    st_sys(dst + 1, s.y);
    st_sys(dst + 2, s.z);
    st_sys(dst + 3, s.w);
    __builtin_amdgcn_s_waitcnt(0);  // the chunk's stores acknowledged before the flag below
  }
  __syncthreads();
  if (threadIdx.x < world) xg_publish(peers.sig[threadIdx.x] + blockIdx.x * XG_MAXW + rank, (unsigned int)e);
}

template <bool OPT>
__global__ __launch_bounds__(XB_THR) void wd_xgmi_gather_opt(
    int stride, XgPeers peers, int world, const unsigned int* __restrict__ my_sig, int* __restrict__ err,
    long long* __restrict__ xctr, float4* __restrict__ out, const int* __restrict__ wsc, float* __restrict__ param,
    float* __restrict__ s0, float* __restrict__ s1, uint16_t* __restrict__ wt_out,
    long long* __restrict__ step_ctr, OptHyper hd, OptHyper hw) {
  const int t = threadIdx.x;
  // one wave: a lane-uniform early exit needs no barrier
  if (xg_failed(err)) return;
  const int q0 = blockIdx.x * XB_THR + t;
  ScState st[4];
  if (OPT) {  // slab-order optimizer state, in flight during the wait
#pragma unroll
    for (int j = 0; j < 4; ++j) st[j] = sc_load(4 * q0 + j, stride, wsc, param, s0, s1);
  }
  const long long e = xctr[blockIdx.x] + 1;  // one wave: every lane reads the slot, no LDS broadcast needed
  const long long step = OPT ? step_ctr[blockIdx.x] + 1 : 0;
  const unsigned int ue = (unsigned int)e;
  const int nchunks = (stride / 4 + RQ - 1) / RQ;
  bool ok = true;
  {  // lane t waits for flag (chunk XB_CHUNKS * blockIdx.x + t / world, rank t % world)
    const int c = XB_CHUNKS * blockIdx.x + t / max(world, 1);
    if (t < XB_CHUNKS * world && c < nchunks) ok = xg_wait(my_sig + c * XG_MAXW + t % world, ue, err);
  }
  // any lane's timeout stops the whole wave: no update, no counter advance (err is set)
  if (__ballot(!ok) != 0ull) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // the peers' partials published before their flags
  const int S4 = stride / 4;
  const int q = blockIdx.x * XB_THR + t;
  if (q < S4) {
    const size_t off = (size_t)(e & 1) * stride + 4 * q;
    float v[XG_MAXW][4];
#pragma unroll
    for (int p = 0; p < XG_MAXW; ++p)
      if (p < world) {
#pragma unroll
        for (int j = 0; j < 4; ++j) v[p][j] = ld_sys(peers.part[p] + off + j);
      }
    float g4[4] = {v[0][0], v[0][1], v[0][2], v[0][3]};
#pragma unroll
    for (int p = 1; p < XG_MAXW; ++p)
      if (p < world) {
#pragma unroll
        for (int j = 0; j < 4; ++j) g4[j] += v[p][j];
      }
    if (!OPT) {
      out[q] = make_float4(g4[0], g4[1], g4[2], g4[3]);
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) sc_update(4 * q + j, st[j], g4[j], hd, hw, step, param, s0, s1, wt_out);
    }
  }
  __syncthreads();  // every lane read its slots before lane 0 moves them on
  if (t == 0) {
    xctr[blockIdx.x] = e;
    if (OPT) step_ctr[blockIdx.x] = step;
  }
  // keep the slots no workgroup of this grid owns equal to the canonical values
  if (blockIdx.x == 0)
    for (int i = gridDim.x + t; i < STEP_SLOTS; i += XB_THR) {
      xctr[i] = e;
      if (OPT) step_ctr[i] = step;
    }
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
                  float* logits_out, float grad_scale, int grid, int train, const int* tmap, int stride,
                  const int* stage_dims, long long feed_stride, long long feed_offset, unsigned long long shuffle_key,
                  hipStream_t stream) {
  static bool attr_done = false;
  if (!attr_done) {
    (void)hipFuncSetAttribute((const void*)wd_fused<true>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
    (void)hipFuncSetAttribute((const void*)wd_fused<false>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES);
    attr_done = true;
  }
  if (grid <= 0 || n_data <= 0 || batch <= 0 || batch > n_data) return -1;
  if (train && (tmap == nullptr || stride < WIDE_PAD || stride > STRIDE || stride % 4 != 0)) return -1;
  if (feed_stride < batch || feed_offset < 0 || feed_offset + batch > feed_stride) return -1;
  const MifxFeed fd{feed_stride, feed_offset, shuffle_key};
  // stage_dims (host array of 10 ints: rows[5], granules-per-row[5]); null = the whole padded image
  StageDims sd;
  const int KL[5] = {K1, K2, K3, K4, K5}, NL[5] = {N1, N2, N3, N4, N5};
  sd.total = 0;
  for (int l = 0; l < 5; ++l) {
    sd.rows[l] = stage_dims ? stage_dims[l] : NL[l];
    sd.gpr[l] = stage_dims ? stage_dims[5 + l] : KL[l] / 8;
    if (sd.rows[l] < 1 || sd.rows[l] > NL[l] || sd.gpr[l] < 1 || sd.gpr[l] > KL[l] / 8) return -1;
    sd.total += sd.rows[l] * sd.gpr[l];
  }
  if (train)
    hipLaunchKernelGGL(wd_fused<true>, dim3(grid), dim3(NTHR), LDS_BYTES, stream, (const uint4*)data, n_data, batch,
                       start_fixed, step_ctr, (const uint16_t*)wt, wide, slab, slab_loss, logits_out, grad_scale,
                       tmap, stride, sd, fd);
  else
    hipLaunchKernelGGL(wd_fused<false>, dim3(grid), dim3(NTHR), LDS_BYTES, stream, (const uint4*)data, n_data, batch,
                       start_fixed, step_ctr, (const uint16_t*)wt, wide, slab, slab_loss, logits_out, grad_scale,
                       tmap, stride, sd, fd);
  return (int)hipGetLastError();
}

int mifx_wd_reduce(const float* slab, int G, int nsplit, float* partial, int stride, hipStream_t stream) {
  if (G <= 0 || nsplit <= 0 || stride <= 0 || stride > STRIDE || stride % 4 != 0) return -1;
  const int gchunk = (G + nsplit - 1) / nsplit;
  dim3 grid((stride / 4 + 255) / 256, nsplit);
  hipLaunchKernelGGL(wd_reduce, grid, dim3(256), 0, stream, (const float4*)slab, G, gchunk, (float4*)partial, stride);
  return (int)hipGetLastError();
}

int mifx_wd_optimizer(const float* partial, int nparts, const int* gidx, const uint8_t* mask, float* param,
                      float* s0, float* s1, void* wt_out, long long* step_ctr, const float* hyper_dnn,
                      const float* hyper_wide, int stride, hipStream_t stream) {
  OptHyper hd{(int)hyper_dnn[0], hyper_dnn[1], hyper_dnn[2], hyper_dnn[3], hyper_dnn[4], hyper_dnn[5], hyper_dnn[6],
              hyper_dnn[7]};
  OptHyper hw{(int)hyper_wide[0], hyper_wide[1], hyper_wide[2], hyper_wide[3], hyper_wide[4], hyper_wide[5],
              hyper_wide[6], hyper_wide[7]};
  const int n = WTOT + NWIDE;
  static_assert((WTOT + NWIDE + 255) / 256 <= STEP_SLOTS, "optimizer grid exceeds the step slots");
  hipLaunchKernelGGL(wd_optimizer, dim3((n + 255) / 256), dim3(256), 0, stream, partial, nparts, gidx, mask, param, s0,
                     s1, (uint16_t*)wt_out, step_ctr, hd, hw, stride);
  return (int)hipGetLastError();
}

// slab [G, stride] -> full sum; with inv != null the optimizer is applied in the same launch (out unused),
// otherwise the sum is written to out [stride]. wmap (nullable): canonical DNN index -> bf16 image offset. step_ctr must hold STEP_SLOTS int64 (per-workgroup step slots).
int mifx_wd_reduce_opt(const float* slab, int G, int stride, float* out, const int* inv, float* param, float* s0,
                       float* s1, void* wt_out, const int* wmap, long long* step_ctr, const float* hyper_dnn,
                       const float* hyper_wide, hipStream_t stream) {
  if (G <= 0 || stride <= 0 || stride > STRIDE || stride % 4 != 0) return -1;
  const dim3 grid((stride / 4 + RQ - 1) / RQ);
  if (grid.x > STEP_SLOTS) return -1;
  if (inv == nullptr) {
    if (out == nullptr) return -1;
    hipLaunchKernelGGL(wd_reduce_opt<false>, grid, dim3(256), 0, stream, (const float4*)slab, G, stride,
                       (float4*)out, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, OptHyper{},
                       OptHyper{});
    return (int)hipGetLastError();
  }
  if (param == nullptr || s0 == nullptr || s1 == nullptr || wt_out == nullptr || step_ctr == nullptr) return -1;
  OptHyper hd{(int)hyper_dnn[0], hyper_dnn[1], hyper_dnn[2], hyper_dnn[3], hyper_dnn[4], hyper_dnn[5], hyper_dnn[6],
              hyper_dnn[7]};
  OptHyper hw{(int)hyper_wide[0], hyper_wide[1], hyper_wide[2], hyper_wide[3], hyper_wide[4], hyper_wide[5],
              hyper_wide[6], hyper_wide[7]};
  hipLaunchKernelGGL(wd_reduce_opt<true>, grid, dim3(256), 0, stream, (const float4*)slab, G, stride, nullptr, inv,
                     param, s0, s1, (uint16_t*)wt_out, wmap, step_ctr, hd, hw);
  return (int)hipGetLastError();
}

// slab [G, stride] -> local sum -> xGMI exchange over `world` ranks -> optimizer (inv != null) or the plain
// global sum into out [stride] (inv == null; self-test). Two launches (A publish, B gather). parts / sigs: host
// arrays of world device pointers (peer buffers opened through IPC; [rank] = our own; parts [2][stride] fp32,
// sigs [chunks][8] uint32 uncached). xctr: STEP_SLOTS int64 epoch slots (all equal), err: device int set to 1
// if a peer never published.
int mifx_wd_xgmi_chunks(int stride) { return (stride / 4 + RQ - 1) / RQ; }

int mifx_wd_reduce_xgmi_opt(const float* slab, int G, int stride, const void* const* parts, void* const* sigs,
                            int world, int rank, const unsigned int* my_sig, int* err, long long* xctr, float* out,
                            const int* wsc, float* param, float* s0, float* s1, void* wt_out,
                            long long* step_ctr, const float* hyper_dnn, const float* hyper_wide,
                            const int* xcd_of, float* xpart, int* xok, long long* xep, hipStream_t stream) {
  if (G <= 0 || world < 1 || world > XG_MAXW || rank < 0 || rank >= world || stride <= 0 || stride > STRIDE ||
      stride % 4 != 0 || my_sig == nullptr || err == nullptr || xctr == nullptr)
    return -1;
  XgPeers pe{};
  for (int p = 0; p < world; ++p) {
    if (parts[p] == nullptr || sigs[p] == nullptr) return -1;
    pe.part[p] = (const float*)parts[p];
    pe.sig[p] = (unsigned int*)sigs[p];
  }
  const dim3 ga(mifx_wd_xgmi_chunks(stride)), gb((stride / 4 + XB_THR - 1) / XB_THR);
  if ((int)gb.x > STEP_SLOTS) return -1;
  if (wsc == nullptr && out == nullptr) return -1;
  if (wsc != nullptr && (param == nullptr || s0 == nullptr || s1 == nullptr || wt_out == nullptr ||
                         step_ctr == nullptr))
    return -1;
  if (wsc != nullptr && xcd_of != nullptr && xpart != nullptr && xok != nullptr && xep != nullptr && G <= 256) {
    // XCD-local level 1, then level 2 publishes, waits, gathers and applies the optimizer (wd_xcd_opt_sc<3>)
    const int nc1 = (stride / 4 + X1C - 1) / X1C;
    const dim3 g2((stride + 255) / 256);
    if ((int)g2.x != (int)gb.x) return -1;  // both paths keep the same number of xctr slots
    OptHyper hd{(int)hyper_dnn[0], hyper_dnn[1], hyper_dnn[2], hyper_dnn[3], hyper_dnn[4], hyper_dnn[5],
                hyper_dnn[6], hyper_dnn[7]};
    OptHyper hw{(int)hyper_wide[0], hyper_wide[1], hyper_wide[2], hyper_wide[3], hyper_wide[4], hyper_wide[5],
                hyper_wide[6], hyper_wide[7]};
    hipLaunchKernelGGL(wd_reduce_xcd, dim3(8 * nc1), dim3(256), 0, stream, (const float4*)slab, G, stride, xcd_of,
                       (float4*)xpart, xok, xep);
    static const bool fused_wait = getenv("MIFX_XGMI_FUSED_WAIT") != nullptr && getenv("MIFX_XGMI_FUSED_WAIT")[0] == '1';
    if (fused_wait) {  // (opt-in) publish + wait + gather + optimizer in the 256-thread level-2 workgroups
      hipLaunchKernelGGL(wd_xcd_opt_sc<3>, g2, dim3(256), 0, stream, xpart, xok, slab, G, stride, xcd_of, xep,
                         nullptr, wsc, param, s0, s1, (uint16_t*)wt_out, step_ctr, hd, hw, pe, world, rank, xctr,
                         my_sig, err);
      return (int)hipGetLastError();
    }
    // default: the level-2 workgroups sum the XCD partials and PUBLISH, and never wait; the wait runs in the
    // one-wave workgroups of wd_xgmi_gather_opt (as on the non-XCD path), so no 256-thread workgroup ever spins
    // on a peer: a rank's waiting kernel cannot hold the CU slots a peer's fused kernel needs when ranks share a
    // GPU, and on separate GPUs each spinner is one wave
    hipLaunchKernelGGL(wd_xcd_opt_sc<2>, g2, dim3(256), 0, stream, xpart, xok, slab, G, stride, xcd_of, xep, nullptr,
                       wsc, param, s0, s1, (uint16_t*)wt_out, step_ctr, hd, hw, pe, world, rank, xctr, my_sig, err);
    hipLaunchKernelGGL(wd_xgmi_gather_opt<true>, gb, dim3(XB_THR), 0, stream, stride, pe, world, my_sig, err, xctr,
                       nullptr, wsc, param, s0, s1, (uint16_t*)wt_out, step_ctr, hd, hw);
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL(wd_reduce_xgmi_publish, ga, dim3(256), 0, stream, (const float4*)slab, G, stride, pe, world, rank,
                     xctr, err);
  if (wsc == nullptr) {  // plain sum into out
    hipLaunchKernelGGL(wd_xgmi_gather_opt<false>, gb, dim3(XB_THR), 0, stream, stride, pe, world, my_sig, err, xctr,
                       (float4*)out, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, OptHyper{}, OptHyper{});
    return (int)hipGetLastError();
  }
  OptHyper hd{(int)hyper_dnn[0], hyper_dnn[1], hyper_dnn[2], hyper_dnn[3], hyper_dnn[4], hyper_dnn[5], hyper_dnn[6],
              hyper_dnn[7]};
  OptHyper hw{(int)hyper_wide[0], hyper_wide[1], hyper_wide[2], hyper_wide[3], hyper_wide[4], hyper_wide[5],
              hyper_wide[6], hyper_wide[7]};
  hipLaunchKernelGGL(wd_xgmi_gather_opt<true>, gb, dim3(XB_THR), 0, stream, stride, pe, world, my_sig, err, xctr,
                     nullptr, wsc, param, s0, s1, (uint16_t*)wt_out, step_ctr, hd, hw);
  return (int)hipGetLastError();
}

// slab [G, stride] -> sum -> optimizer on slab-column-order state (param/s0/s1 [stride], wsc [stride]: -1 padding,
// -2 wide, >= 0 DNN weight-image offset). step_ctr: STEP_SLOTS per-workgroup step slots.
int mifx_wd_reduce_opt_sc(const float* slab, int G, int stride, const int* wsc, float* param, float* s0, float* s1,
                          void* wt_out, long long* step_ctr, const float* hyper_dnn, const float* hyper_wide,
                          hipStream_t stream) {
  if (G <= 0 || stride <= 0 || stride > STRIDE || stride % 4 != 0 || wsc == nullptr || param == nullptr ||
      s0 == nullptr || s1 == nullptr || wt_out == nullptr || step_ctr == nullptr)
    return -1;
  const dim3 grid((stride / 4 + RQ - 1) / RQ);
  if (grid.x > STEP_SLOTS) return -1;
  OptHyper hd{(int)hyper_dnn[0], hyper_dnn[1], hyper_dnn[2], hyper_dnn[3], hyper_dnn[4], hyper_dnn[5], hyper_dnn[6],
              hyper_dnn[7]};
  OptHyper hw{(int)hyper_wide[0], hyper_wide[1], hyper_wide[2], hyper_wide[3], hyper_wide[4], hyper_wide[5],
              hyper_wide[6], hyper_wide[7]};
  if (G == 1)
    hipLaunchKernelGGL(wd_opt1_sc, dim3((stride + 255) / 256), dim3(256), 0, stream, slab, stride, wsc, param, s0, s1,
                       (uint16_t*)wt_out, step_ctr, hd, hw);
  else
    hipLaunchKernelGGL(wd_reduce_opt_sc, grid, dim3(256), 0, stream, (const float4*)slab, G, stride, wsc, param, s0,
                       s1, (uint16_t*)wt_out, step_ctr, hd, hw);
  return (int)hipGetLastError();
}

// XCD-local slab reduction [+ optimizer on slab-column-order state] (see wd_reduce_xcd). xcd_of [G] from the fused
// kernel (mifx_wdc_fused_x); part [16][stride] fp32 and ok [16][chunks] int scratch; xep: STEP_SLOTS int64 epoch
// slots (all equal). wsc == null: plain sum into out [stride].
int mifx_wd_xcd_chunks(int stride) { return (stride / 4 + X1C - 1) / X1C; }

int mifx_wd_reduce_xcd_opt(const float* slab, int G, int stride, const int* xcd_of, float* part, int* ok,
                           long long* xep, float* out, const int* wsc, float* param, float* s0, float* s1,
                           void* wt_out, long long* step_ctr, const float* hyper_dnn, const float* hyper_wide,
                           hipStream_t stream) {
  if (G <= 0 || G > 256 || stride <= 0 || stride > STRIDE || stride % 4 != 0 || xcd_of == nullptr ||
      part == nullptr || ok == nullptr || xep == nullptr)
    return -1;
  if (wsc == nullptr && out == nullptr) return -1;
  if (wsc != nullptr && (param == nullptr || s0 == nullptr || s1 == nullptr || wt_out == nullptr ||
                         step_ctr == nullptr))
    return -1;
  const int nc1 = mifx_wd_xcd_chunks(stride);
  const dim3 g2((stride + 255) / 256);
  if ((int)g2.x > STEP_SLOTS) return -1;
  OptHyper hd{}, hw{};
  if (wsc != nullptr) {
    hd = OptHyper{(int)hyper_dnn[0], hyper_dnn[1], hyper_dnn[2], hyper_dnn[3], hyper_dnn[4], hyper_dnn[5],
                  hyper_dnn[6], hyper_dnn[7]};
    hw = OptHyper{(int)hyper_wide[0], hyper_wide[1], hyper_wide[2], hyper_wide[3], hyper_wide[4], hyper_wide[5],
                  hyper_wide[6], hyper_wide[7]};
  }
  hipLaunchKernelGGL(wd_reduce_xcd, dim3(8 * nc1), dim3(256), 0, stream, (const float4*)slab, G, stride, xcd_of,
                     (float4*)part, ok, xep);
  if (wsc == nullptr)
    hipLaunchKernelGGL(wd_xcd_opt_sc<0>, g2, dim3(256), 0, stream, part, ok, slab, G, stride, xcd_of, xep, out, wsc,
                       param, s0, s1, (uint16_t*)wt_out, step_ctr, hd, hw, XgPeers{}, 0, 0, nullptr, nullptr, nullptr);
  else
    hipLaunchKernelGGL(wd_xcd_opt_sc<1>, g2, dim3(256), 0, stream, part, ok, slab, G, stride, xcd_of, xep, out, wsc,
                       param, s0, s1, (uint16_t*)wt_out, step_ctr, hd, hw, XgPeers{}, 0, 0, nullptr, nullptr, nullptr);
  return (int)hipGetLastError();
}

// Residue-class two-level slab reduction [+ optimizer on slab-column-order state] (see wd_reduce_res). part: [8][stride]
// fp32 scratch. wsc == null: plain sum into out [stride].
int mifx_wd_reduce_res_opt(const float* slab, int G, int stride, float* part, float* out, const int* wsc, float* param,
                           float* s0, float* s1, void* wt_out, long long* step_ctr, const float* hyper_dnn,
                           const float* hyper_wide, hipStream_t stream) {
  if (G <= 0 || stride <= 0 || stride > STRIDE || stride % 4 != 0 || part == nullptr) return -1;
  if (wsc == nullptr && out == nullptr) return -1;
  if (wsc != nullptr && (param == nullptr || s0 == nullptr || s1 == nullptr || wt_out == nullptr ||
                         step_ctr == nullptr || hyper_dnn == nullptr || hyper_wide == nullptr))
    return -1;
  const int nc1 = mifx_wd_xcd_chunks(stride);
  const dim3 g2((stride + 255) / 256);
  if ((int)g2.x > STEP_SLOTS) return -1;
  hipLaunchKernelGGL(wd_reduce_res, dim3(8 * nc1), dim3(256), 0, stream, (const float4*)slab, G, stride, (float4*)part);
  if (wsc == nullptr) {
    hipLaunchKernelGGL(wd_res_opt_sc<0>, g2, dim3(256), 0, stream, part, stride, out, nullptr, nullptr, nullptr,
                       nullptr, nullptr, nullptr, OptHyper{}, OptHyper{});
  } else {
    const OptHyper hd{(int)hyper_dnn[0], hyper_dnn[1], hyper_dnn[2], hyper_dnn[3], hyper_dnn[4], hyper_dnn[5],
                      hyper_dnn[6], hyper_dnn[7]};
    const OptHyper hw{(int)hyper_wide[0], hyper_wide[1], hyper_wide[2], hyper_wide[3], hyper_wide[4], hyper_wide[5],
                      hyper_wide[6], hyper_wide[7]};
    hipLaunchKernelGGL(wd_res_opt_sc<1>, g2, dim3(256), 0, stream, part, stride, nullptr, wsc, param, s0, s1,
                       (uint16_t*)wt_out, step_ctr, hd, hw);
  }
  return (int)hipGetLastError();
}

// The same with both levels in one launch (wd_reduce_res_fused; optimizer only). ticket: nchunks int32, all zero
// before the first call (each call leaves them zero again).
int mifx_wd_reduce_res_opt_fused(const float* slab, int G, int stride, float* part, int* ticket, const int* wsc,
                                 float* param, float* s0, float* s1, void* wt_out, long long* step_ctr,
                                 const float* hyper_dnn, const float* hyper_wide, hipStream_t stream) {
  if (G <= 0 || stride <= 0 || stride > STRIDE || stride % 4 != 0 || part == nullptr || ticket == nullptr) return -1;
  if (wsc == nullptr || param == nullptr || s0 == nullptr || s1 == nullptr || wt_out == nullptr ||
      step_ctr == nullptr || hyper_dnn == nullptr || hyper_wide == nullptr)
    return -1;
  const int nc1 = mifx_wd_xcd_chunks(stride);
  if (nc1 > STEP_SLOTS || nc1 != (stride + 255) / 256) return -1;
  const OptHyper hd{(int)hyper_dnn[0], hyper_dnn[1], hyper_dnn[2], hyper_dnn[3], hyper_dnn[4], hyper_dnn[5],
                    hyper_dnn[6], hyper_dnn[7]};
  const OptHyper hw{(int)hyper_wide[0], hyper_wide[1], hyper_wide[2], hyper_wide[3], hyper_wide[4], hyper_wide[5],
                    hyper_wide[6], hyper_wide[7]};
  hipLaunchKernelGGL(wd_reduce_res_fused, dim3(8 * nc1), dim3(256), 0, stream, (const float4*)slab, G, stride, part,
                     ticket, wsc, param, s0, s1, (uint16_t*)wt_out, step_ctr, hd, hw);
  return (int)hipGetLastError();
}

#ifdef WD_STAMPS
int mifx_wd_stamps(unsigned long long* out) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_stamps), sizeof(g_stamps), 0, hipMemcpyDeviceToHost);
}
int mifx_wd_blk_times(unsigned long long* out) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_blk), sizeof(g_blk), 0, hipMemcpyDeviceToHost);
}
#endif

}  // extern "C"
