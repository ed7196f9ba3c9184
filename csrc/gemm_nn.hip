// Hand-written bf16 MFMA "NN" GEMM for gfx950: C[M, N] = A[M, K] . B[K, N] (+ R[M, N]) -- the input gradient of a
// linear layer, dX = dY W (+ the residual gradient folded in as the C operand, mifx.ops.gemm.GradSlot).
//
// BASELINE config 4 (BERT-base, 4096 tokens): the four input-gradient GEMMs of a layer (dY of QKV 4096x2304, of
// attention-out 4096x768, of FFN-in 4096x3072, of FFN-out 4096x768, against the nn.Linear weight [out, in]) ran on
// hipBLASLt as 128x128-tile kernels on 192 workgroups (31 us for the 4096x768 outputs with K = 2304 / 3072:
// profiles/archive/bert_steady_kernels_r3_fold.md). The reduction index is the weight's ROW index, so the two operands sit
// differently in memory:
//  * A (dY, [M][K], K contiguous) is staged as in csrc/gemm.hip: [BM rows][64] bf16 per K-tile, 128-byte rows with
//    the 16-byte chunk index XOR-swizzled by ((row >> 1) & 7), fragments read with ds_read_b128 (8 consecutive k);
//  * B (W, [K][N], N contiguous) is staged as in csrc/gemm_tn.hip: [64 k rows][BN] with each row's 16-byte chunks
//    rotated by rot(k) (conflict-free transposed reads), fragments read with two ds_read_b64_tr_b16 (a 16-lane group
//    supplies 4 k rows x 16 columns, each lane receives one column's 4 k values);
//  * both via 16-byte global->LDS DMA into a ring of NS buffers, NS - 1 K-tiles in flight, one barrier per K-tile
//    (counted `s_waitcnt vmcnt` retires only the oldest tile);
//  * 4 waves (2 x 2), 16x16x32 MFMAs with the W fragment as the A operand: the accumulator lane holds
//    C[m][n .. n + 3] -> 8-byte stores; R (optional) is added in fp32 before the single rounding to bf16;
//  * the 4096 x 768 outputs take 128 x 96 tiles: 256 workgroups, one per CU; XCD-aware tile order as in the other
//    GEMMs (each XCD walks a contiguous run of tiles, grouped 4 m-blocks wide).
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

constexpr int BK = 64;

__device__ __forceinline__ int swz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

// chunk rotation of k row t for a row of CPB 16-byte chunks (csrc/gemm_tn.hip, tools/lds_banks_tn.py)
template <int CPB>
__device__ __forceinline__ int rot(int t) {
  static_assert(CPB == 8 || CPB == 12 || CPB == 16 || CPB == 24, "chunks per row");
  if constexpr (CPB == 8) return ((t & 3) + 4 * ((t >> 3) & 3)) & 7;
  if constexpr (CPB == 12) return (2 * ((t >> 3) & 3)) % 12;
  if constexpr (CPB == 24) return (6 * (t & 3) + 6 * ((t >> 3) & 3)) % 24;
  return (2 * (t & 3) + 8 * ((t >> 3) & 3)) & 15;
}
template <int CPB>
__device__ __forceinline__ int slot_of(int t, int c) {
  const int p = c + rot<CPB>(t);
  return p >= CPB ? p - CPB : p;
}

__device__ __forceinline__ v4s tr_read(const unsigned char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(p));
}
__device__ __forceinline__ v8bf cat8(v4s a, v4s b) {
  v8s r = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  return __builtin_bit_cast(v8bf, r);
}

template <int BM, int BN, int NS, bool ADD_R>
__global__ __launch_bounds__(256) void gemm_nn(const bf16* __restrict__ A, const bf16* __restrict__ B,
                                                  const bf16* __restrict__ R, bf16* __restrict__ C, int M, int N,
                                                  int K) {
  constexpr int NT = 256, WM = 2, WN = 2;
  constexpr int TM = BM / WM, TN = BN / WN, MR = TM / 16, NR = TN / 16;
  constexpr int CPB = BN / 8;
  constexpr int AR = BM * 8 / NT, BR = BK * CPB / NT;  // DMA rounds per K-tile
  constexpr int ABYTES = BM * BK * 2, BBYTES = BK * BN * 2, BUF = ABYTES + BBYTES;
  static_assert(TM % 16 == 0 && TN % 16 == 0, "wave tiling");
  static_assert((BM * 8) % NT == 0 && (BK * CPB) % NT == 0, "whole DMA rounds (counted waits)");
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];

  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int wm = w / WN, wn = w % WN;
  const int nwg = gridDim.x, bid = blockIdx.x, xcd = bid % 8, q8 = nwg / 8, r8 = nwg % 8;
  const int tile = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + bid / 8;
  constexpr int GM = 4;
  const int nb_m = M / BM, nb_n = N / BN, per_group = GM * nb_n;
  const int group = tile / per_group, first_m = group * GM, gsz = min(GM, nb_m - first_m);
  const int wi = tile - group * per_group;
  const int m0 = (first_m + wi % gsz) * BM, n0 = (wi / gsz) * BN;
  const int KT = K / BK;

  // per-lane DMA source offsets (elements, relative to the K-tile's first column of A / first row of B)
  int aoff[AR], boff[BR];
#pragma unroll
  for (int i = 0; i < AR; ++i) {
    const int s = i * NT + tid, row = s >> 3, c = swz(row, s & 7);
    aoff[i] = (m0 + row) * K + 8 * c;
  }
#pragma unroll
  for (int i = 0; i < BR; ++i) {
    const int s = i * NT + tid, t = s / CPB, pp = s % CPB;
    int c = pp - rot<CPB>(t);
    c = c < 0 ? c + CPB : c;
    boff[i] = t * N + n0 + 8 * c;
  }
  auto issue = [&](int kt, int buf) {
    unsigned char* ba = lds + buf * BUF;
    unsigned char* bb = ba + ABYTES;
    const int k0 = kt * BK;
    const bf16* b0 = B + (size_t)k0 * N;
#pragma unroll
    for (int i = 0; i < AR; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(A + aoff[i] + k0),
                                       (__attribute__((address_space(3))) void*)(ba + (i * NT + 64 * w) * 16), 16, 0,
                                       0);
#pragma unroll
    for (int i = 0; i < BR; ++i)
      __builtin_amdgcn_global_load_lds((const void*)(b0 + boff[i]),
                                       (__attribute__((address_space(3))) void*)(bb + (i * NT + 64 * w) * 16), 16, 0,
                                       0);
  };

  v4f acc[MR][NR];
#pragma unroll
  for (int a = 0; a < MR; ++a)
#pragma unroll
    for (int b = 0; b < NR; ++b) acc[a][b] = (v4f){0.f, 0.f, 0.f, 0.f};

  // lane (r, h): A fragment row wm TM + 16 a + r, chunk 4 ks + h (8 k values from 32 ks + 8 h); B fragment column
  // wn TN + 16 b + r, k rows 32 ks + 8 h + {0..3} (first transposed read) and + 4 (second)
  const int r = lane & 15, h = lane >> 4, q = r >> 2, p = r & 3;
  auto read_frags = [&](const unsigned char* ba, const unsigned char* bb, int ks, v8bf (&af)[MR], v8bf (&bf)[NR]) {
#pragma unroll
    for (int a = 0; a < MR; ++a) {
      const int row = wm * TM + 16 * a + r;
      af[a] = *(const v8bf*)(ba + row * 128 + swz(row, 4 * ks + h) * 16);
    }
    const int t1 = 32 * ks + 8 * h + q, t2 = t1 + 4;
#pragma unroll
    for (int b = 0; b < NR; ++b) {
      const int c = (wn * TN + 16 * b) / 8 + (p >> 1);
      const unsigned char* p1 = bb + (t1 * CPB + slot_of<CPB>(t1, c)) * 16 + 8 * (p & 1);
      const unsigned char* p2 = bb + (t2 * CPB + slot_of<CPB>(t2, c)) * 16 + 8 * (p & 1);
      bf[b] = cat8(tr_read(p1), tr_read(p2));
    }
  };

  constexpr int G = AR + BR;
  constexpr int INFL = (NS - 2) * G;
  static_assert(INFL < 64, "vmcnt range");
  constexpr int WAIT_STEADY = (INFL & 15) | (7 << 4) | (15 << 8) | ((INFL >> 4) << 14);
#pragma unroll
  for (int i = 0; i < NS - 1; ++i)
    if (i < KT) issue(i, i);
  for (int kt = 0; kt < KT; ++kt) {
    if (kt + NS - 2 <= KT - 1)
      __builtin_amdgcn_s_waitcnt(WAIT_STEADY);  // tile kt retired, the NS - 2 after it still in flight
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (kt + NS - 1 < KT) issue(kt + NS - 1, (kt + NS - 1) % NS);
    const unsigned char* ba = lds + (kt % NS) * BUF;
    const unsigned char* bb = ba + ABYTES;
    v8bf af0[MR], bf0[NR], af1[MR], bf1[NR];
    read_frags(ba, bb, 0, af0, bf0);
    read_frags(ba, bb, 1, af1, bf1);
#pragma unroll
    for (int a = 0; a < MR; ++a)
#pragma unroll
      for (int b = 0; b < NR; ++b) acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf0[b], af0[a], acc[a][b], 0, 0, 0);
#pragma unroll
    for (int a = 0; a < MR; ++a)
#pragma unroll
      for (int b = 0; b < NR; ++b) acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf1[b], af1[a], acc[a][b], 0, 0, 0);
  }

  // ---- epilogue: lane (r, h) holds C[m0 + wm TM + 16 a + r][n0 + wn TN + 16 b + 4 h + 0..3]
#pragma unroll
  for (int a = 0; a < MR; ++a) {
    const int m = m0 + wm * TM + 16 * a + r;
#pragma unroll
    for (int b = 0; b < NR; ++b) {
      const int n = n0 + wn * TN + 16 * b + 4 * h;
      v4f v = acc[a][b];
      if constexpr (ADD_R) {
        const v4bf rv = *(const v4bf*)(R + (size_t)m * N + n);
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] += (float)rv[i];
      }
      v4bf o;
#pragma unroll
      for (int i = 0; i < 4; ++i) o[i] = (bf16)v[i];
      *(v4bf*)(C + (size_t)m * N + n) = o;
    }
  }
}

template <int BM, int BN, int NS>
int launch(const void* A, const void* B, const void* R, void* C, int M, int N, int K, hipStream_t st) {
  constexpr int LDS = NS * (BM * BK + BK * BN) * 2;
  static_assert(LDS <= 160 * 1024, "LDS");
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)gemm_nn<BM, BN, NS, false>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              LDS);
    (void)hipFuncSetAttribute((const void*)gemm_nn<BM, BN, NS, true>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              LDS);
    attr = true;
  }
  const dim3 grid((M / BM) * (N / BN));
  if (R != nullptr)
    hipLaunchKernelGGL((gemm_nn<BM, BN, NS, true>), grid, dim3(256), LDS, st, (const bf16*)A, (const bf16*)B,
                       (const bf16*)R, (bf16*)C, M, N, K);
  else
    hipLaunchKernelGGL((gemm_nn<BM, BN, NS, false>), grid, dim3(256), LDS, st, (const bf16*)A, (const bf16*)B,
                       nullptr, (bf16*)C, M, N, K);
  return (int)hipGetLastError();
}

struct Cfg {
  int bm, bn, ns;
};
constexpr Cfg kCfgs[] = {{128, 96, 4}, {128, 96, 5}, {128, 128, 4}, {128, 192, 3}, {256, 128, 3}, {128, 64, 5},
                         {256, 96, 3}};

}  // namespace

extern "C" {

// out[3 i] = BM, out[3 i + 1] = BN, out[3 i + 2] = ring depth
int mifx_gemm_nn_configs(int* out, int n) {
  const int m = (int)(sizeof(kCfgs) / sizeof(Cfg));
  for (int i = 0; i < m && 3 * i + 2 < n; ++i) {
    out[3 * i] = kCfgs[i].bm;
    out[3 * i + 1] = kCfgs[i].bn;
    out[3 * i + 2] = kCfgs[i].ns;
  }
  return m;
}

// C[M, N] = A[M, K] . B[K, N] (+ R[M, N] when R != null), bf16 row-major in / out, fp32 accumulation, one rounding.
// Requires M % BM == 0, N % BN == 0, K % 64 == 0, 16-byte aligned A / B, 8-byte aligned R / C.
int mifx_gemm_nn(int cfg, const void* A, const void* B, const void* R, void* C, int M, int N, int K, hipStream_t st) {
  const int m = (int)(sizeof(kCfgs) / sizeof(Cfg));
  if (cfg < 0 || cfg >= m || M <= 0 || N <= 0 || K <= 0 || A == nullptr || B == nullptr || C == nullptr) return -1;
  const Cfg c = kCfgs[cfg];
  if (M % c.bm || N % c.bn || K % BK) return -1;
  if ((uintptr_t)A % 16 || (uintptr_t)B % 16 || (uintptr_t)C % 8 || (uintptr_t)R % 8) return -1;
  if ((long long)M * K >= (1ll << 31) || (long long)K * N >= (1ll << 31)) return -1;  // 32-bit element offsets
  switch (cfg) {
    case 0: return launch<128, 96, 4>(A, B, R, C, M, N, K, st);
    case 1: return launch<128, 96, 5>(A, B, R, C, M, N, K, st);
    case 2: return launch<128, 128, 4>(A, B, R, C, M, N, K, st);
    case 3: return launch<128, 192, 3>(A, B, R, C, M, N, K, st);
    case 4: return launch<256, 128, 3>(A, B, R, C, M, N, K, st);
    case 5: return launch<128, 64, 5>(A, B, R, C, M, N, K, st);
    default: return launch<256, 96, 3>(A, B, R, C, M, N, K, st);
  }
}

}  // extern "C"
