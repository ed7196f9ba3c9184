// Hand-written bf16 MFMA GEMM for gfx950 with fused epilogues: Y[M, N] = X[M, K] . W[N, K]^T (+ bias) (-> GELU).
//
// BASELINE config 4 (BERT-base): the four projection GEMMs of a layer (QKV, attention out, FFN in, FFN out) are
// "NT" products of a token-major activation and an nn.Linear weight, both K-contiguous. The FFN-in GEMM is followed
// by bias + GELU(erf), which unfused costs a second pass over the [tokens, 3072] activation (bias_gelu_fwd_v,
// 12 us per call at 4096 tokens: profiles/archive/bert_base_steady_kernels_s3b.md); here it is the GEMM's epilogue, which
// writes both the GELU output and the pre-bias product the backward needs (the saved-tensor contract of
// mifx.ops.fused_bert._BiasGelu, so its backward kernel is reused as is).
//
// Structure (CDNA4 guide section 5: 256x256 tile, 8 waves, BK = 64, two LDS buffers filled by global_load_lds):
//  * each workgroup owns a BM x BN output tile; waves are WM x WN, each owning (BM/WM) x (BN/WN);
//  * per K-tile of 64: every lane issues 16-byte global->LDS DMA loads (no VGPR round trip) for the NEXT tile
//    while the waves run the MFMAs of the current one; one barrier per K-tile;
//  * LDS images are row-major [rows][64] bf16 (128-byte rows) with the 16-byte chunk index XOR-swizzled by
//    ((row >> 1) & 7): the 16 rows of an MFMA fragment read (ds_read_b128, lanes l & 15) then hit 16 distinct 16-byte
//    slots of the 256-byte bank row. glds destinations are lane-linear, so the swizzle is applied to each lane's
//    SOURCE address (guide rule 21) and to the fragment reads;
//  * MFMA 16x16x32 bf16 with the weight fragment as the A operand: the accumulator's lane l holds output row
//    m = l & 15 and four CONSECUTIVE columns n = 4 (l >> 4) + r, so the epilogue stores 8 bytes per lane per tile
//    and reads 4 consecutive bias values at once.
//  * XCD-aware tile order: consecutive workgroups run on different XCDs (round-robin dispatch), so the tile index
//    is remapped (bijectively, guide section 5 "XCD swizzle") so that each XCD walks a contiguous run of tiles
//    sharing activation rows in its own L2.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

typedef __bf16 bf16;
typedef __bf16 v8bf __attribute__((ext_vector_type(8)));
typedef __bf16 v4bf __attribute__((ext_vector_type(4)));
typedef float v4f __attribute__((ext_vector_type(4)));

constexpr int BK = 64;

// EPI_ADD_R: Y = X W^T + R (R bf16 [M, N], passed as `bias`): the input-gradient GEMM dX = dY W computed as an NT
// product against a transposed weight copy, with the residual gradient folded in (mifx.ops.gemm.GradSlot)
// EPI_GELU_BWD: Y = dZ = (X W^T) o GELU'(Z + bias) with Z the saved pre-bias product of the FFN-in GEMM (read), plus
// per-workgroup column sums of the stored dZ (the bias gradient) into part[M / BM][N]: the FFN-out input gradient
// and the bias-GELU backward in one pass (the unfused path writes dGELU [M, N] and reads it back)
enum Epi { EPI_NONE = 0, EPI_BIAS = 1, EPI_BIAS_GELU = 2, EPI_ADD_R = 3, EPI_GELU_BWD = 4 };

// GELU(erf) with a branch-free erf (Abramowitz & Stegun 7.1.26: |error| <= 1.5e-7, far below the bf16 output's
// 2^-9 relative step): the library erff evaluates piecewise polynomials selected per |x|, which diverge inside a
// wave and made the fused epilogue cost more than the separate bias_gelu pass it replaces.
__device__ __forceinline__ float erf_fast(float x) {
  const float ax = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(1.f + 0.3275911f * ax);
  const float poly = t * (0.254829592f + t * (-0.284496736f + t * (1.421413741f + t * (-1.453152027f + t * 1.061405429f))));
  const float r = 1.f - poly * __expf(-ax * ax);
  return copysignf(r, x);
}
__device__ __forceinline__ float gelu_f(float x) { return 0.5f * x * (1.f + erf_fast(x * 0.70710678118654752f)); }
__device__ __forceinline__ float gelu_grad_f(float x) {
  return 0.5f * (1.f + erf_fast(x * 0.70710678118654752f)) + x * 0.3989422804014327f * __expf(-0.5f * x * x);
}

__device__ __forceinline__ int swz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

// OPT bit 0: raise the wave priority around each MFMA block (guide T3: the SQ then issues this wave's MFMAs ahead of
// other waves' LDS / VMEM issue); bit 1: software-pipeline the LDS fragment reads one 32-deep k-step ahead of the
// MFMAs that consume them (two fragment register sets); bit 2: THREE LDS buffers, two K-tiles in flight across each
// barrier -- a counted `s_waitcnt vmcnt(G)` (G = this thread's DMAs per tile) retires only the oldest tile and a raw
// s_barrier (no vmcnt(0) drain) orders it for every wave (guide: "Pipelining across barriers").
template <int BM, int BN, int WM, int WN, int EPI, typename P, int OPT>
__global__ __launch_bounds__(64 * WM * WN, 1) void gemm_nt(const bf16* __restrict__ X, const bf16* __restrict__ W,
                                                            const P* __restrict__ bias, bf16* __restrict__ Y,
                                                            bf16* __restrict__ Z, int M, int N, int K,
                                                            float* __restrict__ part) {
  constexpr int NT = 64 * WM * WN;
  constexpr int TM = BM / WM, TN = BN / WN, MR = TM / 16, NR = TN / 16;
  // 16-byte DMA rounds per K-tile (a partial last round is skipped wave by wave: BM * 8 and BN * 8 are multiples of 64)
  constexpr int XR = (BM * 8 + NT - 1) / NT, WR = (BN * 8 + NT - 1) / NT;
  static_assert(TM % 16 == 0 && TN % 16 == 0 && BM % WM == 0 && BN % WN == 0, "wave tiling");
  constexpr int XBYTES = BM * BK * 2, WBYTES = BN * BK * 2, BUF = XBYTES + WBYTES;
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];

  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int wm = w / WN, wn = w % WN;
  // XCD-aware bijective tile order (guide: q = nwg / 8, r = nwg % 8)
  const int nwg = gridDim.x, bid = blockIdx.x, xcd = bid % 8, q = nwg / 8, rr = nwg % 8;
  const int tile = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + bid / 8;
  const int nb_n = N / BN;
  const int m0 = (tile / nb_n) * BM, n0 = (tile % nb_n) * BN;

  // per-lane DMA source offsets (elements) inside a K-tile, and the wave-uniform LDS destinations
  int xoff[XR], woff[WR];
#pragma unroll
  for (int i = 0; i < XR; ++i) {
    const int qq = min(i * NT + tid, BM * 8 - 1), row = qq >> 3, c = swz(row, qq & 7);
    xoff[i] = (m0 + row) * K + 8 * c;
  }
#pragma unroll
  for (int i = 0; i < WR; ++i) {
    const int qq = min(i * NT + tid, BN * 8 - 1), row = qq >> 3, c = swz(row, qq & 7);
    woff[i] = (n0 + row) * K + 8 * c;
  }
  auto issue = [&](int kt, int buf) {
    unsigned char* bx = lds + buf * BUF;
    unsigned char* bw = bx + XBYTES;
    const int k0 = kt * BK;
#pragma unroll
    for (int i = 0; i < XR; ++i)
      if ((BM * 8) % NT == 0 || i * NT + 64 * w < BM * 8)
        __builtin_amdgcn_global_load_lds((const void*)(X + xoff[i] + k0),
                                         (__attribute__((address_space(3))) void*)(bx + (i * NT + 64 * w) * 16), 16, 0,
                                         0);
#pragma unroll
    for (int i = 0; i < WR; ++i)
      if ((BN * 8) % NT == 0 || i * NT + 64 * w < BN * 8)
        __builtin_amdgcn_global_load_lds((const void*)(W + woff[i] + k0),
                                         (__attribute__((address_space(3))) void*)(bw + (i * NT + 64 * w) * 16), 16, 0,
                                         0);
  };

  v4f acc[NR][MR];
#pragma unroll
  for (int a = 0; a < NR; ++a)
#pragma unroll
    for (int b = 0; b < MR; ++b) acc[a][b] = (v4f){0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fc = lane >> 4;  // fragment row, 16-byte k chunk inside a 32-deep k-step
  const int KT = K / BK;
  auto frags = [&](const unsigned char* bx, const unsigned char* bw, int ks, v8bf (&wf)[NR], v8bf (&xf)[MR]) {
#pragma unroll
    for (int a = 0; a < NR; ++a) {
      const int row = wn * TN + 16 * a + fr;
      wf[a] = *(const v8bf*)(bw + row * 128 + swz(row, 4 * ks + fc) * 16);
    }
#pragma unroll
    for (int b = 0; b < MR; ++b) {
      const int row = wm * TM + 16 * b + fr;
      xf[b] = *(const v8bf*)(bx + row * 128 + swz(row, 4 * ks + fc) * 16);
    }
  };
  auto mma = [&](const v8bf (&wf)[NR], const v8bf (&xf)[MR]) {
    if (OPT & 1) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int a = 0; a < NR; ++a)
#pragma unroll
      for (int b = 0; b < MR; ++b)
        acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[a], xf[b], acc[a][b], 0, 0, 0);
    if (OPT & 1) __builtin_amdgcn_s_setprio(0);
  };
  constexpr bool RING3 = (OPT & 4) != 0;
  static_assert(!RING3 || ((BM * 8) % NT == 0 && (BN * 8) % NT == 0), "3-buffer ring: whole DMA rounds only");
  constexpr int G = XR + WR;  // DMAs per thread per K-tile
  // s_waitcnt immediate (gfx9 encoding): vmcnt = G, expcnt / lgkmcnt not waited on
  constexpr int WAIT_G = (G & 15) | (7 << 4) | (15 << 8) | ((G >> 4) << 14);
  issue(0, 0);
  if (RING3 && KT > 1) issue(1, 1);
  for (int kt = 0; kt < KT; ++kt) {
    int cur;
    if constexpr (RING3) {
      if (kt + 1 < KT)
        __builtin_amdgcn_s_waitcnt(WAIT_G);  // tile kt retired, tile kt + 1 still in flight
      else
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __builtin_amdgcn_s_barrier();  // every wave's tile-kt DMAs retired; buffer (kt + 2) % 3 no longer read
      asm volatile("" ::: "memory");
      if (kt + 2 < KT) issue(kt + 2, (kt + 2) % 3);
      cur = kt % 3;
    } else {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();  // tile kt landed for every wave; buffer (kt + 1) & 1 no longer read
      if (kt + 1 < KT) issue(kt + 1, (kt + 1) & 1);
      cur = kt & 1;
    }
    const unsigned char* bx = lds + cur * BUF;
    const unsigned char* bw = bx + XBYTES;
    if (OPT & 2) {  // fragments of k-step 1 read while k-step 0's MFMAs run
      v8bf wf0[NR], xf0[MR], wf1[NR], xf1[MR];
      frags(bx, bw, 0, wf0, xf0);
      frags(bx, bw, 1, wf1, xf1);
      mma(wf0, xf0);
      mma(wf1, xf1);
    } else {
#pragma unroll
      for (int ks = 0; ks < BK / 32; ++ks) {
        v8bf wf[NR], xf[MR];
        frags(bx, bw, ks, wf, xf);
        mma(wf, xf);
      }
    }
  }

  // ---- epilogue: lane holds Y[m][n .. n + 3]
  if constexpr (EPI == EPI_GELU_BWD) {
    float cs[NR][4];
#pragma unroll
    for (int a = 0; a < NR; ++a) {
      const int n = n0 + wn * TN + 16 * a + 4 * fc;
      float bv[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        bv[r] = (float)bias[n + r];
        cs[a][r] = 0.f;
      }
#pragma unroll
      for (int b = 0; b < MR; ++b) {
        const int m = m0 + wm * TM + 16 * b + fr;
        const v4bf zv = *(const v4bf*)(Z + (size_t)m * N + n);
        v4bf o;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          o[r] = (bf16)(acc[a][b][r] * gelu_grad_f((float)zv[r] + bv[r]));
          cs[a][r] += (float)o[r];  // the bias gradient of the value actually stored
        }
        *(v4bf*)(Y + (size_t)m * N + n) = o;
      }
    }
    // column sums: over the 16 rows of a lane group (xor tree), then over the WM row-waves in order (LDS)
#pragma unroll
    for (int a = 0; a < NR; ++a)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float v = cs[a][r];
        v += __shfl_xor(v, 1);
        v += __shfl_xor(v, 2);
        v += __shfl_xor(v, 4);
        v += __shfl_xor(v, 8);
        cs[a][r] = v;
      }
    __syncthreads();  // every wave is past its last LDS fragment read
    float* red = (float*)lds;  // [WM][BN]
    if (fr == 0) {
#pragma unroll
      for (int a = 0; a < NR; ++a)
#pragma unroll
        for (int r = 0; r < 4; ++r) red[wm * BN + wn * TN + 16 * a + 4 * fc + r] = cs[a][r];
    }
    __syncthreads();
    for (int c = tid; c < BN; c += NT) {
      float t = 0.f;
#pragma unroll
      for (int i = 0; i < WM; ++i) t += red[i * BN + c];
      part[(size_t)(m0 / BM) * N + n0 + c] = t;
    }
    return;
  }
#pragma unroll
  for (int a = 0; a < NR; ++a) {
    const int n = n0 + wn * TN + 16 * a + 4 * fc;
    float bv[4] = {0.f, 0.f, 0.f, 0.f};
    if (EPI == EPI_BIAS || EPI == EPI_BIAS_GELU) {
#pragma unroll
      for (int r = 0; r < 4; ++r) bv[r] = (float)bias[n + r];
    }
#pragma unroll
    for (int b = 0; b < MR; ++b) {
      const int m = m0 + wm * TM + 16 * b + fr;
      v4bf o;
      if (EPI == EPI_BIAS_GELU) {
        v4bf z;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          z[r] = (bf16)acc[a][b][r];                  // the product as the unfused GEMM would store it
          o[r] = (bf16)gelu_f((float)z[r] + bv[r]);   // bias_gelu_fwd on that stored value
        }
        *(v4bf*)(Z + (size_t)m * N + n) = z;
      } else if (EPI == EPI_ADD_R) {
        const v4bf rv = *(const v4bf*)((const bf16*)bias + (size_t)m * N + n);
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = (bf16)(acc[a][b][r] + (float)rv[r]);
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) o[r] = (bf16)(acc[a][b][r] + bv[r]);
      }
      *(v4bf*)(Y + (size_t)m * N + n) = o;
    }
  }
}

template <int BM, int BN, int WM, int WN, int EPI, typename P, int OPT>
int launch(const void* X, const void* W, const void* bias, void* Y, void* Z, int M, int N, int K, hipStream_t st,
           float* part = nullptr) {
  constexpr int LDS = ((OPT & 4) ? 3 : 2) * (BM + BN) * BK * 2;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)gemm_nt<BM, BN, WM, WN, EPI, P, OPT>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    attr = true;
  }
  hipLaunchKernelGGL((gemm_nt<BM, BN, WM, WN, EPI, P, OPT>), dim3((M / BM) * (N / BN)), dim3(64 * WM * WN), LDS, st,
                     (const bf16*)X, (const bf16*)W, (const P*)bias, (bf16*)Y, (bf16*)Z, M, N, K, part);
  return (int)hipGetLastError();
}

template <int BM, int BN, int WM, int WN, int OPT>
int dispatch_epi(int epi, int bias_f32, const void* X, const void* W, const void* bias, void* Y, void* Z, int M, int N,
                 int K, hipStream_t st, float* part = nullptr) {
  if (epi == EPI_GELU_BWD)
    return bias_f32 ? launch<BM, BN, WM, WN, EPI_GELU_BWD, float, OPT>(X, W, bias, Y, Z, M, N, K, st, part)
                    : launch<BM, BN, WM, WN, EPI_GELU_BWD, bf16, OPT>(X, W, bias, Y, Z, M, N, K, st, part);
  if (epi == EPI_NONE) return launch<BM, BN, WM, WN, EPI_NONE, bf16, OPT>(X, W, nullptr, Y, nullptr, M, N, K, st);
  if (epi == EPI_ADD_R) return launch<BM, BN, WM, WN, EPI_ADD_R, bf16, OPT>(X, W, bias, Y, nullptr, M, N, K, st);
  if (epi == EPI_BIAS)
    return bias_f32 ? launch<BM, BN, WM, WN, EPI_BIAS, float, OPT>(X, W, bias, Y, nullptr, M, N, K, st)
                    : launch<BM, BN, WM, WN, EPI_BIAS, bf16, OPT>(X, W, bias, Y, nullptr, M, N, K, st);
  return bias_f32 ? launch<BM, BN, WM, WN, EPI_BIAS_GELU, float, OPT>(X, W, bias, Y, Z, M, N, K, st)
                  : launch<BM, BN, WM, WN, EPI_BIAS_GELU, bf16, OPT>(X, W, bias, Y, Z, M, N, K, st);
}

struct Cfg {
  int bm, bn, opt;
};
// (index = the `cfg` argument; BM x BN tile, OPT bits)
// 9..: whole-wave tilings of BERT-base's shapes at 4096 tokens on 256 CUs (256 tiles each): 256x192 (FFN-in),
// 256x144 (QKV, 6 waves), 128x96 (attention-out / FFN-out)
constexpr Cfg kCfgs[] = {{256, 256, 0}, {256, 128, 0}, {128, 128, 0}, {128, 256, 0}, {256, 256, 3}, {128, 128, 3},
                         {256, 128, 3}, {128, 128, 1}, {256, 128, 2}, {256, 192, 3}, {256, 144, 3}, {128, 96, 3},
                         {128, 96, 1}, {128, 96, 5}, {128, 128, 5}, {256, 128, 5}, {128, 96, 7}, {128, 128, 7},
                         {256, 128, 7}, {256, 144, 7}};

// dst[C][R] = src[R][C] (bf16), 64 x 64 tiles through LDS: 16-byte loads along src rows, 16-byte stores along dst
// rows (8 consecutive src rows of one column gathered from LDS). The transposed weight copy of the dX GEMMs.
__device__ __forceinline__ void transpose_tile(const bf16* __restrict__ src, bf16* __restrict__ dst, int R, int C,
                                               int tile, bf16 (*t)[64 + 2]) {
  const int nbc = C / 64, r0 = (tile / nbc) * 64, c0 = (tile % nbc) * 64;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int q = i * 256 + threadIdx.x, row = q >> 3, ch = q & 7;
    const v8bf v = *(const v8bf*)(src + (size_t)(r0 + row) * C + c0 + 8 * ch);
#pragma unroll
    for (int e = 0; e < 8; ++e) t[row][8 * ch + e] = v[e];
  }
  __syncthreads();
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int q = i * 256 + threadIdx.x, col = q >> 3, ch = q & 7;  // dst row = src column col
    v8bf v;
#pragma unroll
    for (int e = 0; e < 8; ++e) v[e] = t[8 * ch + e][col];
    *(v8bf*)(dst + (size_t)(c0 + col) * R + r0 + 8 * ch) = v;
  }
}

__global__ __launch_bounds__(256) void transpose_bf16(const bf16* __restrict__ src, bf16* __restrict__ dst, int R,
                                                      int C) {
  __shared__ bf16 t[64][64 + 2];
  transpose_tile(src, dst, R, C, blockIdx.x, t);
}

// every weight of a model in one launch (mifx.ops.gemm.TransposeCache): entry e covers tiles [tile0, next tile0)
struct TrEntry {
  const bf16* src;
  bf16* dst;
  int R, C, tile0, pad;
};
__global__ __launch_bounds__(256) void transpose_batch(const TrEntry* __restrict__ ents, int n) {
  __shared__ bf16 t[64][64 + 2];
  int e = 0;
  while (e + 1 < n && ents[e + 1].tile0 <= (int)blockIdx.x) ++e;
  const TrEntry E = ents[e];
  transpose_tile(E.src, E.dst, E.R, E.C, (int)blockIdx.x - E.tile0, t);
}

}  // namespace

extern "C" {

// dZ[M, N] = (X[M, K] . W[N, K]^T) o GELU'(Z + bias) (bf16 out), part[M / BM][N] = per-tile column sums of the
// stored dZ (fp32). Z: bf16 [M, N] (the saved pre-bias product), bias bf16 or fp32 [N]. cfg: index into
// mifx_gemm_configs; M % BM == 0, N % BN == 0, K % 64 == 0.
int mifx_gemm_nt_gelu_bwd(int cfg, int bias_f32, const void* X, const void* W, const void* bias, const void* Z,
                          void* Y, float* part, int M, int N, int K, hipStream_t st) {
  const int m = (int)(sizeof(kCfgs) / sizeof(Cfg));
  if (cfg < 0 || cfg >= m || M <= 0 || N <= 0 || K <= 0 || X == nullptr || W == nullptr || Y == nullptr ||
      Z == nullptr || bias == nullptr || part == nullptr)
    return -1;
  const Cfg c = kCfgs[cfg];
  if (M % c.bm || N % c.bn || K % BK) return -1;
  if ((uintptr_t)X % 16 || (uintptr_t)W % 16 || (uintptr_t)Y % 8 || (uintptr_t)Z % 8) return -1;
  if ((long long)M * K >= (1ll << 31) || (long long)N * K >= (1ll << 31)) return -1;
  void* z = const_cast<void*>(Z);
  switch (cfg) {
    case 9: return dispatch_epi<256, 192, 2, 4, 3>(EPI_GELU_BWD, bias_f32, X, W, bias, Y, z, M, N, K, st, part);
    case 11: return dispatch_epi<128, 96, 2, 2, 3>(EPI_GELU_BWD, bias_f32, X, W, bias, Y, z, M, N, K, st, part);
    case 12: return dispatch_epi<128, 96, 2, 2, 1>(EPI_GELU_BWD, bias_f32, X, W, bias, Y, z, M, N, K, st, part);
    case 7: return dispatch_epi<128, 128, 2, 2, 1>(EPI_GELU_BWD, bias_f32, X, W, bias, Y, z, M, N, K, st, part);
    default: return -2;  // configuration without a GELU-backward build
  }
}

// n transposes in one launch: ents = device array of TrEntry {src, dst, R, C, tile0, 0} with tile0 the running sum
// of (R / 64) (C / 64); every R, C % 64 == 0, 16-byte aligned
int mifx_transpose_bf16_batch(const void* ents, int n, int total_tiles, hipStream_t st) {
  if (ents == nullptr || n <= 0 || total_tiles <= 0) return -1;
  hipLaunchKernelGGL(transpose_batch, dim3(total_tiles), dim3(256), 0, st, (const TrEntry*)ents, n);
  return (int)hipGetLastError();
}

// dst [C, R] = src [R, C]^T, bf16; R % 64 == 0, C % 64 == 0, 16-byte aligned
int mifx_transpose_bf16(const void* src, void* dst, int R, int C, hipStream_t st) {
  if (R <= 0 || C <= 0 || R % 64 || C % 64 || (uintptr_t)src % 16 || (uintptr_t)dst % 16) return -1;
  hipLaunchKernelGGL(transpose_bf16, dim3((R / 64) * (C / 64)), dim3(256), 0, st, (const bf16*)src, (bf16*)dst, R, C);
  return (int)hipGetLastError();
}

// tile configurations: out[3 * i] = BM, out[3 * i + 1] = BN, out[3 * i + 2] = OPT bits
int mifx_gemm_configs(int* out, int n) {
  const int m = (int)(sizeof(kCfgs) / sizeof(Cfg));
  for (int i = 0; i < m && 3 * i + 2 < n; ++i) {
    out[3 * i] = kCfgs[i].bm;
    out[3 * i + 1] = kCfgs[i].bn;
    out[3 * i + 2] = kCfgs[i].opt;
  }
  return m;
}

// Y[M, N] = X[M, K] . W[N, K]^T  (bf16 in / out, fp32 accumulation). epi: 0 none, 1 + bias[N], 2 bias + GELU(erf)
// with Z[M, N] = the bf16 product before the bias (the backward's saved input). bias: bf16 or fp32 (bias_f32).
// cfg: index into mifx_gemm_configs. Requires M % BM == 0, N % BN == 0, K % 64 == 0, 16-byte aligned rows.
int mifx_gemm_nt(int cfg, int epi, int bias_f32, const void* X, const void* W, const void* bias, void* Y, void* Z,
                 int M, int N, int K, hipStream_t st) {
  const int m = (int)(sizeof(kCfgs) / sizeof(Cfg));
  if (cfg < 0 || cfg >= m || M <= 0 || N <= 0 || K <= 0 || X == nullptr || W == nullptr || Y == nullptr) return -1;
  const Cfg c = kCfgs[cfg];
  if (M % c.bm || N % c.bn || K % BK) return -1;
  if (epi < 0 || epi > 3 || (epi > 0 && bias == nullptr) || (epi == 2 && Z == nullptr)) return -1;
  if (epi == 3 && (uintptr_t)bias % 8) return -1;
  if ((uintptr_t)X % 16 || (uintptr_t)W % 16 || (uintptr_t)Y % 8 || (Z != nullptr && (uintptr_t)Z % 8)) return -1;
  if ((long long)M * K >= (1ll << 31) || (long long)N * K >= (1ll << 31)) return -1;  // 32-bit element offsets
  switch (cfg) {
    case 0: return dispatch_epi<256, 256, 2, 4, 0>(epi, bias_f32, X, W, bias, Y, Z, M, N, K, st);
    case 1: return dispatch_epi<256, 128, 4, 2, 0>(epi, bias_f32, X, W, bias, Y, Z, M, N, K, st);
    case 2: return dispatch_epi<128, 128, 2, 2, 0>(epi, bias_f32, X, W, bias, Y, Z, M, N, K, st);
    case 3: return dispatch_epi<128, 256, 2, 4, 0>(epi, bias_f32, X, W, bias, Y, Z, M, N, K, st);
    case 4: return dispatch_epi<256, 256, 2, 4, 3>(epi, bias_f32, X, W, bias, Y, Z, M, N, K, st);
    case 5: return dispatch_epi<128, 128, 2, 2, 3>(epi, bias_f32, X, W, bias, Y, Z, M, N, K, st);
    case 6: return dispatch_epi<256, 128, 4, 2, 3>(epi, bias_f32, X, W, bias, Y, Z, M, N, K, st);
    case 7: return dispatch_epi<128, 128, 2, 2, 1>(epi, bias_f32, X, W, bias, Y, Z, M, N, K, st);
    case 8: return dispatch_epi<256, 128, 2, 2, 2>(epi, bias_f32, X, W, bias, Y, Z, M, N, K, st);
    case 9: return dispatch_epi<256, 192, 2, 4, 3>(epi, bias_f32, X, W, bias, Y, Z, M, N, K, st);
    case 10: return dispatch_epi<256, 144, 2, 3, 3>(epi, bias_f32, X, W, bias, Y, Z, M, N, K, st);
    case 11: return dispatch_epi<128, 96, 2, 2, 3>(epi, bias_f32, X, W, bias, Y, Z, M, N, K, st);
    case 12: return dispatch_epi<128, 96, 2, 2, 1>(epi, bias_f32, X, W, bias, Y, Z, M, N, K, st);
    case 13: return dispatch_epi<128, 96, 2, 2, 5>(epi, bias_f32, X, W, bias, Y, Z, M, N, K, st);
    case 14: return dispatch_epi<128, 128, 2, 2, 5>(epi, bias_f32, X, W, bias, Y, Z, M, N, K, st);
    case 15: return dispatch_epi<256, 128, 4, 2, 5>(epi, bias_f32, X, W, bias, Y, Z, M, N, K, st);
    case 16: return dispatch_epi<128, 96, 2, 2, 7>(epi, bias_f32, X, W, bias, Y, Z, M, N, K, st);
    case 17: return dispatch_epi<128, 128, 2, 2, 7>(epi, bias_f32, X, W, bias, Y, Z, M, N, K, st);
    case 18: return dispatch_epi<256, 128, 4, 2, 7>(epi, bias_f32, X, W, bias, Y, Z, M, N, K, st);
    default: return dispatch_epi<256, 144, 2, 3, 3>(epi, bias_f32, X, W, bias, Y, Z, M, N, K, st);
  }
}

}  // extern "C"
