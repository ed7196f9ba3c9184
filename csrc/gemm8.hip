// Ping-pong pipelined bf16 MFMA GEMM for gfx950: Y[M, N] = X[M, K] . W[N, K]^T (+ fused epilogues).
//
// The projection GEMMs of BERT-base (BASELINE config 4) and ResNet-50's 1x1 convolutions in NHWC (config 5) are all
// "NT" products of a K-contiguous activation and a K-contiguous weight. csrc/gemm.hip runs them with ONE barrier and
// a `vmcnt(0)` drain per 64-deep K-tile (the structure that tops out near 0.9 PFLOP/s, guide section 5 "step-3
// structure"); its counters sat at 18-26 % MFMA busy on BERT's K = 768 shapes (profiles/gemm_pmc_r4.md). This kernel
// is the multi-phase structure instead:
//
//  * 8 waves (512 threads), one workgroup per CU, tile BM x BN, BK = 64, two LDS K-tile buffers, each split into four
//    HALF-tiles: A0 / A1 = X rows [0, BM/2) / [BM/2, BM), B0 / B1 = W rows [0, BN/2) / [BN/2, BN).
//  * a K-tile is four PHASES, one C-quadrant each, in the order Q(A0,B0) Q(A1,B0) Q(A1,B1) Q(A0,B1): every phase
//    each wave reads only what the quadrant needs that is not already in its registers (phase 0: A0 + B0 fragments,
//    1: A1, 2: B1, 3: nothing) and runs (BM/64)*(BN/128)*2 MFMAs 16x16x32 on its (BM/4) x (BN/8) piece of the quadrant.
//  * every phase also issues ONE half-tile of global->LDS DMA (`global_load_lds_dwordx4`, no VGPR round trip) into the
//    slot the schedule has freed: phase j of K-tile t stages half (j + 2) % 4 of K-tile t + 1 (j < 2) or t + 2
//    (j >= 2). A half is restaged two phases after its last read (the WAR margin of the guide's template) and first
//    read at least five phases after it was issued, so one counted `s_waitcnt vmcnt(<one K-tile of DMAs>)` per phase,
//    before the phase's first barrier, retires exactly what the next phase reads: four half-tiles (a whole K-tile,
//    32-64 KB per CU) stay in flight across every barrier and the loop never drains to vmcnt(0) (guide T3+T4).
//  * two raw `s_barrier`s per phase (no __syncthreads: its fence would drain the DMAs). Waves 4-7 run one barrier
//    behind waves 0-3 (the guide's stagger): on each SIMD one wave runs its MFMA block while its partner issues LDS
//    reads and DMAs, then they swap. `s_setprio(1)` around every MFMA block keeps the compiler from moving MFMAs
//    across the barriers (guide T5).
//  * LDS rows are 128 bytes with the 16-byte chunk index XOR-swizzled by (row >> 1) & 7 (conflict-free
//    ds_read_b128 of the 16 rows of a fragment); the DMA destination is lane-linear, so the swizzle is applied to each
//    lane's SOURCE address (guide rule 21) and to the fragment reads.
//  * the weight fragment is the MFMA's A operand, so a lane's accumulator holds one output row and four CONSECUTIVE
//    columns (8-byte stores, 4 consecutive bias values).
//  * XCD-aware bijective tile order (consecutive workgroups land on different XCDs; each XCD walks a contiguous run of
//    tiles that share X row panels in its L2).
//
// TN layout (weight gradients, dW = dY^T X: both operands token-major, the reduction is their ROW index): the same
// schedule with half-tiles of 64 tokens x BM/2 (BN/2) columns; an LDS row is a token's 256 (or 128) bytes with its
// 16-byte chunks rotated per token (conflict-free transposed reads, csrc/gemm_tn.hip's rot<>), and the MFMA fragments
// (8 consecutive tokens of one column per lane) come from two ds_read_b64_tr_b16. GROUPED launch: a table of up to
// 64 problems in the kernel arguments, each workgroup finds its (problem, tile) by binary search over the per-problem
// first-tile indices. A BERT step's 48 weight-gradient products are off the backward's critical path, so they are
// deferred to the end of the backward and run as ONE launch of full 256 x 256 tiles over the whole 4096-token
// reduction (no split-K partials, 1296 tiles = five waves of 256 CUs), instead of 48 small launches whose few output
// tiles had to be split over tokens and summed by a second kernel.
//
// Epilogues: none / + bias[N] / bias + GELU(erf) also storing the pre-bias product Z (the FFN-in forward) / + R[M, N]
// (dX = dY W + residual gradient) / GELU backward dZ = (X W^T) o GELU'(Z + bias) with per-tile column sums (the FFN-out
// input gradient fused with FFN-in's bias-GELU backward) / per-tile column sum and sum of squares of the stored bf16
// output (the BatchNorm statistics of a 1x1 convolution, folded into the GEMM that produces it).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <type_traits>

namespace {

typedef __bf16 bf16;
typedef __bf16 v8bf __attribute__((ext_vector_type(8)));
typedef __bf16 v4bf __attribute__((ext_vector_type(4)));
typedef float v4f __attribute__((ext_vector_type(4)));

constexpr int BK = 64;
constexpr int NT = 512;

enum Epi { EPI_NONE = 0, EPI_BIAS = 1, EPI_BIAS_GELU = 2, EPI_ADD_R = 3, EPI_GELU_BWD = 4, EPI_STATS = 5,
           EPI_ADD_STATS = 6, EPI_F32 = 7, EPI_BNBWD = 8, EPI_ADD_BNBWD = 9 };

__device__ __forceinline__ float erf_fast(float x) {  // Abramowitz & Stegun 7.1.26, |error| <= 1.5e-7, branch-free
  const float ax = fabsf(x);
  const float t = __builtin_amdgcn_rcpf(1.f + 0.3275911f * ax);
  const float poly = t * (0.254829592f + t * (-0.284496736f + t * (1.421413741f + t * (-1.453152027f + t * 1.061405429f))));
  return copysignf(1.f - poly * __expf(-ax * ax), x);
}
__device__ __forceinline__ float gelu_f(float x) { return 0.5f * x * (1.f + erf_fast(x * 0.70710678118654752f)); }
__device__ __forceinline__ float gelu_grad_f(float x) {
  return 0.5f * (1.f + erf_fast(x * 0.70710678118654752f)) + x * 0.3989422804014327f * __expf(-0.5f * x * x);
}

__device__ __forceinline__ int swz(int row, int chunk) { return chunk ^ ((row >> 1) & 7); }

typedef short v4s __attribute__((ext_vector_type(4)));
typedef short v8s __attribute__((ext_vector_type(8)));
typedef __attribute__((address_space(3))) v4s lds_v4s;

// TN images: chunk rotation of token row t for a row of CPR 16-byte chunks (every 32-lane half of a transposed
// fragment read touches 64 distinct banks; tools/lds_banks_tn.py)
template <int CPR>
__device__ __forceinline__ int rot(int t) {
  static_assert(CPR == 4 || CPR == 8 || CPR == 16, "chunks per token row");
  if constexpr (CPR == 4) return 2 * ((t >> 3) & 1);  // 64-byte rows (narrow tiles): the 16-lane groups of a half
                                                      // read tokens 8 apart, shifted 8 banks
  if constexpr (CPR == 8) return ((t & 3) + 4 * ((t >> 3) & 3)) & 7;
  return (2 * (t & 3) + 8 * ((t >> 3) & 3)) & 15;
}
__device__ __forceinline__ v8bf tr_frag(const unsigned char* p1, const unsigned char* p2) {
  const v4s a = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)p1);
  const v4s b = __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)p2);
  const v8s r = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  return __builtin_bit_cast(v8bf, r);
}

// Implicit-GEMM 3x3 convolution over NHWC activations (ResNet-50's bottleneck conv2, BASELINE config 5): input
// [Nb][H][W][C] (C a power of two >= 64), output pixels [Nb][OH][OW], taps (r, s) in 0..2, stride / pad. The GEMM's
// reduction index is k = (3 r + s) C + c, so a 64-deep K-tile is one tap and a 64-channel slice: each DMA row of the
// gathered operand is one pixel shifted by the tap -- or, outside the image, the zero page below (the DMA then fills
// the LDS row with zeros; no predicated loads, no separate padding pass). CV 1 (NT, forward / stride-1 input
// gradient): the X rows are output pixels, gathered per K-tile; weights [Cout][3][3][C] (channels_last). CV 2 (TN,
// weight gradient dW[Cout][3][3][C] = sum_pixels dY^T . X_tap): the B token rows are output pixels, gathered from X;
// a BN-wide column block is one tap (C % BN == 0). Divisions by OW and OH OW in the gather are multiply-high
// (`ow_mul` / `ohw_mul`, host-computed; exact for x < 2^31).
struct Geo {
  int H, W, C, OH, OW, stride, pad, cshift;
  unsigned ow_mul;
  int ow_sh;
  unsigned ohw_mul;
  int ohw_sh;
  int tap0;  // first tap: 0 for a 3x3 convolution (K = 9 C); 4 (the center of a pad-1 3x3) for a strided 1x1 (K = C)
  int ntaps;
};
__device__ __attribute__((aligned(16))) bf16 g_zero_page[64] = {};
__device__ __forceinline__ int fdiv(int x, unsigned mul, int sh) {
  return (int)((__umulhi((unsigned)x, mul) + (unsigned)x) >> sh);
}

// grouped TN problems: C[M, N] (bf16, ldc N) = A[T, M]^T B[T, N]; tiles of problem i are [first[i], first[i + 1])
constexpr int MAXP = 48;  // (the problem table travels in the kernel arguments: 48 x 64 bytes)
// Problem i: C_i[M, N] = A_i[T, M]^T B_i[T, N]. bf16 problems (F32 clear): C bf16, one token split, staged bf16
// stores. fp32 problems (F32 set): the token range is cut into S chunks of `chunk` rows (the last shorter), each
// (tile, chunk) item stores its fp32 partial into P[s][M][N]; gemm8_tn_reduce then ADDS sum_s P[s] (fixed order) into
// the fp32 destination C -- the weight gradients of convolutions, whose token count (N H W = 12k-800k rows) is far
// longer than their output is wide. TILE128: 128 x 128 tiles for this problem (dimensions % 256 != 0).
constexpr int F32 = 1, TILE128 = 2, ACCUM = 4;  // ACCUM: C += sum of the partials (else C = the sum)
// NARROW_N / NARROW_M: 256 x 64 / 64 x 256 tiles (a 64-wide weight-gradient dimension: ResNet-50's first stage)
constexpr int NARROW_N = 16, NARROW_M = 32;
// CONV: B is a 3x3 convolution's input gathered per output pixel (CV 2, geometry in device memory at `geo`); the
// problem is dW[M = Cout][N = 9 C] = dY^T . X_taps, F32 only
constexpr int CONV = 8;
// BNX: B is a BatchNorm + ReLU INPUT; the operand is relu(B scale + shift), applied per column as B's fragments leave
// LDS (aux = fp32 [scale[N], shift[N]]): the weight gradient of a convolution whose input activation is never stored
constexpr int BNX = 64;
struct Prob {
  const bf16* A;
  const bf16* B;
  void* C;
  float* P;
  const void* aux;  // CONV: the Geo; BNX: scale / shift
  int M, N, T, chunk, S, flags;
};
struct Group {
  Prob p[MAXP];
  int first[MAXP + 1];  // first work item (tile x chunk) of each problem
  int n;
  int n_big;  // workgroups [0, n_big) run items [0, n_big); the rest run the (BM/2) x (BN/2) quadrants of items
              // [n_big, first[n]) -- a last partial wave of quarter-size tiles instead of full ones (bf16 groups of
              // uniform 256 x 256 tiles only)
};

// s_waitcnt immediate (gfx9 encoding): vmcnt = n, expcnt / lgkmcnt not waited on
constexpr int vm_wait(int n) { return (n & 15) | (7 << 4) | (15 << 8) | ((n >> 4) << 14); }

// The body: one BM x BN tile of Y = X W^T (NT: X [M, K], W [N, K] row-major) or of C = A^T B (TN: A [K, M],
// B [K, N] row-major; X := A, W := B, "K" = tokens), m0 / n0 its origin. CV: implicit-convolution operand (above);
// tok0: the first token of this item's chunk (CV 2: B is then the whole conv input, gathered by pixel index).
// AX: the BatchNorm + ReLU transform relu(v scale[c] + shift[c]) of channel c applied to one operand -- NT: X (c = the
// K index), TN: B (c = the column) -- so the consumer convolution of a BatchNorm + ReLU reads the BatchNorm's INPUT and
// the activation is never written (bit-identical to the stored-activation path: same fused multiply-add and rounding
// as csrc/bn_relu.hip bn_apply). ax = fp32 [scale[L], shift[L]], L = K (NT) or N (TN); its slice is copied to LDS
// after the two K-tile buffers. The transformed operand's half-tiles are DMA'd as usual; in the phase where a half is
// guaranteed to have landed (its counted wait), each thread rewrites the 16-byte chunks ITS OWN DMAs delivered --
// once per workgroup, not per consuming wave -- BEFORE that phase's first barrier, which precedes every wave's
// fragment reads of that half in both stagger groups. (Staging through registers instead mixes plain loads with the
// LDS DMAs, and the compiler then drains vmcnt to 0 every K-tile.) Duplicated DMAs (narrow B halves) of the
// transformed operand land in a scratch area instead, so no raw copy can overwrite a transformed chunk.
template <int BM, int BN, int EPI, typename P, bool TN, int CV = 0, bool AX = false>
__device__ __forceinline__ void gemm8_tile(const bf16* __restrict__ X, const bf16* __restrict__ W,
                                           const P* __restrict__ bias, bf16* __restrict__ Y, bf16* __restrict__ Z,
                                           int M, int N, int K, float* __restrict__ part, int m0, int n0,
                                           unsigned char* lds, const Geo& geo = Geo{}, int tok0 = 0,
                                           const bf16* __restrict__ R2 = nullptr,
                                           const float* __restrict__ ax = nullptr) {
  static_assert(CV == 0 || (CV == 1 && !TN) || (CV == 2 && TN), "conv gather: NT rows (1) or TN B rows (2)");
  static_assert(!AX || CV == 0, "the BatchNorm operand transform: plain (1x1) operands only (no zero-page rows)");
  constexpr int HA = BM / 2, HB = BN / 2;            // rows (NT) / columns (TN) per half-tile
  constexpr int ABYTES = HA * 128, BBYTES = HB * 128;  // NT: 64 bf16 per row; TN: 64 token rows of HA bf16
  // NARROW (NT, BN = 64: the 64-channel convolutions of ResNet-50's first stage): the 8 waves tile a quadrant 4 x 2
  // instead of 2 x 4 (each wave 16 columns), and the 32-row B half-tile is staged by half the threads, the other half
  // re-issuing the same DMAs (same source, same LDS bytes) so every wave's counted vmcnt stays uniform
  constexpr bool NARROW = BN == 64;
  constexpr int WROWS = NARROW ? 4 : 2, WCOLS = NARROW ? 2 : 4;  // wave grid inside a quadrant
  constexpr int RPW = HA / WROWS, CPW = HB / WCOLS;              // rows / columns per wave per quadrant
  constexpr int ADMA = HA * 8, BDMA = HB * 8;                   // A / B DMAs per half-tile
  constexpr int XR = (ADMA + NT - 1) / NT, WR = (BDMA + NT - 1) / NT;  // DMAs per thread per half-tile
  constexpr bool ADUP = ADMA < NT, WDUP = BDMA < NT;  // half the threads re-issue the other half's DMAs
  constexpr int CPA = HA / 8, CPB = HB / 8;            // TN: 16-byte chunks per token row
  static_assert((ADMA % NT == 0 || NT % ADMA == 0) && (BDMA % NT == 0 || NT % BDMA == 0),
                "whole DMA rounds per half-tile");
  static_assert(!WDUP || NARROW, "duplicated B DMAs are the narrow layout's");
  static_assert(!ADUP || (TN && CV == 0), "duplicated A DMAs: the TN narrow-M tiles only");
  constexpr int MF = RPW / 16, NF = CPW / 16;  // 16-row fragments per wave per quadrant
  static_assert(MF >= 1 && NF >= 1 && RPW % 16 == 0 && CPW % 16 == 0, "tile too small for 8 waves");
  static_assert(!NARROW || EPI != EPI_GELU_BWD, "the GELU-backward epilogue's column sums assume 2 wave rows");
  constexpr int BUF = 2 * (ABYTES + BBYTES);
  constexpr int OFF_A0 = 0, OFF_B0 = ABYTES, OFF_A1 = ABYTES + BBYTES, OFF_B1 = 2 * ABYTES + BBYTES;
  constexpr int KTILE_DMAS = 2 * (XR + WR);  // DMAs per thread per K-tile = per 4 consecutive phases

  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int grp = w >> 2;  // stagger group (waves 4-7 run one barrier behind waves 0-3)
  const int wm = NARROW ? (w & 3) : (w >> 2), wn = NARROW ? (w >> 2) : (w & 3);  // wave position in a quadrant
  const int KT = K / BK;

  // per-lane DMA source offsets (elements, K-tile 0) of each half, pre-swizzled / pre-rotated
  int aoff[XR], boff[WR];
#pragma unroll
  for (int i = 0; i < XR; ++i) {
    const int qq = ADUP ? tid % ADMA : i * NT + tid;
    if constexpr (TN) {
      const int t = qq / CPA, pc = qq % CPA;  // token row, physical chunk
      int c = pc - rot<CPA>(t);
      c = c < 0 ? c + CPA : c;
      aoff[i] = t * M + m0 + 8 * c;
    } else {
      const int row = qq >> 3;
      aoff[i] = (m0 + row) * K + 8 * swz(row, qq & 7);
    }
  }
#pragma unroll
  for (int i = 0; i < WR; ++i) {
    const int qq = WDUP ? tid % BDMA : i * NT + tid;
    if constexpr (TN) {
      const int t = qq / CPB, pc = qq % CPB;
      int c = pc - rot<CPB>(t);
      c = c < 0 ? c + CPB : c;
      boff[i] = t * N + n0 + 8 * c;
    } else {
      const int row = qq >> 3;
      boff[i] = (n0 + row) * K + 8 * swz(row, qq & 7);
    }
  }
  // CV 1: each A DMA row's output pixel, decoded once: image base pixel, top-left input coordinate, swizzled chunk
  int cpix[CV == 1 ? 2 : 1][CV == 1 ? XR : 1], cih[CV == 1 ? 2 : 1][CV == 1 ? XR : 1],
      ciw[CV == 1 ? 2 : 1][CV == 1 ? XR : 1], cch[CV == 1 ? XR : 1];
  if constexpr (CV == 1) {
    const int ohw = geo.OH * geo.OW;
#pragma unroll
    for (int i = 0; i < XR; ++i) {
      const int qq = i * NT + tid, row = qq >> 3;
      cch[i] = 8 * swz(row, qq & 7);
#pragma unroll
      for (int hh = 0; hh < 2; ++hh) {
        const int m = m0 + hh * HA + row, nb = m / ohw, rem = m - nb * ohw, oh = rem / geo.OW, ow = rem - oh * geo.OW;
        cpix[hh][i] = nb * geo.H * geo.W;
        cih[hh][i] = oh * geo.stride - geo.pad;
        ciw[hh][i] = ow * geo.stride - geo.pad;
      }
    }
  }
  // CV 2: each B DMA's token row within the K-tile and its logical chunk
  int btok[CV == 2 ? WR : 1], bcol[CV == 2 ? WR : 1];
  if constexpr (CV == 2) {
#pragma unroll
    for (int i = 0; i < WR; ++i) {
      const int qq = i * NT + tid, t = qq / CPB, pc = qq % CPB;
      int c = pc - rot<CPB>(t);
      c = c < 0 ? c + CPB : c;
      btok[i] = t;
      bcol[i] = 8 * c;
    }
  }
  // AX: table loads (before every DMA: retired by the prologue's counted wait)
  constexpr int XS = AX ? (TN ? WR : XR) : 1;       // 16-byte chunks per thread per transformed half
  constexpr int TABF = AX ? (TN ? 2 * BN : 0) : 0;  // TN table floats ([scale, shift] of this tile's columns)
  float4 axv[2] = {};
  if constexpr (AX && !TN) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int q = (i * NT + tid) * 4;
      if (q < 2 * K) axv[i] = *(const float4*)(ax + q);
    }
  }
  if constexpr (AX && TN) {
    const int q = tid * 4;
    if (q < TABF) axv[0] = *(const float4*)(ax + (q < BN ? n0 + q : N + n0 + q - BN));
  }

  // half h (0 A0, 1 B0, 2 A1, 3 B1) of K-tile t into LDS buffer t & 1
  auto stage = [&](int h, int t) {
    unsigned char* buf = lds + (t & 1) * BUF;
    const int k0 = t * BK;
    if (CV == 1 && (h == 0 || h == 2)) {  // gathered pixel rows of tap k0 / C, channels [k0 % C, + 64)
      unsigned char* dst = buf + (h == 0 ? OFF_A0 : OFF_A1);
      const int hh = h >> 1, tap = (k0 >> geo.cshift) + geo.tap0, c0 = k0 & (geo.C - 1), r = tap / 3,
                sx = tap - 3 * r;
#pragma unroll
      for (int i = 0; i < XR; ++i) {
        const int ih = cih[hh][i] + r, iw = ciw[hh][i] + sx;
        const bool ok = (unsigned)ih < (unsigned)geo.H && (unsigned)iw < (unsigned)geo.W;
        const bf16* src = ok ? X + ((size_t)(cpix[hh][i] + ih * geo.W + iw) << geo.cshift) + c0 + cch[i] : g_zero_page;
        __builtin_amdgcn_global_load_lds((const void*)src,
                                         (__attribute__((address_space(3))) void*)(dst + (i * NT + 64 * w) * 16), 16,
                                         0, 0);
      }
      return;
    }
    if (CV == 2 && (h == 1 || h == 3)) {  // gathered token (pixel) rows for this tile's tap
      unsigned char* dst = buf + (h == 1 ? OFF_B0 : OFF_B1);
      const int col = n0 + (h == 3 ? HB : 0), tap = (col >> geo.cshift) + geo.tap0, c0 = col & (geo.C - 1), r = tap / 3,
                sx = tap - 3 * r, ohw = geo.OH * geo.OW;
#pragma unroll
      for (int i = 0; i < WR; ++i) {
        const int x = tok0 + k0 + btok[i], nb = fdiv(x, geo.ohw_mul, geo.ohw_sh), rem = x - nb * ohw,
                  oh = fdiv(rem, geo.ow_mul, geo.ow_sh), ow = rem - oh * geo.OW;
        const int ih = oh * geo.stride - geo.pad + r, iw = ow * geo.stride - geo.pad + sx;
        const bool ok = (unsigned)ih < (unsigned)geo.H && (unsigned)iw < (unsigned)geo.W;
        const bf16* src =
            ok ? W + ((size_t)((nb * geo.H + ih) * geo.W + iw) << geo.cshift) + c0 + bcol[i] : g_zero_page;
        __builtin_amdgcn_global_load_lds((const void*)src,
                                         (__attribute__((address_space(3))) void*)(dst + (i * NT + 64 * w) * 16), 16,
                                         0, 0);
      }
      return;
    }
    if (h == 0 || h == 2) {
      unsigned char* dst = buf + (h == 0 ? OFF_A0 : OFF_A1);
      const bf16* src = TN ? X + (size_t)k0 * M + (h == 2 ? HA : 0) : X + (h == 2 ? HA * K : 0) + k0;
#pragma unroll
      for (int i = 0; i < XR; ++i)
        __builtin_amdgcn_global_load_lds(
            (const void*)(src + aoff[i]),
            (__attribute__((address_space(3))) void*)(dst + (ADUP ? (64 * w) % ADMA : i * NT + 64 * w) * 16), 16, 0,
            0);
    } else {
      unsigned char* dst = buf + (h == 1 ? OFF_B0 : OFF_B1);
      const bf16* src = TN ? W + (size_t)k0 * N + (h == 3 ? HB : 0) : W + (h == 3 ? HB * K : 0) + k0;
#pragma unroll
      for (int i = 0; i < WR; ++i) {
        // (AX TN: the duplicate DMAs of a transformed narrow half land in the scratch area after the table)
        unsigned char* d = (AX && TN && WDUP && 64 * w >= BDMA) ? lds + 2 * BUF + 4 * TABF + (64 * w - BDMA) * 16
                                                              : dst + (WDUP ? (64 * w) % BDMA : i * NT + 64 * w) * 16;
        __builtin_amdgcn_global_load_lds((const void*)(src + boff[i]), (__attribute__((address_space(3))) void*)d,
                                         16, 0, 0);
      }
    }
  };

  v4f acc[2][2][NF][MF];  // [mq][nq][n-frag][m-frag]
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b)
#pragma unroll
      for (int c = 0; c < NF; ++c)
#pragma unroll
        for (int d = 0; d < MF; ++d) acc[a][b][c][d] = (v4f){0.f, 0.f, 0.f, 0.f};

  const int fr = lane & 15, fc = lane >> 4;
  v8bf ra0[MF][2], ra1[MF][2], rb[NF][2];  // A0 / A1 / current-B fragments, [frag][k-step]
  // TN fragment geometry: lane (r = lane & 15 -> token quad q = r >> 2, column quad p = r & 3; h = lane >> 4): the
  // two transposed reads deliver tokens 32 ks + 8 h + q and + 4 of column 16 f + 4 p .. (4 consecutive per read)
  const int tq = fr >> 2, tp = fr & 3;
  auto tn_frag = [&](const unsigned char* half, int cpr_rot, int col0, int ks) -> v8bf {
    const int t1 = 32 * ks + 8 * fc + tq, t2 = t1 + 4;
    const int c = col0 / 8 + (tp >> 1);
    int s1 = c + (cpr_rot == 16 ? rot<16>(t1) : cpr_rot == 8 ? rot<8>(t1) : rot<4>(t1)),
        s2 = c + (cpr_rot == 16 ? rot<16>(t2) : cpr_rot == 8 ? rot<8>(t2) : rot<4>(t2));
    s1 = s1 >= cpr_rot ? s1 - cpr_rot : s1;
    s2 = s2 >= cpr_rot ? s2 - cpr_rot : s2;
    return tr_frag(half + (t1 * cpr_rot + s1) * 16 + 8 * (tp & 1), half + (t2 * cpr_rot + s2) * 16 + 8 * (tp & 1));
  };
  // AX commit: transform staged half x (0: A0 / B0, 1: A1 / B1) of K-tile t and write it to its LDS slots
  auto commit = [&](int x, int t) {
    unsigned char* buf = lds + (t & 1) * BUF;
    const float* tab = (const float*)(lds + 2 * BUF);
#pragma unroll
    for (int i = 0; i < XS; ++i) {
      int slot, c;  // LDS chunk slot and its first channel (NT: K index; TN: table column)
      if constexpr (!TN) {
        slot = i * NT + tid;
        const int row = slot >> 3;
        c = t * BK + 8 * swz(row, slot & 7);
      } else {
        if (WDUP && tid >= BDMA) continue;  // (its duplicate DMAs went to the scratch area)
        slot = WDUP ? tid : i * NT + tid;
        const int tr = slot / CPB, pc = slot % CPB;
        int cc = pc - rot<CPB>(tr);
        cc = cc < 0 ? cc + CPB : cc;
        c = x * HB + 8 * cc;
      }
      const int L = TN ? BN : K;
      const float4 s0 = *(const float4*)(tab + c), s1 = *(const float4*)(tab + c + 4);
      const float4 h0 = *(const float4*)(tab + L + c), h1 = *(const float4*)(tab + L + c + 4);
      const float sc[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
      const float sh[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
      unsigned char* half = buf + (TN ? (x ? OFF_B1 : OFF_B0) : (x ? OFF_A1 : OFF_A0));
      v8bf v = *(const v8bf*)(half + slot * 16);  // this thread's own DMA, landed (counted wait)
#pragma unroll
      for (int e = 0; e < 8; ++e) v[e] = (bf16)fmaxf(fmaf((float)v[e], sc[e], sh[e]), 0.f);
      *(v8bf*)(half + slot * 16) = v;
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // visible at the next barrier
  };
  auto read_a = [&](const unsigned char* half, v8bf (&r)[MF][2], int k0) {
#pragma unroll
    for (int f = 0; f < MF; ++f) {
      const int row = wm * RPW + 16 * f + fr;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        if constexpr (TN)
          r[f][ks] = tn_frag(half, CPA, wm * RPW + 16 * f, ks);
        else
          r[f][ks] = *(const v8bf*)(half + row * 128 + swz(row, 4 * ks + fc) * 16);
      }
    }
    (void)k0;
  };
  auto read_b = [&](const unsigned char* half, int hb) {
#pragma unroll
    for (int f = 0; f < NF; ++f) {
      const int row = wn * CPW + 16 * f + fr;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        if constexpr (TN)
          rb[f][ks] = tn_frag(half, CPB, wn * CPW + 16 * f, ks);
        else
          rb[f][ks] = *(const v8bf*)(half + row * 128 + swz(row, 4 * ks + fc) * 16);
      }
    }
    (void)hb;
  };
  auto mma = [&](v4f (&c)[NF][MF], const v8bf (&ra)[MF][2]) {
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int a = 0; a < NF; ++a)
#pragma unroll
        for (int b = 0; b < MF; ++b) c[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(rb[a][ks], ra[b][ks], c[a][b], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
  };
  auto barrier = [&]() {
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
  };


  // prologue: K-tile 0 whole, K-tile 1 halves A0 / B0; retire K-tile 0's A0 / B0 (phase 0 reads them)
  stage(0, 0);
  stage(1, 0);
  stage(2, 0);
  stage(3, 0);
  if (KT > 1) {
    stage(0, 1);
    stage(1, 1);
    __builtin_amdgcn_s_waitcnt(vm_wait(KTILE_DMAS));
  } else {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  if constexpr (AX) {  // the table to LDS (all threads' parts visible after the barrier), then tile 0's half 0
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const int q = (i * NT + tid) * 4;
      if (q < (TN ? TABF : 2 * K)) *(float4*)(lds + 2 * BUF + 4 * q) = axv[i];
    }
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    barrier();
    commit(0, 0);
  }
  barrier();
  if (grp == 1) barrier();  // the stagger: waves 4-7 one barrier behind

  // one K-tile: 4 phases. ST1 / ST2: K-tiles t + 1 / t + 2 exist (compile-time in the AX build's peeled loop, so every
  // path through its main loop issues the same vector-memory operations and the compiler's own waits on the staging
  // registers equal the counted ones instead of draining)
  auto ktile = [&](int t, auto S1, auto S2, bool rst1, bool rst2) {
    constexpr int cs1 = decltype(S1)::value, cs2 = decltype(S2)::value;  // 1 / 0, or -1: runtime (rst1 / rst2)
    const bool st1 = cs1 < 0 ? rst1 : cs1 == 1, st2 = cs2 < 0 ? rst2 : cs2 == 1;
    const unsigned char* buf = lds + (t & 1) * BUF;
    auto phase = [&](auto J) {
      constexpr int j = decltype(J)::value;
      // LDS fragment reads of this phase's quadrant
      if constexpr (j == 0) {
        read_a(buf + OFF_A0, ra0, t * BK);
        read_b(buf + OFF_B0, 0);
      } else if constexpr (j == 1) {
        read_a(buf + OFF_A1, ra1, t * BK);
      } else if constexpr (j == 2) {
        read_b(buf + OFF_B1, 1);
      }
      // one half-tile of DMA into the slot freed two phases ago
      const bool issue = j < 2 ? st1 : st2;
      if (issue) {
        if constexpr (j < 2)
          stage(j + 2, t + 1);
        else
          stage(j - 2, t + 2);
        __builtin_amdgcn_s_waitcnt(vm_wait(KTILE_DMAS));  // everything issued >= 4 phases ago has landed
      } else {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // tail: nothing younger to count on
      }
      if constexpr (AX) {  // landed now: j 0 -> A1(t), 1 -> B1(t), 2 -> A0(t + 1), 3 -> B0(t + 1)
        if constexpr (!TN && j == 0) commit(1, t);
        if constexpr (!TN && j == 2) if (st1) commit(0, t + 1);
        if constexpr (TN && j == 1) commit(1, t);
        if constexpr (TN && j == 3) if (st1) commit(0, t + 1);
      }
      barrier();
      if constexpr (j == 0) mma(acc[0][0], ra0);
      if constexpr (j == 1) mma(acc[1][0], ra1);
      if constexpr (j == 2) mma(acc[1][1], ra1);
      if constexpr (j == 3) mma(acc[0][1], ra0);
      barrier();
    };
    phase(std::integral_constant<int, 0>{});
    phase(std::integral_constant<int, 1>{});
    phase(std::integral_constant<int, 2>{});
    phase(std::integral_constant<int, 3>{});
  };
  using c1 = std::integral_constant<int, 1>;
  using c0 = std::integral_constant<int, 0>;
  using cr = std::integral_constant<int, -1>;
  if constexpr (AX) {
    int t = 0;
    for (; t + 2 < KT; ++t) ktile(t, c1{}, c1{}, true, true);
    if (t + 1 < KT) ktile(t++, c1{}, c0{}, true, false);
    if (t < KT) ktile(t, c0{}, c0{}, false, false);
  } else {
    for (int t = 0; t < KT; ++t) ktile(t, cr{}, cr{}, t + 1 < KT, t + 2 < KT);
  }
  if (grp == 0) barrier();  // equal barrier counts for both groups

  // ---- epilogue: acc[mq][nq][a][b][r] = Y[m0 + mq HA + wm HA/2 + 16 b + fr][n0 + nq HB + wn HB/4 + 16 a + 4 fc + r]
  if constexpr (EPI == EPI_GELU_BWD) {
    // per-tile column sums of the stored dZ, over the rows of the 16-lane groups (xor tree), then over the two
    // wave rows in order (LDS), written to part[m0 / BM][...]
    float cs[2][NF][4];
#pragma unroll
    for (int nq = 0; nq < 2; ++nq)
#pragma unroll
      for (int a = 0; a < NF; ++a) {
        const int n = n0 + nq * HB + wn * CPW + 16 * a + 4 * fc;
        float bv[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          bv[r] = (float)bias[n + r];
          cs[nq][a][r] = 0.f;
        }
#pragma unroll
        for (int mq = 0; mq < 2; ++mq)
#pragma unroll
          for (int b = 0; b < MF; ++b) {
            const int m = m0 + mq * HA + wm * RPW + 16 * b + fr;
            const v4bf zv = *(const v4bf*)(Z + (size_t)m * N + n);
            v4bf o;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              o[r] = (bf16)(acc[mq][nq][a][b][r] * gelu_grad_f((float)zv[r] + bv[r]));
              cs[nq][a][r] += (float)o[r];
            }
            *(v4bf*)(Y + (size_t)m * N + n) = o;
          }
      }
#pragma unroll
    for (int nq = 0; nq < 2; ++nq)
#pragma unroll
      for (int a = 0; a < NF; ++a)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          float v = cs[nq][a][r];
          v += __shfl_xor(v, 1);
          v += __shfl_xor(v, 2);
          v += __shfl_xor(v, 4);
          v += __shfl_xor(v, 8);
          cs[nq][a][r] = v;
        }
    __syncthreads();  // all DMAs retired (vmcnt(0) in the tail) and every fragment read done: LDS reusable
    float* red = (float*)lds;  // [2 wave rows][BN]
    if (fr == 0) {
#pragma unroll
      for (int nq = 0; nq < 2; ++nq)
#pragma unroll
        for (int a = 0; a < NF; ++a)
#pragma unroll
          for (int r = 0; r < 4; ++r) red[wm * BN + nq * HB + wn * CPW + 16 * a + 4 * fc + r] = cs[nq][a][r];
    }
    __syncthreads();
    for (int c = tid; c < BN; c += NT) part[(size_t)(m0 / BM) * N + n0 + c] = red[c] + red[BN + c];
    return;
  }
  if constexpr (EPI == EPI_F32) {  // fp32 partial tile into part[M][N] (16-byte stores: 4 consecutive columns)
#pragma unroll
    for (int nq = 0; nq < 2; ++nq)
#pragma unroll
      for (int a = 0; a < NF; ++a) {
        const int n = n0 + nq * HB + wn * CPW + 16 * a + 4 * fc;
#pragma unroll
        for (int mq = 0; mq < 2; ++mq)
#pragma unroll
          for (int b = 0; b < MF; ++b) {
            const int m = m0 + mq * HA + wm * RPW + 16 * b + fr;
            *(v4f*)(part + (size_t)m * N + n) = acc[mq][nq][a][b];
          }
      }
    return;
  }
  if constexpr (EPI == EPI_BIAS_GELU) {  // two outputs (Y and the pre-bias Z): direct 8-byte stores
#pragma unroll
    for (int nq = 0; nq < 2; ++nq)
#pragma unroll
      for (int a = 0; a < NF; ++a) {
        const int n = n0 + nq * HB + wn * CPW + 16 * a + 4 * fc;
        float bv[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) bv[r] = (float)bias[n + r];
#pragma unroll
        for (int mq = 0; mq < 2; ++mq)
#pragma unroll
          for (int b = 0; b < MF; ++b) {
            const int m = m0 + mq * HA + wm * RPW + 16 * b + fr;
            v4bf o, z;
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              z[r] = (bf16)acc[mq][nq][a][b][r];
              o[r] = (bf16)gelu_f((float)z[r] + bv[r]);
            }
            *(v4bf*)(Z + (size_t)m * N + n) = z;
            *(v4bf*)(Y + (size_t)m * N + n) = o;
          }
      }
    return;
  }
  // Staged epilogue (none / bias / + R / statistics): the bf16 tile goes through LDS so that every global store and
  // every R load is a whole 16-byte chunk of a row, consecutive lanes along the row (the fragment layout stores 8
  // bytes per lane, 16 rows apart -- half-line writes that made small-K products output-bound). Chunk c of tile row r
  // sits at physical chunk c ^ (r & (CPR_O - 1)): the 16 rows a fragment store writes land on 16 distinct 16-byte
  // slots (conflict-free), and row reads stay conflict-free.
  constexpr int CPR_O = BN / 8;  // 16-byte chunks per tile row
  constexpr int RPI = NT / CPR_O;  // tile rows per store iteration
  constexpr bool STATS = EPI == EPI_STATS || EPI == EPI_ADD_STATS;
  constexpr bool ADD = EPI == EPI_ADD_R || EPI == EPI_ADD_STATS;
  // BNBWD: Y is the gradient dY of a BatchNorm + ReLU's OUTPUT (the input gradient of the 1x1 convolution it feeds);
  // `bias` = that BatchNorm's input x (bf16 [M, N]), `Z` = its forward statistics (fp32 [4][N]: mean, rstd, scale,
  // shift). Besides storing dY, the epilogue reduces the BatchNorm backward's per-tile sums over the tile rows:
  // part[0][m0 / BM][n] = sum g, part[1][...] = sum g xhat, g = dY [x scale + shift > 0], xhat = (x - mean) rstd --
  // what bn_bwd_reduce would otherwise re-read dY and x for.
  // ADD_BNBWD: as BNBWD for dY = X W^T + R2 (bf16 [M, N]) -- the BatchNorm output feeds two convolutions (a
  // projection block's conv1 and shortcut) and R2 is the other one's input gradient, added before the reduction
  constexpr bool BNB = EPI == EPI_BNBWD || EPI == EPI_ADD_BNBWD;
  auto tslot = [&](int row, int c) -> unsigned char* {
    return lds + (size_t)row * (BN * 2) + ((c ^ (row & (CPR_O - 1))) << 4);
  };
#pragma unroll
  for (int nq = 0; nq < 2; ++nq)
#pragma unroll
    for (int a = 0; a < NF; ++a) {
      const int col = nq * HB + wn * CPW + 16 * a + 4 * fc;
      float bv[4] = {0.f, 0.f, 0.f, 0.f};
      if constexpr (EPI == EPI_BIAS) {
#pragma unroll
        for (int r = 0; r < 4; ++r) bv[r] = (float)bias[n0 + col + r];
      }
#pragma unroll
      for (int mq = 0; mq < 2; ++mq)
#pragma unroll
        for (int b = 0; b < MF; ++b) {
          const int row = mq * HA + wm * RPW + 16 * b + fr;
          v4bf o;
#pragma unroll
          for (int r = 0; r < 4; ++r) o[r] = (bf16)(acc[mq][nq][a][b][r] + bv[r]);
          *(v4bf*)(tslot(row, col >> 3) + ((col >> 2) & 1) * 8) = o;
        }
    }
  __syncthreads();
  const int cc = tid % CPR_O, rr0 = tid / CPR_O;
  float cs[8], cq[8], bsc[8], bsh[8], bmu[8], brs[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) cs[e] = cq[e] = 0.f;
  if constexpr (BNB) {
    const float* st = (const float*)(const void*)Z;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const int c = n0 + 8 * cc + e;
      bmu[e] = st[c];
      brs[e] = st[N + c];
      bsc[e] = st[2 * N + c];
      bsh[e] = st[3 * N + c];
    }
  }
  // rows in groups of G: the group's global operand loads (R, the BatchNorm input x, R2) are all issued before any
  // is used -- the accumulators are dead here, so G x 16 bytes per operand stay in flight per thread (a small-K
  // product is bound by this pass: with one load in flight per row it streamed at ~3.5 TB/s)
  constexpr int NI = BM / RPI, G = NI < 8 ? NI : 8;
  constexpr bool LD1 = ADD || BNB, LD2 = EPI == EPI_ADD_BNBWD;
#pragma unroll 1
  for (int i0 = 0; i0 < NI; i0 += G) {
    v8bf l1[LD1 ? G : 1], l2[LD2 ? G : 1];
#pragma unroll
    for (int j = 0; j < G; ++j) {
      const size_t g = (size_t)(m0 + rr0 + (i0 + j) * RPI) * N + n0 + 8 * cc;
      if constexpr (LD1) l1[j] = *(const v8bf*)((const bf16*)bias + g);
      if constexpr (LD2) l2[j] = *(const v8bf*)(R2 + g);
    }
#pragma unroll
    for (int j = 0; j < G; ++j) {
      const int row = rr0 + (i0 + j) * RPI;
      v8bf v = *(const v8bf*)tslot(row, cc);
      const size_t g = (size_t)(m0 + row) * N + n0 + 8 * cc;
      if constexpr (ADD) {  // Y = X W^T + R, one rounding of the fp32-exact sum of two bf16 values
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = (bf16)((float)v[e] + (float)l1[j][e]);
        if constexpr (STATS) *(v8bf*)tslot(row, cc) = v;  // the stored sum, re-read by the second statistics pass
      }
      if constexpr (STATS) {
#pragma unroll
        for (int e = 0; e < 8; ++e) cs[e] += (float)v[e];
      }
      if constexpr (EPI == EPI_ADD_BNBWD) {  // one rounding of the fp32-exact sum of two bf16 values
#pragma unroll
        for (int e = 0; e < 8; ++e) v[e] = (bf16)((float)v[e] + (float)l2[j][e]);
      }
      if constexpr (BNB) {  // the BatchNorm backward's reduction, with its mask computed as the forward's fmaf
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const float u = (float)l1[j][e];
          const float gg = fmaf(u, bsc[e], bsh[e]) <= 0.f ? 0.f : (float)v[e];
          cs[e] += gg;
          cq[e] += gg * ((u - bmu[e]) * brs[e]);
        }
      }
      *(v8bf*)(Y + g) = v;
    }
  }
  if constexpr (STATS || BNB) {
    // per-tile BatchNorm statistics of the STORED values, two-pass (mean, then the sum of squared deviations from
    // it): part[0][m0 / BM][n] = tile mean, part[1][m0 / BM][n] = M2 = sum (y - mean)^2 over the BM rows; combined
    // across tiles by Chan's formula in fp64 (mifx_bn_relu_fwd_tiles), so no E[y^2] - E[y]^2 cancellation
    float* red = (float*)(lds + (size_t)BM * BN * 2);  // [8 waves][BN]
    float* meanv = red + 8 * BN;                       // [BN]
    auto reduce_cols = [&](float (&v)[8], float* outc, float scale) {
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        if constexpr (CPR_O <= 8) v[e] += __shfl_xor(v[e], 8);
        if constexpr (CPR_O <= 16) v[e] += __shfl_xor(v[e], 16);
        v[e] += __shfl_xor(v[e], 32);
      }
      if (lane < CPR_O) {
#pragma unroll
        for (int e = 0; e < 8; ++e) red[w * BN + 8 * lane + e] = v[e];
      }
      __syncthreads();
      for (int c = tid; c < BN; c += NT) {
        float t = 0.f;
#pragma unroll
        for (int k = 0; k < 8; ++k) t += red[k * BN + c];
        outc[c] = t * scale;
      }
      __syncthreads();
    };
    if constexpr (BNB) {
      reduce_cols(cs, meanv, 1.f);
      for (int c = tid; c < BN; c += NT) part[(size_t)(m0 / BM) * N + n0 + c] = meanv[c];
      reduce_cols(cq, meanv, 1.f);  // (the barrier inside orders the reads of meanv above before the overwrite)
      for (int c = tid; c < BN; c += NT) part[((size_t)(M / BM) + m0 / BM) * N + n0 + c] = meanv[c];
      return;
    }
    reduce_cols(cs, meanv, 1.f / BM);
    float mu[8], m2[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      mu[e] = meanv[8 * cc + e];
      m2[e] = 0.f;
    }
#pragma unroll 4
    for (int i = 0; i < BM / RPI; ++i) {
      const v8bf v = *(const v8bf*)tslot(rr0 + i * RPI, cc);
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float d = (float)v[e] - mu[e];
        m2[e] += d * d;
      }
    }
    for (int c = tid; c < BN; c += NT) part[(size_t)(m0 / BM) * N + n0 + c] = meanv[c];
    reduce_cols(m2, meanv, 1.f);  // (every thread has read its means: the barrier inside precedes the overwrite)
    for (int c = tid; c < BN; c += NT) part[((size_t)(M / BM) + m0 / BM) * N + n0 + c] = meanv[c];
  }
}

__device__ __forceinline__ int xcd_tile() {  // bijective XCD-aware remap of blockIdx.x (guide section 5)
  const int nwg = gridDim.x, bid = blockIdx.x, xcd = bid % 8, q = nwg / 8, rr = nwg % 8;
  return (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + bid / 8;
}

template <int BM, int BN, int EPI, typename P>
__global__ __launch_bounds__(NT, 1) void gemm8_nt(const bf16* __restrict__ X, const bf16* __restrict__ W,
                                                  const P* __restrict__ bias, bf16* __restrict__ Y,
                                                  bf16* __restrict__ Z, int M, int N, int K,
                                                  float* __restrict__ part, const bf16* __restrict__ R2) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int tile = xcd_tile(), nb_n = N / BN;
  gemm8_tile<BM, BN, EPI, P, false>(X, W, bias, Y, Z, M, N, K, part, (tile / nb_n) * BM, (tile % nb_n) * BN, lds,
                                    Geo{}, 0, R2);
}

// Y = relu(X scale + shift) . W^T: the consumer 1x1 convolution of a BatchNorm + ReLU over the BatchNorm's input X
// (ax = [scale[K], shift[K]] fp32, K <= 2048)
template <int BM, int BN, int EPI>
__global__ __launch_bounds__(NT, 1) void gemm8_nt_bnx(const bf16* __restrict__ X, const bf16* __restrict__ W,
                                                      const bf16* __restrict__ bias, bf16* __restrict__ Y, int M,
                                                      int N, int K, float* __restrict__ part,
                                                      const float* __restrict__ ax) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int tile = xcd_tile(), nb_n = N / BN;
  gemm8_tile<BM, BN, EPI, bf16, false, 0, true>(X, W, bias, Y, nullptr, M, N, K, part, (tile / nb_n) * BM,
                                                (tile % nb_n) * BN, lds, Geo{}, 0, nullptr, ax);
}

// implicit-GEMM 3x3 convolution (CV 1): Y[Nb OH OW, N] = gathered X . W[N, 9 C]^T, epilogues as gemm8_nt
template <int BM, int BN, int EPI, typename P>
__global__ __launch_bounds__(NT, 1) void gemm8_conv(const bf16* __restrict__ X, const bf16* __restrict__ W,
                                                    const P* __restrict__ bias, bf16* __restrict__ Y,
                                                    bf16* __restrict__ Z, int M, int N, int K,
                                                    float* __restrict__ part, const Geo geo) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int tile = xcd_tile(), nb_n = N / BN;
  gemm8_tile<BM, BN, EPI, P, false, 1>(X, W, bias, Y, Z, M, N, K, part, (tile / nb_n) * BM, (tile % nb_n) * BN, lds,
                                       geo);
}

// grouped TN: each workgroup's (problem, item) from the table by binary search; an item is (tile, token chunk); tiles
// of a problem run m-fastest in groups of 4 m-blocks (an XCD's consecutive tiles share B column strips in its L2)
template <int BM, int BN, bool TN>
__device__ __forceinline__ void grouped_item(const Prob& p, int item, int quad, unsigned char* lds) {
  constexpr int GM = 4;
  const int bm = (p.flags & TILE128) ? BM / 2 : (p.flags & NARROW_M) ? 64 : BM,
            bn = (p.flags & TILE128) ? BN / 2 : (p.flags & NARROW_N) ? 64 : BN;
  const int nb_m = p.M / bm, nb_n = p.N / bn, tiles = nb_m * nb_n;
  const int sp = item / tiles, t = item - sp * tiles;
  const int per_group = GM * nb_n, grp = t / per_group, first_m = grp * GM, gsz = min(GM, nb_m - first_m);
  const int wi = t - grp * per_group;
  const int m0 = (first_m + wi % gsz) * bm, n0 = (wi / gsz) * bn;
  const int t0 = sp * p.chunk, len = min(p.chunk, p.T - t0);
  const bf16* A = p.A + (size_t)t0 * p.M;
  if (p.flags & CONV) {  // (F32 only; the B rows are gathered from the whole input by pixel index t0 + ...)
    const Geo geo = *(const Geo*)p.aux;
    float* P = p.P + (size_t)sp * p.M * p.N;
    if (p.flags & NARROW_N)
      gemm8_tile<BM, 64, EPI_F32, bf16, true, 2>(A, p.B, nullptr, nullptr, nullptr, p.M, p.N, len, P, m0, n0, lds,
                                                 geo, t0);
    else if (p.flags & TILE128)
      gemm8_tile<BM / 2, BN / 2, EPI_F32, bf16, true, 2>(A, p.B, nullptr, nullptr, nullptr, p.M, p.N, len, P, m0, n0,
                                                         lds, geo, t0);
    else
      gemm8_tile<BM, BN, EPI_F32, bf16, true, 2>(A, p.B, nullptr, nullptr, nullptr, p.M, p.N, len, P, m0, n0, lds,
                                                 geo, t0);
    return;
  }
  const bf16* B = p.B + (size_t)t0 * p.N;
  if (p.flags & BNX) {  // (F32 only: a convolution weight gradient over a BatchNorm + ReLU input)
    float* P = p.P + (size_t)sp * p.M * p.N;
    const float* bx = (const float*)p.aux;
    if (p.flags & NARROW_N)
      gemm8_tile<BM, 64, EPI_F32, bf16, true, 0, true>(A, B, nullptr, nullptr, nullptr, p.M, p.N, len, P, m0, n0, lds,
                                                       Geo{}, 0, nullptr, bx);
    else if (p.flags & NARROW_M)
      gemm8_tile<64, BN, EPI_F32, bf16, true, 0, true>(A, B, nullptr, nullptr, nullptr, p.M, p.N, len, P, m0, n0, lds,
                                                       Geo{}, 0, nullptr, bx);
    else  // (TILE128: the 256 x 256 build with the staging registers would exceed the register file)
      gemm8_tile<BM / 2, BN / 2, EPI_F32, bf16, true, 0, true>(A, B, nullptr, nullptr, nullptr, p.M, p.N, len, P, m0,
                                                               n0, lds, Geo{}, 0, nullptr, bx);
    return;
  }
  if (p.flags & F32) {
    float* P = p.P + (size_t)sp * p.M * p.N;
    if (p.flags & NARROW_N)
      gemm8_tile<BM, 64, EPI_F32, bf16, true>(A, B, nullptr, nullptr, nullptr, p.M, p.N, len, P, m0, n0, lds);
    else if (p.flags & NARROW_M)
      gemm8_tile<64, BN, EPI_F32, bf16, true>(A, B, nullptr, nullptr, nullptr, p.M, p.N, len, P, m0, n0, lds);
    else if (p.flags & TILE128)
      gemm8_tile<BM / 2, BN / 2, EPI_F32, bf16, true>(A, B, nullptr, nullptr, nullptr, p.M, p.N, len, P, m0, n0, lds);
    else
      gemm8_tile<BM, BN, EPI_F32, bf16, true>(A, B, nullptr, nullptr, nullptr, p.M, p.N, len, P, m0, n0, lds);
    return;
  }
  bf16* C = (bf16*)p.C;
  if (quad >= 0 || (p.flags & TILE128)) {
    const int mq = quad >= 0 ? m0 + (quad >> 1) * (BM / 2) : m0, nq = quad >= 0 ? n0 + (quad & 1) * (BN / 2) : n0;
    gemm8_tile<BM / 2, BN / 2, EPI_NONE, bf16, true>(A, B, nullptr, C, nullptr, p.M, p.N, len, nullptr, mq, nq, lds);
    return;
  }
  gemm8_tile<BM, BN, EPI_NONE, bf16, true>(A, B, nullptr, C, nullptr, p.M, p.N, len, nullptr, m0, n0, lds);
}

__global__ __launch_bounds__(NT, 1) void gemm8_tn_grouped(const Group g) {
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  int item, quad = -1;
  if ((int)blockIdx.x < g.n_big) {  // bijective XCD-aware remap over the full-size items
    const int nwg = g.n_big, bid = blockIdx.x, xcd = bid % 8, q = nwg / 8, rr = nwg % 8;
    item = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + bid / 8;
  } else {
    const int sidx = blockIdx.x - g.n_big;
    item = g.n_big + sidx / 4;
    quad = sidx % 4;
  }
  int lo = 0, hi = g.n - 1;  // largest i with first[i] <= item
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if (g.first[mid] <= item) lo = mid; else hi = mid - 1;
  }
  grouped_item<256, 256, true>(g.p[lo], item - g.first[lo], quad, lds);
}

// C_i[M, N] (fp32) += sum over s of P_i[s][M][N], s in order; one thread per 4 elements, problems back to back
struct RedProb {
  const float* P;
  float* C;
  long long n4, first4;  // float4 count, first global float4 index
  int S, accum;
};
struct RedGroup {
  RedProb p[MAXP];
  int n;
};
__global__ __launch_bounds__(256) void gemm8_tn_reduce(const RedGroup g, long long total4) {
  const long long q = (long long)blockIdx.x * 256 + threadIdx.x;
  if (q >= total4) return;
  int i = 0;
  while (i + 1 < g.n && g.p[i + 1].first4 <= q) ++i;
  const RedProb& r = g.p[i];
  const long long k = q - r.first4;
  v4f acc = ((const v4f*)r.P)[k];
  for (int s = 1; s < r.S; ++s) acc += ((const v4f*)r.P)[(size_t)s * r.n4 + k];
  if (r.accum) acc += ((v4f*)r.C)[k];
  ((v4f*)r.C)[k] = acc;
}

// dynamic LDS: the main loop's two K-tile buffers, or the staged epilogue's bf16 tile (+ statistics scratch)
template <int BM, int BN, int EPI>
constexpr int lds_bytes() {
  const int loop = 2 * 2 * (BM / 2 + BN / 2) * 128;
  const int epi = BM * BN * 2 +
                  ((EPI == EPI_STATS || EPI == EPI_ADD_STATS || EPI == EPI_BNBWD || EPI == EPI_ADD_BNBWD) ? 9 * BN * 4
                                                                                                         : 0);
  return loop > epi ? loop : epi;
}

template <int BM, int BN, int EPI, typename P>
int launch(const void* X, const void* W, const void* bias, void* Y, void* Z, int M, int N, int K, float* part,
           hipStream_t st, const void* R2 = nullptr) {
  constexpr int LDS = lds_bytes<BM, BN, EPI>();
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)gemm8_nt<BM, BN, EPI, P>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    attr = true;
  }
  hipLaunchKernelGGL((gemm8_nt<BM, BN, EPI, P>), dim3((M / BM) * (N / BN)), dim3(NT), LDS, st, (const bf16*)X,
                     (const bf16*)W, (const P*)bias, (bf16*)Y, (bf16*)Z, M, N, K, part, (const bf16*)R2);
  return (int)hipGetLastError();
}

constexpr int BNX_MAXK = 2048;
template <int BM, int BN, int EPI>
int launch_bnx(const void* X, const void* W, const void* bias, void* Y, int M, int N, int K, float* part,
               const float* ax, hipStream_t st) {
  constexpr int LOOP = 2 * 2 * (BM / 2 + BN / 2) * 128, BASE = lds_bytes<BM, BN, EPI>();
  constexpr int MAXL = (LOOP + 8 * BNX_MAXK > BASE ? LOOP + 8 * BNX_MAXK : BASE);
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)gemm8_nt_bnx<BM, BN, EPI>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              MAXL);
    attr = true;
  }
  const int lds = LOOP + 8 * K > BASE ? LOOP + 8 * K : BASE;
  hipLaunchKernelGGL((gemm8_nt_bnx<BM, BN, EPI>), dim3((M / BM) * (N / BN)), dim3(NT), lds, st, (const bf16*)X,
                     (const bf16*)W, (const bf16*)bias, (bf16*)Y, M, N, K, part, ax);
  return (int)hipGetLastError();
}
template <int BM, int BN>
int dispatch_bnx(int epi, const void* X, const void* W, const void* bias, void* Y, int M, int N, int K, float* part,
                 const float* ax, hipStream_t st) {
  switch (epi) {
    case EPI_NONE: return launch_bnx<BM, BN, EPI_NONE>(X, W, nullptr, Y, M, N, K, nullptr, ax, st);
    case EPI_STATS: return launch_bnx<BM, BN, EPI_STATS>(X, W, nullptr, Y, M, N, K, part, ax, st);
    case EPI_ADD_STATS: return launch_bnx<BM, BN, EPI_ADD_STATS>(X, W, bias, Y, M, N, K, part, ax, st);
  }
  return -1;
}

template <int BM, int BN, int EPI>
int launch_conv(const void* X, const void* W, const void* bias, void* Y, void* Z, int M, int N, int K, float* part,
                const Geo& geo, hipStream_t st) {
  constexpr int LDS = lds_bytes<BM, BN, EPI>();
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)gemm8_conv<BM, BN, EPI, bf16>, hipFuncAttributeMaxDynamicSharedMemorySize,
                              LDS);
    attr = true;
  }
  hipLaunchKernelGGL((gemm8_conv<BM, BN, EPI, bf16>), dim3((M / BM) * (N / BN)), dim3(NT), LDS, st, (const bf16*)X,
                     (const bf16*)W, (const bf16*)bias, (bf16*)Y, (bf16*)Z, M, N, K, part, geo);
  return (int)hipGetLastError();
}

template <int BM, int BN>
int dispatch_conv(int epi, const void* X, const void* W, const void* bias, void* Y, void* Z, int M, int N, int K,
                  float* part, const Geo& geo, hipStream_t st) {
  switch (epi) {
    case EPI_NONE: return launch_conv<BM, BN, EPI_NONE>(X, W, nullptr, Y, nullptr, M, N, K, nullptr, geo, st);
    case EPI_STATS: return launch_conv<BM, BN, EPI_STATS>(X, W, nullptr, Y, nullptr, M, N, K, part, geo, st);
    case EPI_BNBWD: return launch_conv<BM, BN, EPI_BNBWD>(X, W, bias, Y, Z, M, N, K, part, geo, st);
  }
  return -1;
}

Geo make_geo(int H, int W, int C, int OH, int OW, int stride, int pad, int tap0 = 0, int ntaps = 9) {
  Geo g{H, W, C, OH, OW, stride, pad, 0, 0u, 0, 0u, 0, tap0, ntaps};
  while ((1 << g.cshift) < C) ++g.cshift;
  auto magic = [](unsigned d, unsigned& mul, int& sh) {  // x / d == (umulhi(x, mul) + x) >> sh for x < 2^31
    sh = 0;
    while ((1ull << sh) < d) ++sh;
    mul = (unsigned)(((1ull << 32) * ((1ull << sh) - d)) / d + 1);
  };
  magic((unsigned)OW, g.ow_mul, g.ow_sh);
  magic((unsigned)(OH * OW), g.ohw_mul, g.ohw_sh);
  return g;
}

bool geo_ok(int Nb, int H, int W, int C, int OH, int OW, int stride, int pad) {
  return Nb > 0 && H > 0 && W > 0 && C >= 64 && (C & (C - 1)) == 0 && stride >= 1 && stride <= 2 && pad >= 0 &&
         pad <= 2 && OH == (H + 2 * pad - 3) / stride + 1 && OW == (W + 2 * pad - 3) / stride + 1 &&
         (long long)Nb * H * W * C < (1ll << 31) && (long long)Nb * OH * OW < (1ll << 31);
}

template <int BM, int BN>
int dispatch(int epi, int bias_f32, const void* X, const void* W, const void* bias, void* Y, void* Z, int M, int N,
             int K, float* part, hipStream_t st, const void* R2) {
  switch (epi) {
    case EPI_NONE: return launch<BM, BN, EPI_NONE, bf16>(X, W, nullptr, Y, nullptr, M, N, K, nullptr, st);
    case EPI_BIAS:
      return bias_f32 ? launch<BM, BN, EPI_BIAS, float>(X, W, bias, Y, nullptr, M, N, K, nullptr, st)
                      : launch<BM, BN, EPI_BIAS, bf16>(X, W, bias, Y, nullptr, M, N, K, nullptr, st);
    case EPI_BIAS_GELU:
      return bias_f32 ? launch<BM, BN, EPI_BIAS_GELU, float>(X, W, bias, Y, Z, M, N, K, nullptr, st)
                      : launch<BM, BN, EPI_BIAS_GELU, bf16>(X, W, bias, Y, Z, M, N, K, nullptr, st);
    case EPI_ADD_R: return launch<BM, BN, EPI_ADD_R, bf16>(X, W, bias, Y, nullptr, M, N, K, nullptr, st);
    case EPI_GELU_BWD:
      if constexpr (BN == 64) {
        return -1;  // (not built for the narrow tiles)
      } else {
        return bias_f32 ? launch<BM, BN, EPI_GELU_BWD, float>(X, W, bias, Y, Z, M, N, K, part, st)
                        : launch<BM, BN, EPI_GELU_BWD, bf16>(X, W, bias, Y, Z, M, N, K, part, st);
      }
    case EPI_STATS: return launch<BM, BN, EPI_STATS, bf16>(X, W, nullptr, Y, nullptr, M, N, K, part, st);
    case EPI_ADD_STATS: return launch<BM, BN, EPI_ADD_STATS, bf16>(X, W, bias, Y, nullptr, M, N, K, part, st);
    case EPI_BNBWD: return launch<BM, BN, EPI_BNBWD, bf16>(X, W, bias, Y, Z, M, N, K, part, st);
    case EPI_ADD_BNBWD: return launch<BM, BN, EPI_ADD_BNBWD, bf16>(X, W, bias, Y, Z, M, N, K, part, st, R2);
  }
  return -1;
}

struct Cfg {
  int bm, bn;
};
constexpr Cfg kCfgs[] = {{256, 256}, {256, 128}, {128, 256}, {128, 128}, {256, 64}, {128, 64}};

}  // namespace

extern "C" {

int mifx_gemm8_configs(int* out, int n) {
  const int m = (int)(sizeof(kCfgs) / sizeof(Cfg));
  for (int i = 0; i < m && 2 * i + 1 < n; ++i) {
    out[2 * i] = kCfgs[i].bm;
    out[2 * i + 1] = kCfgs[i].bn;
  }
  return m;
}

// Y[M, N] = X[M, K] . W[N, K]^T, bf16 in / out, fp32 accumulation. epi: 0 none; 1 + bias[N]; 2 GELU(. + bias) with
// Z = bf16(X W^T) (pre-bias); 3 + R (bias = bf16 [M, N]); 4 dZ = (X W^T) o GELU'(Z + bias) with part[M / BM][N] the
// per-tile column sums of dZ; 5 part[2][M / BM][N] = per-tile column mean / sum of squared deviations (M2) of the
// stored Y; 6 = 3 and 5: Y = X W^T + R with the statistics of the stored sum; 8: Y = X W^T is the gradient of a
// BatchNorm + ReLU output, bias = the BatchNorm's input (bf16 [M, N]), Z = its statistics (fp32 [4][N]: mean, rstd,
// scale, shift), part[2][M / BM][N] = per-tile (sum g, sum g xhat) of the BatchNorm backward; 9: as 8 for
// Y = X W^T + R2 (bf16 [M, N]). bias bf16 or fp32 (bias_f32). M % BM == 0, N % BN == 0, K % 64 == 0, 16-byte aligned operands.
int mifx_gemm8_nt(int cfg, int epi, int bias_f32, const void* X, const void* W, const void* bias, void* Y, void* Z,
                  float* part, int M, int N, int K, const void* R2, hipStream_t st) {
  const int m = (int)(sizeof(kCfgs) / sizeof(Cfg));
  if (cfg < 0 || cfg >= m || M <= 0 || N <= 0 || K <= 0 || X == nullptr || W == nullptr || Y == nullptr) return -1;
  const Cfg c = kCfgs[cfg];
  if (M % c.bm || N % c.bn || K % BK) return -1;
  if (epi < 0 || epi > 9 || epi == 7) return -1;
  if ((epi >= 1 && epi <= 4) || epi == 6 || epi >= 8) {
    if (bias == nullptr) return -1;
  }
  if ((epi == 2 || epi == 4 || epi >= 8) && Z == nullptr) return -1;
  if (epi >= 4 && part == nullptr) return -1;
  if (epi >= 8 && (uintptr_t)bias % 16) return -1;
  if (epi == 9 && (R2 == nullptr || (uintptr_t)R2 % 16)) return -1;
  if ((uintptr_t)X % 16 || (uintptr_t)W % 16 || (uintptr_t)Y % 16 || (Z != nullptr && (uintptr_t)Z % 8)) return -1;
  if ((epi == 3 || epi == 6) && (uintptr_t)bias % 16) return -1;
  if ((long long)M * K >= (1ll << 31) || (long long)N * K >= (1ll << 31)) return -1;  // 32-bit element offsets
  switch (cfg) {
    case 0: return dispatch<256, 256>(epi, bias_f32, X, W, bias, Y, Z, M, N, K, part, st, R2);
    case 1: return dispatch<256, 128>(epi, bias_f32, X, W, bias, Y, Z, M, N, K, part, st, R2);
    case 2: return dispatch<128, 256>(epi, bias_f32, X, W, bias, Y, Z, M, N, K, part, st, R2);
    case 3: return dispatch<128, 128>(epi, bias_f32, X, W, bias, Y, Z, M, N, K, part, st, R2);
    case 4: return dispatch<256, 64>(epi, bias_f32, X, W, bias, Y, Z, M, N, K, part, st, R2);
    default: return dispatch<128, 64>(epi, bias_f32, X, W, bias, Y, Z, M, N, K, part, st, R2);
  }
}

// Y[M, N] = relu(X scale + shift) . W[N, K]^T (+ R: epi 6) with ax = fp32 [scale[K], shift[K]] (a BatchNorm's
// finalized statistics): the 1x1 convolution consuming a BatchNorm + ReLU, reading the BatchNorm's input X. epi 0, 5
// (statistics of Y), 6 (bias = R bf16 [M, N], statistics of the stored sum). K <= 2048; otherwise as mifx_gemm8_nt.
int mifx_gemm8_nt_bnx(int cfg, int epi, const void* X, const void* W, const void* bias, void* Y, float* part, int M,
                      int N, int K, const float* ax, hipStream_t st) {
  const int m = (int)(sizeof(kCfgs) / sizeof(Cfg));
  if (cfg < 0 || cfg >= m || M <= 0 || N <= 0 || K <= 0 || K > BNX_MAXK || X == nullptr || W == nullptr ||
      Y == nullptr || ax == nullptr)
    return -1;
  const Cfg c = kCfgs[cfg];
  if (M % c.bm || N % c.bn || K % BK) return -1;
  if (epi != 0 && epi != 5 && epi != 6) return -1;
  if (epi != 0 && part == nullptr) return -1;
  if (epi == 6 && (bias == nullptr || (uintptr_t)bias % 16)) return -1;
  if ((uintptr_t)X % 16 || (uintptr_t)W % 16 || (uintptr_t)Y % 16 || (uintptr_t)ax % 16) return -1;
  if ((long long)M * K >= (1ll << 31) || (long long)N * K >= (1ll << 31)) return -1;
  switch (cfg) {
    case 0: return dispatch_bnx<256, 256>(epi, X, W, bias, Y, M, N, K, part, ax, st);
    case 1: return dispatch_bnx<256, 128>(epi, X, W, bias, Y, M, N, K, part, ax, st);
    case 2: return dispatch_bnx<128, 256>(epi, X, W, bias, Y, M, N, K, part, ax, st);
    case 3: return dispatch_bnx<128, 128>(epi, X, W, bias, Y, M, N, K, part, ax, st);
    case 4: return dispatch_bnx<256, 64>(epi, X, W, bias, Y, M, N, K, part, ax, st);
    default: return dispatch_bnx<128, 64>(epi, X, W, bias, Y, M, N, K, part, ax, st);
  }
}

// 3x3 convolution as an implicit GEMM (see Geo): x bf16 NHWC [Nb][H][W][C], w bf16 [N][3][3][C] (channels_last
// weight), y bf16 [Nb OH OW][N]; epi 0 none, 5 per-tile BatchNorm statistics of y (as mifx_gemm8_nt), 8 y is a
// BatchNorm + ReLU output gradient (bias = that BatchNorm's input [Nb OH OW][N], Z = its statistics) with the per-tile
// backward sums. Nb OH OW % BM == 0, N % BN == 0.
int mifx_gemm8_conv3x3(int cfg, int epi, const void* x, const void* w, const void* bias, void* y, void* Z, float* part,
                       int Nb, int H, int W, int C, int N, int stride, int pad, hipStream_t st) {
  const int m = (int)(sizeof(kCfgs) / sizeof(Cfg));
  if (cfg < 0 || cfg >= m || x == nullptr || w == nullptr || y == nullptr) return -1;
  const int OH = (H + 2 * pad - 3) / stride + 1, OW = (W + 2 * pad - 3) / stride + 1;
  if (!geo_ok(Nb, H, W, C, OH, OW, stride, pad)) return -1;
  const Cfg c = kCfgs[cfg];
  const int M = Nb * OH * OW, K = 9 * C;
  if (M % c.bm || N <= 0 || N % c.bn || (long long)N * K >= (1ll << 31)) return -1;
  if (epi != 0 && epi != 5 && epi != 8) return -1;
  if (epi != 0 && part == nullptr) return -1;
  if (epi == 8 && (bias == nullptr || Z == nullptr || (uintptr_t)bias % 16)) return -1;
  if ((uintptr_t)x % 16 || (uintptr_t)w % 16 || (uintptr_t)y % 16) return -1;
  const Geo g = make_geo(H, W, C, OH, OW, stride, pad);
  switch (cfg) {
    case 0: return dispatch_conv<256, 256>(epi, x, w, bias, y, Z, M, N, K, part, g, st);
    case 1: return dispatch_conv<256, 128>(epi, x, w, bias, y, Z, M, N, K, part, g, st);
    case 2: return dispatch_conv<128, 256>(epi, x, w, bias, y, Z, M, N, K, part, g, st);
    case 3: return dispatch_conv<128, 128>(epi, x, w, bias, y, Z, M, N, K, part, g, st);
    case 4: return dispatch_conv<256, 64>(epi, x, w, bias, y, Z, M, N, K, part, g, st);
    default: return dispatch_conv<128, 64>(epi, x, w, bias, y, Z, M, N, K, part, g, st);
  }
}

// The device-side geometry record of a convolution for mifx_gemm8_tn_grouped's CONV problems: a 3x3 pad-`pad`
// convolution (center1x1 = 0, N = 9 C), or a strided 1x1 (center1x1 = 1: the center tap of a pad-1 3x3, N = C).
int mifx_gemm8_geo_bytes() { return (int)sizeof(Geo); }
int mifx_gemm8_geo(int Nb, int H, int W, int C, int stride, int pad, int center1x1, void* out) {
  if (center1x1) pad = 1;
  const int OH = (H + 2 * pad - 3) / stride + 1, OW = (W + 2 * pad - 3) / stride + 1;
  if (out == nullptr || !geo_ok(Nb, H, W, C, OH, OW, stride, pad)) return -1;
  const Geo g = center1x1 ? make_geo(H, W, C, OH, OW, stride, pad, 4, 1) : make_geo(H, W, C, OH, OW, stride, pad);
  __builtin_memcpy(out, &g, sizeof(Geo));
  return 0;
}

// Strided 1x1 convolution (stride 2 ResNet shortcuts) as the center tap of the implicit GEMM: y [Nb OH OW][N] =
// x[Nb][stride oh][stride ow][:] . w[N][C]^T, OH = (H - 1) / stride + 1; epi 0 or 5 (statistics).
int mifx_gemm8_conv1x1s(int cfg, int epi, const void* x, const void* w, void* y, float* part, int Nb, int H, int W,
                        int C, int N, int stride, hipStream_t st) {
  const int m = (int)(sizeof(kCfgs) / sizeof(Cfg));
  if (cfg < 0 || cfg >= m || x == nullptr || w == nullptr || y == nullptr || stride < 1 || stride > 2) return -1;
  const int OH = (H - 1) / stride + 1, OW = (W - 1) / stride + 1;
  if (!geo_ok(Nb, H, W, C, OH, OW, stride, 1)) return -1;
  const Cfg c = kCfgs[cfg];
  const int M = Nb * OH * OW;
  if (M % c.bm || N <= 0 || N % c.bn || (long long)N * C >= (1ll << 31)) return -1;
  if (epi != 0 && epi != 5) return -1;
  if (epi == 5 && part == nullptr) return -1;
  if ((uintptr_t)x % 16 || (uintptr_t)w % 16 || (uintptr_t)y % 16) return -1;
  const Geo g = make_geo(H, W, C, OH, OW, stride, 1, 4, 1);
  switch (cfg) {
    case 0: return dispatch_conv<256, 256>(epi, x, w, nullptr, y, nullptr, M, N, C, part, g, st);
    case 1: return dispatch_conv<256, 128>(epi, x, w, nullptr, y, nullptr, M, N, C, part, g, st);
    case 2: return dispatch_conv<128, 256>(epi, x, w, nullptr, y, nullptr, M, N, C, part, g, st);
    case 3: return dispatch_conv<128, 128>(epi, x, w, nullptr, y, nullptr, M, N, C, part, g, st);
    case 4: return dispatch_conv<256, 64>(epi, x, w, nullptr, y, nullptr, M, N, C, part, g, st);
    default: return dispatch_conv<128, 64>(epi, x, w, nullptr, y, nullptr, M, N, C, part, g, st);
  }
}

// Grouped TN GEMM: for i < n, C_i[M_i, N_i] = A_i[T_i, M_i]^T B_i[T_i, N_i] (bf16 row-major operands, fp32
// accumulation), all in ONE launch. flags_i: bit 0 F32 -- C_i is fp32 and receives the product (+= with bit 2 ACCUM,
// else =), computed in
// token chunks of chunk_i rows (fp32 partials in ws, summed in order by a second launch); bit 1 TILE128 -- 128 x 128
// tiles (M_i, N_i % 128) instead of 256 x 256 (% 256). bf16 problems need chunk_i = T_i. T_i % 64 == 0, chunk_i % 64
// == 0, 16-byte aligned operands, n <= 64. Bit 3 CONV: B is a convolution input gathered by geos[i] (a Geo); bit 6
// BNX: the B operand is relu(B scale + shift) per column, geos[i] = fp32 [scale[N], shift[N]]. ws: fp32 workspace of sum over F32 problems of S_i M_i N_i floats
// (S_i = ceil(T_i / chunk_i)), may be null without F32 problems. Returns the number of work items (> 0) or < 0.
int mifx_gemm8_tn_grouped(int n, const void* const* A, const void* const* B, void* const* C, const int* M,
                          const int* N, const int* T, const int* chunk, const int* flags, float* ws,
                          const void* const* geos, hipStream_t st) {
  if (n <= 0 || n > MAXP) return -1;
  Group g{};
  RedGroup rg{};
  int items = 0, nred = 0;
  bool uniform256 = true;
  long long woff = 0, r4 = 0;
  for (int i = 0; i < n; ++i) {
    const int fl = flags[i], tb = (fl & TILE128) ? 128 : 256;
    const int tm = (fl & NARROW_M) ? 64 : tb, tn = (fl & NARROW_N) ? 64 : tb;
    if (A[i] == nullptr || B[i] == nullptr || C[i] == nullptr || M[i] <= 0 || N[i] <= 0 || T[i] <= 0) return -1;
    if (M[i] % tm || N[i] % tn || T[i] % BK || chunk[i] <= 0 || chunk[i] % BK) return -1;
    if ((fl & (NARROW_M | NARROW_N)) && (!(fl & F32) || (fl & TILE128) || (fl & NARROW_M && fl & NARROW_N) ||
                                         (fl & NARROW_M && fl & CONV)))
      return -1;
    if (!(fl & F32) && chunk[i] != T[i]) return -1;
    if ((uintptr_t)A[i] % 16 || (uintptr_t)B[i] % 16 || (uintptr_t)C[i] % 16) return -1;
    if ((long long)T[i] * M[i] >= (1ll << 31)) return -1;
    if (!(fl & CONV) && (long long)T[i] * N[i] >= (1ll << 31)) return -1;
    const void* aux = nullptr;
    if (fl & CONV) {  // geometry in device memory; N = 9 C with C % (tile width) == 0 (one tap per column block)
      if (!(fl & F32) || geos == nullptr || geos[i] == nullptr || N[i] % tn) return -1;  // (N = taps x C, host-side)
      aux = geos[i];
    }
    if (fl & BNX) {  // aux[i]: the BatchNorm's fp32 [scale[N], shift[N]]; 128 x 128 or narrow tiles only
      if (!(fl & F32) || (fl & CONV) || geos == nullptr || geos[i] == nullptr || (uintptr_t)geos[i] % 16) return -1;
      if (!(fl & (TILE128 | NARROW_M | NARROW_N))) return -1;
      aux = geos[i];
    }
    const int S = (T[i] + chunk[i] - 1) / chunk[i];
    float* P = nullptr;
    if (fl & F32) {
      if (ws == nullptr) return -1;
      P = ws + woff;
      const long long n4 = (long long)M[i] * N[i] / 4;
      rg.p[nred++] = RedProb{P, (float*)C[i], n4, r4, S, (fl & ACCUM) ? 1 : 0};
      r4 += n4;
      woff += (long long)S * M[i] * N[i];
      uniform256 = false;
    }
    if (fl & (TILE128 | NARROW_M | NARROW_N)) uniform256 = false;
    g.p[i] = Prob{(const bf16*)A[i], (const bf16*)B[i], C[i], P, aux, M[i], N[i], T[i], chunk[i], S, fl};
    g.first[i] = items;
    items += (M[i] / tm) * (N[i] / tn) * S;
  }
  g.first[n] = items;
  g.n = n;
  // a last partial wave of at most a quarter of the chip runs as quarter-size tiles (4x the workgroups, 1/4 the time)
  const int cus = 256, rem = items % cus;
  g.n_big = (uniform256 && items > cus && rem > 0 && rem <= cus / 4) ? items - rem : items;
  const int grid = g.n_big + 4 * (items - g.n_big);
  constexpr int LDS = lds_bytes<256, 256, EPI_NONE>() + 2 * 256 * 4 + NT * 16;  // + BNX column table, dup scratch
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)gemm8_tn_grouped, hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    attr = true;
  }
  hipLaunchKernelGGL(gemm8_tn_grouped, dim3(grid), dim3(NT), LDS, st, g);
  if (nred) {
    rg.n = nred;
    hipLaunchKernelGGL(gemm8_tn_reduce, dim3((unsigned)((r4 + 255) / 256)), dim3(256), 0, st, rg, r4);
  }
  const int rc = (int)hipGetLastError();
  return rc ? -rc : items;
}

}  // extern "C"
