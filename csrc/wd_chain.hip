// Register-chained fused Wide&Deep training step for gfx950 (second-generation kernel).
//
// Parity target: reference `airflow-dags/taxi_utils.py:148-191` (_build_estimator: DNNLinearCombinedClassifier,
// DNN [100, 70, 48, 34] on 3 dense floats, linear part over 9 categorical identity columns, sigmoid CE) with
// the hidden sizes of `trainer_fn` (`taxi_utils.py:300-345`). Same math and gradient-slab contract as
// csrc/wide_deep.hip (wd_fused); the data flow inside a workgroup is different:
//
//  * 4 waves x 32 examples = 128 examples per iteration. A wave carries ITS 32 examples (two 16-column
//    blocks) through the whole forward in registers: layer l's 16x16 MFMA output tiles (lane = example,
//    4 consecutive output features per lane) are ReLU'd, packed to bf16 and used directly as the B operand of
//    layer l+1 (tiles 2s and 2s+1 form k-step s). This makes layer l+1's k order a fixed permutation of the
//    natural feature order inside every 32-block (position 8H + E <-> feature 16(E/4) + 4H + E%4), so each
//    layer's weight image is stored with its COLUMNS in that "C order" (host: models.wide_deep.chain_perm).
//    No LDS activation traffic and no block barrier in the forward; each weight fragment read from LDS
//    feeds two MFMAs (both column blocks).
//  * The activation-gradient chain dA_{l-1} = W_l^T dZ_l stays in registers the same way (output tiles of
//    one layer are the B operand of the next); its A operand is read from the same weight image with
//    ds_read_b64_tr_b16 at the permuted rows that match (rows 32s + 16(h%2) + 4(h/2) + {0..3, 8..11}).
//    Layer 5 (one logit row) is a rank-1 product done on the VALU.
//  * Weight gradients dW_l^T = dZ_l^T A_{l-1} reduce over examples, so they need the transpose: per layer the
//    128 x N_l gradient (natural order) and the 128 x K_l activation (C order) are staged in LDS once and read
//    back with ds_read_b64_tr_b16; every wave owns a fixed set of 16x16 dW tiles and keeps their fp32
//    accumulators in registers across ALL iterations (MFMA K-accumulation == batch reduction), so the
//    workgroup writes one gradient slab at the end, in the same tile-native layout as wd_fused.
//    The ReLU masks of the backward come from the staged activations (C order, 8-byte reads).
//  * Wide part: embedding-bag gather of 9 fp32 weights per example (issued before the forward), fixed-point
//    LDS histogram for its gradient (order-independent -> deterministic), as in wd_fused.
//
// MIFX_HIPCC_FLAGS: -fno-honor-nans -fno-honor-infinities
#include <hip/hip_runtime.h>
#include "xcd.h"
#include "feed.h"
#include <stdint.h>

namespace {

typedef __bf16 bf16;
typedef __bf16 v8bf __attribute__((ext_vector_type(8)));
typedef __bf16 v4bf __attribute__((ext_vector_type(4)));
typedef __bf16 v2bf __attribute__((ext_vector_type(2)));
typedef short v4s __attribute__((ext_vector_type(4)));
typedef short v8s __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4s lds_v4s;

#include "wd_opt.h"

#ifndef WDC_T
#define WDC_T 128
#endif
// examples per workgroup iteration: 128 (this file's library), 64 (csrc/wd_chain64.hip: the same kernel built
// for one 4-wave workgroup of 4 x 16 examples, the small-batch shape) or 256 (csrc/wd_chain256.hip: 8 waves x 32
// examples, two column blocks per wave -- the large-batch shape: one iteration per workgroup at B = 65536 on 256
// workgroups, the forward and activation-gradient chains of both blocks interleaved in one wave)
constexpr int T = WDC_T;
static_assert(T == 128 || T == 64 || T == 256, "T");
constexpr bool ONE_ITER = T == 256 || T == 64;  // see the iteration loop of wdc_fused
constexpr int MAXW = 8;  // waves per workgroup: T / (16 TBN), TBN = 16-example column blocks per wave (1 or 2)
// Row padding (elements): WPAD for the weight images, PAD for the staging images; with the row permutations below
// (wperm, sperm16) every LDS access site is conflict-free in the bank model (tools/lds_banks.py). (XOR swizzles
// of 8-byte granules reach the same in the model, but their per-lane XORs defeat the compiler's immediate-offset
// addressing and the kernels then spill: measured, not adopted.)
constexpr int WPAD = 16;
constexpr int PAD = 8;

constexpr int K1 = 32, N1 = 128;
constexpr int K2 = 128, N2 = 96;
constexpr int K3 = 96, N3 = 64;
constexpr int K4 = 64, N4 = 64;
constexpr int K5 = 64, N5 = 16;

// weight image (bf16, LDS layout == global image layout): W_l^T [N_l][K_l + WPAD], columns in C order
constexpr int LW1 = 0;
constexpr int LW2 = LW1 + N1 * (K1 + WPAD);
constexpr int LW3 = LW2 + N2 * (K2 + WPAD);
constexpr int LW4 = LW3 + N3 * (K3 + WPAD);
constexpr int LW5 = LW4 + N4 * (K4 + WPAD);
constexpr int LWEND = LW5 + N5 * (K5 + WPAD);  // 33536
// dW staging: dZ_l [T][N_l + PAD] (natural order) followed by A_{l-1} [T][K_l + PAD] (C order)
constexpr int stage_len(int K, int N) { return T * (N + PAD) + T * (K + PAD); }
constexpr int cmax(int a, int b) { return a > b ? a : b; }
// LDS left for staging next to the weight image and the wide histogram. A layer whose full staging (T rows of dZ
// and A) does not fit is staged and reduced in two passes of T / 2 rows -- column block 0 of every wave, then
// block 1 (T = 256: layers 1-3; never at T <= 128)
constexpr int WIDE_PAD = 2176;  // the wide (linear) weights / histogram, padded
constexpr int LDS_FIXED_B = LWEND * 2 + WIDE_PAD * 4 + 64 * 4;
constexpr int STAGE_MAX = ((163840 - LDS_FIXED_B) / 2) & ~7;
constexpr bool split_stage(int K, int N) { return stage_len(K, N) > STAGE_MAX; }
constexpr int stage_eff(int K, int N) { return split_stage(K, N) ? stage_len(K, N) / 2 : stage_len(K, N); }
constexpr int LSLEN = cmax(cmax(cmax(stage_eff(K1, N1), stage_eff(K2, N2)), cmax(stage_eff(K3, N3), stage_eff(K4, N4))),
                           stage_eff(K5, N5));
static_assert(T == 256 || !(split_stage(K1, N1) || split_stage(K2, N2) || split_stage(K3, N3) ||
                            split_stage(K4, N4) || split_stage(K5, N5)), "split staging is the T = 256 shape's");
static_assert(!split_stage(K4, N4) && !split_stage(K5, N5), "layers 4-5 stage whole");
constexpr int LS = LWEND;
constexpr int LSEND = LS + LSLEN;
constexpr int NWIDE = 2128;
constexpr int WIDE_BIAS = 2127;
constexpr int NTILE = 108;
constexpr int LDS_BYTES = LSEND * 2 + WIDE_PAD * 4 + 64 * 4;
static_assert(LDS_BYTES <= 163840, "LDS budget");
static_assert((LSEND * 2) % 16 == 0 && (LS * 2) % 16 == 0, "16-B aligned regions");

constexpr int TB1 = 0, TB2 = TB1 + (N1 / 16) * (K1 / 16), TB3 = TB2 + (N2 / 16) * (K2 / 16),
              TB4 = TB3 + (N3 / 16) * (K3 / 16), TB5 = TB4 + (N4 / 16) * (K4 / 16);
static_assert(TB5 + (N5 / 16) * (K5 / 16) == NTILE, "tile count");

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
// Packed-bf16 activation math: 2 values per 32-bit lane op instead of a compare/select or max per value.
typedef short s16x2 __attribute__((ext_vector_type(2)));
typedef unsigned short u16x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ unsigned int cvt_pk(float lo, float hi) {  // v_cvt_pk_bf16_f32 (round to nearest even)
  return __builtin_bit_cast(unsigned int, (v2bf){(bf16)lo, (bf16)hi});
}
// relu on two packed bf16: as signed 16-bit integers negative bf16 values (and -0) are negative, non-negative ones
// order like their floats, so max(x, 0) in int16 is relu(x) (= relu before rounding: rounding keeps the sign)
__device__ __forceinline__ unsigned int relu_pk(unsigned int x) {
  return __builtin_bit_cast(unsigned int, __builtin_elementwise_max(__builtin_bit_cast(s16x2, x), (s16x2){0, 0}));
}
// zero the bf16 halves of g whose activation half in a is zero (a >= 0 after relu): g * min(a, 1) in u16
// (asm: written as u16 vector math the compiler turns it back into a compare + select per half)
__device__ __forceinline__ unsigned int mask_pk(unsigned int g, unsigned int a) {
  unsigned int m, r;
  // the (1, 1) operand from a register: a packed op's inline constant only fills the low half
  asm("v_pk_min_u16 %0, %1, %2" : "=v"(m) : "v"(a), "v"(0x00010001u));
  asm("v_pk_mul_lo_u16 %0, %1, %2" : "=v"(r) : "v"(g), "v"(m));
  return r;
}
__device__ __forceinline__ v8bf pack_relu(v4f a, v4f b) {
  const unsigned int u[4] = {relu_pk(cvt_pk(a[0], a[1])), relu_pk(cvt_pk(a[2], a[3])), relu_pk(cvt_pk(b[0], b[1])),
                             relu_pk(cvt_pk(b[2], b[3]))};
  return __builtin_bit_cast(v8bf, u);
}
__device__ __forceinline__ v4bf to_bf4(v4f a) {
  v4bf o;
#pragma unroll
  for (int i = 0; i < 4; ++i) o[i] = (bf16)a[i];
  return o;
}
__device__ __forceinline__ v8bf cat_bf(v4bf a, v4bf b) {
  v8bf o;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    o[i] = a[i];
    o[4 + i] = b[i];
  }
  return o;
}
__device__ __forceinline__ void block_sync_lds() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
constexpr v4f kZero4 = {0.f, 0.f, 0.f, 0.f};

// ---- LDS row permutations (bank-conflict control; tools/lds_banks.py models every access site of this kernel and
// finds all of them conflict-free with these layouts, padding alone leaves 2x on the transposed reads):
//  * weight images: physical row wperm(n) = n ^ (bit 4 of n) << 2. The activation-gradient transposed reads of a
//    32-lane half touch rows q and 16 + q (+8); with 8 + 16 k dword rows (WPAD 16) rows 16 + q would share banks
//    with rows q, as rows 20 + q they do not. The lane part of every permuted row is known per lane (bit 4 of the
//    row is lane-dependent in the transposed read, one of two constants in the forward read).
//  * staging images: inside every 16-row block, row bits (b3 b2 b1 b0) -> (b3 b1 b0 b2): the 8 rows a 32-lane half
//    of a dW transposed read touches (q, 8 + q) become physical rows of one parity, which with 4 mod 8 dword rows
//    (PAD 8) are 8 dwords apart mod 64; the 16-byte stores and 8-byte mask reads of 16 consecutive rows stay
//    conflict-free. models.wide_deep.chain_image_offsets applies wperm on the host.
__host__ __device__ constexpr int wperm(int n) { return n ^ (((n >> 4) & 1) << 2); }
__host__ __device__ constexpr int sperm16(int t) { return (t & 8) | ((t & 3) << 1) | ((t >> 2) & 1); }

#ifdef WDC_STAMPS  // diagnostic build only (tools/build_stamps.sh): per-wave shader-clock stamps of block 0
__device__ unsigned long long g_wdc_stamps[MAXW][32];
#define STAMP(i)                                                                                  \
  do {                                                                                            \
    __builtin_amdgcn_sched_barrier(0);                                                            \
    if (blockIdx.x == 0 && lane == 0 && stamp_on) g_wdc_stamps[w][i] = __builtin_amdgcn_s_memtime(); \
    __builtin_amdgcn_sched_barrier(0);                                                            \
  } while (0)
// per-block 100 MHz global clock: [block][0] start, [1] prologue done, [2] end (wave 0)
__device__ unsigned long long g_wdc_blk[4096][3];
#define BSTAMP(i)                                                                                       \
  do {                                                                                                  \
    __builtin_amdgcn_sched_barrier(0);                                                                  \
    if (w == 0 && lane == 0 && blockIdx.x < 4096) g_wdc_blk[blockIdx.x][i] = __builtin_amdgcn_s_memrealtime(); \
    __builtin_amdgcn_sched_barrier(0);                                                                  \
  } while (0)
#else
#define BSTAMP(i) \
  do {            \
  } while (0)
#define STAMP(i) \
  do {           \
  } while (0)
#endif

// ---- forward layer for the wave's two column blocks: acc[tb][nt] = W^T[16 nt ..][.] . B[tb][.]
// W image rows natural, columns C order; B[tb][s] is the k-step-s fragment (C order) of the layer input.
template <int K, int N, int TBN>
__device__ __forceinline__ void fwd(const uint16_t* W, const v8bf (&B)[TBN][K / 32], v4f (&acc)[TBN][N / 16], int r,
                                    int h) {
  constexpr int KS = K / 32, NT = N / 16;
#pragma unroll
  for (int nt = 0; nt < NT; ++nt)
#pragma unroll
    for (int tb = 0; tb < TBN; ++tb) acc[tb][nt] = kZero4;
  const int rw[2] = {r, r ^ 4};  // physical row in a 32-row block: 16 nt + rw[nt & 1]
  v8bf wa[2][NT];
#pragma unroll
  for (int nt = 0; nt < NT; ++nt) wa[0][nt] = ld8(W + (16 * nt + rw[nt & 1]) * (K + WPAD) + 8 * h);
#pragma unroll
  for (int s = 0; s < KS; ++s) {
    if (s + 1 < KS) {
#pragma unroll
      for (int nt = 0; nt < NT; ++nt) wa[(s + 1) & 1][nt] = ld8(W + (16 * nt + rw[nt & 1]) * (K + WPAD) + 32 * (s + 1) + 8 * h);
    }
#pragma unroll
    for (int nt = 0; nt < NT; ++nt)
#pragma unroll
      for (int tb = 0; tb < TBN; ++tb) acc[tb][nt] = mfma(wa[s & 1][nt], B[tb][s], acc[tb][nt]);
  }
}

template <int N, int TBN>
__device__ __forceinline__ void relu_pack(const v4f (&acc)[TBN][N / 16], v8bf (&out)[TBN][N / 32]) {
#pragma unroll
  for (int tb = 0; tb < TBN; ++tb)
#pragma unroll
    for (int s = 0; s < N / 32; ++s) out[tb][s] = pack_relu(acc[tb][2 * s], acc[tb][2 * s + 1]);
}

// ---- activation gradient: dA^T[k][t] = sum_n W[n][k] dZ[n][t] for the W image of a layer (K x N), its
// rows (n, natural) read transposed at the rows that match the chained dZ fragments (C order of the layer
// above). dz[tb][kt'] are the previous gradient tiles (N/16 of them); out[tb][kt] the K/16 output tiles.
template <int K, int N, int TBN>
__device__ __forceinline__ void bwd_dA(const uint16_t* W, const v4bf (&dz)[TBN][N / 16], v4f (&out)[TBN][K / 16], int r,
                                       int h) {
  constexpr int NS = N / 32, KT = K / 16;
  const int q = r >> 2, p = r & 3;
  const int rb = wperm(16 * (h & 1) + 4 * (h >> 1) + q);  // + 32 s (+8): bits 3, 5, 6 untouched by wperm
  v8bf b[TBN][NS];
#pragma unroll
  for (int tb = 0; tb < TBN; ++tb)
#pragma unroll
    for (int s = 0; s < NS; ++s) b[tb][s] = cat_bf(dz[tb][2 * s], dz[tb][2 * s + 1]);
#pragma unroll
  for (int kt = 0; kt < KT; ++kt)
#pragma unroll
    for (int tb = 0; tb < TBN; ++tb) out[tb][kt] = kZero4;
#pragma unroll
  for (int kt = 0; kt < KT; ++kt) {
    v8bf a[NS];
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      const uint16_t* pa = W + (32 * s + rb) * (K + WPAD) + 16 * kt + 4 * p;
      a[s] = cat8(tr_read(pa), tr_read(pa + 8 * (K + WPAD)));
    }
#pragma unroll
    for (int s = 0; s < NS; ++s)
#pragma unroll
      for (int tb = 0; tb < TBN; ++tb) out[tb][kt] = mfma(a[s], b[tb][s], out[tb][kt]);
  }
}

// ReLU mask of the layer input from the staged activation (C order) and bf16 pack of the gradient
template <int K, int TBN>
__device__ __forceinline__ void mask_grad(const v4f (&g)[TBN][K / 16], const uint16_t* SA, int w, int r, int h,
                                          v4bf (&dz)[TBN][K / 16]) {
  const int rp = sperm16(r);
#pragma unroll
  for (int tb = 0; tb < TBN; ++tb)
#pragma unroll
    for (int kt = 0; kt < K / 16; ++kt) {
      const int row = 16 * TBN * w + 16 * tb + rp;
      const uint2 m = *(const uint2*)(SA + row * (K + PAD) + 16 * kt + 4 * h);
      const unsigned int u[2] = {mask_pk(cvt_pk(g[tb][kt][0], g[tb][kt][1]), m.x),
                                 mask_pk(cvt_pk(g[tb][kt][2], g[tb][kt][3]), m.y)};
      dz[tb][kt] = __builtin_bit_cast(v4bf, u);
    }
}

// stage dZ (gradient tiles, C order of the layer above: tiles 2m, 2m+1 = the 16-byte fragment of C positions
// 32 m + 8 h, as bwd_dA consumes them) and the layer's input activation fragments (C order) for the dW product
// of a layer with dims K x N; rows permuted by sperm16 inside each 16-row block
template <int K, int N, int TBN>
__device__ __forceinline__ void stage(uint16_t* S, const v4bf (&dz)[TBN][N / 16], const v8bf (&a)[TBN][K / 32], int w,
                                      int r, int h) {
  uint16_t* SZ = S;
  uint16_t* SA = S + T * (N + PAD);
  const int rp = sperm16(r);
#pragma unroll
  for (int tb = 0; tb < TBN; ++tb) {
    const int row = 16 * TBN * w + 16 * tb + rp;
#pragma unroll
    for (int m = 0; m < N / 32; ++m) *(v8bf*)(SZ + row * (N + PAD) + 32 * m + 8 * h) = cat_bf(dz[tb][2 * m], dz[tb][2 * m + 1]);
#pragma unroll
    for (int s = 0; s < K / 32; ++s) *(v8bf*)(SA + row * (K + PAD) + 32 * s + 8 * h) = a[tb][s];
  }
}

// ---- split staging (T = 256, layers 1-3): pass `tb` stages column block tb of every wave (rows 16 w + sperm16(r) of
// a T / 2-row image), the activation gradient waits as unmasked bf16 tiles until its pass's A rows give the mask
template <int K, int N, int TBN>
__device__ __forceinline__ void stage_half(uint16_t* S, const v4bf (&dz)[TBN][N / 16], const v8bf (&a)[TBN][K / 32],
                                           int w, int r, int h, int tb) {
  constexpr int R = T / 2;
  uint16_t* SZ = S;
  uint16_t* SA = S + R * (N + PAD);
  const int row = 16 * w + sperm16(r);
#pragma unroll
  for (int t = 0; t < TBN; ++t) {
    if (t != tb) continue;
#pragma unroll
    for (int m = 0; m < N / 32; ++m) *(v8bf*)(SZ + row * (N + PAD) + 32 * m + 8 * h) = cat_bf(dz[t][2 * m], dz[t][2 * m + 1]);
#pragma unroll
    for (int s2 = 0; s2 < K / 32; ++s2) *(v8bf*)(SA + row * (K + PAD) + 32 * s2 + 8 * h) = a[t][s2];
  }
}
template <int K, int TBN>
__device__ __forceinline__ void to_bf_tiles(const v4f (&g)[TBN][K / 16], unsigned int (&gb)[TBN][K / 16][2]) {
#pragma unroll
  for (int tb = 0; tb < TBN; ++tb)
#pragma unroll
    for (int kt = 0; kt < K / 16; ++kt) {
      gb[tb][kt][0] = cvt_pk(g[tb][kt][0], g[tb][kt][1]);
      gb[tb][kt][1] = cvt_pk(g[tb][kt][2], g[tb][kt][3]);
    }
}
template <int K, int TBN>
__device__ __forceinline__ void mask_half(const unsigned int (&gb)[TBN][K / 16][2], const uint16_t* SA, int w, int r,
                                          int h, v4bf (&dz)[TBN][K / 16], int tb) {
  const int row = 16 * w + sperm16(r);
#pragma unroll
  for (int t = 0; t < TBN; ++t) {
    if (t != tb) continue;
#pragma unroll
    for (int kt = 0; kt < K / 16; ++kt) {
      const uint2 m = *(const uint2*)(SA + row * (K + PAD) + 16 * kt + 4 * h);
      const unsigned int u[2] = {mask_pk(gb[t][kt][0], m.x), mask_pk(gb[t][kt][1], m.y)};
      dz[t][kt] = __builtin_bit_cast(v4bf, u);
    }
  }
}

// ---- weight gradient: the wave's NTW x KTW tiles (nt = nt0 + i ntS, kt = kt0 + j ktS) accumulate
// dW^T[n][k] += sum_t dZ[t][n] A[t][k] over the T staged rows (4 k-steps of 32 examples)
template <int K, int N, int NTW, int KTW, int ROWS = T>
__device__ __forceinline__ void dw_phase(v4f (&acc)[NTW * KTW], const uint16_t* S, int nt0, int ntS, int kt0, int ktS,
                                         int r, int h) {
  const uint16_t* SZ = S;
  const uint16_t* SA = S + ROWS * (N + PAD);
  const int q = r >> 2, p = r & 3;
  // example rows 32 ts + 8 h + q (first read) and + 4 (second): inside the 16-row block 16 (h >> 1) they are
  // rows 8 (h & 1) + q and + 4, physical sperm16() = 8 (h & 1) + 2 q and + 1
  const int rl = 16 * (h >> 1) + 8 * (h & 1) + 2 * q;
#pragma unroll
  for (int ts = 0; ts < ROWS / 32; ++ts) {
    v8bf fa[NTW], fb[KTW];
#pragma unroll
    for (int i = 0; i < NTW; ++i) {
      const uint16_t* pa = SZ + (32 * ts + rl) * (N + PAD) + 16 * (nt0 + i * ntS) + 4 * p;
      fa[i] = cat8(tr_read(pa), tr_read(pa + (N + PAD)));
    }
#pragma unroll
    for (int j = 0; j < KTW; ++j) {
      const uint16_t* pb = SA + (32 * ts + rl) * (K + PAD) + 16 * (kt0 + j * ktS) + 4 * p;
      fb[j] = cat8(tr_read(pb), tr_read(pb + (K + PAD)));
    }
#pragma unroll
    for (int i = 0; i < NTW; ++i)
#pragma unroll
      for (int j = 0; j < KTW; ++j) acc[i * KTW + j] = mfma(fa[i], fb[j], acc[i * KTW + j]);
  }
}

template <int K, int NTW, int KTW>
__device__ __forceinline__ void load_ct(int (&ct)[NTW * KTW], int tbase, int nt0, int ntS, int kt0, int ktS,
                                        const int* __restrict__ tmap) {
#pragma unroll
  for (int i = 0; i < NTW; ++i)
#pragma unroll
    for (int j = 0; j < KTW; ++j) ct[i * KTW + j] = tmap[tbase + (nt0 + i * ntS) * (K / 16) + kt0 + j * ktS];
}


// WDC_NT_SLAB (diagnostic builds): slab stores with the non-temporal hint, so the 24 MB of per-step partials
// stream out of L2 during the kernel instead of sitting dirty until the end-of-kernel write-back
#ifndef WDC_NT_SLAB
#define WDC_NT_SLAB 0
#endif
template <class V>
__device__ __forceinline__ void slab_store(V* p, V v) {
  if constexpr (WDC_NT_SLAB) __builtin_nontemporal_store(v, p);
  else *p = v;
}

template <int NT>
__device__ __forceinline__ void store_tiles(float* slab, const v4f (&acc)[NT], const int (&ct)[NT], int lane) {
#pragma unroll
  for (int i = 0; i < NT; ++i) {
    if (ct[i] < 0) continue;
    float* dst = slab + (size_t)ct[i] * 256 + lane;
#pragma unroll
    for (int e = 0; e < 4; ++e) slab_store(dst + e * 64, acc[i][e]);
  }
}

// ---- in-kernel step tail (TAIL = true): slab reduction + optimizer inside the training kernel itself.
// With one workgroup per CU and grid <= #CUs every workgroup of the launch is resident, so the launch can
// synchronise grid-wide. After its last iteration every workgroup has written its slab row (into the L2 of the
// XCD it runs on); then
//   barrier 1 -> level 1: the workgroups of each XCD split the columns and sum the rows written on THAT XCD
//                (ascending row order, L2 hits), storing the per-XCD partials write-through (system scope);
//   barrier 2 -> level 2: workgroup b sums the per-XCD partials of its ~stride/G columns (XCDs in the order of
//                their first row: the same association for any rotation of the round-robin dispatch, so the
//                step is run-to-run deterministic) and applies the optimizer (wd_opt.h sc_update) in place.
// This replaces the two tail kernels (csrc/wide_deep.hip wd_reduce_xcd + wd_xcd_opt_sc, 11.8 us per step at
// B=65536, profiles/archive/bench_r2_final_kernels.md) and their launch ramps; the slab never has to leave its XCD.
// Barrier: a monotonic 64-bit arrival counter (no reset, no generation flag): the workgroup whose arrival
// returned `old` waits until the counter reaches (old / G + 1) G. The wait is bounded by wall-clock time: on a
// timeout (a workgroup never arrived: not co-resident) it sets the sticky `err` flag, and the tail then skips
// the update and the step-counter advance (the host raises at its next check).
struct TailArgs {
  float* xpart;                  // [XMAX][stride] per-XCD partial column sums
  unsigned long long* bar;       // arrival counter (monotonic)
  int* err;                      // sticky failure flag
  const int* wsc;                // slab column -> -1 padding / -2 wide / >= 0 bf16 image offset
  float* param;
  float* s0;
  float* s1;
  uint16_t* wt_out;              // the bf16 weight image (the kernel's own staging source)
  long long* step_slots;         // STEP_SLOTS per-workgroup optimizer step slots (slot 0 = the data offset step)
  OptHyper hd, hw;
  long long* dbg;                // optional [grid][8] real-time stamps (tools/tail_stamps.py); null = off
  int nsteps;                    // PERSIST: training steps per launch
  int helpers;                   // > 0: the one-row tail (help_update) with this many optimizer workgroups
};
#define TSTAMP(i)                                                                      \
  do {                                                                                 \
    if (ta.dbg != nullptr && threadIdx.x == 0) ta.dbg[blockIdx.x * 8 + (i)] = wall_clock64(); \
  } while (0)
constexpr int XMAXT = 16;  // XCC_ID range
constexpr long long TAIL_TIMEOUT_TICKS = 200ll * 1000 * 1000;  // 2 s at the 100 MHz real-time clock

__device__ __forceinline__ void st_sys4(float* p, float4 v) {
  __hip_atomic_store((unsigned int*)p + 0, __float_as_uint(v.x), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store((unsigned int*)p + 1, __float_as_uint(v.y), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store((unsigned int*)p + 2, __float_as_uint(v.z), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
  __hip_atomic_store((unsigned int*)p + 3, __float_as_uint(v.w), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ float ld_sys1(const float* p) {
  return __uint_as_float(__hip_atomic_load((const unsigned int*)p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM));
}

// every thread's outstanding stores acknowledged, then one arrival per workgroup; false on timeout / earlier error
__device__ __forceinline__ bool grid_sync(unsigned long long* bar, int* err, int G, int* s_flag) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    int ok = __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0;
    const unsigned long long old = __hip_atomic_fetch_add(bar, 1ull, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const unsigned long long target = (old / (unsigned long long)G + 1ull) * (unsigned long long)G;
    const long long t0 = wall_clock64();
    while (ok && __hip_atomic_load(bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < target) {
      __builtin_amdgcn_s_sleep(1);
      if (wall_clock64() - t0 > TAIL_TIMEOUT_TICKS) {
        __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ok = 0;
      }
    }
    *s_flag = ok;
  }
  __syncthreads();
  return *s_flag != 0;
}

// ---- one-row tail (TAIL with ta.helpers = H > 0), for batches ONE workgroup trains (the reference batch of 40):
// the launch is 1 + H workgroups. Workgroup 0 runs the step and publishes its gradient row (ta.bar = the step);
// workgroups 1..H are the optimizer -- one thread per slab column and step slot h - 1, exactly wd_opt1_sc's
// workgroups (csrc/wide_deep.hip), so the update is bit-identical -- which load their columns' master weights and
// optimizer state at launch, under workgroup 0's step, then wait for the row. This replaces the separate optimizer
// launch: its ramp, kernel-argument and state loads no longer follow the step. The wait is bounded by wall-clock
// time (a timeout sets ta.err and skips the update; the host raises). ta.bar holds the last published step and is
// reset by the host whenever the step counters are rewritten (resume), so a stale value can never match.
template <int NTHR>
__device__ void help_update(const TailArgs& ta, const float* __restrict__ slab, int stride, int* s_flag) {
  const int hb = (int)blockIdx.x - 1;
  const int gi = hb * NTHR + (int)threadIdx.x;
  const ScState st = sc_load(gi, stride, ta.wsc, ta.param, ta.s0, ta.s1);
  const long long step = ta.step_slots[hb] + 1;
  if (threadIdx.x == 0) {
    int ok = 1;
    const long long t0 = wall_clock64();
    // relaxed polls: an acquire load per poll would invalidate this XCD's L2 every time (workgroup 0 may share it);
    // the row itself is read past the caches below
    while ((long long)__hip_atomic_load(ta.bar, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != step) {
      __builtin_amdgcn_s_sleep(1);
      if (wall_clock64() - t0 > TAIL_TIMEOUT_TICKS) {
        __hip_atomic_store(ta.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ok = 0;
        break;
      }
    }
    *s_flag = ok;
  }
  __syncthreads();
  if (!*s_flag) return;
  if (gi < stride) {
    const float g = ld_sys1(slab + gi);  // written by workgroup 0, possibly on another XCD: read past the caches
    sc_update(gi, st, g, ta.hd, ta.hw, step, ta.param, ta.s0, ta.s1, ta.wt_out);
  }
  if (threadIdx.x == 0) ta.step_slots[hb] = step;
}

// ---- persistent small-batch training (PERSIST = true): ONE workgroup runs `nsteps` whole training steps of a
// batch <= T in one launch. Its dW tiles are the whole gradient (no slab, no reduction): right after a layer's dW
// phase every lane applies the optimizer to the columns its accumulators hold (column ct * 256 + 64 e + lane of
// the compact layout) and writes the new bf16 weight straight into the LDS weight image -- that layer's weights are
// not read again in the step (its activation gradient ran before the dW barrier). The wide weights stay in LDS as
// fp32 and are updated from the LDS histogram at the end of the step. The weight image is staged once per launch;
// the fp32 master weights / optimizer state stay in global memory (L2-resident, each column read and written by
// the one lane that owns it). Bit-identical to the slab path with grid 1 (same fp32 gradient, same update).
// Measured on MI355X at B=40: 25.6 us/step against 14.8 us for the grid-1 fused kernel + 370-workgroup optimizer
// launch -- the ~750 KB of per-step optimizer traffic (slab, master weights, accumulators, column map) through one
// CU's memory path outweighs the staging and launch it saves -- so the trainer keeps it opt-in.
constexpr int LDS_BYTES_P = LDS_BYTES + WIDE_PAD * 4;
static_assert(LDS_BYTES_P <= 163840, "LDS budget (persistent)");

// The optimizer over the lane's own dW columns (column ct[i] * 256 + 64 e + lane of the compact layout, which
// this lane stored to the slab row earlier in the step -- same lane, same addresses, so program order suffices):
// the 4-column tiles are processed GS at a time with their loads batched. Run at the end of the step, where no
// accumulators are live (applying each layer's update right after its dW phase instead spills the kernel).
template <int NT>
__device__ __forceinline__ void opt_tiles(const int (&ct)[NT], int lane, const TailArgs& ta, long long step,
                                          bool last_step, uint16_t* img, const float* slab_row) {
  constexpr int GS = 3;  // 4+ spills the persistent kernel (tiles of 4 columns x 5 loads each)
  const bool s1_live = ta.hd.kind >= 2;
#pragma unroll
  for (int i0 = 0; i0 < NT; i0 += GS) {
    int wo[GS][4];
    float p[GS][4], a0[GS][4], a1[GS][4], g[GS][4];
#pragma unroll
    for (int j = 0; j < GS; ++j) {
      const int i = i0 + j;
      if (i >= NT || ct[i] < 0) continue;
      const unsigned g0 = (unsigned)ct[i] * 256u + (unsigned)lane;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const unsigned gi = g0 + 64u * e;
        wo[j][e] = ta.wsc[gi];
        p[j][e] = ta.param[gi];
        a0[j][e] = ta.s0[gi];
        a1[j][e] = s1_live ? ta.s1[gi] : 0.f;
        g[j][e] = slab_row[gi];
      }
    }
#pragma unroll
    for (int j = 0; j < GS; ++j) {
      const int i = i0 + j;
      if (i >= NT || ct[i] < 0) continue;
      const unsigned g0 = (unsigned)ct[i] * 256u + (unsigned)lane;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        if (wo[j][e] < 0) continue;  // padding column
        const unsigned gi = g0 + 64u * e;
        const float w = opt_update(ta.hd, p[j][e], g[j][e], a0[j][e], a1[j][e], step);
        ta.param[gi] = w;
        ta.s0[gi] = a0[j][e];
        if (s1_live) ta.s1[gi] = a1[j][e];
        const uint16_t wb = __builtin_bit_cast(uint16_t, (bf16)w);
        img[wo[j][e]] = wb;
        if (last_step) ta.wt_out[wo[j][e]] = wb;
      }
    }
  }
}

template <bool TRAIN, int TBN, bool TAIL, bool PERSIST = false>
__global__ __launch_bounds__(64 * (T / (16 * TBN)), 1) void wdc_fused(const uint4* __restrict__ data, long long n_data, long long batch,
                                                     long long start_fixed, const long long* __restrict__ step_ctr,
                                                     const uint4* __restrict__ wimg, const float* __restrict__ wide,
                                                     float* __restrict__ slab, float* __restrict__ slab_loss,
                                                     float* __restrict__ logits_out, float grad_scale,
                                                     const int* __restrict__ tmap, int stride,
                                                     int* __restrict__ xcd_of, TailArgs ta, MifxFeed feed) {
  extern __shared__ __attribute__((aligned(16))) uint16_t lds[];
  float* wgrad = (float*)(lds + LSEND);
  float* red = wgrad + WIDE_PAD;
  int* wgi = (int*)wgrad;
  constexpr int NWAVE = T / (16 * TBN), NTHR = 64 * NWAVE, EPW = 16 * TBN;  // waves, threads, examples per wave
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, r = lane & 15, h = lane >> 4;
  bool stamp_on = true;
  (void)stamp_on;
  STAMP(0);
  BSTAMP(0);
  if constexpr (TRAIN && TAIL) {
    if (ta.helpers > 0 && blockIdx.x > 0) {  // one-row tail: an optimizer workgroup
      help_update<NTHR>(ta, slab, stride, (int*)lds);
      return;
    }
  }
  // the XCD this workgroup's slab row is written from (its L2 holds the row for the XCD-local reduction,
  // csrc/wide_deep.hip wd_reduce_xcd)
  if constexpr (TAIL) TSTAMP(0);
  if (TRAIN && xcd_of != nullptr && tid == 0) {
    if (TAIL)  // read by workgroups on every XCD after the first barrier: write-through
      __hip_atomic_store(xcd_of + blockIdx.x, mifx_xcc_id(), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    else
      xcd_of[blockIdx.x] = mifx_xcc_id();
  }

#ifndef WDC_REG_STAGE
#define WDC_REG_STAGE 0
#endif
  // WDC_REG_STAGE (diagnostic builds): stage the weight image through registers (global_load_dwordx4 +
  // ds_write_b128) instead of LDS-DMA
  constexpr bool REG_STAGE = WDC_REG_STAGE && !PERSIST;
  constexpr int NCH_STAGE = LWEND / 8, PER_STAGE = (NCH_STAGE + NTHR - 1) / NTHR;
  uint4 wst[REG_STAGE ? PER_STAGE : 1];
  (void)wst;
  {  // stage the bf16 weight image (already in LDS layout) with direct-to-LDS loads: no VGPR round trip, no
     // ds_write transfer cycles. Wave w's lanes fill 16-byte chunks i * NTHR + 64 w + lane; the last wave's
     // lanes past the image end re-read its last chunk and land in the staging area, written before any read.
#ifndef WDC_DIAG_NOIMG
#define WDC_DIAG_NOIMG 0
#endif
    // WDC_DIAG_NOIMG (stamp builds only, wrong results): skip the image load, so the prologue stamp times the
    // step-counter -> feed -> record chain alone
    if constexpr (!REG_STAGE && !WDC_DIAG_NOIMG) {
#pragma unroll
      for (int i = 0; i < PER_STAGE; ++i) {
        const int c0 = i * NTHR + 64 * w;  // wave-uniform
        if (c0 < NCH_STAGE)
          __builtin_amdgcn_global_load_lds((const void*)(wimg + min(c0 + lane, NCH_STAGE - 1)),
                                           (__attribute__((address_space(3))) void*)(lds + c0 * 8), 16, 0, 0);
      }
    } else if constexpr (REG_STAGE) {  // register staging: loads now, ds_write_b128 after the first record fetch
#pragma unroll
      for (int i = 0; i < PER_STAGE; ++i) wst[i] = wimg[min(i * NTHR + tid, NCH_STAGE - 1)];
    }
    // (one launch = one step: the wait for the image and the block barrier come after the first iteration's
    // record fetch below, so the step-counter -> records latency chain runs under the staging instead of after it)
    if constexpr (PERSIST) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  }
  float* wlds = red + 64;  // PERSIST: the fp32 wide weights [WIDE_PAD], resident for the launch
  if (TRAIN)
    for (int c = tid; c < WIDE_PAD; c += NTHR) wgrad[c] = 0.f;
  if constexpr (PERSIST) {
    for (int c = tid; c < WIDE_PAD; c += NTHR) wlds[c] = wide[c];
    __syncthreads();
  }

#ifndef WDC_DIAG_NOSTEP
#define WDC_DIAG_NOSTEP 0
#endif
  // WDC_DIAG_NOSTEP (stamp builds only, wrong record order): step 0's records, no step-counter load ahead of them
  const long long step0 = (step_ctr && !WDC_DIAG_NOSTEP) ? step_ctr[0] : 0;
  constexpr bool kPersist = PERSIST;
  const int nsteps = kPersist ? ta.nsteps : 1;
  for (int ps = 0; ps < nsteps; ++ps) {
  // record feed (csrc/feed.h): the step's place in the (optionally shuffled) global record stream; a fixed start
  // (eval / predict) reads records start_fixed.. in stored order
  MifxFeed fd = feed;
  MifxFeedStep fs;
  if (step_ctr) {
    fs = mifx_feed_step(fd, step0 + ps, n_data);
  } else {
    fd.key = 0;
    fs.e0 = 0;
    fs.i0 = start_fixed;
    fs.h = 1;
  }
  const int niters = (int)((batch + T - 1) / T);
  const int my_iters = (niters - (int)blockIdx.x + (int)gridDim.x - 1) / (int)gridDim.x;
  const float qbound = fmaxf(fabsf(grad_scale) * (float)(max(my_iters, 1) * T), 1e-30f);
  const float qscale = exp2f(fminf(floorf(log2f(1073741824.f / qbound)), 100.f));
  const float qinv = 1.f / qscale;
  const float qmax = 1073741824.f / (float)(max(my_iters, 1) * T);

  // dW tile ownership (wave w); 4 waves: L1 nt {2w, 2w+1} x kt 0 (kt 1 holds only padding columns);
  // L2 nt 0..5 x kt {2w, 2w+1}; L3 nt w x kt 0..5; L4 nt w x kt 0..3; L5 nt 0 x kt w.
  // 8 waves: L1 nt w x kt 0; L2 nt 3(w%2)..+2 x kt 2(w/2)..+1 (3 x 2 blocks: 5 operand fragments per k-step
  // instead of 7 for 6 x 1); L3 nt w%4 x kt 3(w/4)..+2; L4 nt w%4 x kt 2(w/4)..+1; L5 nt 0 x kt w (waves 0..3)
  constexpr bool W4 = NWAVE == 4;  // 4-wave shapes (TBN 2 at T 128, TBN 1 at T 64) share one tile ownership
  static_assert(NWAVE == 4 || NWAVE == 8, "waves");
  constexpr int O1N = W4 ? 2 : 1, O2N = W4 ? 6 : 3, O2K = 2, O3K = W4 ? 6 : 3, O4K = W4 ? 4 : 2;
  const int n1 = W4 ? 2 * w : w, n2 = W4 ? 0 : 3 * (w & 1), k2 = W4 ? 2 * w : 2 * (w >> 1),
            n3 = w & 3, k3 = W4 ? 0 : 3 * (w >> 2), n4 = w & 3, k4 = W4 ? 0 : 2 * (w >> 2);
  const bool l5 = w < 4;
  v4f acc1[O1N], acc2[O2N * O2K], acc3[O3K], acc4[O4K], acc5[1];
  int ct1[O1N], ct2[O2N * O2K], ct3[O3K], ct4[O4K], ct5[1];
  if (TRAIN) {
#pragma unroll
    for (int i = 0; i < O1N; ++i) acc1[i] = kZero4;
#pragma unroll
    for (int i = 0; i < O2N * O2K; ++i) acc2[i] = kZero4;
#pragma unroll
    for (int i = 0; i < O3K; ++i) acc3[i] = kZero4;
#pragma unroll
    for (int i = 0; i < O4K; ++i) acc4[i] = kZero4;
    acc5[0] = kZero4;
    load_ct<K1, O1N, 1>(ct1, TB1, n1, 1, 0, 0, tmap);
    load_ct<K2, O2N, O2K>(ct2, TB2, n2, 1, k2, 1, tmap);
    load_ct<K3, 1, O3K>(ct3, TB3, n3, 0, k3, 1, tmap);
    load_ct<K4, 1, O4K>(ct4, TB4, n4, 0, k4, 1, tmap);
    load_ct<K5, 1, 1>(ct5, TB5, 0, 0, w & 3, 0, tmap);
    if (!l5) ct5[0] = -1;
  }
  float loss_sum = 0.f, dl_sum = 0.f;
  // the column block whose wide part / loss this lane computes (lanes h < TBN own one each)
  const int mtb = TBN == 2 ? (h & 1) : 0;

  auto fetch = [&](int it, uint4 (&u)[TBN][2]) {
#pragma unroll
    for (int tb = 0; tb < TBN; ++tb) {
      const long long row = min((long long)it * T + EPW * w + 16 * tb + r, batch - 1);
      const long long di = mifx_feed_record(fd, fs, row, n_data);  // host guarantees batch <= n_data
      u[tb][0] = data[2 * di];
      u[tb][1] = data[2 * di + 1];
    }
  };
  uint4 nu[TBN][2];
  fetch(blockIdx.x, nu);
  if constexpr (REG_STAGE) {
#pragma unroll
    for (int i = 0; i < PER_STAGE; ++i)
      if (i * NTHR + tid < NCH_STAGE) *(uint4*)(lds + (i * NTHR + tid) * 8) = wst[i];
  }
  if constexpr (!PERSIST) {  // weight image (LDS-DMA) and the first records landed; wgrad zeroed
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }

  STAMP(1);
  BSTAMP(1);
  // PERSIST (grid 1, batch <= T): exactly one iteration, known at compile time, so the dW accumulators die at
  // their layer's emission instead of living across a loop back-edge
  // ONE_ITER (T = 256: the host launches grid >= ceil(batch / T)): every workgroup runs exactly its own iteration,
  // also known at compile time -- the dW accumulators live only through their layer's phase, and no prefetch
  constexpr bool SINGLE = PERSIST || ONE_ITER;
  const int it_end = SINGLE ? 1 : niters, it_inc = SINGLE ? 1 : (int)gridDim.x;
  for (int itv = SINGLE ? 0 : (int)blockIdx.x; itv < it_end; itv += it_inc) {
    const int it = ONE_ITER ? (int)blockIdx.x : itv;
#ifdef WDC_STAMPS
    stamp_on = niters > (int)gridDim.x ? it == (int)(blockIdx.x + gridDim.x) : it == (int)blockIdx.x;
#endif
    STAMP(2);
    const bool last = SINGLE || it + (int)gridDim.x >= niters;  // this workgroup's final iteration: dW final
    float* my_slab = TRAIN ? slab + (size_t)blockIdx.x * stride : nullptr;
    const long long pstep = step0 + ps + 1;  // PERSIST: the optimizer step (Adam bias correction)
    const bool plast = ps + 1 == nsteps;
#define WDC_EMIT(NT, ACC, CT)                          \
  do {                                                 \
    if (last) store_tiles<NT>(my_slab, ACC, CT, lane); \
  } while (0)
    uint4 u[TBN][2];
#pragma unroll
    for (int tb = 0; tb < TBN; ++tb) {
      u[tb][0] = nu[tb][0];
      u[tb][1] = nu[tb][1];
    }
    if constexpr (!SINGLE) fetch(it + gridDim.x, nu);  // next iteration's records

    // wide gather for the lane's column block (issued before the forward: its latency hides under MFMAs)
    const uint4 m0 = mtb ? u[TBN - 1][0] : u[0][0], m1 = mtb ? u[TBN - 1][1] : u[0][1];
    const uint32_t idw[5] = {m0.w, m1.x, m1.y, m1.z, m1.w};
    int ids[9];
    float wv[9];
#pragma unroll
    for (int f = 0; f < 9; ++f) {
      int id = (f & 1) ? (idw[f >> 1] >> 16) : (idw[f >> 1] & 0xffff);
      id = id < kWideNb[f] ? id : 0;
      ids[f] = kWideOff[f] + id;
      wv[f] = PERSIST ? wlds[ids[f]] : wide[ids[f]];
    }
    const float wbias = PERSIST ? wlds[WIDE_BIAS] : wide[WIDE_BIAS];

    // ---- forward, in registers
    v8bf a0[TBN][1];
#pragma unroll
    for (int tb = 0; tb < TBN; ++tb) {
      const v8bf x = {(bf16)__uint_as_float(u[tb][0].x), (bf16)__uint_as_float(u[tb][0].y),
                      (bf16)__uint_as_float(u[tb][0].z), (bf16)1.0f, (bf16)0.f, (bf16)0.f, (bf16)0.f, (bf16)0.f};
      a0[tb][0] = h == 0 ? x : (v8bf){};
    }
    v8bf a1[TBN][N1 / 32], a2[TBN][N2 / 32], a3[TBN][N3 / 32], a4[TBN][N4 / 32];
    v4f z5[TBN][1];
    {
      v4f acc[TBN][N1 / 16];
      fwd<K1, N1, TBN>(lds + LW1, a0, acc, r, h);
      relu_pack<N1, TBN>(acc, a1);
    }
    {
      v4f acc[TBN][N2 / 16];
      fwd<K2, N2, TBN>(lds + LW2, a1, acc, r, h);
      relu_pack<N2, TBN>(acc, a2);
    }
    {
      v4f acc[TBN][N3 / 16];
      fwd<K3, N3, TBN>(lds + LW3, a2, acc, r, h);
      relu_pack<N3, TBN>(acc, a3);
    }
    {
      v4f acc[TBN][N4 / 16];
      fwd<K4, N4, TBN>(lds + LW4, a3, acc, r, h);
      relu_pack<N4, TBN>(acc, a4);
    }
    fwd<K5, N5, TBN>(lds + LW5, a4, z5, r, h);

    STAMP(3);
    // ---- logit = deep (row 0 of the layer-5 tile: lane (r, h = 0)) + wide; loss and dlogit
    const float zd0 = __shfl(z5[0][0][0], r), zd1 = __shfl(z5[TBN - 1][0][0], r);
    float wl = wbias;
#pragma unroll
    for (int f = 0; f < 9; ++f) wl += wv[f];
    const float x = (mtb ? zd1 : zd0) + wl;
    const long long grow = (long long)it * T + EPW * w + 16 * mtb + r;
    const bool own = h < TBN && grow < batch;
    const float y = (float)(idw[4] >> 16);
    const float lossv = fmaxf(x, 0.f) - x * y + log1pf(__expf(-fabsf(x)));
    if (!TRAIN) {
      if (own) {
        logits_out[grow] = x;
        loss_sum += lossv;
      }
      continue;
    }
    const float dl = own ? (1.f / (1.f + __expf(-x)) - y) * grad_scale : 0.f;
    if (own) {
      loss_sum += lossv;
      dl_sum += dl;
    }
    // dlogit of the lane's example in both column blocks, rounded to bf16 like the staged dZ5 the dW5 MFMA reads
    float dlb[TBN];
#pragma unroll
    for (int tb = 0; tb < TBN; ++tb) dlb[tb] = (float)(bf16)__shfl(dl, 16 * tb + r);

    // ---- layer 5: stage (dZ5, A4); dW5; dA4 = w5 (x) dl on the VALU, masked
    STAMP(4);
    uint16_t* S = lds + LS;
    block_sync_lds();  // previous iteration's dW1 reads of the staging area are done
    STAMP(5);
    if (own) {
      const int q = __float2int_rn(fminf(fmaxf(dl * qscale, -qmax), qmax));
#pragma unroll
      for (int f = 0; f < 9; ++f) atomicAdd(&wgi[ids[f]], q);
    }
    {
      v4bf d5[TBN][1];
#pragma unroll
      for (int tb = 0; tb < TBN; ++tb) {
        v4bf o = {(bf16)0.f, (bf16)0.f, (bf16)0.f, (bf16)0.f};
        if (h == 0) o[0] = (bf16)dlb[tb];
        d5[tb][0] = o;
      }
      // dZ5 has one natural-order tile (N5 = 16): stage it directly (row t: [dl, 0 ... 0])
#pragma unroll
      for (int tb = 0; tb < TBN; ++tb) {
        const int row = EPW * w + 16 * tb + sperm16(r);
        *(v4bf*)(S + row * (N5 + PAD) + 4 * h) = d5[tb][0];
#pragma unroll
        for (int s = 0; s < K5 / 32; ++s)
          *(v8bf*)(S + T * (N5 + PAD) + row * (K5 + PAD) + 32 * s + 8 * h) = a4[tb][s];
      }
    }
    v4bf dz4[TBN][K5 / 16];
    {  // dA4 (VALU) + mask: own rows only, before the barrier (see layer 4)
      v4f g[TBN][K5 / 16];
#pragma unroll
      for (int kt = 0; kt < K5 / 16; ++kt) {
        const uint2 wv2 = *(const uint2*)(lds + LW5 + 16 * kt + 4 * h);  // W5 row 0 (the logit row; X(0) = 0)
        const float w5[4] = {__uint_as_float(wv2.x << 16), __uint_as_float(wv2.x & 0xffff0000u),
                             __uint_as_float(wv2.y << 16), __uint_as_float(wv2.y & 0xffff0000u)};
#pragma unroll
        for (int tb = 0; tb < TBN; ++tb)
#pragma unroll
          for (int e = 0; e < 4; ++e) g[tb][kt][e] = w5[e] * dlb[tb];
      }
      mask_grad<K5, TBN>(g, S + T * (N5 + PAD), w, r, h, dz4);
    }
    block_sync_lds();
    STAMP(6);
    if (l5) dw_phase<K5, N5, 1, 1>(acc5, S, 0, 0, w & 3, 0, r, h);
    WDC_EMIT(1, acc5, ct5);
    block_sync_lds();

    // ---- layer 4
    STAMP(7);
    stage<K4, N4, TBN>(S, dz4, a3, w, r, h);
    // the activation gradient needs only the weights, this wave's dZ and its own staged rows (the relu mask):
    // issued before the barrier so its MFMAs and weight reads overlap the other waves' staging
    v4bf dz3[TBN][K4 / 16];
    {
      v4f g[TBN][K4 / 16];
      bwd_dA<K4, N4, TBN>(lds + LW4, dz4, g, r, h);
      mask_grad<K4, TBN>(g, S + T * (N4 + PAD), w, r, h, dz3);
    }
    block_sync_lds();
    STAMP(8);
    dw_phase<K4, N4, 1, O4K>(acc4, S, n4, 0, k4, 1, r, h);
    WDC_EMIT(O4K, acc4, ct4);
    block_sync_lds();

    // ---- layer 3
    STAMP(9);
    v4bf dz2[TBN][K3 / 16];
    if constexpr (split_stage(K3, N3)) {  // two passes of T / 2 staged rows (column block 0, then 1)
      unsigned int gb[TBN][K3 / 16][2];
      {
        stage_half<K3, N3, TBN>(S, dz3, a2, w, r, h, 0);
        v4f g[TBN][K3 / 16];
        bwd_dA<K3, N3, TBN>(lds + LW3, dz3, g, r, h);
        to_bf_tiles<K3, TBN>(g, gb);
      }
      mask_half<K3, TBN>(gb, S + (T / 2) * (N3 + PAD), w, r, h, dz2, 0);
      block_sync_lds();
      dw_phase<K3, N3, 1, O3K, T / 2>(acc3, S, n3, 0, k3, 1, r, h);
      block_sync_lds();
      stage_half<K3, N3, TBN>(S, dz3, a2, w, r, h, 1);
      mask_half<K3, TBN>(gb, S + (T / 2) * (N3 + PAD), w, r, h, dz2, 1);
      block_sync_lds();
      STAMP(10);
      dw_phase<K3, N3, 1, O3K, T / 2>(acc3, S, n3, 0, k3, 1, r, h);
    } else {
      stage<K3, N3, TBN>(S, dz3, a2, w, r, h);
      // the activation gradient needs only the weights, this wave's dZ and its own staged rows (the relu mask):
      // issued before the barrier so its MFMAs and weight reads overlap the other waves' staging
      {
        v4f g[TBN][K3 / 16];
        bwd_dA<K3, N3, TBN>(lds + LW3, dz3, g, r, h);
        mask_grad<K3, TBN>(g, S + T * (N3 + PAD), w, r, h, dz2);
      }
      block_sync_lds();
      STAMP(10);
      dw_phase<K3, N3, 1, O3K>(acc3, S, n3, 0, k3, 1, r, h);
    }
    WDC_EMIT(O3K, acc3, ct3);
    block_sync_lds();

    // ---- layer 2
    STAMP(11);
    v4bf dz1[TBN][K2 / 16];
    if constexpr (split_stage(K2, N2)) {  // two passes of T / 2 staged rows (column block 0, then 1)
      unsigned int gb[TBN][K2 / 16][2];
      {
        stage_half<K2, N2, TBN>(S, dz2, a1, w, r, h, 0);
        v4f g[TBN][K2 / 16];
        bwd_dA<K2, N2, TBN>(lds + LW2, dz2, g, r, h);
        to_bf_tiles<K2, TBN>(g, gb);
      }
      mask_half<K2, TBN>(gb, S + (T / 2) * (N2 + PAD), w, r, h, dz1, 0);
      block_sync_lds();
      dw_phase<K2, N2, O2N, O2K, T / 2>(acc2, S, n2, 1, k2, 1, r, h);
      block_sync_lds();
      stage_half<K2, N2, TBN>(S, dz2, a1, w, r, h, 1);
      mask_half<K2, TBN>(gb, S + (T / 2) * (N2 + PAD), w, r, h, dz1, 1);
      block_sync_lds();
      STAMP(12);
      dw_phase<K2, N2, O2N, O2K, T / 2>(acc2, S, n2, 1, k2, 1, r, h);
    } else {
      stage<K2, N2, TBN>(S, dz2, a1, w, r, h);
      // the activation gradient needs only the weights, this wave's dZ and its own staged rows (the relu mask):
      // issued before the barrier so its MFMAs and weight reads overlap the other waves' staging
      {
        v4f g[TBN][K2 / 16];
        bwd_dA<K2, N2, TBN>(lds + LW2, dz2, g, r, h);
        mask_grad<K2, TBN>(g, S + T * (N2 + PAD), w, r, h, dz1);
      }
      block_sync_lds();
      STAMP(12);
      dw_phase<K2, N2, O2N, O2K>(acc2, S, n2, 1, k2, 1, r, h);
    }
    WDC_EMIT(O2N * O2K, acc2, ct2);
    block_sync_lds();

    // ---- layer 1
    STAMP(13);
    if constexpr (split_stage(K1, N1)) {  // two passes of T / 2 staged rows
      stage_half<K1, N1, TBN>(S, dz1, a0, w, r, h, 0);
      block_sync_lds();
      dw_phase<K1, N1, O1N, 1, T / 2>(acc1, S, n1, 1, 0, 0, r, h);
      block_sync_lds();
      stage_half<K1, N1, TBN>(S, dz1, a0, w, r, h, 1);
      block_sync_lds();
      STAMP(14);
      dw_phase<K1, N1, O1N, 1, T / 2>(acc1, S, n1, 1, 0, 0, r, h);
    } else {
      stage<K1, N1, TBN>(S, dz1, a0, w, r, h);
      block_sync_lds();
      STAMP(14);
      dw_phase<K1, N1, O1N, 1>(acc1, S, n1, 1, 0, 0, r, h);
    }
    WDC_EMIT(O1N, acc1, ct1);
    if constexpr (PERSIST) {  // the whole DNN update of this lane's columns (see opt_tiles)
      constexpr int NA = O1N + O2N * O2K + O3K + O4K + 1;
      int cta[NA];
#pragma unroll
      for (int i = 0; i < O1N; ++i) cta[i] = ct1[i];
#pragma unroll
      for (int i = 0; i < O2N * O2K; ++i) cta[O1N + i] = ct2[i];
#pragma unroll
      for (int i = 0; i < O3K; ++i) cta[O1N + O2N * O2K + i] = ct3[i];
#pragma unroll
      for (int i = 0; i < O4K; ++i) cta[O1N + O2N * O2K + O3K + i] = ct4[i];
      cta[NA - 1] = ct5[0];
      opt_tiles<NA>(cta, lane, ta, pstep, plast, lds, my_slab);
    }
    STAMP(15);
  }
#ifdef WDC_STAMPS
  stamp_on = true;
#endif
  STAMP(16);

  // ---- epilogue: per-workgroup slab (same layout as wd_fused)
  for (int o = 32; o > 0; o >>= 1) {
    loss_sum += __shfl_xor(loss_sum, o);
    dl_sum += __shfl_xor(dl_sum, o);
  }
  __syncthreads();  // last dW reads done; red/wgrad final
  if (lane == 0) {
    red[w] = loss_sum;
    red[NWAVE + w] = dl_sum;
  }
  // (the dW tiles went out in the last iteration, each right after its layer's dW phase: their stores drain
  // under the remaining layers' compute instead of here)
  __syncthreads();
  if constexpr (TRAIN && PERSIST) {  // wide weights: optimizer on the histogram gradient, in LDS + master copy
    const bool s1_live = ta.hw.kind >= 2;
    const int w0 = stride - WIDE_PAD;
    for (int c = tid; c < WIDE_PAD; c += NTHR) {
      float v = (float)wgi[c] * qinv;
      wgi[c] = 0;  // next step's histogram (read back only after the step-end barrier)
      if (c == WIDE_BIAS) {
#pragma unroll
        for (int i = 0; i < NWAVE; ++i) v += red[NWAVE + i];
      }
      if (ta.wsc[w0 + c] == -1) continue;  // padding
      float a0 = ta.s0[w0 + c], a1 = s1_live ? ta.s1[w0 + c] : 0.f;
      const float nw = opt_update(ta.hw, wlds[c], v, a0, a1, step0 + ps + 1);
      wlds[c] = nw;
      ta.param[w0 + c] = nw;
      ta.s0[w0 + c] = a0;
      if (s1_live) ta.s1[w0 + c] = a1;
    }
  } else if (TRAIN) {
    // 16-byte stores (stride and WIDE_PAD are multiples of 4 floats; the histogram sits 16-B aligned in LDS)
    static_assert(WIDE_PAD % 4 == 0 && (LSEND * 2) % 16 == 0, "vector wide-gradient epilogue");
    v4f* my4 = (v4f*)(slab + (size_t)blockIdx.x * stride + (stride - WIDE_PAD));
    const int4* wgi4 = (const int4*)wgi;
    for (int c4 = tid; c4 < WIDE_PAD / 4; c4 += NTHR) {
      const int4 qv = wgi4[c4];
      float4 v = make_float4((float)qv.x * qinv, (float)qv.y * qinv, (float)qv.z * qinv, (float)qv.w * qinv);
      static_assert(WIDE_BIAS % 4 == 3, "bias column is the .w lane of its float4");
      if (c4 == WIDE_BIAS / 4) {  // the wave sums added one by one onto the bias column, in wave order
#pragma unroll
        for (int i = 0; i < NWAVE; ++i) v.w += red[NWAVE + i];
      }
      slab_store(my4 + c4, v4f{v.x, v.y, v.z, v.w});
    }
  }
  if (tid == 0 && slab_loss) {
    float l = 0.f;
#pragma unroll
    for (int i = 0; i < NWAVE; ++i) l += red[i];
    slab_loss[blockIdx.x] = l;
  }
  if constexpr (PERSIST) {
    // the step's LDS weight / wide updates and histogram reset before the next step's forward; the master
    // state's stores acknowledged and the vector L1 invalidated before the owning lanes read it back
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  }
  }  // step loop
  if constexpr (PERSIST) {
    for (int i = tid; i < STEP_SLOTS; i += NTHR) ta.step_slots[i] = step0 + nsteps;
  }
  STAMP(17);
  BSTAMP(2);
  if constexpr (TRAIN && TAIL) {
    if (ta.helpers > 0) {  // one-row tail: publish the gradient row (slab row 0) to the optimizer workgroups
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (tid == 0) {
        __threadfence();  // agent-scope release: this XCD's L2 written back, the row visible to every XCD
        __hip_atomic_store(ta.bar, (unsigned long long)(step0 + 1), __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
      }
      return;
    }
    const int G = gridDim.x, b = blockIdx.x, S4 = stride / 4;
    int* tl = (int*)(lds + LS);  // the staging area is free now
    int* rows = tl;              // [256] rows written on this XCD, ascending
    int* first = tl + 256;       // [XMAXT] first row per XCD
    int* order = tl + 256 + XMAXT;
    int* misc = tl + 256 + 2 * XMAXT;  // [0] barrier flag, [1] nrows, [2] my index, [3] nord, [4..7] wave counts
    float4* rsum = (float4*)(tl + 512);  // [4][128] level-1 row-group partials
    // optimizer state of this workgroup's level-2 columns: in flight across both barriers
    const int per = (stride + G - 1) / G;
    const int gi = b * per + tid;
    ScState st{-1, 0.f, 0.f, 0.f};
    if (tid < per) st = sc_load(gi, stride, ta.wsc, ta.param, ta.s0, ta.s1);
    const long long step = ta.step_slots[b] + 1;
    TSTAMP(1);
    if (!grid_sync(ta.bar, ta.err, G, misc)) return;
    TSTAMP(2);
    // ---- level 1
    const int x = mifx_xcc_id();
    if (tid < XMAXT) first[tid] = 1 << 30;
    const int xo = tid < G ? __hip_atomic_load(xcd_of + tid, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) : -1;
    const bool sel = tid < G && xo == x;
    const unsigned long long m = __ballot(sel);
    if (lane == 0 && w < 4) misc[4 + w] = __popcll(m);
    __syncthreads();
    if (tid < G) atomicMin(&first[xo & (XMAXT - 1)], tid);
    int base = 0;
    for (int i = 0; i < w && i < 4; ++i) base += misc[4 + i];
    if (sel) {
      const int pos = base + __popcll(m & ((1ull << lane) - 1));
      rows[pos] = tid;
      if (tid == b) misc[2] = pos;
    }
    if (tid == 0) misc[1] = misc[4] + misc[5] + misc[6] + misc[7];
    __syncthreads();
    if (tid < XMAXT) {  // XCDs holding rows, ordered by their first row (lane tid's rank among the valid ones)
      const int f = first[tid];
      const bool valid = f < (1 << 30);
      int rank = 0;
#pragma unroll
      for (int y = 0; y < XMAXT; ++y) rank += first[y] < f ? 1 : 0;
      if (valid) order[rank] = tid;
      const unsigned long long vm = __ballot(valid);
      if (tid == 0) misc[3] = __popcll(vm);
    }
    const int nr = misc[1], me = misc[2];
    const int q0 = (int)((long long)me * S4 / nr), q1 = (int)((long long)(me + 1) * S4 / nr);
    const float4* slab4 = (const float4*)slab;
    for (int qb = q0; qb < q1; qb += 128) {
      const int lq = tid & 127, rg = tid >> 7;  // 4 row groups (NTHR = 512)
      const int q = qb + lq;
      float4 a = make_float4(0.f, 0.f, 0.f, 0.f);
      if (q < q1) {
        constexpr int U = 8;
        for (int i0 = rg; i0 < nr; i0 += 4 * U) {
          float4 v[U];
#pragma unroll
          for (int u = 0; u < U; ++u) {
            const int i = i0 + 4 * u;
            v[u] = i < nr ? slab4[(size_t)rows[i] * S4 + q] : make_float4(0.f, 0.f, 0.f, 0.f);
          }
#pragma unroll
          for (int u = 0; u < U; ++u) {
            a.x += v[u].x; a.y += v[u].y; a.z += v[u].z; a.w += v[u].w;
          }
        }
      }
      rsum[rg * 128 + lq] = a;
      __syncthreads();
      if (rg == 0 && q < q1) {
        float4 sm = rsum[lq];
#pragma unroll
        for (int k2 = 1; k2 < 4; ++k2) {
          const float4 v = rsum[k2 * 128 + lq];
          sm.x += v.x; sm.y += v.y; sm.z += v.z; sm.w += v.w;
        }
        st_sys4(ta.xpart + (size_t)x * stride + 4 * q, sm);
      }
      __syncthreads();
    }
    TSTAMP(3);
    if (!grid_sync(ta.bar, ta.err, G, misc)) return;
    TSTAMP(4);
    // ---- level 2 + optimizer
    if (tid < per && gi < stride) {
      const int nord = misc[3];
      float pv[XMAXT];
#pragma unroll
      for (int k2 = 0; k2 < XMAXT; ++k2) pv[k2] = k2 < nord ? ld_sys1(ta.xpart + (size_t)order[k2] * stride + gi) : 0.f;
      float g = pv[0];
#pragma unroll
      for (int k2 = 1; k2 < XMAXT; ++k2)
        if (k2 < nord) g += pv[k2];
      sc_update(gi, st, g, ta.hd, ta.hw, step, ta.param, ta.s0, ta.s1, ta.wt_out);
    }
    if (tid == 0) ta.step_slots[b] = step;
    if (b == 0)
      for (int i = G + tid; i < STEP_SLOTS; i += NTHR) ta.step_slots[i] = step;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    TSTAMP(5);
  }
}

template <bool TRAIN, int TBN, bool TAIL = false, bool PERSIST = false>
void launch(dim3 grid, hipStream_t stream, const void* data, long long n_data, long long batch, long long start_fixed,
            const long long* step_ctr, const void* wimg, const float* wide, float* slab, float* slab_loss,
            float* logits_out, float grad_scale, const int* tmap, int stride, int* xcd_of, MifxFeed feed,
            TailArgs ta = TailArgs{}) {
  constexpr int lds_bytes = PERSIST ? LDS_BYTES_P : LDS_BYTES;
  static bool attr_done = false;
  if (!attr_done) {
    (void)hipFuncSetAttribute((const void*)wdc_fused<TRAIN, TBN, TAIL, PERSIST>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, lds_bytes);
    attr_done = true;
  }
  hipLaunchKernelGGL((wdc_fused<TRAIN, TBN, TAIL, PERSIST>), grid, dim3(64 * (T / (16 * TBN))), lds_bytes, stream,
                     (const uint4*)data, n_data, batch, start_fixed, step_ctr, (const uint4*)wimg, wide, slab,
                     slab_loss, logits_out, grad_scale, tmap, stride, xcd_of, ta, feed);
}

}  // namespace

// exported names: the T = 64 build (csrc/wd_chain64.hip) suffixes them, so neither library's calls can bind to the
// other's definitions when both are loaded RTLD_GLOBAL
#if WDC_T == 128
#define WDC_SYM(n) n
#elif WDC_T == 64
#define WDC_SYM(n) n##_t64
#else
#define WDC_SYM(n) n##_t256
#endif

extern "C" {

// T, LWEND (weight image elements), LDS_BYTES, WPAD (weight-image row pad), NTILE, WIDE_PAD
int WDC_SYM(mifx_wdc_constants)(int* out, int n) {
  const int v[] = {T, LWEND, LDS_BYTES, WPAD, NTILE, WIDE_PAD, LW1, LW2, LW3, LW4, LW5};
  const int m = (int)(sizeof(v) / sizeof(int));
  for (int i = 0; i < n && i < m; ++i) out[i] = v[i];
  return m;
}

// One launch = forward (+ loss) [+ backward into the per-workgroup slab] over `batch` records starting at
// waves: 4 (4 waves x 32 examples, one wave per SIMD) or 8 (8 waves x 16 examples, two waves per SIMD).
// (step_ctr[0] * batch) % n_data (or start_fixed when step_ctr is null). wimg: the bf16 weight image in LDS
// layout (LWEND elements, C-ordered columns, see models.wide_deep.chain_image).
// xcd_of (nullable, >= grid ints): receives the XCD each workgroup ran on (training only).
// (T = 64 build: waves must be 4, 4 x 16 examples)
int WDC_SYM(mifx_wdc_fused_f)(const void* data, long long n_data, long long batch, long long start_fixed,
                              const long long* step_ctr, const void* wimg, const float* wide, float* slab,
                              float* slab_loss, float* logits_out, float grad_scale, int grid, int train,
                              const int* tmap, int stride, int waves, int* xcd_of, long long feed_stride,
                              long long feed_offset, unsigned long long shuffle_key, hipStream_t stream) {
  if (grid <= 0 || n_data <= 0 || batch <= 0 || batch > n_data || wimg == nullptr || wide == nullptr) return -1;
  if ((uintptr_t)wimg % 16 != 0 || (uintptr_t)data % 16 != 0) return -1;
  if (train && (tmap == nullptr || slab == nullptr || stride < WIDE_PAD || stride % 4 != 0)) return -1;
  if (!train && logits_out == nullptr) return -1;
  if (feed_stride < batch || feed_offset < 0 || feed_offset + batch > feed_stride) return -1;
  const MifxFeed fd{feed_stride, feed_offset, shuffle_key};
  const dim3 g(grid);
#if WDC_T == 64
  if (waves != 4) return -1;
  if ((long long)grid * T < batch) return -1;  // ONE_ITER: one iteration per workgroup
  if (train)
    launch<true, 1>(g, stream, data, n_data, batch, start_fixed, step_ctr, wimg, wide, slab, slab_loss, logits_out,
                    grad_scale, tmap, stride, xcd_of, fd);
  else
    launch<false, 1>(g, stream, data, n_data, batch, start_fixed, step_ctr, wimg, wide, slab, slab_loss, logits_out,
                     grad_scale, tmap, stride, nullptr, fd);
  return (int)hipGetLastError();
#elif WDC_T == 256
  if (waves != 8) return -1;  // 8 waves x 2 column blocks of 16 examples
  if ((long long)grid * T < batch) return -1;  // ONE_ITER: one iteration per workgroup
  if (train)
    launch<true, 2>(g, stream, data, n_data, batch, start_fixed, step_ctr, wimg, wide, slab, slab_loss, logits_out,
                    grad_scale, tmap, stride, xcd_of, fd);
  else
    launch<false, 2>(g, stream, data, n_data, batch, start_fixed, step_ctr, wimg, wide, slab, slab_loss, logits_out,
                     grad_scale, tmap, stride, nullptr, fd);
  return (int)hipGetLastError();
#else
  if (waves != 4 && waves != 8) return -1;
  if (train && waves == 4)
    launch<true, 2>(g, stream, data, n_data, batch, start_fixed, step_ctr, wimg, wide, slab, slab_loss, logits_out,
                    grad_scale, tmap, stride, xcd_of, fd);
  else if (train)
    launch<true, 1>(g, stream, data, n_data, batch, start_fixed, step_ctr, wimg, wide, slab, slab_loss, logits_out,
                    grad_scale, tmap, stride, xcd_of, fd);
  else  // eval / predict: the 4-wave shape for either request (forward only, no dW phases to overlap)
    launch<false, 2>(g, stream, data, n_data, batch, start_fixed, step_ctr, wimg, wide, slab, slab_loss, logits_out,
                     grad_scale, tmap, stride, nullptr, fd);
  return (int)hipGetLastError();
#endif
}

// the same launch with the records in stored order, one replica (feed stride = batch, offset 0, no shuffle)
int WDC_SYM(mifx_wdc_fused_x)(const void* data, long long n_data, long long batch, long long start_fixed,
                              const long long* step_ctr, const void* wimg, const float* wide, float* slab,
                              float* slab_loss, float* logits_out, float grad_scale, int grid, int train,
                              const int* tmap, int stride, int waves, int* xcd_of, hipStream_t stream) {
  return WDC_SYM(mifx_wdc_fused_f)(data, n_data, batch, start_fixed, step_ctr, wimg, wide, slab, slab_loss,
                                   logits_out, grad_scale, grid, train, tmap, stride, waves, xcd_of, batch, 0, 0,
                                   stream);
}

int WDC_SYM(mifx_wdc_fused)(const void* data, long long n_data, long long batch, long long start_fixed,
                            const long long* step_ctr, const void* wimg, const float* wide, float* slab,
                            float* slab_loss, float* logits_out, float grad_scale, int grid, int train,
                            const int* tmap, int stride, int waves, hipStream_t stream) {
  return WDC_SYM(mifx_wdc_fused_x)(data, n_data, batch, start_fixed, step_ctr, wimg, wide, slab, slab_loss,
                                   logits_out, grad_scale, grid, train, tmap, stride, waves, nullptr, stream);
}

// One training step of a batch ONE workgroup trains, with the optimizer in the same launch (help_update): grid
// 1 + helpers, helpers = ceil(stride / threads per workgroup) (wd_opt1_sc's workgroup count at 256 threads). State in
// slab-column order (wsc / param / s0 / s1, step slots); bar / err as mifx_wdc_fused_tail. T = 64 build: 4 waves;
// T = 128 build: 8 waves.
int WDC_SYM(mifx_wdc_fused_help)(const void* data, long long n_data, long long batch, long long* step_ctr, void* wimg,
                                 float* wide, float* slab, float* slab_loss, float grad_scale, const int* tmap,
                                 int stride, unsigned long long* bar, int* err, const int* wsc, float* param,
                                 float* s0, float* s1, const float* hyper_dnn, const float* hyper_wide, int helpers,
                                 long long feed_stride, long long feed_offset, unsigned long long shuffle_key,
                                 hipStream_t stream) {
#if WDC_T == 256
  return -1;
#else
  constexpr int NTHR_H = WDC_T == 64 ? 256 : 512;  // threads of the TBN = 1 shape (4 / 8 waves)
  if (n_data <= 0 || batch <= 0 || batch > T || batch > n_data || helpers <= 0 || helpers + 1 > STEP_SLOTS ||
      (long long)helpers * NTHR_H < stride)
    return -1;
  if (wimg == nullptr || wide == nullptr || slab == nullptr || tmap == nullptr || bar == nullptr || err == nullptr ||
      wsc == nullptr || param == nullptr || s0 == nullptr || s1 == nullptr || step_ctr == nullptr ||
      hyper_dnn == nullptr || hyper_wide == nullptr)
    return -1;
  if ((uintptr_t)wimg % 16 != 0 || (uintptr_t)data % 16 != 0 || stride < WIDE_PAD || stride % 4 != 0) return -1;
  if (feed_stride < batch || feed_offset < 0 || feed_offset + batch > feed_stride) return -1;
  TailArgs ta{};
  ta.bar = bar;
  ta.err = err;
  ta.wsc = wsc;
  ta.param = param;
  ta.s0 = s0;
  ta.s1 = s1;
  ta.wt_out = (uint16_t*)wimg;
  ta.step_slots = step_ctr;
  ta.helpers = helpers;
  ta.hd = OptHyper{(int)hyper_dnn[0], hyper_dnn[1], hyper_dnn[2], hyper_dnn[3], hyper_dnn[4], hyper_dnn[5],
                   hyper_dnn[6], hyper_dnn[7]};
  ta.hw = OptHyper{(int)hyper_wide[0], hyper_wide[1], hyper_wide[2], hyper_wide[3], hyper_wide[4], hyper_wide[5],
                   hyper_wide[6], hyper_wide[7]};
  launch<true, 1, true>(dim3(1 + helpers), stream, data, n_data, batch, 0, step_ctr, wimg, wide, slab, slab_loss,
                        nullptr, grad_scale, tmap, stride, nullptr, MifxFeed{feed_stride, feed_offset, shuffle_key},
                        ta);
  return (int)hipGetLastError();
#endif
}

#if WDC_T == 128  // the in-kernel tail and the persistent kernel exist for the 8-wave T = 128 shape only

// Training step with the in-kernel tail (slab reduction + optimizer inside the launch; see TailArgs): 8-wave
// shape, grid <= the number of CUs (every workgroup must be resident), the whole step in ONE launch.
// xpart: [16][stride] fp32 scratch; bar: one uint64 arrival counter (zero at creation, never reset while the
// trainer lives); err: sticky int flag; wsc / param / s0 / s1 / wt (the kernel's own weight image) / step_ctr
// (STEP_SLOTS slots): the slab-column-order optimizer state of csrc/wide_deep.hip wd_reduce_opt_sc.
int mifx_wdc_fused_tail(const void* data, long long n_data, long long batch, long long* step_ctr, void* wimg,
                        float* wide, float* slab, float* slab_loss, float grad_scale, int grid, const int* tmap,
                        int stride, int* xcd_of, float* xpart, unsigned long long* bar, int* err, const int* wsc,
                        float* param, float* s0, float* s1, const float* hyper_dnn, const float* hyper_wide,
                        long long* dbg, long long feed_stride, long long feed_offset, unsigned long long shuffle_key,
                        hipStream_t stream) {
  int dev = 0, ncu = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) !=
                                              hipSuccess)
    return -1;
  if (grid <= 0 || grid > ncu || grid > 256 || grid > STEP_SLOTS || n_data <= 0 || batch <= 0 || batch > n_data)
    return -1;
  if (wimg == nullptr || wide == nullptr || slab == nullptr || tmap == nullptr || xcd_of == nullptr ||
      xpart == nullptr || bar == nullptr || err == nullptr || wsc == nullptr || param == nullptr || s0 == nullptr ||
      s1 == nullptr || step_ctr == nullptr)
    return -1;
  if ((uintptr_t)wimg % 16 != 0 || (uintptr_t)data % 16 != 0 || stride < WIDE_PAD || stride % 4 != 0) return -1;
  if (feed_stride < batch || feed_offset < 0 || feed_offset + batch > feed_stride) return -1;
  TailArgs ta{};
  ta.xpart = xpart;
  ta.bar = bar;
  ta.err = err;
  ta.wsc = wsc;
  ta.param = param;
  ta.s0 = s0;
  ta.s1 = s1;
  ta.wt_out = (uint16_t*)wimg;
  ta.step_slots = step_ctr;
  ta.dbg = dbg;
  ta.hd = OptHyper{(int)hyper_dnn[0], hyper_dnn[1], hyper_dnn[2], hyper_dnn[3], hyper_dnn[4], hyper_dnn[5],
                   hyper_dnn[6], hyper_dnn[7]};
  ta.hw = OptHyper{(int)hyper_wide[0], hyper_wide[1], hyper_wide[2], hyper_wide[3], hyper_wide[4], hyper_wide[5],
                   hyper_wide[6], hyper_wide[7]};
  launch<true, 1, true>(dim3(grid), stream, data, n_data, batch, 0, step_ctr, wimg, wide, slab, slab_loss, nullptr,
                        grad_scale, tmap, stride, xcd_of, MifxFeed{feed_stride, feed_offset, shuffle_key}, ta);
  return (int)hipGetLastError();
}

// Persistent small-batch training (see opt_tiles): `nsteps` whole training steps of a batch <= T in ONE launch of
// one 8-wave workgroup -- forward, backward, Adagrad/FTRL/Adam/SGD update of every weight, step counter advance.
// State in slab-column order as mifx_wdc_fused_tail (wsc / param / s0 / s1, STEP_SLOTS step slots; wimg is the
// global bf16 image, rewritten at the last step). Bit-identical to nsteps grid-1 slab steps + wd_reduce_opt_sc.
int mifx_wdc_persist(const void* data, long long n_data, long long batch, long long* step_ctr, void* wimg,
                     float* wide, float* slab, float* slab_loss, float grad_scale, const int* tmap, int stride, const int* wsc,
                     float* param, float* s0, float* s1, const float* hyper_dnn, const float* hyper_wide, int nsteps,
                     long long feed_stride, long long feed_offset, unsigned long long shuffle_key, hipStream_t stream) {
  if (nsteps <= 0 || n_data <= 0 || batch <= 0 || batch > T || batch > n_data) return -1;
  if (wimg == nullptr || wide == nullptr || tmap == nullptr || wsc == nullptr || param == nullptr || s0 == nullptr ||
      s1 == nullptr || step_ctr == nullptr || hyper_dnn == nullptr || hyper_wide == nullptr || slab == nullptr)
    return -1;
  if ((uintptr_t)wimg % 16 != 0 || (uintptr_t)data % 16 != 0 || stride < WIDE_PAD || stride % 4 != 0) return -1;
  if (feed_stride < batch || feed_offset < 0 || feed_offset + batch > feed_stride) return -1;
  TailArgs ta{};
  ta.wsc = wsc;
  ta.param = param;
  ta.s0 = s0;
  ta.s1 = s1;
  ta.wt_out = (uint16_t*)wimg;
  ta.step_slots = step_ctr;
  ta.nsteps = nsteps;
  ta.hd = OptHyper{(int)hyper_dnn[0], hyper_dnn[1], hyper_dnn[2], hyper_dnn[3], hyper_dnn[4], hyper_dnn[5],
                   hyper_dnn[6], hyper_dnn[7]};
  ta.hw = OptHyper{(int)hyper_wide[0], hyper_wide[1], hyper_wide[2], hyper_wide[3], hyper_wide[4], hyper_wide[5],
                   hyper_wide[6], hyper_wide[7]};
  launch<true, 1, false, true>(dim3(1), stream, data, n_data, batch, 0, step_ctr, wimg, wide, slab, slab_loss,
                               nullptr, grad_scale, tmap, stride, nullptr, MifxFeed{feed_stride, feed_offset, shuffle_key},
                               ta);
  return (int)hipGetLastError();
}

#endif  // WDC_T == 128

#ifdef WDC_STAMPS
int mifx_wdc_stamps(unsigned long long* out) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wdc_stamps), sizeof(g_wdc_stamps), 0, hipMemcpyDeviceToHost);
}
int mifx_wdc_blk_stamps(unsigned long long* out) {
  return (int)hipMemcpyFromSymbol(out, HIP_SYMBOL(g_wdc_blk), sizeof(g_wdc_blk), 0, hipMemcpyDeviceToHost);
}
#endif

}  // extern "C"
