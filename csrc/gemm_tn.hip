// Hand-written bf16 MFMA "TN" GEMM for gfx950: C[M, N] = A[T, M]^T . B[T, N] -- the weight gradient of a linear layer,
// dW = dY^T X, with the token dimension T (the reduction) as the row index of BOTH operands.
//
// BASELINE config 4 (BERT-base, 4096 tokens): the four weight-gradient GEMMs of a layer (QKV 2304x768, attention-out
// 768x768, FFN-in 3072x768, FFN-out 768x3072, all with K = 4096 tokens) were hipBLASLt's slowest products in the
// training step: 144-216 workgroups of 128x128 / 64x64 tiles on 256 CUs (one K-reduction per tile, no split), 30-46 us
// each, 160-420 TFLOP/s (profiles/archive/bert_steady_kernels_r3.md). Here every shape gets a whole wave of workgroups: the
// 96 x 96 tile puts 3072 x 768 (and 768 x 3072) on exactly 256 workgroups, and small outputs split the token range
// over gridDim.y with an fp32 partial per split, summed in split order by a second kernel (deterministic).
//
// Structure:
//  * 4 waves (2 x 2), each owning a (BM/2) x (BN/2) block of 16 x 16 MFMA tiles (mfma_f32_16x16x32_bf16);
//  * per 64-token K-tile every lane issues 16-byte global->LDS DMA loads (no VGPR round trip) of A rows [64][BM] and
//    B rows [64][BN] into a ring of NS buffers (~144 KB), NS - 1 tiles ahead of the MFMAs; one barrier per K-tile;
//  * both operands sit in LDS token-major, so the MFMA fragments (8 consecutive tokens per lane) are read with
//    ds_read_b64_tr_b16: a 16-lane group supplies 4 token rows x 16 columns, each lane receives one column's 4
//    tokens; two reads (+4 rows) make the 8-token fragment. The 16-byte chunks of row t sit rotated by rot(t)
//    inside their row (applied to each lane's DMA SOURCE address, as DMA destinations are lane-linear): with the
//    rotation below every 32-lane half of every fragment read touches 64 distinct banks (checked by
//    tools/lds_banks_tn.py for each chunk count);
//  * the MFMA takes the B fragment as its A operand, so the accumulator lane holds C[m][n .. n + 3]: 8-byte bf16
//    stores (or 16-byte fp32 partial stores) in the epilogue;
//  * XCD-aware tile order: consecutive workgroups run on different XCDs (round-robin dispatch), so the tile index is
//    remapped bijectively so that each XCD walks a contiguous run of tiles, grouped 4 m-blocks wide, in its own L2.
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

// chunk rotation of token row t for a row of CPA 16-byte chunks (conflict-free transposed fragment reads)
template <int CPA>
__device__ __forceinline__ int rot(int t) {
  static_assert(CPA == 8 || CPA == 12 || CPA == 16 || CPA == 24, "chunks per row");
  if constexpr (CPA == 8) return ((t & 3) + 4 * ((t >> 3) & 3)) & 7;
  if constexpr (CPA == 12) return (2 * ((t >> 3) & 3)) % 12;
  if constexpr (CPA == 24) return (6 * (t & 3) + 6 * ((t >> 3) & 3)) % 24;
  return (2 * (t & 3) + 8 * ((t >> 3) & 3)) & 15;
}
template <int CPA>
__device__ __forceinline__ int slot_of(int t, int c) {  // physical chunk of logical chunk c in row t
  const int p = c + rot<CPA>(t);
  return p >= CPA ? p - CPA : p;
}

__device__ __forceinline__ v4s tr_read(const unsigned char* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(p));
}
__device__ __forceinline__ v8bf cat8(v4s a, v4s b) {
  v8s r = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  return __builtin_bit_cast(v8bf, r);
}

// OUT_F32: store the fp32 partial of split blockIdx.y at P + blockIdx.y * M * N (else bf16 C directly).
// OPT bit 0: raise the wave priority around each MFMA block (bit 1 in the config table: the 8-wave gemm_tn_k2).
template <int BM, int BN, bool OUT_F32, int OPT, int NS>
__global__ __launch_bounds__(256) void gemm_tn(const bf16* __restrict__ A, const bf16* __restrict__ B,
                                                  bf16* __restrict__ C, float* __restrict__ P, int M, int N, int T,
                                                  int tps) {
  constexpr int NT = 256, WM = 2, WN = 2;
  constexpr int TM = BM / WM, TN = BN / WN, MR = TM / 16, NR = TN / 16;
  constexpr int CPA = BM / 8, CPB = BN / 8;  // 16-byte chunks per token row
  constexpr int AR = (BK * CPA + NT - 1) / NT, BR = (BK * CPB + NT - 1) / NT;  // DMA rounds per K-tile
  constexpr int ABYTES = BK * BM * 2, BBYTES = BK * BN * 2, BUF = ABYTES + BBYTES;
  static_assert(TM % 16 == 0 && TN % 16 == 0, "wave tiling");
  static_assert((BK * CPA) % NT == 0 && (BK * CPB) % NT == 0, "whole DMA rounds (counted waits)");
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];

  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int wm = w / WN, wn = w % WN;
  const int nwg = gridDim.x, bid = blockIdx.x, xcd = bid % 8, q8 = nwg / 8, r8 = nwg % 8;
  const int tile = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + bid / 8;
  // grouped order: runs of GM m-blocks x all n-blocks, m fastest, so an XCD's run of consecutive tiles covers a
  // GM x (run / GM) block of the output and re-reads few A and B strips per K-tile from its L2
  constexpr int GM = 4;
  const int nb_m = M / BM, nb_n = N / BN, per_group = GM * nb_n;
  const int group = tile / per_group, first_m = group * GM, gsz = min(GM, nb_m - first_m);
  const int wi = tile - group * per_group;
  const int m0 = (first_m + wi % gsz) * BM, n0 = (wi / gsz) * BN;
  const int t_begin = blockIdx.y * tps, KT = tps / BK;

  // per-lane DMA source offsets (elements, relative to the K-tile's first token row)
  int aoff[AR], boff[BR];
#pragma unroll
  for (int i = 0; i < AR; ++i) {
    const int s = min(i * NT + tid, BK * CPA - 1), t = s / CPA, p = s % CPA;
    int c = p - rot<CPA>(t);
    c = c < 0 ? c + CPA : c;
    aoff[i] = t * M + m0 + 8 * c;
  }
#pragma unroll
  for (int i = 0; i < BR; ++i) {
    const int s = min(i * NT + tid, BK * CPB - 1), t = s / CPB, p = s % CPB;
    int c = p - rot<CPB>(t);
    c = c < 0 ? c + CPB : c;
    boff[i] = t * N + n0 + 8 * c;
  }
  auto issue = [&](int kt, int buf) {
    unsigned char* ba = lds + buf * BUF;
    unsigned char* bb = ba + ABYTES;
    const size_t t0 = (size_t)(t_begin + kt * BK);
    const bf16* a0 = A + t0 * M;
    const bf16* b0 = B + t0 * N;
#pragma unroll
    for (int i = 0; i < AR; ++i)
      if ((BK * CPA) % NT == 0 || i * NT + 64 * w < BK * CPA)
        __builtin_amdgcn_global_load_lds((const void*)(a0 + aoff[i]),
                                         (__attribute__((address_space(3))) void*)(ba + (i * NT + 64 * w) * 16), 16, 0,
                                         0);
#pragma unroll
    for (int i = 0; i < BR; ++i)
      if ((BK * CPB) % NT == 0 || i * NT + 64 * w < BK * CPB)
        __builtin_amdgcn_global_load_lds((const void*)(b0 + boff[i]),
                                         (__attribute__((address_space(3))) void*)(bb + (i * NT + 64 * w) * 16), 16, 0,
                                         0);
  };

  v4f acc[MR][NR];
#pragma unroll
  for (int a = 0; a < MR; ++a)
#pragma unroll
    for (int b = 0; b < NR; ++b) acc[a][b] = (v4f){0.f, 0.f, 0.f, 0.f};

  // fragment read geometry: lane (r, h), r = lane & 15 -> (row quad q = r >> 2, column quad p = r & 3)
  const int r = lane & 15, h = lane >> 4, q = r >> 2, p = r & 3;
  auto read_frags = [&](const unsigned char* ba, const unsigned char* bb, int ks, v8bf (&af)[MR], v8bf (&bf)[NR]) {
    const int t1 = 32 * ks + 8 * h + q, t2 = t1 + 4;
#pragma unroll
    for (int a = 0; a < MR; ++a) {
      const int c = (wm * TM + 16 * a) / 8 + (p >> 1);
      const unsigned char* p1 = ba + (t1 * CPA + slot_of<CPA>(t1, c)) * 16 + 8 * (p & 1);
      const unsigned char* p2 = ba + (t2 * CPA + slot_of<CPA>(t2, c)) * 16 + 8 * (p & 1);
      af[a] = cat8(tr_read(p1), tr_read(p2));
    }
#pragma unroll
    for (int b = 0; b < NR; ++b) {
      const int c = (wn * TN + 16 * b) / 8 + (p >> 1);
      const unsigned char* p1 = bb + (t1 * CPB + slot_of<CPB>(t1, c)) * 16 + 8 * (p & 1);
      const unsigned char* p2 = bb + (t2 * CPB + slot_of<CPB>(t2, c)) * 16 + 8 * (p & 1);
      bf[b] = cat8(tr_read(p1), tr_read(p2));
    }
  };

  // NS-buffer ring, NS - 1 K-tiles in flight: one K-tile's MFMAs (~300 cycles) are far shorter than a DMA's
  // latency from L2 / MALL, so the loads of the next NS - 2 tiles overlap the wait for this one. A counted
  // `s_waitcnt vmcnt` retires only the oldest tile (G DMAs per thread per tile); the barrier then orders it for
  // every wave and frees the buffer read in the previous iteration, which the next issue refills.
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
    if (OPT & 1) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int a = 0; a < MR; ++a)
#pragma unroll
      for (int b = 0; b < NR; ++b) acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf0[b], af0[a], acc[a][b], 0, 0, 0);
#pragma unroll
    for (int a = 0; a < MR; ++a)
#pragma unroll
      for (int b = 0; b < NR; ++b) acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bf1[b], af1[a], acc[a][b], 0, 0, 0);
    if (OPT & 1) __builtin_amdgcn_s_setprio(0);
  }

  // ---- epilogue: lane (r, h) holds C[m0 + wm TM + 16 a + r][n0 + wn TN + 16 b + 4 h + 0..3]
#pragma unroll
  for (int a = 0; a < MR; ++a) {
    const int m = m0 + wm * TM + 16 * a + r;
#pragma unroll
    for (int b = 0; b < NR; ++b) {
      const int n = n0 + wn * TN + 16 * b + 4 * h;
      if constexpr (OUT_F32) {
        *(v4f*)(P + (size_t)blockIdx.y * M * N + (size_t)m * N + n) = acc[a][b];
      } else {
        v4bf o;
#pragma unroll
        for (int i = 0; i < 4; ++i) o[i] = (bf16)acc[a][b][i];
        *(v4bf*)(C + (size_t)m * N + n) = o;
      }
    }
  }
}

// Measured (profiles/archive/gemm_tn_r3b_k2.jsonl): 50 us on FFN-in's dW at S = 1 against 54 for the 4-wave deep ring and
// 38 for two 4-wave workgroups per CU with a 2-way token split -- two independent barrier pipelines per CU beat one
// 8-wave pipeline, so the tuned table keeps the split; this form stays selectable (config 18).
// 8-wave form of the 96 x 96 tile (one workgroup per CU, two waves per SIMD, no token split across workgroups):
// waves w and w + 4 own the same 48 x 48 quadrant and take the two 32-token k-steps of every K-tile, so each SIMD
// runs two independent MFMA chains (the one-wave-per-SIMD 4-wave form idles at every barrier and fragment read);
// the k-step-1 waves hand their accumulators to the k-step-0 waves through LDS at the end (fixed order: k-step 0
// + k-step 1). DMA: each K-tile's 12 + 12 wave-instructions are dealt 2 + 1 / 1 + 2 to waves 0-3 / 4-7 (3 each, so
// the counted vmcnt is the same for every wave).
template <bool OUT_F32, int NS>
__global__ __launch_bounds__(512) void gemm_tn_k2(const bf16* __restrict__ A, const bf16* __restrict__ B,
                                                 bf16* __restrict__ C, float* __restrict__ P, int M, int N, int T,
                                                 int tps) {
  constexpr int BM = 96, BN = 96, TM = 48, TN = 48, MR = 3, NR = 3, CPA = 12, CPB = 12;
  constexpr int ABYTES = BK * BM * 2, BBYTES = BK * BN * 2, BUF = ABYTES + BBYTES;
  constexpr int G = 3;
  extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int qd = w & 3, kg = w >> 2, wm = qd >> 1, wn = qd & 1;
  const int nwg = gridDim.x, bid = blockIdx.x, xcd = bid % 8, q8 = nwg / 8, r8 = nwg % 8;
  const int tile = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + bid / 8;
  constexpr int GM = 4;
  const int nb_m = M / BM, nb_n = N / BN, per_group = GM * nb_n;
  const int group = tile / per_group, first_m = group * GM, gsz = min(GM, nb_m - first_m);
  const int wi = tile - group * per_group;
  const int m0 = (first_m + wi % gsz) * BM, n0 = (wi / gsz) * BN;
  const int t_begin = blockIdx.y * tps, KT = tps / BK;
  // this wave's 3 DMA wave-instructions: (operand, instruction index) -> LDS slots [64 i, 64 i + 64)
  int doff[G], dslot[G];
  bool dis_a[G];
#pragma unroll
  for (int j = 0; j < G; ++j) {
    // waves 0-3: A {w, w + 8}, B {w + 4}; waves 4-7: A {w}, B {w - 4, w + 4}
    const bool isa = kg == 0 ? j < 2 : j == 0;
    const int i = isa ? w + 8 * j : (kg == 0 ? w + 4 : (w - 4) + 8 * (j - 1));
    const int sl = 64 * i + lane, t = sl / 12, pp = sl % 12;
    int c = pp - rot<12>(t);
    c = c < 0 ? c + 12 : c;
    dis_a[j] = isa;
    dslot[j] = 64 * i;
    doff[j] = isa ? t * M + m0 + 8 * c : t * N + n0 + 8 * c;
  }
  auto issue = [&](int kt, int buf) {
    unsigned char* ba = lds + buf * BUF;
    const size_t t0 = (size_t)(t_begin + kt * BK);
#pragma unroll
    for (int j = 0; j < G; ++j) {
      const bf16* src = dis_a[j] ? A + t0 * M + doff[j] : B + t0 * N + doff[j];
      unsigned char* dst = dis_a[j] ? ba + dslot[j] * 16 : ba + ABYTES + dslot[j] * 16;
      __builtin_amdgcn_global_load_lds((const void*)src, (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
    }
  };
  v4f acc[MR][NR];
#pragma unroll
  for (int a = 0; a < MR; ++a)
#pragma unroll
    for (int b = 0; b < NR; ++b) acc[a][b] = (v4f){0.f, 0.f, 0.f, 0.f};
  const int r = lane & 15, h = lane >> 4, q = r >> 2, p = r & 3;
  const int t1 = 32 * kg + 8 * h + q, t2 = t1 + 4;
  int ao1[MR], ao2[MR], bo1[NR], bo2[NR];  // byte offsets of this lane's fragment reads inside a buffer
#pragma unroll
  for (int a = 0; a < MR; ++a) {
    const int c = (wm * TM + 16 * a) / 8 + (p >> 1);
    ao1[a] = (t1 * CPA + slot_of<CPA>(t1, c)) * 16 + 8 * (p & 1);
    ao2[a] = (t2 * CPA + slot_of<CPA>(t2, c)) * 16 + 8 * (p & 1);
  }
#pragma unroll
  for (int b = 0; b < NR; ++b) {
    const int c = (wn * TN + 16 * b) / 8 + (p >> 1);
    bo1[b] = ABYTES + (t1 * CPB + slot_of<CPB>(t1, c)) * 16 + 8 * (p & 1);
    bo2[b] = ABYTES + (t2 * CPB + slot_of<CPB>(t2, c)) * 16 + 8 * (p & 1);
  }
  constexpr int INFL = (NS - 2) * G;
  constexpr int WAIT_STEADY = (INFL & 15) | (7 << 4) | (15 << 8) | ((INFL >> 4) << 14);
#pragma unroll
  for (int i = 0; i < NS - 1; ++i)
    if (i < KT) issue(i, i);
  for (int kt = 0; kt < KT; ++kt) {
    if (kt + NS - 2 <= KT - 1)
      __builtin_amdgcn_s_waitcnt(WAIT_STEADY);
    else
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (kt + NS - 1 < KT) issue(kt + NS - 1, (kt + NS - 1) % NS);
    const unsigned char* bf = lds + (kt % NS) * BUF;
    v8bf af[MR], bfr[NR];
#pragma unroll
    for (int a = 0; a < MR; ++a) af[a] = cat8(tr_read(bf + ao1[a]), tr_read(bf + ao2[a]));
#pragma unroll
    for (int b = 0; b < NR; ++b) bfr[b] = cat8(tr_read(bf + bo1[b]), tr_read(bf + bo2[b]));
#pragma unroll
    for (int a = 0; a < MR; ++a)
#pragma unroll
      for (int b = 0; b < NR; ++b) acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[b], af[a], acc[a][b], 0, 0, 0);
  }
  // k-step-1 waves -> LDS -> k-step-0 waves add (every buffer is free once all waves passed this barrier)
  __syncthreads();
  v4f* red = (v4f*)lds;
  if (kg == 1) {
#pragma unroll
    for (int a = 0; a < MR; ++a)
#pragma unroll
      for (int b = 0; b < NR; ++b) red[((qd * MR + a) * NR + b) * 64 + lane] = acc[a][b];
  }
  __syncthreads();
  if (kg == 1) return;
#pragma unroll
  for (int a = 0; a < MR; ++a) {
    const int m = m0 + wm * TM + 16 * a + r;
#pragma unroll
    for (int b = 0; b < NR; ++b) {
      const v4f o4 = acc[a][b] + red[((qd * MR + a) * NR + b) * 64 + lane];
      const int n = n0 + wn * TN + 16 * b + 4 * h;
      if constexpr (OUT_F32) {
        *(v4f*)(P + (size_t)blockIdx.y * M * N + (size_t)m * N + n) = o4;
      } else {
        v4bf o;
#pragma unroll
        for (int i = 0; i < 4; ++i) o[i] = (bf16)o4[i];
        *(v4bf*)(C + (size_t)m * N + n) = o;
      }
    }
  }
}

// C = bf16(sum over s of P[s]) in split order; 8 elements per thread
__global__ __launch_bounds__(256) void splits_sum(const float4* __restrict__ P, int S, long long n8, v8bf* __restrict__ C) {
  const long long i = (long long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n8) return;
  float4 lo = P[2 * i], hi = P[2 * i + 1];
  for (int s = 1; s < S; ++s) {
    const float4 a = P[(size_t)s * 2 * n8 + 2 * i], b = P[(size_t)s * 2 * n8 + 2 * i + 1];
    lo.x += a.x; lo.y += a.y; lo.z += a.z; lo.w += a.w;
    hi.x += b.x; hi.y += b.y; hi.z += b.z; hi.w += b.w;
  }
  C[i] = v8bf{(bf16)lo.x, (bf16)lo.y, (bf16)lo.z, (bf16)lo.w, (bf16)hi.x, (bf16)hi.y, (bf16)hi.z, (bf16)hi.w};
}

// NS0 = 0: the deepest ring within ~144 KB of LDS (one workgroup per CU); else NS0 buffers (smaller rings let 2-3
// workgroups share a CU)
template <int BM, int BN, bool OUT_F32, int OPT, int NS0>
int launch(const void* A, const void* B, void* C, float* P, int M, int N, int T, int S, hipStream_t st) {
  constexpr int BUF = (BM + BN) * BK * 2;
  constexpr int NS = NS0 ? NS0 : ((147456 / BUF) < 8 ? (147456 / BUF) : 8);
  constexpr int LDS = NS * BUF;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)gemm_tn<BM, BN, OUT_F32, OPT, NS>,
                              hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    attr = true;
  }
  hipLaunchKernelGGL((gemm_tn<BM, BN, OUT_F32, OPT, NS>), dim3((M / BM) * (N / BN), S), dim3(256), LDS, st,
                     (const bf16*)A, (const bf16*)B, (bf16*)C, P, M, N, T, T / S);
  return (int)hipGetLastError();
}

template <bool OUT_F32>
int launch_k2(const void* A, const void* B, void* C, float* P, int M, int N, int T, int S, hipStream_t st) {
  constexpr int BUF = 2 * 96 * BK * 2, NS = 6, LDS = NS * BUF;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)gemm_tn_k2<OUT_F32, NS>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS);
    attr = true;
  }
  hipLaunchKernelGGL((gemm_tn_k2<OUT_F32, NS>), dim3((M / 96) * (N / 96), S), dim3(512), LDS, st, (const bf16*)A,
                     (const bf16*)B, (bf16*)C, P, M, N, T, T / S);
  return (int)hipGetLastError();
}

int dispatch_k2(const void* A, const void* B, void* C, float* P, int M, int N, int T, int S, hipStream_t st) {
  if (S == 1) return launch_k2<false>(A, B, C, nullptr, M, N, T, 1, st);
  const int rc = launch_k2<true>(A, B, nullptr, P, M, N, T, S, st);
  if (rc != 0) return rc;
  const long long n8 = (long long)M * N / 8;
  hipLaunchKernelGGL(splits_sum, dim3((unsigned)((n8 + 255) / 256)), dim3(256), 0, st, (const float4*)P, S, n8,
                     (v8bf*)C);
  return (int)hipGetLastError();
}

struct Cfg {
  int bm, bn, opt, ns;
};
constexpr Cfg kCfgs[] = {{96, 96, 0, 0},  {96, 96, 1, 0},   {128, 128, 0, 0}, {128, 96, 0, 0}, {96, 128, 0, 0},
                         {64, 64, 0, 0},  {128, 64, 0, 0},  {64, 128, 0, 0},  {96, 96, 0, 3},  {96, 96, 0, 2},
                         {128, 128, 0, 2}, {128, 128, 0, 3}, {64, 64, 0, 3},   {128, 64, 0, 3}, {64, 128, 0, 3},
                         {192, 192, 0, 3}, {192, 96, 0, 3},  {96, 192, 0, 3},  {96, 96, 2, 6},  {96, 96, 1, 2},
                         {128, 128, 1, 2}};

template <int BM, int BN, int OPT, int NS0 = 0>
int dispatch(const void* A, const void* B, void* C, float* P, int M, int N, int T, int S, hipStream_t st) {
  if (S == 1) return launch<BM, BN, false, OPT, NS0>(A, B, C, nullptr, M, N, T, 1, st);
  const int rc = launch<BM, BN, true, OPT, NS0>(A, B, nullptr, P, M, N, T, S, st);
  if (rc != 0) return rc;
  const long long n8 = (long long)M * N / 8;
  hipLaunchKernelGGL(splits_sum, dim3((unsigned)((n8 + 255) / 256)), dim3(256), 0, st, (const float4*)P, S, n8,
                     (v8bf*)C);
  return (int)hipGetLastError();
}

}  // namespace

extern "C" {

// tile configurations: out[3 i] = BM, out[3 i + 1] = BN, out[3 i + 2] = OPT bits + 16 x ring depth (0: deepest)
int mifx_gemm_tn_configs(int* out, int n) {
  const int m = (int)(sizeof(kCfgs) / sizeof(Cfg));
  for (int i = 0; i < m && 3 * i + 2 < n; ++i) {
    out[3 * i] = kCfgs[i].bm;
    out[3 * i + 1] = kCfgs[i].bn;
    out[3 * i + 2] = kCfgs[i].opt + 16 * kCfgs[i].ns;
  }
  return m;
}

// C[M, N] (bf16) = A[T, M]^T . B[T, N] (bf16, row-major, fp32 accumulation). S > 1 splits T over S workgroup rows
// with fp32 partials P [S, M, N] summed in split order. Requires M % BM == 0, N % BN == 0, T % (64 S) == 0,
// 16-byte aligned rows (M % 8 == 0, N % 8 == 0 follow).
int mifx_gemm_tn(int cfg, const void* A, const void* B, void* C, float* P, int M, int N, int T, int S,
                 hipStream_t st) {
  const int m = (int)(sizeof(kCfgs) / sizeof(Cfg));
  if (cfg < 0 || cfg >= m || M <= 0 || N <= 0 || T <= 0 || S <= 0 || A == nullptr || B == nullptr || C == nullptr)
    return -1;
  const Cfg c = kCfgs[cfg];
  if (M % c.bm || N % c.bn || T % (BK * S)) return -1;
  if (S > 1 && P == nullptr) return -1;
  if ((uintptr_t)A % 16 || (uintptr_t)B % 16 || (uintptr_t)C % 16 || (P != nullptr && (uintptr_t)P % 16)) return -1;
  if ((long long)T * M >= (1ll << 31) || (long long)T * N >= (1ll << 31)) return -1;  // 32-bit element offsets
  switch (cfg) {
    case 0: return dispatch<96, 96, 0>(A, B, C, P, M, N, T, S, st);
    case 1: return dispatch<96, 96, 1>(A, B, C, P, M, N, T, S, st);
    case 2: return dispatch<128, 128, 0>(A, B, C, P, M, N, T, S, st);
    case 3: return dispatch<128, 96, 0>(A, B, C, P, M, N, T, S, st);
    case 4: return dispatch<96, 128, 0>(A, B, C, P, M, N, T, S, st);
    case 5: return dispatch<64, 64, 0>(A, B, C, P, M, N, T, S, st);
    case 6: return dispatch<128, 64, 0>(A, B, C, P, M, N, T, S, st);
    case 7: return dispatch<64, 128, 0>(A, B, C, P, M, N, T, S, st);
    case 8: return dispatch<96, 96, 0, 3>(A, B, C, P, M, N, T, S, st);
    case 9: return dispatch<96, 96, 0, 2>(A, B, C, P, M, N, T, S, st);
    case 10: return dispatch<128, 128, 0, 2>(A, B, C, P, M, N, T, S, st);
    case 11: return dispatch<128, 128, 0, 3>(A, B, C, P, M, N, T, S, st);
    case 12: return dispatch<64, 64, 0, 3>(A, B, C, P, M, N, T, S, st);
    case 13: return dispatch<128, 64, 0, 3>(A, B, C, P, M, N, T, S, st);
    case 14: return dispatch<64, 128, 0, 3>(A, B, C, P, M, N, T, S, st);
    case 15: return dispatch<192, 192, 0, 3>(A, B, C, P, M, N, T, S, st);
    case 16: return dispatch<192, 96, 0, 3>(A, B, C, P, M, N, T, S, st);
    case 17: return dispatch<96, 192, 0, 3>(A, B, C, P, M, N, T, S, st);
    case 18: return dispatch_k2(A, B, C, P, M, N, T, S, st);  // 8 waves, k-steps split over wave pairs
    case 19: return dispatch<96, 96, 1, 2>(A, B, C, P, M, N, T, S, st);
    default: return dispatch<128, 128, 1, 2>(A, B, C, P, M, N, T, S, st);
  }
}

}  // extern "C"
