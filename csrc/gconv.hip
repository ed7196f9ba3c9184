// Grouped convolution as an implicit GEMM on bf16 MFMA (NHWC): forward (any stride), input gradient (stride 1:
// the forward kernel on the flipped weight; stride > 1: a phase-split kernel), weight gradient (any stride).
//
// Reference workload: the PATE-2017 `deep_cnn.inference` CNN (5x5 convs 64/128 channels,
// `research/pate_2017/deep_cnn.py:84-191`) trained for every teacher of the ensemble
// (`train_teachers.py:44-96`). `mifx/privacy/pate/ensemble.py` trains all teachers at once as ONE grouped
// network (group g = teacher g), and MIOpen's grouped NHWC solvers run those shapes (G = 250 groups of
// 64 -> 128 channels, 5x5, 14x14, B = 128) at 20-40 TFLOP/s. Here each group is an implicit GEMM:
//   y[m = (n,p,q), g*K + k] = b[g*K + k] + sum_{r,s,c} x[n, p+r-pad, q+s-pad, g*C + c] * w[g][k][r][s][c]
// with M = N*Ho*Wo output pixels, N_gemm = K output channels, reduction = R*S*C ordered tap-major, so a
// 32-wide reduction chunk is 32 contiguous channels of one input pixel (one 64-byte row).
//
//  * Tiles: 128 pixels x BN channels (BN = 128 or 64) per 256-thread workgroup; 4 waves, each 64 x BN/2, on
//    v_mfma_f32_16x16x32_bf16 with fp32 accumulators. A (pixel rows, zero-filled outside the image) and B
//    (weight rows [k][tap][c]) chunks are staged global -> registers -> LDS, double-buffered (one barrier
//    per 32-wide chunk); LDS rows are padded to 80 bytes so the 16-byte fragment reads are conflict-free.
//  * Grid (pixel tiles, K / BN, G): tiles of one group are consecutive, so a group's weights and its input
//    halo rows are reused from L2 while they are hot.
//  * The input gradient of a stride-1 convolution is the same operation on dy with the weight flipped
//    spatially and transposed ([g][c][R-1-r][S-1-s][k]) and pad' = R-1-pad, so one kernel serves both.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

typedef __bf16 bf16;
typedef __bf16 v8bf __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));
typedef unsigned int u4 __attribute__((ext_vector_type(4)));

constexpr int kThreads = 256;
constexpr int BM = 128, BK = 32, LDR = 40;  // LDS row: 32 bf16 + 8 pad (80 B)

__device__ __forceinline__ v4f mfma(v8bf a, v8bf b, v4f c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

struct Geo {
  int N, Hi, Wi, Ho, Wo, G, C, K, R, S, pad, stride;
};

// optional residual epilogue (inference of a pre-activation block): y = bf16(bf16(conv + bias) + res) and
// y2 = bf16(relu(y * scale2 + shift2)) -- the residual sum and the next block's BatchNorm + ReLU, rounded exactly as
// the separate add and csrc/bn_relu.hip apply kernels round them
struct ResEpi {
  const bf16* res;      // [M, G*K] like y, or null
  const float* scale2;  // [G*K] (with y2)
  const float* shift2;
  bf16* y2;             // or null
};

// one 16-byte output chunk (8 channels from c) through the residual epilogue; returns the chunk for y
__device__ __forceinline__ u4 res_epi(u4 v, const ResEpi& re, size_t off, int c) {
  if (re.res == nullptr) return v;
  const u4 r = *(const u4*)(re.res + off);
  v8bf a = __builtin_bit_cast(v8bf, v), b = __builtin_bit_cast(v8bf, r), o2;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    a[e] = (bf16)((float)a[e] + (float)b[e]);
    if (re.y2 != nullptr) o2[e] = (bf16)fmaxf(fmaf((float)a[e], re.scale2[c + e], re.shift2[c + e]), 0.f);
  }
  if (re.y2 != nullptr) *(v8bf*)(re.y2 + off) = o2;
  return __builtin_bit_cast(u4, a);
}

// amdgpu_waves_per_eu(4): 4 workgroups per CU (40 KB LDS each) -- the loop is latency-bound, occupancy pays
// (profiles/archive/gconv_bk_ab_r2.txt, gconv_prefetch_ab_r2.txt: deeper prefetch / wider chunks that cost occupancy lose)
// ksplit > 1 (few pixel tiles, e.g. batch-1 inference): blockIdx.z = g * ksplit + split, the workgroup reduces
// steps [nsteps split / ksplit, nsteps (split + 1) / ksplit) and writes its fp32 partial to part[split][M][G*K]
// (gconv_splitk_finish adds the splits in order, + bias, ReLU)
template <int BN>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(4, 8))) void gconv_fwd(const bf16* __restrict__ x, const bf16* __restrict__ w,
                                                      const float* __restrict__ bias, bf16* __restrict__ y, Geo d,
                                                      int relu, float* __restrict__ part, int ksplit, ResEpi re) {
  constexpr int BCH = (BN * 4 + kThreads - 1) / kThreads;  // 16-byte weight chunks per thread per step (2, 1, 1)
  // one LDS block: double-buffered A and B staging, reused as the epilogue's output tile
  __shared__ __attribute__((aligned(16))) bf16 smem[2 * BM * LDR + 2 * BN * LDR];
  bf16(*As)[BM * LDR] = reinterpret_cast<bf16(*)[BM * LDR]>(smem);
  bf16(*Bs)[BN * LDR] = reinterpret_cast<bf16(*)[BN * LDR]>(smem + 2 * BM * LDR);
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int g = (int)blockIdx.z / ksplit, split = (int)blockIdx.z - g * ksplit, n0 = blockIdx.y * BN;
  const long long M = (long long)d.N * d.Ho * d.Wo;
  const long long m0 = (long long)blockIdx.x * BM;
  const int CT = d.G * d.C;  // input row stride (channels)
  const int chunks_c = d.C / BK, nsteps_all = d.R * d.S * chunks_c;
  const int s_begin = (int)((long long)nsteps_all * split / ksplit);
  const int s_end = (int)((long long)nsteps_all * (split + 1) / ksplit);

  // this thread's two A chunks: pixel rows ap[j] = (t >> 2) + 64 j, 16-byte part (t & 3)
  int an[2], ah[2], aw[2];
  bool am[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const long long m = m0 + (t >> 2) + 64 * j;
    am[j] = m < M;
    const long long mm = am[j] ? m : 0;
    aw[j] = (int)(mm % d.Wo);
    ah[j] = (int)((mm / d.Wo) % d.Ho);
    an[j] = (int)(mm / ((long long)d.Wo * d.Ho));
  }
  const int apart = (t & 3) * 8;
  const bf16* wg = w + (size_t)g * d.K * d.R * d.S * d.C;

  u4 ra[2], rb[BCH];
  auto load = [&](int step) {
    const int tap = step / chunks_c, c0 = (step - tap * chunks_c) * BK;
    const int r = tap / d.S, s = tap - r * d.S;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int hh = ah[j] * d.stride + r - d.pad, ww = aw[j] * d.stride + s - d.pad;
      if (am[j] && hh >= 0 && hh < d.Hi && ww >= 0 && ww < d.Wi) {
        const bf16* src = x + ((size_t)(an[j] * d.Hi + hh) * d.Wi + ww) * CT + g * d.C + c0 + apart;
        ra[j] = *(const u4*)src;
      } else {
        ra[j] = u4{0, 0, 0, 0};
      }
    }
#pragma unroll
    for (int j = 0; j < BCH; ++j) {
      const int c = t + kThreads * j, k = c >> 2, part = (c & 3) * 8;
      if ((BN * 4) % kThreads == 0 || c < BN * 4) rb[j] = *(const u4*)(wg + ((size_t)(n0 + k) * d.R * d.S + tap) * d.C + c0 + part);
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int j = 0; j < 2; ++j) *(u4*)(&As[buf][((t >> 2) + 64 * j) * LDR + apart]) = ra[j];
#pragma unroll
    for (int j = 0; j < BCH; ++j) {
      const int c = t + kThreads * j;
      if ((BN * 4) % kThreads == 0 || c < BN * 4) *(u4*)(&Bs[buf][(c >> 2) * LDR + (c & 3) * 8]) = rb[j];
    }
  };

  constexpr int TN = BN / 32;  // 16-wide column tiles per wave (wave owns BN/2 columns; BN = 32: one tile)
  v4f acc[4][TN];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};
  const int wm = (wv >> 1) * 64, wn = (wv & 1) * (BN / 2);
  const int fr = lane & 15, fk = (lane >> 4) * 8;

  load(s_begin);
  store(0);
  __syncthreads();
  for (int step = s_begin; step < s_end; ++step) {
    const int buf = (step - s_begin) & 1;
    if (step + 1 < s_end) load(step + 1);
    v8bf af[4], bfr[TN];
#pragma unroll
    for (int i = 0; i < 4; ++i) af[i] = *(const v8bf*)(&As[buf][(wm + 16 * i + fr) * LDR + fk]);
#pragma unroll
    for (int j = 0; j < TN; ++j) bfr[j] = *(const v8bf*)(&Bs[buf][(wn + 16 * j + fr) * LDR + fk]);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = mfma(af[i], bfr[j], acc[i][j]);
    if (step + 1 < s_end) store(buf ^ 1);
    __syncthreads();
  }

  if (part != nullptr) {  // split-K: this split's fp32 partial (bias / ReLU in gconv_splitk_finish)
    const int KT = d.G * d.K;
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int ch = g * d.K + n0 + wn + 16 * j + fr;
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const long long m = m0 + wm + 16 * i + 4 * (lane >> 4) + e;
          if (m < M) part[((size_t)split * M + m) * KT + ch] = acc[i][j][e];
        }
    }
    return;
  }

  // epilogue: acc[i][j][e] = y[pixel m0 + wm + 16 i + 4 (lane >> 4) + e][channel n0 + wn + 16 j + (lane & 15)].
  // (+ bias, optional ReLU) -> bf16 tile in LDS (the staging buffers are free after the last barrier), then
  // 16-byte coalesced row stores: a pixel's BN channels are contiguous in y.
  constexpr int CLD = BN + 8;
  static_assert(BM * CLD <= 2 * BM * LDR + 2 * BN * LDR, "epilogue tile fits the staging buffers");
  bf16* Cs = smem;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int cl = wn + 16 * j + fr;
    const float b = bias ? bias[g * d.K + n0 + cl] : 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float v = acc[i][j][e] + b;
        if (relu) v = fmaxf(v, 0.f);
        Cs[(wm + 16 * i + 4 * (lane >> 4) + e) * CLD + cl] = (bf16)v;
      }
  }
  __syncthreads();
  const int KT = d.G * d.K;
  constexpr int CPR = BN / 8;  // 16-byte chunks per pixel row
  for (int c = t; c < BM * CPR; c += kThreads) {
    const int row = c / CPR, part = (c % CPR) * 8;
    const long long m = m0 + row;
    if (m < M) {
      const size_t off = (size_t)m * KT + g * d.K + n0 + part;
      *(u4*)(y + off) = res_epi(*(const u4*)(&Cs[row * CLD + part]), re, off, g * d.K + n0 + part);
    }
  }
}

// y = bf16(relu(sum over splits of part[s] + bias)), splits added in order; 8 channels per thread
__global__ __launch_bounds__(kThreads) void gconv_splitk_finish(const float* __restrict__ part, int ksplit, long long M,
                                                               int KT, const float* __restrict__ bias, int relu,
                                                               bf16* __restrict__ y, ResEpi re) {
  const long long i = (long long)blockIdx.x * kThreads + threadIdx.x;
  if (i >= M * KT / 8) return;
  const size_t base = (size_t)i * 8;
  float a[8];
  {
    const float4 lo = *(const float4*)(part + base), hi = *(const float4*)(part + base + 4);
    a[0] = lo.x, a[1] = lo.y, a[2] = lo.z, a[3] = lo.w, a[4] = hi.x, a[5] = hi.y, a[6] = hi.z, a[7] = hi.w;
  }
  for (int s = 1; s < ksplit; ++s) {
    const float* p = part + (size_t)s * M * KT + base;
    const float4 lo = *(const float4*)p, hi = *(const float4*)(p + 4);
    a[0] += lo.x, a[1] += lo.y, a[2] += lo.z, a[3] += lo.w, a[4] += hi.x, a[5] += hi.y, a[6] += hi.z, a[7] += hi.w;
  }
  const int c = (int)(base % KT);
  v8bf o;
#pragma unroll
  for (int e = 0; e < 8; ++e) {
    float v = a[e] + (bias ? bias[c + e] : 0.f);
    if (relu) v = fmaxf(v, 0.f);
    o[e] = (bf16)v;
  }
  *(u4*)(y + base) = res_epi(__builtin_bit_cast(u4, o), re, base, c);
}

// ---- input gradient of a STRIDED convolution -----------------------------------------------------------
// dx[n, h, w, g*C + c] = sum over taps (r, s) with (h + pad - r) % st == 0 and (w + pad - s) % st == 0 of
//   dy[n, (h + pad - r) / st, (w + pad - s) / st, g*K + k] * w[g][k][c][r][s].
// Split by output phase (h % st, w % st): inside a phase every pixel takes the SAME taps
// (r = r0 + st a, r0 = (ph + pad) % st; likewise s), and the dy row of tap a is p = i - a + bh for dx row
// h = ph + st i (bh = (ph + pad - r0) / st) -- a stride-1 implicit GEMM per phase with no wasted (zero) taps.
// blockIdx.z = g * st^2 + phase, pixel tiles are phase-major (pixels of one tile share the phase), reduction =
// (phase taps) x K in 32-wide chunks; same tile / LDS / MFMA structure as gconv_fwd. Weight image: the transposed
// (unflipped) [G][C][R][S][K] layout; dx rows are scattered back to (n, h, w) in the epilogue.
template <int BN>
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(4, 8))) void gconv_dgrad_s(
    const bf16* __restrict__ dy, const bf16* __restrict__ wt, bf16* __restrict__ dx, Geo d) {
  constexpr int BCH = (BN * 4 + kThreads - 1) / kThreads;
  __shared__ __attribute__((aligned(16))) bf16 smem[2 * BM * LDR + 2 * BN * LDR];
  bf16(*As)[BM * LDR] = reinterpret_cast<bf16(*)[BM * LDR]>(smem);
  bf16(*Bs)[BN * LDR] = reinterpret_cast<bf16(*)[BN * LDR]>(smem + 2 * BM * LDR);
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int st = d.stride, nph = st * st;
  const int g = blockIdx.z / nph, ph = (blockIdx.z % nph) / st, pw = blockIdx.z % st;
  const int n0 = blockIdx.y * BN;
  const int Hp = (d.Hi - ph + st - 1) / st, Wp = (d.Wi - pw + st - 1) / st;  // dx rows / cols of this phase
  const long long Mp = (long long)d.N * Hp * Wp;
  const long long m0 = (long long)blockIdx.x * BM;
  if (Hp <= 0 || Wp <= 0 || m0 >= Mp) return;
  const int r0 = (ph + d.pad) % st, s0 = (pw + d.pad) % st;
  const int Ra = r0 < d.R ? (d.R - r0 + st - 1) / st : 0, Sa = s0 < d.S ? (d.S - s0 + st - 1) / st : 0;
  const int bh = (ph + d.pad - r0) / st, bw = (pw + d.pad - s0) / st;
  const int KT = d.G * d.K;  // dy row stride (channels)
  const int chunks_k = d.K / BK, nsteps = Ra * Sa * chunks_k;

  int an[2], ai[2], aj[2];
  bool am[2];
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const long long m = m0 + (t >> 2) + 64 * j;
    am[j] = m < Mp;
    const long long mm = am[j] ? m : 0;
    aj[j] = (int)(mm % Wp);
    ai[j] = (int)((mm / Wp) % Hp);
    an[j] = (int)(mm / ((long long)Wp * Hp));
  }
  const int apart = (t & 3) * 8;
  const bf16* wg = wt + (size_t)g * d.C * d.R * d.S * d.K;

  u4 ra[2], rb[BCH];
  auto load = [&](int step) {
    const int tap = step / chunks_k, k0 = (step - tap * chunks_k) * BK;
    const int a = tap / Sa, b = tap - a * Sa;
    const int r = r0 + st * a, s = s0 + st * b;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int p = ai[j] - a + bh, q = aj[j] - b + bw;
      if (am[j] && p >= 0 && p < d.Ho && q >= 0 && q < d.Wo) {
        ra[j] = *(const u4*)(dy + ((size_t)(an[j] * d.Ho + p) * d.Wo + q) * KT + g * d.K + k0 + apart);
      } else {
        ra[j] = u4{0, 0, 0, 0};
      }
    }
#pragma unroll
    for (int j = 0; j < BCH; ++j) {
      const int c = t + kThreads * j, cr = c >> 2, part = (c & 3) * 8;
      if ((BN * 4) % kThreads == 0 || c < BN * 4)
        rb[j] = *(const u4*)(wg + (((size_t)(n0 + cr) * d.R + r) * d.S + s) * d.K + k0 + part);
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int j = 0; j < 2; ++j) *(u4*)(&As[buf][((t >> 2) + 64 * j) * LDR + apart]) = ra[j];
#pragma unroll
    for (int j = 0; j < BCH; ++j) {
      const int c = t + kThreads * j;
      if ((BN * 4) % kThreads == 0 || c < BN * 4) *(u4*)(&Bs[buf][(c >> 2) * LDR + (c & 3) * 8]) = rb[j];
    }
  };

  constexpr int TN = BN / 32;
  v4f acc[4][TN];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};
  const int wm = (wv >> 1) * 64, wn = (wv & 1) * (BN / 2);
  const int fr = lane & 15, fk = (lane >> 4) * 8;

  if (nsteps > 0) {
    load(0);
    store(0);
  }
  __syncthreads();
  for (int step = 0; step < nsteps; ++step) {
    const int buf = step & 1;
    if (step + 1 < nsteps) load(step + 1);
    v8bf af[4], bfr[TN];
#pragma unroll
    for (int i = 0; i < 4; ++i) af[i] = *(const v8bf*)(&As[buf][(wm + 16 * i + fr) * LDR + fk]);
#pragma unroll
    for (int j = 0; j < TN; ++j) bfr[j] = *(const v8bf*)(&Bs[buf][(wn + 16 * j + fr) * LDR + fk]);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = mfma(af[i], bfr[j], acc[i][j]);
    if (step + 1 < nsteps) store(buf ^ 1);
    __syncthreads();
  }

  constexpr int CLD = BN + 8;
  static_assert(BM * CLD <= 2 * BM * LDR + 2 * BN * LDR, "epilogue tile fits the staging buffers");
  bf16* Cs = smem;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int cl = wn + 16 * j + fr;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) Cs[(wm + 16 * i + 4 * (lane >> 4) + e) * CLD + cl] = (bf16)acc[i][j][e];
  }
  __syncthreads();
  const int CT = d.G * d.C;
  constexpr int CPR = BN / 8;
  for (int c = t; c < BM * CPR; c += kThreads) {
    const int row = c / CPR, part = (c % CPR) * 8;
    const long long m = m0 + row;
    if (m < Mp) {
      const int jj = (int)(m % Wp), ii = (int)((m / Wp) % Hp), nn = (int)(m / ((long long)Wp * Hp));
      const int h = ph + st * ii, w = pw + st * jj;
      *(u4*)(dx + ((size_t)(nn * d.Hi + h) * d.Wi + w) * CT + g * d.C + n0 + part) = *(const u4*)(&Cs[row * CLD + part]);
    }
  }
}

// ---- weight gradient ------------------------------------------------------------------------------------
// dw[g*K + k][c][r][s] = sum_m dy[m][g*K + k] * x[pixel(m) + (r - pad, s - pad)][g*C + c]: a GEMM of
// 128 k-rows x 128 (tap, c) columns per workgroup (the flattened tap-major column space), reduced over output pixels m in
// chunks of 32. Both operands arrive pixel-major (channels contiguous), so the chunks are staged as
// [32 pixels][128] bf16 images (rows padded to 288 B) and the MFMA fragments, which need 8 consecutive reduction
// elements per lane, come from ds_read_b64_tr_b16 transposed reads. The reduction order inside a 32-chunk is
// permuted identically for both operands (element j of lane group g <-> pixel row 4g + j for j < 4,
// 16 + 4g + j - 4 for j >= 4), which makes every transposed read conflict-free.
typedef short v4s __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4s lds_v4s;
constexpr int WLD = 144;  // LDS row (bf16 elements): 128 + 16 pad = 288 B

__device__ __forceinline__ v4s tr_read(const bf16* p) { return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)p); }
__device__ __forceinline__ v8bf cat8(v4s a, v4s b) {
  const v4s r0 = a, r1 = b;
  typedef short v8s __attribute__((ext_vector_type(8)));
  const v8s r = {r0[0], r0[1], r0[2], r0[3], r1[0], r1[1], r1[2], r1[3]};
  return __builtin_bit_cast(v8bf, r);
}

// Split over output pixels (splits > 1, blockIdx.z = g * splits + split): few (tap, k, group) tiles -- a single
// group, e.g. ResNet-50's convs -- would leave most CUs idle, so the pixel reduction is cut into `splits` ranges of
// whole 32-pixel chunks; each writes its partial dW into part[split] and gconv_wgrad_sum adds the splits in split
// order (deterministic: no atomics).
__global__ __launch_bounds__(kThreads) __attribute__((amdgpu_waves_per_eu(4, 8))) void gconv_wgrad(const bf16* __restrict__ x, const bf16* __restrict__ dy,
                                                        float* __restrict__ dw, Geo d, int splits) {
  __shared__ __attribute__((aligned(16))) bf16 As[2][32 * WLD];  // dy chunk [pixel][k]
  __shared__ __attribute__((aligned(16))) bf16 Bs[2][32 * WLD];  // x chunk [pixel][(tap, c)]
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int g = blockIdx.z / splits, sp = blockIdx.z - g * splits, k0 = blockIdx.y * 128;
  const int RS = d.R * d.S, col0 = blockIdx.x * 128;  // 128 columns of the flattened (tap, c) space
  const long long M = (long long)d.N * d.Ho * d.Wo;
  const int KT = d.G * d.K, CT = d.G * d.C;
  const int total = (int)((M + 31) / 32), per = (total + splits - 1) / splits;
  const int s_begin = sp * per, nsteps = max(0, min(total, s_begin + per) - s_begin);
  if (splits > 1) dw += (size_t)sp * d.G * d.K * d.C * RS;  // this split's partial
  // this thread's chunks: pixel rows pr[j] = (t >> 4) + 16 j, 16-byte chunk (t & 15) of the 256-byte row
  const int ch = t & 15;
  const int bcol = col0 + ch * 8;  // C % 8 == 0: an 8-channel chunk never straddles two taps
  const bool btap_ok = bcol < RS * d.C;
  const int btap = bcol / d.C, bc = bcol - btap * d.C;
  const int br = btap / d.S, bs = btap - br * d.S;

  u4 ra[2], rb[2];
  auto load = [&](int step) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const long long m = (long long)(s_begin + step) * 32 + (t >> 4) + 16 * j;
      ra[j] = u4{0, 0, 0, 0};
      rb[j] = u4{0, 0, 0, 0};
      if (m < M) {
        if (k0 + ch * 8 < d.K) ra[j] = *(const u4*)(dy + m * KT + g * d.K + k0 + ch * 8);
        const int q = (int)(m % d.Wo), p = (int)((m / d.Wo) % d.Ho), n = (int)(m / ((long long)d.Wo * d.Ho));
        const int hh = p * d.stride + br - d.pad, ww = q * d.stride + bs - d.pad;
        if (btap_ok && hh >= 0 && hh < d.Hi && ww >= 0 && ww < d.Wi)
          rb[j] = *(const u4*)(x + ((size_t)(n * d.Hi + hh) * d.Wi + ww) * CT + g * d.C + bc);
      }
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int row = (t >> 4) + 16 * j;
      *(u4*)(&As[buf][row * WLD + ch * 8]) = ra[j];
      *(u4*)(&Bs[buf][row * WLD + ch * 8]) = rb[j];
    }
  };

  v4f acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = v4f{0.f, 0.f, 0.f, 0.f};
  const int wm = (wv >> 1) * 64, wn = (wv & 1) * 64;
  // transposed-read address of lane 4q + p of its 16-lane group G: rows 4G + q (and 16 + 4G + q), cols 4p..4p+3
  const int grp = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int rd_row = 4 * grp + q, rd_col = 4 * p;

  if (nsteps > 0) {
    load(0);
    store(0);
  }
  __syncthreads();
  for (int step = 0; step < nsteps; ++step) {
    const int buf = step & 1;
    if (step + 1 < nsteps) load(step + 1);
    v8bf af[4], bfr[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const bf16* pa = &As[buf][rd_row * WLD + wm + 16 * i + rd_col];
      af[i] = cat8(tr_read(pa), tr_read(pa + 16 * WLD));
      const bf16* pb = &Bs[buf][rd_row * WLD + wn + 16 * i + rd_col];
      bfr[i] = cat8(tr_read(pb), tr_read(pb + 16 * WLD));
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = mfma(af[i], bfr[j], acc[i][j]);
    if (step + 1 < nsteps) store(buf ^ 1);
    __syncthreads();
  }

  // acc[i][j][e]: k = k0 + wm + 16 i + 4 (lane >> 4) + e, column wn + 16 j + (lane & 15) = (tap, c)
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int col = col0 + wn + 16 * j + (lane & 15);
    if (col >= RS * d.C) continue;
    const int tap = col / d.C, c = col - tap * d.C;
    const int r = tap / d.S, s = tap - r * d.S;
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int k = k0 + wm + 16 * i + 4 * (lane >> 4) + e;
        if (k < d.K) dw[(((size_t)(g * d.K + k) * d.C + c) * d.R + r) * d.S + s] = acc[i][j][e];
      }
  }
}

// dw[i] = sum over splits (in split order) of part[split][i]
__global__ __launch_bounds__(256) void gconv_wgrad_sum(const float4* __restrict__ part, long long n4, int splits,
                                                       float4* __restrict__ dw) {
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n4; i += (long long)gridDim.x * 256) {
    float4 a = part[i];
    for (int s = 1; s < splits; ++s) {
      const float4 v = part[(size_t)s * n4 + i];
      a.x += v.x; a.y += v.y; a.z += v.z; a.w += v.w;
    }
    dw[i] = a;
  }
}

}  // namespace

extern "C" {

// pixel splits the weight gradient takes for a shape: ~1024 workgroups (4 per CU: the kernel's occupancy) when the
// pixel count allows, every split >= 16 chunks of 32 pixels, at most 256 splits and 64 M floats of partials; the
// caller provides splits x |dw| floats of scratch when it is > 1
int mifx_gconv_wgrad_splits(int N, int Hi, int Wi, int G, int C, int K, int R, int S, int pad, int stride) {
  if (stride <= 0) return 1;
  const long long Ho = (Hi + 2 * pad - R) / stride + 1, Wo = (Wi + 2 * pad - S) / stride + 1;
  const long long tiles = (long long)((R * S * C + 127) / 128) * ((K + 127) / 128) * G;
  const long long chunks = ((long long)N * Ho * Wo + 31) / 32;
  const long long dwn = (long long)G * K * C * R * S;
  long long sp = (1024 + tiles - 1) / tiles;
  sp = sp < chunks / 16 ? sp : chunks / 16;
  sp = sp < 256 ? sp : 256;
  while (sp > 1 && sp * dwn > (64ll << 20)) --sp;
  return (int)(sp > 1 ? sp : 1);
}

// dw [G*K][C][R][S] fp32 (PyTorch layout) from x [N, Hi, Wi, G*C] and dy [N, Ho, Wo, G*K] bf16 (NHWC).
// Needs C % 8 == 0 and K % 8 == 0 (tiles of 128 k x 128 (tap, c) columns; partial last tiles are masked).
// splits / part: mifx_gconv_wgrad_splits(...) and its scratch (part may be null when splits == 1).
int mifx_gconv_wgrad(const void* x, const void* dy, float* dw, int N, int Hi, int Wi, int G, int C, int K, int R,
                     int S, int pad, int stride, int splits, float* part, hipStream_t st) {
  if (stride <= 0) return -1;
  const int Ho = (Hi + 2 * pad - R) / stride + 1, Wo = (Wi + 2 * pad - S) / stride + 1;
  if (N <= 0 || G <= 0 || C <= 0 || C % 8 != 0 || K <= 0 || K % 8 != 0 || Hi + 2 * pad < R ||
      Wi + 2 * pad < S || pad < 0 || pad >= R || pad >= S || splits < 1 || (splits > 1 && part == nullptr))
    return -1;
  if ((long long)N * Ho * Wo > 0x3fffffffLL || (long long)G * splits > 65535) return -1;
  const Geo d{N, Hi, Wi, Ho, Wo, G, C, K, R, S, pad, stride};
  hipLaunchKernelGGL(gconv_wgrad, dim3((R * S * C + 127) / 128, (K + 127) / 128, G * splits), dim3(kThreads), 0, st,
                     (const bf16*)x, (const bf16*)dy, splits > 1 ? part : dw, d, splits);
  if (splits > 1) {
    const long long n4 = (long long)G * K * C * R * S / 4;  // C % 8 == 0: divisible
    const long long blocks = (n4 + 255) / 256;
    hipLaunchKernelGGL(gconv_wgrad_sum, dim3((unsigned)(blocks < 4096 ? blocks : 4096)), dim3(256), 0, st,
                       (const float4*)part, n4, splits, (float4*)dw);
  }
  return (int)hipGetLastError();
}

// Input gradient of a convolution with stride >= 1: dy [N, Ho, Wo, G*K] bf16, wt [G][C][R][S][K] bf16 (the weight
// transposed, NOT flipped), dx [N, Hi, Wi, G*C] bf16 (every element written). Needs C % 32 == 0, K % 32 == 0.
int mifx_gconv_dgrad_strided(const void* dy, const void* wt, void* dx, int N, int Hi, int Wi, int G, int C, int K,
                             int R, int S, int pad, int stride, hipStream_t st) {
  if (stride <= 0 || stride > 8) return -1;
  const int Ho = (Hi + 2 * pad - R) / stride + 1, Wo = (Wi + 2 * pad - S) / stride + 1;
  if (N <= 0 || G <= 0 || C <= 0 || C % 32 != 0 || K <= 0 || K % BK != 0 || Hi + 2 * pad < R || Wi + 2 * pad < S ||
      pad < 0 || pad >= R || pad >= S || Ho <= 0 || Wo <= 0)
    return -1;
  if ((long long)G * stride * stride > 65535) return -1;
  const Geo d{N, Hi, Wi, Ho, Wo, G, C, K, R, S, pad, stride};
  const long long Hp = (Hi + stride - 1) / stride, Wp = (Wi + stride - 1) / stride;  // the largest phase
  const long long mt = ((long long)N * Hp * Wp + BM - 1) / BM;
  if (mt > 0x7fffffffLL) return -1;
  const dim3 z((unsigned)mt, 1, (unsigned)(G * stride * stride));
  if (C % 128 == 0)
    hipLaunchKernelGGL(gconv_dgrad_s<128>, dim3(z.x, C / 128, z.z), dim3(kThreads), 0, st, (const bf16*)dy,
                       (const bf16*)wt, (bf16*)dx, d);
  else if (C % 64 == 0)
    hipLaunchKernelGGL(gconv_dgrad_s<64>, dim3(z.x, C / 64, z.z), dim3(kThreads), 0, st, (const bf16*)dy,
                       (const bf16*)wt, (bf16*)dx, d);
  else
    hipLaunchKernelGGL(gconv_dgrad_s<32>, dim3(z.x, C / 32, z.z), dim3(kThreads), 0, st, (const bf16*)dy,
                       (const bf16*)wt, (bf16*)dx, d);
  return (int)hipGetLastError();
}

// x [N, Hi, Wi, G*C] bf16, w [G][K][R][S][C] bf16, bias [G*K] fp32 or null, y [N, Ho, Wo, G*K] bf16;
// zero padding `pad` on every side, Ho = (Hi + 2 pad - R) / stride + 1, relu != 0: y = max(y, 0).
// Needs C % 32 == 0 and K % 32 == 0.
// res / scale2 / shift2 / y2 (nullable): the residual epilogue (ResEpi) -- y = conv (+ bias, ReLU) + res, and
// y2 = relu(y * scale2 + shift2)
int mifx_gconv_fwd_ex(const void* x, const void* w, const float* bias, void* y, int N, int Hi, int Wi, int G, int C,
                      int K, int R, int S, int pad, int stride, int relu, float* part, int ksplit, const void* res,
                      const float* scale2, const float* shift2, void* y2, hipStream_t st) {
  if (stride <= 0 || ksplit <= 0 || (ksplit > 1 && part == nullptr)) return -1;
  if (y2 != nullptr && (res == nullptr || scale2 == nullptr || shift2 == nullptr)) return -1;
  const ResEpi re{(const bf16*)res, scale2, shift2, (bf16*)y2};
  const int Ho = (Hi + 2 * pad - R) / stride + 1, Wo = (Wi + 2 * pad - S) / stride + 1;
  if (N <= 0 || G <= 0 || (long long)G * ksplit > 65535 || C <= 0 || C % BK != 0 || K <= 0 || K % 32 != 0 ||
      Hi + 2 * pad < R || Wi + 2 * pad < S || pad < 0 || pad >= R || pad >= S || ksplit > R * S * (C / BK))
    return -1;
  const Geo d{N, Hi, Wi, Ho, Wo, G, C, K, R, S, pad, stride};
  const long long M = (long long)N * Ho * Wo;
  const long long mt = (M + BM - 1) / BM;
  if (mt > 0x7fffffffLL) return -1;
  float* pp = ksplit > 1 ? part : nullptr;
  const unsigned gz = (unsigned)(G * ksplit);
  if (K % 128 == 0) {
    hipLaunchKernelGGL(gconv_fwd<128>, dim3((unsigned)mt, K / 128, gz), dim3(kThreads), 0, st, (const bf16*)x,
                       (const bf16*)w, bias, (bf16*)y, d, relu, pp, ksplit, re);
  } else if (K % 64 == 0) {
    hipLaunchKernelGGL(gconv_fwd<64>, dim3((unsigned)mt, K / 64, gz), dim3(kThreads), 0, st, (const bf16*)x,
                       (const bf16*)w, bias, (bf16*)y, d, relu, pp, ksplit, re);
  } else {  // e.g. the 96-channel layers of PATE's inference_deeper
    hipLaunchKernelGGL(gconv_fwd<32>, dim3((unsigned)mt, K / 32, gz), dim3(kThreads), 0, st, (const bf16*)x,
                       (const bf16*)w, bias, (bf16*)y, d, relu, pp, ksplit, re);
  }
  if (ksplit > 1) {
    const long long n8 = M * G * K / 8;
    hipLaunchKernelGGL(gconv_splitk_finish, dim3((unsigned)((n8 + kThreads - 1) / kThreads)), dim3(kThreads), 0, st,
                       (const float*)part, ksplit, M, G * K, bias, relu, (bf16*)y, re);
  }
  return (int)hipGetLastError();
}

int mifx_gconv_fwd_splitk(const void* x, const void* w, const float* bias, void* y, int N, int Hi, int Wi, int G,
                          int C, int K, int R, int S, int pad, int stride, int relu, float* part, int ksplit,
                          hipStream_t st) {
  return mifx_gconv_fwd_ex(x, w, bias, y, N, Hi, Wi, G, C, K, R, S, pad, stride, relu, part, ksplit, nullptr, nullptr,
                           nullptr, nullptr, st);
}

// x [N, Hi, Wi, G*C] bf16, w [G][K][R][S][C] bf16, bias [G*K] fp32 or null, y [N, Ho, Wo, G*K] bf16;
// zero padding `pad` on every side, Ho = (Hi + 2 pad - R) / stride + 1, relu != 0: y = max(y, 0).
// Needs C % 32 == 0 and K % 32 == 0.
int mifx_gconv_fwd(const void* x, const void* w, const float* bias, void* y, int N, int Hi, int Wi, int G, int C,
                   int K, int R, int S, int pad, int stride, int relu, hipStream_t st) {
  return mifx_gconv_fwd_splitk(x, w, bias, y, N, Hi, Wi, G, C, K, R, S, pad, stride, relu, nullptr, 1, st);
}

// reduction splits for a forward whose pixel x channel tiles cannot fill the chip (batch-1 inference): enough
// workgroups for ~all CUs, >= 4 reduction steps of 32 channels per split, at most 32 splits; 1 = no split
int mifx_gconv_fwd_ksplit(int N, int Hi, int Wi, int G, int C, int K, int R, int S, int pad, int stride) {
  if (stride <= 0 || C % BK != 0 || K % 32 != 0) return 1;
  const long long Ho = (Hi + 2 * pad - R) / stride + 1, Wo = (Wi + 2 * pad - S) / stride + 1;
  const long long M = (long long)N * Ho * Wo;
  const int bn = K % 128 == 0 ? 128 : K % 64 == 0 ? 64 : 32;
  const long long tiles = ((M + BM - 1) / BM) * (K / bn) * G;
  const int nsteps = R * S * (C / BK);
  if (tiles >= 128) return 1;
  int ks = (int)((256 + tiles - 1) / tiles);
  ks = ks < nsteps / 4 ? ks : nsteps / 4;
  ks = ks < 32 ? ks : 32;
  return ks > 1 ? ks : 1;
}

}  // extern "C"
