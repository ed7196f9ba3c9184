// Fused multi-head self-attention for BERT (BASELINE config 4) on gfx950: forward and backward, key-padding
// mask, counter-based attention-probability dropout. Replaces scaled_dot_product_attention, whose ROCm
// backends are Triton-generated (AOTriton attn_fwd / bwd_kernel_fuse: 0.96 ms of a 7.4 ms BERT-base step,
// profiles/archive/bert_base_steady_kernels_s3b.md).
//
// S = 64 / 128: one workgroup per (batch, local head): the whole S x S problem of a BERT sequence (head dim 64)
// lives in one CU. S/16 waves, wave w owns queries 16w .. 16w+15 and works in the TRANSPOSED orientation so the
// MFMA outputs chain (same idiom as csrc/wd_chain.hip):
//  * S^T = K Q^T (16x16x32 bf16 MFMA, K rows from LDS, Q^T fragments = the wave's own query rows): lane = query,
//    4 consecutive keys per lane per key tile. Softmax statistics per query reduce over the lane's registers and
//    across the 4 lane groups with two xor shuffles.
//  * O^T = V^T P^T: the P^T tiles 2s, 2s+1 ARE the B operand of k-step s (keys in the chained order
//    32s + 16(e/4) + 4h + e%4), so the V^T operand is read with ds_read_b64_tr_b16 at those key rows.
//  * backward: S^T and dP_d^T = V dO^T recomputed per wave; dS^T = P^T (dP^T - D), D = rowsum(dO o O);
//    dQ^T = K^T dS^T chained the same way; P_d, then dS, are staged in LDS ([query][key], over the no longer
//    needed K / V images: 74 KB per workgroup, two workgroups per CU) and each wave then owns 16 keys for
//    dV^T = dO^T P_d and dK^T = Q^T dS, reading both operands with transposed LDS reads.
// qkv is the fused projection output [B, S, 3, H, 64] (this rank's H heads), out / dout are [B, S, H, 64]; no
// transposes around the kernels. Longer sequences (S % 64 == 0, <= 512) take the chunked kernels described further
// down. Dropout element (b, global head, i, j) uses the flat index
// ((b Htot + h0 + h) S + i) S + j into the counter-based mask of csrc/counter_rng.h, so the mask does not depend
// on how heads are split over tensor-parallel ranks.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <stdlib.h>

#include "counter_rng.h"

namespace {

typedef __bf16 bf16;
typedef __bf16 v8bf __attribute__((ext_vector_type(8)));
typedef __bf16 v4bf __attribute__((ext_vector_type(4)));
typedef short v4s __attribute__((ext_vector_type(4)));
typedef short v8s __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4s lds_v4s;

constexpr int D = 64;        // head dim
constexpr int LD = D + 8;    // LDS row of a [token][d] image (elements): 144 B rows (the S > 128 kernels)
// the S <= 128 kernels' row: 160 B. With 144-B rows the score reads (ds_read_b128, rows 16 kt + r) and the transposed
// V^T / K^T reads (rows 32 ks + 4 h + q) put two rows of a lane group on one bank set (2-way); 160-B rows are
// conflict-free for both (bank model: tools/lds_banks_attn.py). The backward's 4 images then take 80 KB: still two
// workgroups per CU. (The long kernels keep 144 B: K and V of S = 512 must fit 160 KB.)
#ifndef ATTN_LD_SHORT
#define ATTN_LD_SHORT 80
#endif
constexpr int LDS_ = ATTN_LD_SHORT;
static_assert(LDS_ % 8 == 0 && LDS_ >= D, "16-B aligned rows");
constexpr v4f kZero4 = {0.f, 0.f, 0.f, 0.f};

__device__ __forceinline__ v4s tr_read(const bf16* p) {
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)(p));
}
__device__ __forceinline__ v8bf cat8(v4s a, v4s b) {
  v8s r = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  return __builtin_bit_cast(v8bf, r);
}
__device__ __forceinline__ v8bf ld8(const bf16* p) { return *(const v8bf*)p; }
__device__ __forceinline__ v4f mfma(v8bf a, v8bf b, v4f c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ v8bf pack8(v4f a, v4f b) {
  v8bf o;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    o[i] = (bf16)a[i];
    o[4 + i] = (bf16)b[i];
  }
  return o;
}
__device__ __forceinline__ v4bf pack4(v4f a) {
  v4bf o;
#pragma unroll
  for (int i = 0; i < 4; ++i) o[i] = (bf16)a[i];
  return o;
}

struct Drop {
  const int64_t* rng;
  int site;
  uint32_t thr;  // 0: no dropout
  float scale;   // 1 / (1 - p)
};

// load S rows x 64 of one [B, S, *, 64]-strided tensor into an LDS [S][LDS_] image (16-B chunks)
template <int S, int NTHR>
__device__ __forceinline__ void load_rows(bf16* dst, const bf16* src, size_t row_stride) {
  for (int c = threadIdx.x; c < S * 8; c += NTHR) {
    const int row = c >> 3, ch = c & 7;
    *(uint4*)(dst + row * LDS_ + ch * 8) = *(const uint4*)(src + (size_t)row * row_stride + ch * 8);
  }
}

// scores S^T for the wave's 16 queries: acc[kt][e] = q_i . k_{16kt + 4h + e}, q_i = query 16w + r
template <int S>
__device__ __forceinline__ void scores(const bf16* Ks, const v8bf (&qf)[2], v4f (&acc)[S / 16], int r, int h) {
#pragma unroll
  for (int kt = 0; kt < S / 16; ++kt) {
    v4f a = kZero4;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) a = mfma(ld8(Ks + (16 * kt + r) * LDS_ + 32 * ks + 8 * h), qf[ks], a);
    acc[kt] = a;
  }
}

// P^T (probabilities, before dropout) from the scores, the key bias and the per-query logsumexp
template <int S>
__device__ __forceinline__ void probs(v4f (&p)[S / 16], float scale, const float* kb, float lse, int h) {
#pragma unroll
  for (int kt = 0; kt < S / 16; ++kt) {
    const float4 b = kb ? *(const float4*)(kb + 16 * kt + 4 * h) : make_float4(0.f, 0.f, 0.f, 0.f);
    p[kt][0] = __expf(p[kt][0] * scale + b.x - lse);
    p[kt][1] = __expf(p[kt][1] * scale + b.y - lse);
    p[kt][2] = __expf(p[kt][2] * scale + b.z - lse);
    p[kt][3] = __expf(p[kt][3] * scale + b.w - lse);
  }
}

// dropout keep bits of the lane's 4 keys of tile kt for query i: flat index ((bh_global) S + i) S + 16kt + 4h
template <int S>
__device__ __forceinline__ uint32_t keep_bits(const Drop& dp, uint64_t key, uint64_t row_base, int kt, int h) {
  if (!dp.thr) return 0xf;
  return mifx_rng::keep4(key, (row_base + 16 * kt + 4 * h) >> 2, dp.thr);
}

// QS: query split -- QS workgroups per (batch, head), each with S / 16 / QS waves over its S / QS queries (the K / V
// images loaded by each): B H QS workgroups, so BERT-base's 384 (batch, head) pairs do not leave a half-empty second
// wave on 256 CUs
template <int S, int QS = 1>
__global__ __launch_bounds__(64 * (S / 16) / QS) void attn_fwd(const bf16* __restrict__ qkv,
                                                              const float* __restrict__ kbias, float scale, Drop dp,
                                                              int H, int h0, int Htot, bf16* __restrict__ out,
                                                              float* __restrict__ lse_out) {
  constexpr int NTHR = 64 * (S / 16) / QS, KT = S / 16, KS = S / 32;
  __shared__ __attribute__((aligned(16))) bf16 Ks[S * LDS_];
  __shared__ __attribute__((aligned(16))) bf16 Vs[S * LDS_];
  const int bh = blockIdx.x / QS, qpart = blockIdx.x % QS;
  const int b = bh / H, hh = bh % H;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, r = lane & 15, h = lane >> 4;
  const size_t tok = (size_t)3 * H * D;
  const bf16* base = qkv + (size_t)b * S * tok;
  load_rows<S, NTHR>(Ks, base + (size_t)(H + hh) * D, tok);
  load_rows<S, NTHR>(Vs, base + (size_t)(2 * H + hh) * D, tok);
  const int qi = qpart * (S / QS) + 16 * w + r;
  v8bf qf[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) qf[ks] = *(const v8bf*)(base + (size_t)qi * tok + (size_t)hh * D + 32 * ks + 8 * h);
  __syncthreads();

  v4f s[KT];
  scores<S>(Ks, qf, s, r, h);
  const float* kb = kbias ? kbias + (size_t)b * S : nullptr;
  float m = -3.0e38f;
#pragma unroll
  for (int kt = 0; kt < KT; ++kt) {
    const float4 bb = kb ? *(const float4*)(kb + 16 * kt + 4 * h) : make_float4(0.f, 0.f, 0.f, 0.f);
    s[kt][0] = s[kt][0] * scale + bb.x;
    s[kt][1] = s[kt][1] * scale + bb.y;
    s[kt][2] = s[kt][2] * scale + bb.z;
    s[kt][3] = s[kt][3] * scale + bb.w;
    m = fmaxf(m, fmaxf(fmaxf(s[kt][0], s[kt][1]), fmaxf(s[kt][2], s[kt][3])));
  }
  m = fmaxf(m, __shfl_xor(m, 16));
  m = fmaxf(m, __shfl_xor(m, 32));
  float l = 0.f;
#pragma unroll
  for (int kt = 0; kt < KT; ++kt)
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      s[kt][e] = __expf(s[kt][e] - m);
      l += s[kt][e];
    }
  l += __shfl_xor(l, 16);
  l += __shfl_xor(l, 32);
  const float inv = 1.f / l;
  const uint64_t key = dp.thr ? mifx_rng::drop_key(dp.rng, dp.site) : 0;
  const uint64_t row_base = (((uint64_t)b * Htot + h0 + hh) * S + qi) * S;
  v8bf pb[KS];
#pragma unroll
  for (int kt = 0; kt < KT; ++kt) {
    const uint32_t k = keep_bits<S>(dp, key, row_base, kt, h);
    const float sc = dp.thr ? inv * dp.scale : inv;
#pragma unroll
    for (int e = 0; e < 4; ++e) s[kt][e] = (k >> e) & 1 ? s[kt][e] * sc : 0.f;
  }
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) pb[ks] = pack8(s[2 * ks], s[2 * ks + 1]);
  // O^T = V^T P^T (V^T rows read transposed at the chained key order)
  const int q = r >> 2, p = r & 3;
#pragma unroll
  for (int dt = 0; dt < D / 16; ++dt) {
    v4f o = kZero4;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const bf16* pa = Vs + (32 * ks + 4 * h + q) * LDS_ + 16 * dt + 4 * p;
      o = mfma(cat8(tr_read(pa), tr_read(pa + 16 * LDS_)), pb[ks], o);
    }
    *(v4bf*)(out + ((size_t)b * S + qi) * H * D + (size_t)hh * D + 16 * dt + 4 * h) = pack4(o);
  }
  if (h == 0) lse_out[((size_t)b * H + hh) * S + qi] = m + __logf(l);
}

template <int S>
__global__ __launch_bounds__(64 * (S / 16)) void attn_bwd(const bf16* __restrict__ qkv, const float* __restrict__ kbias,
                                                         const bf16* __restrict__ o, const bf16* __restrict__ dout,
                                                         const float* __restrict__ lse, float scale, Drop dp, int H,
                                                         int h0, int Htot, bf16* __restrict__ dqkv) {
  constexpr int NTHR = 64 * (S / 16), KT = S / 16, KS = S / 32, LP = S + 8;
  extern __shared__ __attribute__((aligned(16))) bf16 smem[];
  bf16* Qs = smem;
  bf16* Ks = Qs + S * LDS_;
  bf16* Vs = Ks + S * LDS_;
  bf16* dOs = Vs + S * LDS_;
  // P_d and dS are staged, one after the other, over the K / V images once those are no longer read
  // ([query][key] rows of S + 8: 17 KB <= the 18 KB of K + V at S = 128): 74 KB of LDS -> two workgroups per CU
  bf16* KV = Ks;
  const int b = blockIdx.x / H, hh = blockIdx.x % H;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, r = lane & 15, h = lane >> 4;
  const size_t tok = (size_t)3 * H * D, otok = (size_t)H * D;
  const bf16* base = qkv + (size_t)b * S * tok;
  load_rows<S, NTHR>(Qs, base + (size_t)hh * D, tok);
  load_rows<S, NTHR>(Ks, base + (size_t)(H + hh) * D, tok);
  load_rows<S, NTHR>(Vs, base + (size_t)(2 * H + hh) * D, tok);
  load_rows<S, NTHR>(dOs, dout + (size_t)b * S * otok + (size_t)hh * D, otok);
  const int qi = 16 * w + r;
  // D_i = sum_d dO o O over the lane group's 16 d values, reduced over the 4 groups
  float di;
  {
    const bf16* po = o + ((size_t)b * S + qi) * otok + (size_t)hh * D + 16 * h;
    const bf16* pd = dout + ((size_t)b * S + qi) * otok + (size_t)hh * D + 16 * h;
    const v8bf o0 = ld8(po), o1 = ld8(po + 8), d0 = ld8(pd), d1 = ld8(pd + 8);
    di = 0.f;
#pragma unroll
    for (int e = 0; e < 8; ++e) di += (float)o0[e] * (float)d0[e] + (float)o1[e] * (float)d1[e];
    di += __shfl_xor(di, 16);
    di += __shfl_xor(di, 32);
  }
  const float lq = lse[((size_t)b * H + hh) * S + qi];
  __syncthreads();

  v8bf qf[2], dof[2];
#pragma unroll
  for (int ks = 0; ks < 2; ++ks) {
    qf[ks] = ld8(Qs + qi * LDS_ + 32 * ks + 8 * h);
    dof[ks] = ld8(dOs + qi * LDS_ + 32 * ks + 8 * h);
  }
  v4f pp[KT];
  scores<S>(Ks, qf, pp, r, h);
  probs<S>(pp, scale, kbias ? kbias + (size_t)b * S : nullptr, lq, h);
  // dP_d^T = V dO^T
  v4f dp_[KT];
#pragma unroll
  for (int kt = 0; kt < KT; ++kt) {
    v4f a = kZero4;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) a = mfma(ld8(Vs + (16 * kt + r) * LDS_ + 32 * ks + 8 * h), dof[ks], a);
    dp_[kt] = a;
  }
  const uint64_t key = dp.thr ? mifx_rng::drop_key(dp.rng, dp.site) : 0;
  const uint64_t row_base = (((uint64_t)b * Htot + h0 + hh) * S + qi) * S;
  v8bf dsb[KS];
  v4f ds[KT];
  v4bf pdv[KT], dsv[KT];
#pragma unroll
  for (int kt = 0; kt < KT; ++kt) {
    const uint32_t k = keep_bits<S>(dp, key, row_base, kt, h);
    const float dsc = dp.thr ? dp.scale : 1.f;
    v4f pd;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const bool kept = (k >> e) & 1;
      const float dpv = kept ? dp_[kt][e] * dsc : 0.f;  // dP = dP_d o M / (1 - p)
      ds[kt][e] = pp[kt][e] * (dpv - di) * scale;        // dS (with the score scale folded in)
      pd[e] = kept ? pp[kt][e] * dsc : 0.f;              // P_d
    }
    pdv[kt] = pack4(pd);
    dsv[kt] = pack4(ds[kt]);
  }
#pragma unroll
  for (int ks = 0; ks < KS; ++ks) dsb[ks] = pack8(ds[2 * ks], ds[2 * ks + 1]);
  // dQ^T = K^T dS^T (K rows read transposed at the chained key order)
  const int q = r >> 2, p = r & 3;
#pragma unroll
  for (int dt = 0; dt < D / 16; ++dt) {
    v4f a = kZero4;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const bf16* pa = Ks + (32 * ks + 4 * h + q) * LDS_ + 16 * dt + 4 * p;
      a = mfma(cat8(tr_read(pa), tr_read(pa + 16 * LDS_)), dsb[ks], a);
    }
    *(v4bf*)(dqkv + ((size_t)b * S + qi) * tok + (size_t)hh * D + 16 * dt + 4 * h) = pack4(a);
  }
  // wave w owns keys 16w .. 16w+15: dV^T = dO^T P_d, then dK^T = Q^T dS (queries are the reduction, natural
  // order); each staged over K / V once every wave is past its reads of them
  const int kj = 16 * w;
  __syncthreads();  // K / V reads (scores, dP, dQ) done
#pragma unroll
  for (int kt = 0; kt < KT; ++kt) *(v4bf*)(KV + qi * LP + 16 * kt + 4 * h) = pdv[kt];
  __syncthreads();
#pragma unroll
  for (int dt = 0; dt < D / 16; ++dt) {
    v4f av = kZero4;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int row = 32 * s + 8 * h + q;
      const bf16* pdo = dOs + row * LDS_ + 16 * dt + 4 * p;
      const bf16* ppd = KV + row * LP + kj + 4 * p;
      av = mfma(cat8(tr_read(pdo), tr_read(pdo + 4 * LDS_)), cat8(tr_read(ppd), tr_read(ppd + 4 * LP)), av);
    }
    *(v4bf*)(dqkv + ((size_t)b * S + kj + r) * tok + (size_t)(2 * H + hh) * D + 16 * dt + 4 * h) = pack4(av);
  }
  __syncthreads();  // P_d reads done
#pragma unroll
  for (int kt = 0; kt < KT; ++kt) *(v4bf*)(KV + qi * LP + 16 * kt + 4 * h) = dsv[kt];
  __syncthreads();
#pragma unroll
  for (int dt = 0; dt < D / 16; ++dt) {
    v4f ak = kZero4;
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int row = 32 * s + 8 * h + q;
      const bf16* pq = Qs + row * LDS_ + 16 * dt + 4 * p;
      const bf16* pds = KV + row * LP + kj + 4 * p;
      ak = mfma(cat8(tr_read(pq), tr_read(pq + 4 * LDS_)), cat8(tr_read(pds), tr_read(pds + 4 * LP)), ak);
    }
    *(v4bf*)(dqkv + ((size_t)b * S + kj + r) * tok + (size_t)(H + hh) * D + 16 * dt + 4 * h) = pack4(ak);
  }
}

// ---- sequences of 192 .. 512 tokens (S % 64 == 0) -------------------------------------------------------------
// The whole S x S problem no longer fits one CU's registers and LDS, so the long kernels tile it flash-style while
// keeping the chained MFMA orientation of the S <= 128 kernels:
//  * forward: a workgroup owns 128 queries of one (batch, head) (8 waves x 16), the head's K and V rows resident in
//    LDS (S x 144 B each: 147 KB at S = 512); keys stream in chunks of 64 with an online softmax (running max and
//    row sum per query lane, the O^T accumulators rescaled per chunk), the dropout mask drawn per chunk.
//  * backward, dQ: the same partition; with the forward's logsumexp the probabilities of a key chunk need nothing
//    from other chunks, so dS^T is formed chunk by chunk and dQ^T = K^T dS^T accumulates in registers. It also
//    writes D_i = rowsum(dO o O) for the second kernel.
//  * backward, dK / dV: a workgroup owns 128 keys (wave = 16 keys), Q and dO resident; query chunks of 64 give
//    S = Q K^T and dP_d = dO V^T in the [query][key] orientation, so P_d and dS chain straight into
//    dV^T = dO^T P_d and dK^T = Q^T dS with dO / Q read transposed -- the forward's structure with the roles of
//    queries and keys exchanged. The lane holds 4 query rows of one key column; the dropout bits come from one
//    mask draw per lane (row 4h + lane % 4, its quad's 4 keys) exchanged within the quad.
constexpr int LQB = 128, LNT = 512, LKC = 64, LMAXS = 512;

constexpr int long_lds(int S) { return 2 * S * LD * 2; }

// the query (key) blocks of one head are consecutive logical blocks: keep them on one XCD (dispatch round-robins
// consecutive workgroups over the 8 XCDs), so the head's K / V (Q / dO) rows are fetched into one L2
__device__ __forceinline__ int xcd_block(int bid, int nwg) { return (nwg & 7) ? bid : (bid & 7) * (nwg >> 3) + (bid >> 3); }

__device__ __forceinline__ void load_rows_n(bf16* dst, const bf16* src, size_t row_stride, int rows) {
#pragma unroll 4
  for (int c = threadIdx.x; c < rows * 8; c += LNT) {
    const int row = c >> 3, ch = c & 7;
    *(uint4*)(dst + row * LD + ch * 8) = *(const uint4*)(src + (size_t)row * row_stride + ch * 8);
  }
}

__global__ __launch_bounds__(LNT) void attn_fwd_long(const bf16* __restrict__ qkv, const float* __restrict__ kbias,
                                                     int S, float scale, Drop dp, int H, int h0, int Htot,
                                                     bf16* __restrict__ out, float* __restrict__ lse_out) {
  extern __shared__ __attribute__((aligned(16))) bf16 smem[];
  bf16* Ks = smem;
  bf16* Vs = smem + S * LD;
  const int nqb = (S + LQB - 1) / LQB, lb = xcd_block(blockIdx.x, gridDim.x);
  const int qb = lb % nqb, bh = lb / nqb, b = bh / H, hh = bh % H;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, r = lane & 15, h = lane >> 4, q = r >> 2, p = r & 3;
  const size_t tok = (size_t)3 * H * D;
  const bf16* base = qkv + (size_t)b * S * tok;
  load_rows_n(Ks, base + (size_t)(H + hh) * D, tok, S);
  load_rows_n(Vs, base + (size_t)(2 * H + hh) * D, tok, S);
  const bool live = qb * LQB + 16 * w < S;
  const int qi = qb * LQB + 16 * w + r;
  v8bf qf[2];
  if (live)
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) qf[ks] = ld8(base + (size_t)qi * tok + (size_t)hh * D + 32 * ks + 8 * h);
  __syncthreads();
  if (!live) return;  // no barrier follows

  const float* kb = kbias ? kbias + (size_t)b * S : nullptr;
  const uint64_t key = dp.thr ? mifx_rng::drop_key(dp.rng, dp.site) : 0;
  const uint64_t row_base = (((uint64_t)b * Htot + h0 + hh) * S + qi) * S;
  float m = -3.0e38f, l = 0.f;
  v4f o[D / 16];
#pragma unroll
  for (int dt = 0; dt < D / 16; ++dt) o[dt] = kZero4;
  for (int c = 0; c < S; c += LKC) {
    v4f s[LKC / 16];
    float mc = m;
#pragma unroll
    for (int kt = 0; kt < LKC / 16; ++kt) {
      v4f a = kZero4;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) a = mfma(ld8(Ks + (c + 16 * kt + r) * LD + 32 * ks + 8 * h), qf[ks], a);
      const float4 bb = kb ? *(const float4*)(kb + c + 16 * kt + 4 * h) : make_float4(0.f, 0.f, 0.f, 0.f);
      a[0] = a[0] * scale + bb.x;
      a[1] = a[1] * scale + bb.y;
      a[2] = a[2] * scale + bb.z;
      a[3] = a[3] * scale + bb.w;
      mc = fmaxf(mc, fmaxf(fmaxf(a[0], a[1]), fmaxf(a[2], a[3])));
      s[kt] = a;
    }
    mc = fmaxf(mc, __shfl_xor(mc, 16));
    mc = fmaxf(mc, __shfl_xor(mc, 32));
    const float alpha = __expf(m - mc);
    m = mc;
    l *= alpha;
#pragma unroll
    for (int dt = 0; dt < D / 16; ++dt) o[dt] *= alpha;
#pragma unroll
    for (int kt = 0; kt < LKC / 16; ++kt) {
      const uint32_t kbits = dp.thr ? mifx_rng::keep4(key, (row_base + c + 16 * kt + 4 * h) >> 2, dp.thr) : 0xf;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float pe = __expf(s[kt][e] - m);
        l += pe;
        s[kt][e] = (kbits >> e) & 1 ? pe : 0.f;
      }
    }
    const v8bf pb[2] = {pack8(s[0], s[1]), pack8(s[2], s[3])};
    // O^T += V^T P^T over this chunk (V rows read transposed at the chained key order)
#pragma unroll
    for (int dt = 0; dt < D / 16; ++dt)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const bf16* pa = Vs + (c + 32 * ks + 4 * h + q) * LD + 16 * dt + 4 * p;
        o[dt] = mfma(cat8(tr_read(pa), tr_read(pa + 16 * LD)), pb[ks], o[dt]);
      }
  }
  l += __shfl_xor(l, 16);
  l += __shfl_xor(l, 32);
  const float inv = (dp.thr ? dp.scale : 1.f) / l;
#pragma unroll
  for (int dt = 0; dt < D / 16; ++dt)
    *(v4bf*)(out + ((size_t)b * S + qi) * H * D + (size_t)hh * D + 16 * dt + 4 * h) = pack4(o[dt] * inv);
  if (h == 0) lse_out[(size_t)bh * S + qi] = m + __logf(l);
}

__global__ __launch_bounds__(LNT) void attn_bwd_dq_long(const bf16* __restrict__ qkv, const float* __restrict__ kbias,
                                                        const bf16* __restrict__ o, const bf16* __restrict__ dout,
                                                        const float* __restrict__ lse, int S, float scale, Drop dp,
                                                        int H, int h0, int Htot, bf16* __restrict__ dqkv,
                                                        float* __restrict__ dsum) {
  extern __shared__ __attribute__((aligned(16))) bf16 smem[];
  bf16* Ks = smem;
  bf16* Vs = smem + S * LD;
  const int nqb = (S + LQB - 1) / LQB, lb = xcd_block(blockIdx.x, gridDim.x);
  const int qb = lb % nqb, bh = lb / nqb, b = bh / H, hh = bh % H;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, r = lane & 15, h = lane >> 4, q = r >> 2, p = r & 3;
  const size_t tok = (size_t)3 * H * D, otok = (size_t)H * D;
  const bf16* base = qkv + (size_t)b * S * tok;
  load_rows_n(Ks, base + (size_t)(H + hh) * D, tok, S);
  load_rows_n(Vs, base + (size_t)(2 * H + hh) * D, tok, S);
  const bool live = qb * LQB + 16 * w < S;
  const int qi = qb * LQB + 16 * w + r;
  v8bf qf[2], dof[2];
  float di = 0.f, lq = 0.f;
  if (live) {
    const bf16* pdo = dout + ((size_t)b * S + qi) * otok + (size_t)hh * D;
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      qf[ks] = ld8(base + (size_t)qi * tok + (size_t)hh * D + 32 * ks + 8 * h);
      dof[ks] = ld8(pdo + 32 * ks + 8 * h);
    }
    const bf16* po = o + ((size_t)b * S + qi) * otok + (size_t)hh * D + 16 * h;
    const v8bf o0 = ld8(po), o1 = ld8(po + 8), d0 = ld8(pdo + 16 * h), d1 = ld8(pdo + 16 * h + 8);
#pragma unroll
    for (int e = 0; e < 8; ++e) di += (float)o0[e] * (float)d0[e] + (float)o1[e] * (float)d1[e];
    di += __shfl_xor(di, 16);
    di += __shfl_xor(di, 32);
    if (h == 0) dsum[(size_t)bh * S + qi] = di;
    lq = lse[(size_t)bh * S + qi];
  }
  __syncthreads();
  if (!live) return;

  const float* kb = kbias ? kbias + (size_t)b * S : nullptr;
  const uint64_t key = dp.thr ? mifx_rng::drop_key(dp.rng, dp.site) : 0;
  const uint64_t row_base = (((uint64_t)b * Htot + h0 + hh) * S + qi) * S;
  const float dsc = dp.thr ? dp.scale : 1.f;
  v4f dq[D / 16];
#pragma unroll
  for (int dt = 0; dt < D / 16; ++dt) dq[dt] = kZero4;
  for (int c = 0; c < S; c += LKC) {
    v4f ds[LKC / 16];
#pragma unroll
    for (int kt = 0; kt < LKC / 16; ++kt) {
      v4f sc = kZero4, dpd = kZero4;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        sc = mfma(ld8(Ks + (c + 16 * kt + r) * LD + 32 * ks + 8 * h), qf[ks], sc);
        dpd = mfma(ld8(Vs + (c + 16 * kt + r) * LD + 32 * ks + 8 * h), dof[ks], dpd);
      }
      const float4 bb = kb ? *(const float4*)(kb + c + 16 * kt + 4 * h) : make_float4(0.f, 0.f, 0.f, 0.f);
      const float bv[4] = {bb.x, bb.y, bb.z, bb.w};
      const uint32_t kbits = dp.thr ? mifx_rng::keep4(key, (row_base + c + 16 * kt + 4 * h) >> 2, dp.thr) : 0xf;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const float pe = __expf(sc[e] * scale + bv[e] - lq);
        const float dpv = (kbits >> e) & 1 ? dpd[e] * dsc : 0.f;
        ds[kt][e] = pe * (dpv - di) * scale;
      }
    }
    const v8bf dsb[2] = {pack8(ds[0], ds[1]), pack8(ds[2], ds[3])};
#pragma unroll
    for (int dt = 0; dt < D / 16; ++dt)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const bf16* pa = Ks + (c + 32 * ks + 4 * h + q) * LD + 16 * dt + 4 * p;
        dq[dt] = mfma(cat8(tr_read(pa), tr_read(pa + 16 * LD)), dsb[ks], dq[dt]);
      }
  }
#pragma unroll
  for (int dt = 0; dt < D / 16; ++dt)
    *(v4bf*)(dqkv + ((size_t)b * S + qi) * tok + (size_t)hh * D + 16 * dt + 4 * h) = pack4(dq[dt]);
}

__global__ __launch_bounds__(LNT) void attn_bwd_dkv_long(const bf16* __restrict__ qkv, const float* __restrict__ kbias,
                                                         const bf16* __restrict__ dout, const float* __restrict__ lse,
                                                         const float* __restrict__ dsum, int S, float scale, Drop dp,
                                                         int H, int h0, int Htot, bf16* __restrict__ dqkv) {
  extern __shared__ __attribute__((aligned(16))) bf16 smem[];
  bf16* Qs = smem;
  bf16* dOs = smem + S * LD;
  const int nkb = (S + LQB - 1) / LQB, lb = xcd_block(blockIdx.x, gridDim.x);
  const int kb_ = lb % nkb, bh = lb / nkb, b = bh / H, hh = bh % H;
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63, r = lane & 15, h = lane >> 4, q = r >> 2, p = r & 3;
  const size_t tok = (size_t)3 * H * D, otok = (size_t)H * D;
  const bf16* base = qkv + (size_t)b * S * tok;
  load_rows_n(Qs, base + (size_t)hh * D, tok, S);
  load_rows_n(dOs, dout + (size_t)b * S * otok + (size_t)hh * D, otok, S);
  const bool live = kb_ * LQB + 16 * w < S;
  const int kj = kb_ * LQB + 16 * w + r;
  v8bf kf[2], vf[2];
  float bj = 0.f;
  if (live) {
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      kf[ks] = ld8(base + (size_t)kj * tok + (size_t)(H + hh) * D + 32 * ks + 8 * h);
      vf[ks] = ld8(base + (size_t)kj * tok + (size_t)(2 * H + hh) * D + 32 * ks + 8 * h);
    }
    if (kbias) bj = kbias[(size_t)b * S + kj];
  }
  __syncthreads();
  if (!live) return;

  const float* lq = lse + (size_t)bh * S;
  const float* dd = dsum + (size_t)bh * S;
  const uint64_t key = dp.thr ? mifx_rng::drop_key(dp.rng, dp.site) : 0;
  const uint64_t mrow = ((uint64_t)b * Htot + h0 + hh) * S;
  const float dsc = dp.thr ? dp.scale : 1.f;
  v4f dk[D / 16], dv[D / 16];
#pragma unroll
  for (int dt = 0; dt < D / 16; ++dt) dk[dt] = dv[dt] = kZero4;
  for (int c = 0; c < S; c += LKC) {
    v4f pd[LKC / 16], ds[LKC / 16];
#pragma unroll
    for (int it = 0; it < LKC / 16; ++it) {
      // lane: S[i][j], i = c + 16 it + 4h + e, j = kj
      v4f sc = kZero4, dpd = kZero4;
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        sc = mfma(ld8(Qs + (c + 16 * it + r) * LD + 32 * ks + 8 * h), kf[ks], sc);
        dpd = mfma(ld8(dOs + (c + 16 * it + r) * LD + 32 * ks + 8 * h), vf[ks], dpd);
      }
      const int i0 = c + 16 * it + 4 * h;
      const float4 L = *(const float4*)(lq + i0);
      const float4 Dq = *(const float4*)(dd + i0);
      const float lv[4] = {L.x, L.y, L.z, L.w}, dv4[4] = {Dq.x, Dq.y, Dq.z, Dq.w};
      uint32_t nib = 0xf;
      if (dp.thr) nib = mifx_rng::keep4(key, ((mrow + i0 + p) * S + (kj & ~3)) >> 2, dp.thr);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const bool kept = dp.thr ? ((__shfl(nib, (lane & ~3) | e) >> p) & 1) : true;
        const float pe = __expf(sc[e] * scale + bj - lv[e]);
        pd[it][e] = kept ? pe * dsc : 0.f;
        ds[it][e] = pe * ((kept ? dpd[e] * dsc : 0.f) - dv4[e]) * scale;
      }
    }
    const v8bf pdb[2] = {pack8(pd[0], pd[1]), pack8(pd[2], pd[3])};
    const v8bf dsb[2] = {pack8(ds[0], ds[1]), pack8(ds[2], ds[3])};
#pragma unroll
    for (int dt = 0; dt < D / 16; ++dt)
#pragma unroll
      for (int ks = 0; ks < 2; ++ks) {
        const bf16* pa = dOs + (c + 32 * ks + 4 * h + q) * LD + 16 * dt + 4 * p;
        dv[dt] = mfma(cat8(tr_read(pa), tr_read(pa + 16 * LD)), pdb[ks], dv[dt]);
        const bf16* pq = Qs + (c + 32 * ks + 4 * h + q) * LD + 16 * dt + 4 * p;
        dk[dt] = mfma(cat8(tr_read(pq), tr_read(pq + 16 * LD)), dsb[ks], dk[dt]);
      }
  }
  bf16* dst = dqkv + ((size_t)b * S + kj) * tok;
#pragma unroll
  for (int dt = 0; dt < D / 16; ++dt) {
    *(v4bf*)(dst + (size_t)(H + hh) * D + 16 * dt + 4 * h) = pack4(dk[dt]);
    *(v4bf*)(dst + (size_t)(2 * H + hh) * D + 16 * dt + 4 * h) = pack4(dv[dt]);
  }
}

bool long_seq(int S) { return S > 128 && S <= LMAXS && S % LKC == 0; }

uint32_t drop_threshold(float p) {
  if (!(p > 0.f)) return 0;
  const float t = p * 65536.f + 0.5f;
  return t >= 65536.f ? 65536u : (uint32_t)t;
}

template <int S>
constexpr int bwd_lds() {
  static_assert(S * (S + 8) <= 2 * S * LDS_, "P_d / dS staging must fit over the K and V images");
  return 4 * S * LDS_ * 2;
}

}  // namespace

extern "C" {

// qkv [B, S, 3, H, 64] bf16 (contiguous), kbias [B, S] fp32 additive key bias or null, out [B, S, H, 64] bf16,
// lse [B, H, S] fp32. p: attention-probability dropout (rng: device int64 [seed, counter]; site per layer).
// h0 / Htot: this rank's first global head and the model's head count (dropout indexing only).
int mifx_attn_fwd(const void* qkv, const float* kbias, int B, int S, int H, int h0, int Htot, float scale, float p,
                  const int64_t* rng, int site, void* out, float* lse, hipStream_t st) {
  if (B <= 0 || H <= 0 || (S != 64 && S != 128 && !long_seq(S)) || p < 0.f || p >= 1.f || (p > 0.f && rng == nullptr))
    return -1;
  if (((uintptr_t)qkv | (uintptr_t)out | (uintptr_t)kbias) % 16 != 0) return -1;
  const Drop dp{rng, site, drop_threshold(p), 1.f / (1.f - p)};
  const dim3 grid(B * H);
  if (long_seq(S)) {
    static bool attr = false;
    if (!attr) {
      (void)hipFuncSetAttribute((const void*)attn_fwd_long, hipFuncAttributeMaxDynamicSharedMemorySize,
                                long_lds(LMAXS));
      attr = true;
    }
    hipLaunchKernelGGL(attn_fwd_long, dim3(B * H * ((S + LQB - 1) / LQB)), dim3(LNT), long_lds(S), st,
                       (const bf16*)qkv, kbias, S, scale, dp, H, h0, Htot, (bf16*)out, lse);
  } else if (S == 128) {
    // MIFX_ATTN_QSPLIT: 1 (default), 2 or 4 workgroups per (batch, head). BERT-base step: 6,206 / 6,179 seq/s at 1,
    // 6,190 / 6,184 at 2, 5,992 / 6,004 at 4 (profiles/bert_attn_qsplit_ab_r5.txt): the kernel is latency-bound per
    // workgroup, not by the 1.5-wave quantisation of 384 workgroups
    static const int qs = [] {
      const char* e = getenv("MIFX_ATTN_QSPLIT");
      const int v = e ? atoi(e) : 1;
      return v == 2 || v == 4 ? v : 1;
    }();
    if (qs == 1)
      hipLaunchKernelGGL((attn_fwd<128, 1>), grid, dim3(512), 0, st, (const bf16*)qkv, kbias, scale, dp, H, h0, Htot,
                         (bf16*)out, lse);
    else if (qs == 2)
      hipLaunchKernelGGL((attn_fwd<128, 2>), dim3(B * H * 2), dim3(256), 0, st, (const bf16*)qkv, kbias, scale, dp, H,
                         h0, Htot, (bf16*)out, lse);
    else
      hipLaunchKernelGGL((attn_fwd<128, 4>), dim3(B * H * 4), dim3(128), 0, st, (const bf16*)qkv, kbias, scale, dp, H,
                         h0, Htot, (bf16*)out, lse);
  } else
    hipLaunchKernelGGL(attn_fwd<64>, grid, dim3(256), 0, st, (const bf16*)qkv, kbias, scale, dp, H, h0, Htot,
                       (bf16*)out, lse);
  return (int)hipGetLastError();
}

// dqkv [B, S, 3, H, 64] bf16 (every element written); dsum: fp32 [B, H, S] workspace for S > 128 (else unused)
int mifx_attn_bwd(const void* qkv, const float* kbias, const void* out, const void* dout, const float* lse, int B,
                  int S, int H, int h0, int Htot, float scale, float p, const int64_t* rng, int site, void* dqkv,
                  float* dsum, hipStream_t st) {
  if (B <= 0 || H <= 0 || (S != 64 && S != 128 && !long_seq(S)) || p < 0.f || p >= 1.f || (p > 0.f && rng == nullptr))
    return -1;
  if (long_seq(S) && dsum == nullptr) return -1;
  if (((uintptr_t)qkv | (uintptr_t)out | (uintptr_t)dout | (uintptr_t)dqkv | (uintptr_t)kbias) % 16 != 0) return -1;
  static bool attr = false;
  if (!attr) {
    (void)hipFuncSetAttribute((const void*)attn_bwd<128>, hipFuncAttributeMaxDynamicSharedMemorySize, bwd_lds<128>());
    (void)hipFuncSetAttribute((const void*)attn_bwd<64>, hipFuncAttributeMaxDynamicSharedMemorySize, bwd_lds<64>());
    attr = true;
  }
  const Drop dp{rng, site, drop_threshold(p), 1.f / (1.f - p)};
  const dim3 grid(B * H);
  if (long_seq(S)) {
    static bool lattr = false;
    if (!lattr) {
      (void)hipFuncSetAttribute((const void*)attn_bwd_dq_long, hipFuncAttributeMaxDynamicSharedMemorySize,
                                long_lds(LMAXS));
      (void)hipFuncSetAttribute((const void*)attn_bwd_dkv_long, hipFuncAttributeMaxDynamicSharedMemorySize,
                                long_lds(LMAXS));
      lattr = true;
    }
    const dim3 lgrid(B * H * ((S + LQB - 1) / LQB));
    hipLaunchKernelGGL(attn_bwd_dq_long, lgrid, dim3(LNT), long_lds(S), st, (const bf16*)qkv, kbias, (const bf16*)out,
                       (const bf16*)dout, lse, S, scale, dp, H, h0, Htot, (bf16*)dqkv, dsum);
    hipLaunchKernelGGL(attn_bwd_dkv_long, lgrid, dim3(LNT), long_lds(S), st, (const bf16*)qkv, kbias,
                       (const bf16*)dout, lse, (const float*)dsum, S, scale, dp, H, h0, Htot, (bf16*)dqkv);
  } else if (S == 128)
    hipLaunchKernelGGL(attn_bwd<128>, grid, dim3(512), bwd_lds<128>(), st, (const bf16*)qkv, kbias, (const bf16*)out,
                       (const bf16*)dout, lse, scale, dp, H, h0, Htot, (bf16*)dqkv);
  else
    hipLaunchKernelGGL(attn_bwd<64>, grid, dim3(256), bwd_lds<64>(), st, (const bf16*)qkv, kbias, (const bf16*)out,
                       (const bf16*)dout, lse, scale, dp, H, h0, Htot, (bf16*)dqkv);
  return (int)hipGetLastError();
}

}  // extern "C"
