// Weight gradient of the narrow 3x3 convolutions (C, Cout multiples of 64; pad 1; stride 1 or 2) for gfx950:
// dW[co][r][s][c] = sum over output pixels (n, oh, ow) of dY[n][oh][ow][co] * X[n][S oh + r - 1][S ow + s - 1][c].
//
// Reference workload: ResNet-50 of the reference's TFJob examples (SURVEY KN14,
// `install-kubeflow/ks_app/vendor/kubeflow/examples/prototypes/tf-job-simple-v1beta2.jsonnet:28-38`). Stages 1-2 have
// 64- and 128-channel 3x3 convolutions; the grouped split-K TN GEMM of mifx.ops.gemm serves the 256+-channel ones
// but loses on these (its 128-wide column tiles re-gather the input once per tap pair), and MIOpen's igemm_wrw ran
// them at 336-455 TFLOP/s (176 / 130-138 us at B = 256, profiles/conv3x3_routes_r5.jsonl). Here ONE staged patch of
// the input serves all nine taps:
//
//  * Workgroup = (pixel split, 64-output-channel slice, 64-input-channel slice); output tile 64 x (9 taps x 64 c) =
//    64 x 576, i.e. 36 16-wide column tiles, nine per wave (4 waves), all 4 16-row tiles per wave: 144 fp32
//    accumulators per lane on v_mfma_f32_16x16x32_bf16, the 32 PIXELS of a K-step as the reduction.
//  * The split's output rows go CR at a time (never across an image): the dY rows [pixel][64 co] and the input rows
//    they need ((CR - 1) S + 3 rows of W + 2 pixels, zeros outside the image) [pixel][64 c] are staged in LDS with
//    16-byte loads and stores, plus a table of each output pixel's tap-(0,0) input pixel.
//  * Both operands are pixel-major, so every fragment is a pair of ds_read_b64_tr_b16 transposed reads (a lane's 8
//    reduction elements are 8 pixels). Element j of lane group g is pixel 4 g + j (j < 4) / 16 + 4 g + j - 4, the same
//    permutation for both operands, so a 32-lane half reads 8 CONSECUTIVE pixel rows; rows are 128 B with the
//    32-byte block index XORed with (row >> 1) & 3, which puts any 8 consecutive rows on 8 distinct bank octets
//    (conflict-free for dY and the input reads). Stride 2 stages each input row as its even columns then its odd
//    ones, so consecutive output pixels read consecutive staged pixels for every tap there too.
//  * A tap's B fragment is the table entry + the tap's staged-pixel offset: no im2col, no per-tap reload.
//  * Each workgroup writes its fp32 partial [Cout][3][3][C] slice into part[split]; conv3_wgrad_sum adds the splits
//    in split order (deterministic) into the parameter's layout (channels_last or contiguous).
//  * blockIdx -> work is XCD-aware: the slices of a split (same pixels) and neighbouring splits (shared halo rows)
//    run on one XCD, whose L2 then serves the re-reads.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

typedef __bf16 bf16;
typedef __bf16 v8bf __attribute__((ext_vector_type(8)));
typedef float v4f __attribute__((ext_vector_type(4)));
typedef short v4s __attribute__((ext_vector_type(4)));
typedef short v8s __attribute__((ext_vector_type(8)));
typedef unsigned int u4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) v4s lds_v4s;

constexpr int NT = 256;
constexpr int CS = 64;  // channels per slice (both operands): one 128-byte LDS row per pixel
#ifndef STAGE_BATCH
#define STAGE_BATCH 4
#endif
#ifndef C3_WS
#define C3_WS 0  // the wave-specialised build (below): measured no faster, profiles/conv3_wgrad_shapes_r6.jsonl
#endif

__device__ __forceinline__ v4f mfma(v8bf a, v8bf b, v4f c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ v4s tr_read(const bf16* p) { return __builtin_amdgcn_ds_read_tr16_b64_v4i16((lds_v4s*)p); }
__device__ __forceinline__ v8bf cat8(v4s a, v4s b) {
  const v8s r = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  return __builtin_bit_cast(v8bf, r);
}
// element offset of (row, 16-channel block cb, element e) in a swizzled [rows][64] image
__device__ __forceinline__ int sw(int row, int cb, int e) { return row * CS + 16 * (cb ^ ((row >> 1) & 3)) + e; }

struct Geo {
  int N, H, W, C, Cout, OH, OW, S, CR, NPS;  // NPS: pixel slots per chunk (multiple of 32)
  int XW, HW, c1, c2;  // staged row width; stride 2: phase width; staged column of taps s = 1, 2
  int splits, ncs, nslices;
};

// one staged chunk: dY rows [NPS][64], the pixel table [NPS], the input rows [XR][XW][64]
struct Bufs {
  bf16* ys;
  int* poff;
  bf16* xs;
};
__device__ __forceinline__ Bufs bufs_at(bf16* base, const Geo& g) {
  Bufs r;
  r.ys = base;
  r.poff = (int*)(base + g.NPS * CS);
  r.xs = (bf16*)(r.poff + g.NPS);
  return r;
}
__host__ __device__ inline int buf_elems(int nps, int xr, int xw) { return nps * CS + nps * 2 + xr * xw * CS; }

struct Chunk {
  int n, oh0, cr;
};
__device__ __forceinline__ Chunk chunk_at(int gr, int r_end, const Geo& g) {
  Chunk c;
  c.n = gr / g.OH;
  c.oh0 = gr - c.n * g.OH;
  c.cr = min(min(g.CR, g.OH - c.oh0), r_end - gr);
  return c;
}

// stage chunk ch into B: threads tl = 0 .. LT - 1 (STAGE_BATCH 16-byte loads in flight per thread before their
// LDS stores)
template <int LT>
__device__ __forceinline__ void stage(const bf16* __restrict__ x, const bf16* __restrict__ dy, const Geo& g, int os,
                                      int cs, Chunk ch, Bufs B, int tl) {
  const int npix = ch.cr * g.OW, np32 = (npix + 31) & ~31;
  const int xr = (ch.cr - 1) * g.S + 3;
  // dY rows oh0 .. oh0 + cr - 1 of this output-channel slice; zero slots up to the K-step multiple
  const bf16* dsrc = dy + ((size_t)ch.n * g.OH + ch.oh0) * g.OW * g.Cout + CS * os;
  for (int i0 = tl; i0 < np32 * 8; i0 += STAGE_BATCH * LT) {
    u4 v[STAGE_BATCH];
#pragma unroll
    for (int k = 0; k < STAGE_BATCH; ++k) {
      const int i = i0 + k * LT, px = i >> 3, c8 = i & 7;
      v[k] = (u4){0u, 0u, 0u, 0u};
      if (px < npix) v[k] = *(const u4*)(dsrc + (size_t)px * g.Cout + 8 * c8);
    }
#pragma unroll
    for (int k = 0; k < STAGE_BATCH; ++k) {
      const int i = i0 + k * LT, px = i >> 3, c8 = i & 7;
      if (px < np32) *(u4*)(B.ys + sw(px, c8 >> 1, 8 * (c8 & 1))) = v[k];
    }
  }
  // input rows S oh0 - 1 .. of this input-channel slice, columns -1 .. W (zeros outside the image)
  const int ih0 = g.S * ch.oh0 - 1;
  const int nx = xr * g.XW * 8;
  for (int i0 = tl; i0 < nx; i0 += STAGE_BATCH * LT) {
    u4 v[STAGE_BATCH];
#pragma unroll
    for (int k = 0; k < STAGE_BATCH; ++k) {
      const int i = i0 + k * LT, sp = i >> 3, c8 = i & 7;
      const int ir = sp / g.XW, sc = sp - ir * g.XW;
      const int ic = g.S == 1 ? sc : (sc < g.HW ? 2 * sc : 2 * (sc - g.HW) + 1);  // stride 2: even | odd columns
      const int ih = ih0 + ir, iw = ic - 1;
      v[k] = (u4){0u, 0u, 0u, 0u};
      if (i < nx && ih >= 0 && ih < g.H && iw >= 0 && iw < g.W)
        v[k] = *(const u4*)(x + (((size_t)ch.n * g.H + ih) * g.W + iw) * g.C + CS * cs + 8 * c8);
    }
#pragma unroll
    for (int k = 0; k < STAGE_BATCH; ++k) {
      const int i = i0 + k * LT, sp = i >> 3, c8 = i & 7;
      if (i < nx) *(u4*)(B.xs + sw(sp, c8 >> 1, 8 * (c8 & 1))) = v[k];
    }
  }
  for (int i = tl; i < np32; i += LT) {
    const int pc = min(i, npix - 1), orl = pc / g.OW;
    B.poff[i] = orl * g.S * g.XW + (pc - orl * g.OW);  // (slots past npix: any in-range pixel, dY is 0 there)
  }
}

// the compute wave wv (0..3) of one staged chunk: nine 16-column tiles x all four 16-row tiles
__device__ __forceinline__ void compute(const Geo& g, Bufs B, int npix, int wv, int lane, v4f (&acc)[4][9]) {
  const int grp = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
  const int np32 = (npix + 31) & ~31;
  for (int p0 = 0; p0 < np32; p0 += 32) {
    const int ra = p0 + 4 * grp + q, rb = ra + 16;  // this lane's transposed-read rows (pixel slots)
    v8bf af[4];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) af[mt] = cat8(tr_read(B.ys + sw(ra, mt, 4 * p)), tr_read(B.ys + sw(rb, mt, 4 * p)));
    const int xa = B.poff[ra], xb = B.poff[rb];
#pragma unroll
    for (int j = 0; j < 9; ++j) {
      const int J = 9 * wv + j, tap = J >> 2, cb = J & 3;
      const int ts = tap % 3, to = (tap / 3) * g.XW + (ts == 0 ? 0 : ts == 1 ? g.c1 : g.c2);
      const v8bf bfr = cat8(tr_read(B.xs + sw(xa + to, cb, 4 * p)), tr_read(B.xs + sw(xb + to, cb, 4 * p)));
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) acc[mt][j] = mfma(af[mt], bfr, acc[mt][j]);
    }
  }
}

#if C3_WS
// Wave-specialised build (-DC3_WS=1): 8 waves, one workgroup per CU. Waves 0-3 multiply the staged chunk c while
// waves 4-7 stage chunk c + 1 into the other LDS buffer; one barrier per chunk. Aimed at the staging latency of the
// default 4-wave build (two workgroups per CU, 19 % MFMA busy: profiles/conv3_wgrad_pmc_r6.md), it measured no
// faster (131 / 140 vs 137 / 123 us): one multiplying wave per SIMD exposes the transposed-read latency instead.
constexpr int NTK = 512;
#else
constexpr int NTK = NT;
#endif

__global__ __launch_bounds__(NTK) __attribute__((amdgpu_waves_per_eu(2, 2))) void conv3_wgrad(
    const bf16* __restrict__ x, const bf16* __restrict__ dy, float* __restrict__ part, Geo g) {
  extern __shared__ __attribute__((aligned(16))) bf16 lds[];
  const int t = threadIdx.x, lane = t & 63;
  const int wv = __builtin_amdgcn_readfirstlane(t >> 6);
  // XCD-aware work index: consecutive u share an XCD when the grid divides by 8
  const int G = gridDim.x, b = blockIdx.x;
  const int u = (G % 8 == 0) ? (b % 8) * (G / 8) + b / 8 : b;
  const int split = u / g.nslices, slice = u - split * g.nslices;
  const int os = slice / g.ncs, cs = slice - os * g.ncs;
  const int rows_total = g.N * g.OH;
  const int r_begin = (int)((long long)rows_total * split / g.splits);
  const int r_end = (int)((long long)rows_total * (split + 1) / g.splits);

#if C3_WS
  // the two roles run separate loops with the same number of barriers (one per chunk, after the prologue), so the
  // loaders carry no accumulators and the multipliers no staging registers
  const int bel = buf_elems(g.NPS, (g.CR - 1) * g.S + 3, g.XW);
  const Bufs B0 = bufs_at(lds, g), B1 = bufs_at(lds + bel, g);
  if (wv >= 4) {
    int gr = r_begin;
    Chunk cur = chunk_at(gr, r_end, g);
    if (gr < r_end) stage<256>(x, dy, g, os, cs, cur, B0, t - 256);
    __syncthreads();
    int bsel = 0;
    while (gr < r_end) {
      const int gn = gr + cur.cr;
      const Chunk nxt = chunk_at(gn, r_end, g);
      if (gn < r_end) stage<256>(x, dy, g, os, cs, nxt, bsel ? B0 : B1, t - 256);
      __syncthreads();  // chunk c consumed, chunk c + 1 staged
      gr = gn;
      cur = nxt;
      bsel ^= 1;
    }
    return;
  }
  v4f acc[4][9];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 9; ++j) acc[i][j] = (v4f){0.f, 0.f, 0.f, 0.f};
  __syncthreads();  // chunk 0 staged
  {
    int bsel = 0;
    for (int gr = r_begin; gr < r_end;) {
      const Chunk cur = chunk_at(gr, r_end, g);
      compute(g, bsel ? B1 : B0, cur.cr * g.OW, wv, lane, acc);
      __syncthreads();
      gr += cur.cr;
      bsel ^= 1;
    }
  }
#else
  v4f acc[4][9];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 9; ++j) acc[i][j] = (v4f){0.f, 0.f, 0.f, 0.f};
  const Bufs B0 = bufs_at(lds, g);
  for (int gr = r_begin; gr < r_end;) {
    const Chunk cur = chunk_at(gr, r_end, g);
    gr += cur.cr;
    __syncthreads();  // the previous chunk's reads are done
    stage<NT>(x, dy, g, os, cs, cur, B0, t);
    __syncthreads();
    compute(g, B0, cur.cr * g.OW, wv, lane, acc);
  }
#endif
  // acc[mt][j][e] = dW[co = 64 os + 16 mt + 4 grp + e][tap J >> 2][c = 64 cs + 16 (J & 3) + (lane & 15)]
  const int grp = lane >> 4;
  float* dst = part + (size_t)split * g.Cout * 9 * g.C;
#pragma unroll
  for (int j = 0; j < 9; ++j) {
    const int J = 9 * wv + j, tap = J >> 2;
    const int c = CS * cs + 16 * (J & 3) + (lane & 15);
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int co = CS * os + 16 * mt + 4 * grp + e;
        dst[((size_t)co * 9 + tap) * g.C + c] = acc[mt][j][e];
      }
  }
}

// dw = sum over splits of part[split], part in [Cout][3][3][C] order; dw channels_last (cl = 1, the same order) or
// contiguous [Cout][C][3][3]. Block: 16 float4 columns x 16 split lanes; lane l adds splits l, l + 16, ... in order,
// then one thread per column adds the 16 lane sums in lane order (a fixed order: deterministic)
__global__ __launch_bounds__(256) void conv3_wgrad_sum(const float4* __restrict__ part, int n4, int splits, int C,
                                                       int cl, float* __restrict__ dw) {
  __shared__ float4 red[16][17];
  const int col = threadIdx.x & 15, sl = threadIdx.x >> 4;
  const int i = blockIdx.x * 16 + col;  // n4 % 16 == 0 (C % 64 == 0)
  float4 a = {0.f, 0.f, 0.f, 0.f};
  int s = sl;
  for (; s + 48 < splits; s += 64) {
    float4 v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) v[k] = part[(size_t)(s + 16 * k) * n4 + i];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      a.x += v[k].x;
      a.y += v[k].y;
      a.z += v[k].z;
      a.w += v[k].w;
    }
  }
  for (; s < splits; s += 16) {
    const float4 v = part[(size_t)s * n4 + i];
    a.x += v.x;
    a.y += v.y;
    a.z += v.z;
    a.w += v.w;
  }
  red[sl][col] = a;
  __syncthreads();
  if (sl != 0) return;
  for (int l = 1; l < 16; ++l) {
    const float4 v = red[l][col];
    a.x += v.x;
    a.y += v.y;
    a.z += v.z;
    a.w += v.w;
  }
  if (cl) {
    ((float4*)dw)[i] = a;
  } else {
    const float av[4] = {a.x, a.y, a.z, a.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int e = 4 * i + k, c = e % C, tap = (e / C) % 9, co = e / (9 * C);
      dw[((size_t)co * C + c) * 9 + tap] = av[k];
    }
  }
}

// chunk rows and LDS bytes for a shape: the most output rows (<= 256 pixel slots) that keep two workgroups per CU
int staged_width(int W, int S) { return S == 1 ? W + 2 : 2 * ((W + 3) / 2); }

void plan(int W, int OW, int S, int OH, int* cr_out, int* nps_out, int* lds_out) {
  const int XW = staged_width(W, S);
  int cr = 256 / OW;
  cr = cr < 1 ? 1 : (cr > OH ? OH : cr);
  for (;; --cr) {
    const int nps = (cr * OW + 31) & ~31, xr = (cr - 1) * S + 3;
    const int lds = buf_elems(nps, xr, XW) * 2;  // one staged chunk (bytes)
    if (lds <= 78 * 1024 || cr == 1) {
      *cr_out = cr;
      *nps_out = nps;
      *lds_out = C3_WS ? 2 * lds : lds;  // (wave-specialised: two buffers, one workgroup per CU)
      return;
    }
  }
}

}  // namespace

extern "C" {

// pixel splits for a shape (~256 workgroups, one per CU, wave-specialised; 512 otherwise: two per CU), so the caller
// can size part = splits * Cout * 9 * C floats
int mifx_conv3_wgrad_splits(int N, int H, int W, int C, int Cout, int S) {
  if (N <= 0 || H <= 0 || W <= 0 || C % 64 || Cout % 64 || (S != 1 && S != 2)) return -1;
  const int OH = (H - 1) / S + 1, slices = (C / 64) * (Cout / 64);
  const int target = C3_WS ? 256 : 512;
  int sp = (target + slices - 1) / slices;
  if (sp > N * OH) sp = N * OH;
  return sp < 1 ? 1 : sp;
}

// LDS bytes the kernel takes for a shape (-1: not supported)
int mifx_conv3_wgrad_lds_bytes(int W, int H, int S) {
  const int OH = (H - 1) / S + 1, OW = (W - 1) / S + 1;
  int cr, nps, lds;
  plan(W, OW, S, OH, &cr, &nps, &lds);
  return lds <= 160 * 1024 ? lds : -1;
}

// x bf16 NHWC [N, H, W, C], dy bf16 NHWC [N, OH, OW, Cout] (pad 1, stride S in {1, 2}, OH = (H - 1) / S + 1);
// part fp32 scratch of splits * Cout * 9 * C; dw fp32 [Cout, C, 3, 3] (dw_cl: channels_last storage)
int mifx_conv3_wgrad(const void* x, const void* dy, float* part, float* dw, int dw_cl, int N, int H, int W, int C,
                     int Cout, int S, int splits, hipStream_t st) {
  if (x == nullptr || dy == nullptr || part == nullptr || dw == nullptr) return -1;
  if (N <= 0 || H <= 0 || W <= 0 || C <= 0 || Cout <= 0 || C % 64 || Cout % 64 || (S != 1 && S != 2)) return -1;
  if ((uintptr_t)x % 16 || (uintptr_t)dy % 16 || (uintptr_t)part % 16 || (uintptr_t)dw % 16) return -1;
  const int OH = (H - 1) / S + 1, OW = (W - 1) / S + 1;
  if ((long long)N * H * W * C >= (1ll << 31) || (long long)N * OH * OW * Cout >= (1ll << 31)) return -1;
  if (splits < 1 || splits > N * OH) return -1;
  Geo g;
  g.N = N; g.H = H; g.W = W; g.C = C; g.Cout = Cout; g.OH = OH; g.OW = OW; g.S = S;
  g.XW = staged_width(W, S); g.HW = (W + 3) / 2; g.c1 = S == 1 ? 1 : g.HW; g.c2 = S == 1 ? 2 : 1;
  int lds;
  plan(W, OW, S, OH, &g.CR, &g.NPS, &lds);
  if (lds > 160 * 1024) return -1;
  g.splits = splits; g.ncs = C / 64; g.nslices = (C / 64) * (Cout / 64);
  const long long blocks = (long long)splits * g.nslices;
  if (blocks > 0x7fffffff || (long long)splits * Cout * 9 * C >= (1ll << 31)) return -1;
  static int attr_lds = 0;
  if (lds > 64 * 1024 && lds > attr_lds) {
    (void)hipFuncSetAttribute((const void*)conv3_wgrad, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    attr_lds = lds;
  }
  hipLaunchKernelGGL(conv3_wgrad, dim3((unsigned)blocks), dim3(NTK), lds, st, (const bf16*)x, (const bf16*)dy, part, g);
  const int n4 = Cout * 9 * C / 4;
  hipLaunchKernelGGL(conv3_wgrad_sum, dim3(n4 / 16), dim3(256), 0, st, (const float4*)part, n4, splits, C, dw_cl, dw);
  return (int)hipGetLastError();
}

}  // extern "C"
