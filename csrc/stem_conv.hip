// ResNet-50's stem convolution (7x7, stride 2, pad 3, 3 -> 64 channels) as an MFMA implicit GEMM for gfx950.
//
// Reference workload: the ImageNet ResNet-50 training job of the reference's TFJob examples (SURVEY KN14,
// `install-kubeflow/ks_app/vendor/kubeflow/examples/prototypes/tf-job-simple-v1beta2.jsonnet:28-38`). On MIOpen the
// forward ran as `igemm_fwd_gtcx35 ... bt256x64x8` at ~150 TFLOP/s (366-400 us per B=256 step,
// profiles/resnet_steady_r5za.md): three input channels give the generic implicit GEMM a K-tile of 3 and nothing to
// reuse. Here the reduction is laid out by KERNEL ROW: for output pixel (oh, ow) and kernel row r the 21 values
// (s, c) = x[2 oh - 3 + r][2 ow - 3 + s][c], s < 7, are CONTIGUOUS in an NHWC input row (7 pixels x 3 channels), so one
// MFMA K-step of 32 is one kernel row: elements q < 21 are the real taps, q = 21..31 read the next pixels of the same
// row and meet zero weights. 7 K-steps of v_mfma_f32_16x16x32_bf16 per 16 x 16 output tile, 34 % of them on padding --
// cheap next to the memory traffic, and no im2col gather or masking in the inner loop.
//
//  * Workgroup: ROWS = 16 output rows of one image (16 x OW pixels) x all 64 output channels, 4 waves. Each wave loads
//    its 28 weight fragments (bf16 image [64][7][32], L2-resident) into registers while the 37 input rows the
//    workgroup needs (zero rows / columns outside the image) are staged in LDS; after one barrier it runs, for every
//    4th 16-pixel tile, 7 x 4 MFMAs fed by 4-byte window reads.
//  * The weight is the MFMA A operand (16 output channels x 32 taps: one 16-byte LDS read per lane) and the input
//    window the B operand (32 taps x 16 pixels: 4 aligned 4-byte LDS reads per lane), so a lane's accumulator holds
//    four consecutive output channels of one pixel: 8-byte NHWC stores.
//  * stem_weight_image converts the fp32 parameter (NCHW or channels_last) to the padded bf16 image each step.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

typedef __bf16 bf16;
typedef __bf16 v8bf __attribute__((ext_vector_type(8)));
typedef __bf16 v4bf __attribute__((ext_vector_type(4)));
typedef float v4f __attribute__((ext_vector_type(4)));

constexpr int KH = 7, KW = 7, CIN = 3, COUT = 64, STR = 2, PAD = 3;
constexpr int Q = KW * CIN;                 // 21 taps per kernel row
constexpr int QP = 32;                      // one MFMA K-step
#ifndef STEM_ROWS
#define STEM_ROWS 16  // (8 / 12 / 16 same-box step A/B: 16 fastest, profiles/resnet_stem_rows_ab_r6.jsonl)
#endif
constexpr int ROWS = STEM_ROWS;             // output rows per workgroup
constexpr int IR = STR * (ROWS - 1) + KH;   // input rows staged
constexpr int NT = 256;

__device__ __forceinline__ v4f mfma(v8bf a, v8bf b, v4f c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}

// LDS input row length (bf16): (W + 2 PAD) CIN real/zero columns + slack for the padding taps of the last window
__host__ __device__ constexpr int lrow(int W) { return ((W + 2 * PAD) * CIN + 16 + 7) / 8 * 8; }

// w fp32 [64][3][7][7] (cl = 0: NCHW-contiguous; 1: channels_last, i.e. [64][7][7][3]) -> bf16 [64][7][32],
// q = s * 3 + c, zero for q >= 21
__global__ __launch_bounds__(256) void stem_weight_image(const float* __restrict__ w, int cl, bf16* __restrict__ img) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= COUT * KH * QP) return;
  const int q = i % QP, r = (i / QP) % KH, o = i / (QP * KH);
  float v = 0.f;
  if (q < Q) {
    const int s = q / CIN, c = q % CIN;
    v = cl ? w[o * (KH * Q) + r * Q + q] : w[((o * CIN + c) * KH + r) * KW + s];
  }
  img[i] = (bf16)v;
}

// grid (ceil(OH / ROWS), N); dynamic LDS: the input rows [IR][lrow(W)]
__global__ __launch_bounds__(NT) void stem_fwd(const bf16* __restrict__ x, const bf16* __restrict__ wimg,
                                               bf16* __restrict__ y, int H, int W, int OH, int OW) {
  extern __shared__ __attribute__((aligned(16))) bf16 lds[];
  bf16* xl = lds;
  const int LR = lrow(W);
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int n = blockIdx.y, oh0 = blockIdx.x * ROWS;

  const int pl = lane & 15, kg = lane >> 4;
  // the wave's A operands for every (kernel row, 16-channel tile), straight from the (L2-resident) weight image into
  // registers -- issued before the input staging so their latency overlaps it
  v8bf wa[KH][4];
#pragma unroll
  for (int r = 0; r < KH; ++r)
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) wa[r][nt] = *(const v8bf*)(wimg + (size_t)(nt * 16 + pl) * KH * QP + r * QP + 8 * kg);
  // ---- stage the input rows 2 oh0 - 3 .. (zeros outside the image; element (iw + 3) * 3 + c). Rows whose 3W
  // elements are 16-byte aligned in global memory (W % 8 == 0) move as 16-byte loads and 2-byte LDS stores (the LDS
  // image starts 9 elements into the row, which keeps the B reads 4-byte aligned); others element by element.
  const int row_elems = W * CIN;
  if (row_elems % 8 == 0 && (uintptr_t)x % 16 == 0) {
    const int nv = row_elems / 8;
    for (int i = t; i < IR * LR; i += NT) {  // zero the padding columns / out-of-image rows / slack
      const int ir = i / LR, e = i % LR, j = e - PAD * CIN, ih = STR * oh0 - PAD + ir;
      if (!(ih >= 0 && ih < H && j >= 0 && j < row_elems)) xl[i] = (bf16)0.f;
    }
    for (int i = t; i < IR * nv; i += NT) {
      const int ir = i / nv, v = i % nv, ih = STR * oh0 - PAD + ir;
      if (ih < 0 || ih >= H) continue;
      const v8bf d = *(const v8bf*)(x + ((size_t)n * H + ih) * row_elems + 8 * v);
      bf16* dst = xl + ir * LR + PAD * CIN + 8 * v;
#pragma unroll
      for (int u = 0; u < 8; ++u) dst[u] = d[u];
    }
  } else {
    for (int ir = 0; ir < IR; ++ir) {
      const int ih = STR * oh0 - PAD + ir;
      bf16* dst = xl + ir * LR;
      const bool in = ih >= 0 && ih < H;
      const bf16* src = x + ((size_t)n * H + (in ? ih : 0)) * row_elems;
      for (int e = t; e < LR; e += NT) {
        const int j = e - PAD * CIN;  // element of the image row
        dst[e] = (in && j >= 0 && j < row_elems) ? src[j] : (bf16)0.f;
      }
    }
  }
  __syncthreads();

  const int npix = ROWS * OW, ntiles = (npix + 15) / 16;
  for (int pt = wv; pt < ntiles; pt += 4) {
    const int p = pt * 16 + pl;
    const int orl = p < npix ? p / OW : 0, ow = p < npix ? p % OW : 0;
    const bool valid = p < npix && oh0 + orl < OH;
    v4f acc[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) acc[nt] = (v4f){0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int r = 0; r < KH; ++r) {
      // B: taps 8 kg .. 8 kg + 7 of kernel row r for this lane's pixel (4-byte aligned: even element offset)
      const uint32_t* bp = (const uint32_t*)(xl + (STR * orl + r) * LR + STR * CIN * ow + 8 * kg);
      const uint32_t bw[4] = {bp[0], bp[1], bp[2], bp[3]};
      const v8bf b = __builtin_bit_cast(v8bf, bw);
#pragma unroll
      for (int nt = 0; nt < 4; ++nt) acc[nt] = mfma(wa[r][nt], b, acc[nt]);
    }
    if (!valid) continue;
    // acc[nt][i] = y[pixel pl][channel nt 16 + 4 kg + i]
    bf16* dst = y + (((size_t)n * OH + oh0 + orl) * OW + ow) * COUT + 4 * kg;
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
      const v4bf o = {(bf16)acc[nt][0], (bf16)acc[nt][1], (bf16)acc[nt][2], (bf16)acc[nt][3]};
      *(v4bf*)(dst + nt * 16) = o;
    }
  }
}

// ---- weight gradient: dW[o][r][q] = sum over output pixels of dY[pixel][o] * X[2 oh + r][6 ow + q] (q = s 3 + c).
// C[64][224] = A[64 x pixels] B[pixels x 224] with the PIXELS as the MFMA reduction. One workgroup per (image, row
// split); it walks its output rows CR at a time: stage the 2 CR + 5 input rows (as the forward), the dY rows
// TRANSPOSED ([64][yrow]: an A fragment is 8 consecutive pixels of one channel, one 16-byte read; each thread moves
// 8 x 8 blocks, transposed in registers, so the LDS writes are 16 bytes too) and a table of the pixels' window offsets;
// then per 32-pixel K-step each wave multiplies the 4 channel tiles by its k-tiles {w, w + 4, ...} of the 14 (B
// fragment: 8 pixels of one tap, 8 2-byte reads at table offset + tap offset). Every workgroup writes its fp32 partial
// [64][224]; a second kernel sums the partials in workgroup order (deterministic) into the parameter layout.
constexpr int CR = 4;                       // output rows per staged chunk
constexpr int WIR = STR * (CR - 1) + KH;    // input rows per chunk
constexpr int KT = KH * QP / 16;            // 14 k-tiles of 16
// transposed dY row: the chunk's pixels rounded up to the 32-pixel K-step (zero-filled), + 8 to stagger the banks
__host__ __device__ constexpr int yrow(int OW) { return (CR * OW + 31) / 32 * 32 + 8; }

__global__ __launch_bounds__(NT) void stem_wgrad(const bf16* __restrict__ x, const bf16* __restrict__ dy,
                                                 float* __restrict__ part, int H, int W, int OH, int OW, int splits) {
  extern __shared__ __attribute__((aligned(16))) bf16 lds[];
  const int LR = lrow(W), YR = yrow(OW);  // input row / transposed dY row lengths
  const int NPM = YR - 8;                 // pixel slots per chunk (multiple of 32)
  bf16* yt = lds;                           // [64][YR]
  int* poff = (int*)(lds + COUT * YR);      // [NPM] window offset of each pixel slot
  bf16* xl = (bf16*)(poff + NPM);           // [WIR][LR]
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int n = blockIdx.x / splits, sp = blockIdx.x % splits;
  const int oh_b = (int)((long long)OH * sp / splits), oh_e = (int)((long long)OH * (sp + 1) / splits);
  const int pl = lane & 15, kg = lane >> 4;
  // this lane's tap offsets (kernel row r, element q) for its k-tiles
  int toff[4];
#pragma unroll
  for (int slot = 0; slot < 4; ++slot) {
    const int k = (wv + 4 * slot) * 16 + pl;
    toff[slot] = (k / QP) * LR + k % QP;
  }
  v4f acc[4][4];  // [o tile][own k-tile slot]
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 4; ++b) acc[a][b] = (v4f){0.f, 0.f, 0.f, 0.f};
  const int row_elems = W * CIN;
  const bool vec = row_elems % 8 == 0 && (uintptr_t)x % 16 == 0;
  for (int oh0 = oh_b; oh0 < oh_e; oh0 += CR) {
    const int rows = min(CR, oh_e - oh0), npix = rows * OW, np32 = (npix + 31) / 32 * 32;
    __syncthreads();  // the previous chunk's reads are done
    // input rows 2 oh0 - 3 .. (zeros outside the image)
    if (vec) {
      const int nv = row_elems / 8;
      for (int i = t; i < WIR * LR; i += NT) {
        const int ir = i / LR, e = i % LR, j = e - PAD * CIN, ih = STR * oh0 - PAD + ir;
        if (!(ih >= 0 && ih < H && j >= 0 && j < row_elems)) xl[i] = (bf16)0.f;
      }
      for (int i = t; i < WIR * nv; i += NT) {
        const int ir = i / nv, v = i % nv, ih = STR * oh0 - PAD + ir;
        if (ih < 0 || ih >= H) continue;
        const v8bf d = *(const v8bf*)(x + ((size_t)n * H + ih) * row_elems + 8 * v);
        bf16* dst = xl + ir * LR + PAD * CIN + 8 * v;
#pragma unroll
        for (int u = 0; u < 8; ++u) dst[u] = d[u];
      }
    } else {
      for (int i = t; i < WIR * LR; i += NT) {
        const int ir = i / LR, e = i % LR, j = e - PAD * CIN, ih = STR * oh0 - PAD + ir;
        xl[i] = (ih >= 0 && ih < H && j >= 0 && j < row_elems) ? x[((size_t)n * H + ih) * row_elems + j] : (bf16)0.f;
      }
    }
    // window offsets; slots beyond npix repeat the last pixel (dY is zero there)
    for (int p = t; p < np32; p += NT) {
      const int pc = min(p, npix - 1), orl = pc / OW;
      poff[p] = STR * orl * LR + STR * CIN * (pc - orl * OW);
    }
    // dY rows oh0 .. oh0 + rows - 1 transposed, in 8 (pixel) x 8 (channel) blocks, pixel block fastest over the
    // threads (conflict-free 16-byte LDS writes); pixels beyond npix are zero
    const int nb8 = np32 / 8;
    for (int i = t; i < nb8 * (COUT / 8); i += NT) {
      const int p8 = i % nb8, o8 = (i / nb8) * 8;
      v8bf d[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int p = 8 * p8 + u;
        d[u] = p < npix ? *(const v8bf*)(dy + (((size_t)n * OH + oh0) * OW + p) * COUT + o8) : (v8bf){};
      }
#pragma unroll
      for (int c = 0; c < 8; ++c) {
        const v8bf col = {d[0][c], d[1][c], d[2][c], d[3][c], d[4][c], d[5][c], d[6][c], d[7][c]};
        *(v8bf*)(yt + (o8 + c) * YR + 8 * p8) = col;
      }
    }
    __syncthreads();
    for (int p0 = 0; p0 < npix; p0 += 32) {
      v8bf af[4];
#pragma unroll
      for (int mt = 0; mt < 4; ++mt) af[mt] = *(const v8bf*)(yt + (mt * 16 + pl) * YR + p0 + 8 * kg);
      int po[8];
      *(int4*)po = *(const int4*)(poff + p0 + 8 * kg);
      *(int4*)(po + 4) = *(const int4*)(poff + p0 + 8 * kg + 4);
#pragma unroll
      for (int slot = 0; slot < 4; ++slot) {
        if (wv + 4 * slot >= KT) break;
        v8bf b;
#pragma unroll
        for (int u = 0; u < 8; ++u) b[u] = xl[po[u] + toff[slot]];
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) acc[mt][slot] = mfma(af[mt], b, acc[mt][slot]);
      }
    }
  }
  // acc[mt][slot][i] = C[o = mt 16 + 4 kg + i][k = ktile 16 + pl]
  float* dst = part + (size_t)blockIdx.x * COUT * KH * QP;
#pragma unroll
  for (int slot = 0; slot < 4; ++slot) {
    const int ktile = wv + 4 * slot;
    if (ktile >= KT) break;
#pragma unroll
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
      for (int i = 0; i < 4; ++i) dst[(size_t)(mt * 16 + 4 * kg + i) * (KH * QP) + ktile * 16 + pl] = acc[mt][slot][i];
  }
}

// dW (fp32, the parameter's layout) = sum of the G partials in order, taps q < 21 only
__global__ __launch_bounds__(256) void stem_wgrad_reduce(const float* __restrict__ part, int G, float* __restrict__ dw,
                                                         int cl) {
  const int i = blockIdx.x * 256 + threadIdx.x;  // over 64 x 7 x 21
  if (i >= COUT * KH * Q) return;
  const int q = i % Q, r = (i / Q) % KH, o = i / (Q * KH);
  const size_t col = (size_t)o * KH * QP + r * QP + q;
  float a = 0.f;
  int g = 0;
  for (; g + 8 <= G; g += 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = part[(size_t)(g + u) * COUT * KH * QP + col];
#pragma unroll
    for (int u = 0; u < 8; ++u) a += v[u];
  }
  for (; g < G; ++g) a += part[(size_t)g * COUT * KH * QP + col];
  const int s = q / CIN, c = q % CIN;
  dw[cl ? (size_t)o * (KH * Q) + r * Q + q : ((size_t)(o * CIN + c) * KH + r) * KW + s] = a;
}

}  // namespace

extern "C" {

int mifx_stem_lds_bytes(int W) { return IR * lrow(W) * 2; }

// x: bf16 NHWC [N, H, W, 3]; w: fp32 [64, 3, 7, 7] (w_cl: channels_last storage); wimg: bf16 scratch [64 * 7 * 32];
// y: bf16 NHWC [N, OH, OW, 64], OH = (H - 1) / 2 + 1, OW = (W - 1) / 2 + 1
int mifx_stem_fwd(const void* x, const float* w, int w_cl, void* wimg, void* y, int N, int H, int W,
                  hipStream_t st) {
  if (x == nullptr || w == nullptr || wimg == nullptr || y == nullptr || N <= 0 || H < 1 || W < 1 || W > 4096)
    return -1;
  if ((uintptr_t)x % 2 || (uintptr_t)wimg % 16 || (uintptr_t)y % 8) return -1;
  const int OH = (H + 2 * PAD - KH) / STR + 1, OW = (W + 2 * PAD - KW) / STR + 1;
  const int lds = mifx_stem_lds_bytes(W);
  if (lds > 160 * 1024) return -1;
  static int attr_lds = 0;
  if (lds > 64 * 1024 && lds > attr_lds) {
    (void)hipFuncSetAttribute((const void*)stem_fwd, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    attr_lds = lds;
  }
  hipLaunchKernelGGL(stem_weight_image, dim3((COUT * KH * QP + 255) / 256), dim3(256), 0, st, w, w_cl, (bf16*)wimg);
  hipLaunchKernelGGL(stem_fwd, dim3((OH + ROWS - 1) / ROWS, N), dim3(NT), lds, st, (const bf16*)x,
                     (const bf16*)wimg, (bf16*)y, H, W, OH, OW);
  return (int)hipGetLastError();
}


// workgroups per image: at least 512 in all (two per CU: one stages while the other multiplies)
int mifx_stem_wgrad_splits(int N) { return N >= 512 ? 1 : (512 + N - 1) / N; }
int mifx_stem_wgrad_lds_bytes(int W) {
  const int OW = (W + 2 * PAD - KW) / STR + 1;
  return COUT * yrow(OW) * 2 + (yrow(OW) - 8) * 4 + WIR * lrow(W) * 2;
}

// dW of the stem: x bf16 NHWC [N, H, W, 3], dy bf16 NHWC [N, OH, OW, 64]; part: fp32 scratch of
// N * splits * 64 * 224 floats (splits = mifx_stem_wgrad_splits(N)); dw: fp32 [64, 3, 7, 7] (dw_cl: channels_last)
int mifx_stem_wgrad(const void* x, const void* dy, float* part, float* dw, int dw_cl, int N, int H, int W,
                    hipStream_t st) {
  if (x == nullptr || dy == nullptr || part == nullptr || dw == nullptr || N <= 0 || H < 1 || W < 1 || W > 4096)
    return -1;
  if ((uintptr_t)dy % 16) return -1;
  const int OH = (H + 2 * PAD - KH) / STR + 1, OW = (W + 2 * PAD - KW) / STR + 1;
  const int lds = mifx_stem_wgrad_lds_bytes(W);
  if (lds > 160 * 1024) return -1;
  static int attr_lds = 0;
  if (lds > 64 * 1024 && lds > attr_lds) {
    (void)hipFuncSetAttribute((const void*)stem_wgrad, hipFuncAttributeMaxDynamicSharedMemorySize, lds);
    attr_lds = lds;
  }
  const int splits = mifx_stem_wgrad_splits(N);
  hipLaunchKernelGGL(stem_wgrad, dim3(N * splits), dim3(NT), lds, st, (const bf16*)x, (const bf16*)dy, part, H, W, OH,
                     OW, splits);
  hipLaunchKernelGGL(stem_wgrad_reduce, dim3((COUT * KH * Q + 255) / 256), dim3(256), 0, st, part, N * splits, dw,
                     dw_cl);
  return (int)hipGetLastError();
}

}  // extern "C"
