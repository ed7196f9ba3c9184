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
//  * Workgroup: ROWS = 4 output rows of one image (4 x OW pixels) x all 64 output channels, 4 waves. The 11 input rows
//    it needs (zero rows / columns outside the image) and the bf16 weight image [64][7][32] (+8 pad per channel row:
//    conflict-free 16-byte fragment reads) are staged in LDS once; then each wave loads its 28 weight fragments into registers once
//    and, for every 4th 16-pixel tile, runs 7 x 4 MFMAs fed by 4-byte window reads, with no further barrier.
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
constexpr int WROW = KH * QP + 8;           // weight image row (one output channel) in LDS, bf16 elements
#ifndef STEM_ROWS
#define STEM_ROWS 4
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

// grid (ceil(OH / ROWS), N); dynamic LDS: weights [64][WROW] then input rows [IR][lrow(W)]
__global__ __launch_bounds__(NT) void stem_fwd(const bf16* __restrict__ x, const bf16* __restrict__ wimg,
                                               bf16* __restrict__ y, int H, int W, int OH, int OW) {
  extern __shared__ __attribute__((aligned(16))) bf16 lds[];
  bf16* wl = lds;
  bf16* xl = lds + COUT * WROW;
  const int LR = lrow(W);
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  const int n = blockIdx.y, oh0 = blockIdx.x * ROWS;

  // ---- stage the weight image (16-byte chunks: [64][7][32] -> rows of WROW)
  for (int i = t; i < COUT * KH * QP / 8; i += NT) {
    const int o = i / (KH * QP / 8), j = i % (KH * QP / 8);
    *(v8bf*)(wl + o * WROW + 8 * j) = *(const v8bf*)(wimg + (size_t)o * KH * QP + 8 * j);
  }
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
  const int pl = lane & 15, kg = lane >> 4;
  // the wave's A operands for every (kernel row, 16-channel tile): read once, kept in registers over its pixel tiles
  v8bf wa[KH][4];
#pragma unroll
  for (int r = 0; r < KH; ++r)
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) wa[r][nt] = *(const v8bf*)(wl + (nt * 16 + pl) * WROW + r * QP + 8 * kg);
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

}  // namespace

extern "C" {

int mifx_stem_lds_bytes(int W) { return (COUT * WROW + IR * lrow(W)) * 2; }

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

}  // extern "C"
