// Exact-fp32 MFMA GEMM with edge tiles for gfx950: C[M, N] = A[M, K] . B[K, N] (row-major, any M, N, K).
//
// KN18, the reference's only recorded number: an eager 1000 x 1000 fp32 matmul on CPU, 9.87 ms
// (`notebooks/tf2.0/EagerExecution.ipynb:L491-L511`, output `:528-530`). torch.matmul sends that shape to hipBLASLt;
// the bf16 kernels of csrc/gemm.hip need whole 256-wide tiles and K % 64 and are bf16. This kernel is the
// reference's op as written -- fp32 in, fp32 accumulate, fp32 out -- on the f32 matrix cores
// (v_mfma_f32_16x16x4_f32: exact fp32 products and sums, 64 FLOP / cycle / SIMD, the fp32 vector rate), with
// ragged edges handled in the tile loads (zero fill outside the matrix) and masked stores.
//
// Tiling: 64 x 64 output tile per 256-thread workgroup (1000 x 1000 -> 16 x 16 = 256 tiles: one per CU), 4 waves
// each owning a 32 x 32 quarter (2 x 2 MFMA tiles); K in tiles of 16, staged k-major in LDS ([16][64 + 4] per
// operand: conflict-free fragment reads) and double-buffered, so the next tile's global loads are in flight while
// the current tile's 16 MFMAs per wave run. Per k-step of 4 an MFMA lane holds A[row l % 16][k l / 16] and
// B[k l / 16][col l % 16]; the accumulator lane holds C[4 (l / 16) + i][l % 16].
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

constexpr int BM = 64, BN = 64, BK = 16, LDP = 64 + 4, NT = 256;
typedef float v4f __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(NT) void gemm_f32_nn(const float* __restrict__ A, const float* __restrict__ B,
                                                  float* __restrict__ C, int M, int N, int K, int lda, int ldb,
                                                  int ldc) {
  __shared__ float As[2][BK][LDP];
  __shared__ float Bs[2][BK][LDP];
  const int tid = threadIdx.x, w = tid >> 6, lane = tid & 63;
  const int nb_n = (N + BN - 1) / BN;
  // XCD-aware tile order: the 8 workgroups dispatched together land on 8 XCDs; give each XCD a contiguous run of
  // tiles (shared A rows / B columns in its L2)
  const int nwg = gridDim.x, bid = blockIdx.x, xcd = bid % 8, q = nwg / 8, rr = nwg % 8;
  const int tile = (xcd < rr ? xcd * (q + 1) : rr * (q + 1) + (xcd - rr) * q) + bid / 8;
  const int m0 = (tile / nb_n) * BM, n0 = (tile % nb_n) * BN;
  const int wm = w >> 1, wn = w & 1;

  // staging: thread t loads A[m0 + t / 4][k0 + 4 (t % 4) .. +3] and B[k0 + t / 16][n0 + 4 (t % 16) .. +3]
  const int ar = tid >> 2, ak = (tid & 3) * 4;
  const int bk = tid >> 4, bc = (tid & 15) * 4;
  float ra[4], rb[4];
  auto load = [&](int k0) {
    const int gm = m0 + ar;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int gk = k0 + ak + i;
      ra[i] = (gm < M && gk < K) ? A[(size_t)gm * lda + gk] : 0.f;
    }
    const int gk = k0 + bk;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int gn = n0 + bc + i;
      rb[i] = (gk < K && gn < N) ? B[(size_t)gk * ldb + gn] : 0.f;
    }
  };
  auto store = [&](int buf) {
#pragma unroll
    for (int i = 0; i < 4; ++i) As[buf][ak + i][ar] = ra[i];
#pragma unroll
    for (int i = 0; i < 4; ++i) Bs[buf][bk][bc + i] = rb[i];
  };

  v4f acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) acc[i][j] = (v4f){0.f, 0.f, 0.f, 0.f};

  const int KT = (K + BK - 1) / BK;
  load(0);
  store(0);
  __syncthreads();
  const int fr = lane & 15, fk = lane >> 4;
  for (int kt = 0; kt < KT; ++kt) {
    const int cur = kt & 1;
    if (kt + 1 < KT) load((kt + 1) * BK);  // next tile's global loads in flight under this tile's MFMAs
#pragma unroll
    for (int s = 0; s < BK / 4; ++s) {
      float a[2], b[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) a[i] = As[cur][4 * s + fk][wm * 32 + 16 * i + fr];
#pragma unroll
      for (int j = 0; j < 2; ++j) b[j] = Bs[cur][4 * s + fk][wn * 32 + 16 * j + fr];
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 2; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a[i], b[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < KT) store(cur ^ 1);  // the other buffer: its last readers finished before the previous barrier
    __syncthreads();
  }
  // acc[i][j] lane l: C[m0 + wm 32 + 16 i + 4 (l / 16) + e][n0 + wn 32 + 16 j + l % 16]
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int gn = n0 + wn * 32 + 16 * j + fr;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int gm = m0 + wm * 32 + 16 * i + 4 * fk + e;
        if (gm < M && gn < N) C[(size_t)gm * ldc + gn] = acc[i][j][e];
      }
    }
}

}  // namespace

extern "C" {

// C[M, N] = A[M, K] . B[K, N], fp32 row-major with leading dimensions lda >= K, ldb >= N, ldc >= N (elements).
int mifx_gemm_f32_nn(const float* A, const float* B, float* C, int M, int N, int K, int lda, int ldb, int ldc,
                     hipStream_t st) {
  if (M <= 0 || N <= 0 || K <= 0 || A == nullptr || B == nullptr || C == nullptr || lda < K || ldb < N || ldc < N)
    return -1;
  if ((long long)M * lda >= (1ll << 40) || (long long)K * ldb >= (1ll << 40)) return -1;
  const int tiles = ((M + BM - 1) / BM) * ((N + BN - 1) / BN);
  hipLaunchKernelGGL(gemm_f32_nn, dim3(tiles), dim3(NT), 0, st, A, B, C, M, N, K, lda, ldb, ldc);
  return (int)hipGetLastError();
}

}  // extern "C"
