// Full-pass analyzer + evaluation kernels for gfx950 (Transform / StatisticsGen / Evaluator).
//
// Reference ops: tft.scale_to_z_score mean/var reduction
// (`airflow-dags/taxi_utils.py:116-119`), tft.bucketize apply (`taxi_utils.py:128-130`), TFDV
// numeric column statistics, TFMA sliced metrics with bucketed confusion-matrix AUC.
//
//  * col_moments: grid-stride fp64 Welford/Chan reduction (count, mean, M2, min, max, zeros):
//    wave-level shuffle combine, one LDS pass per block, per-block partials combined by a single
//    block in the second launch (deterministic: fixed combine order).
//  * bucketize: boundaries staged in LDS, branch-free binary search per element, 4 elements/thread.
//  * segment_hist: per-slice (count, label sum, pred sum, loss sum, correct) + a NB-bucket prediction
//    histogram split by label, accumulated in LDS with ds_add then flushed with one global atomic
//    per non-zero bin (host turns the histograms into AUC / precision / recall).
//  * hist / select: equal-width or explicit-edge histograms (TFDV), and the exact order-statistic selection behind
//    tft.quantiles / bucketize boundaries and TFDV quantiles / median: a uniform histogram narrows every wanted
//    rank to one bin, the few values of those bins are gathered and ordered on the host (repeated on a bin that is
//    too full) -- exact np.quantile results without a device sort.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

struct Mom {
  double n, mean, m2, mn, mx, zeros;
};

__device__ __forceinline__ Mom combine(const Mom& a, const Mom& b) {
  if (a.n == 0) return b;
  if (b.n == 0) return a;
  Mom r;
  r.n = a.n + b.n;
  const double d = b.mean - a.mean;
  r.mean = a.mean + d * (b.n / r.n);
  r.m2 = a.m2 + b.m2 + d * d * (a.n * b.n / r.n);
  r.mn = fmin(a.mn, b.mn);
  r.mx = fmax(a.mx, b.mx);
  r.zeros = a.zeros + b.zeros;
  return r;
}

__device__ __forceinline__ Mom shfl_down(const Mom& m, int o) {
  Mom r;
  r.n = __shfl_down(m.n, o);
  r.mean = __shfl_down(m.mean, o);
  r.m2 = __shfl_down(m.m2, o);
  r.mn = __shfl_down(m.mn, o);
  r.mx = __shfl_down(m.mx, o);
  r.zeros = __shfl_down(m.zeros, o);
  return r;
}

__device__ Mom block_reduce(Mom m) {
  __shared__ Mom part[16];
  for (int o = 32; o > 0; o >>= 1) m = combine(m, shfl_down(m, o));
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  if (lane == 0) part[w] = m;
  __syncthreads();
  Mom r = {0, 0, 0, INFINITY, -INFINITY, 0};
  if (threadIdx.x == 0) {
    for (int i = 0; i < (int)(blockDim.x >> 6); ++i) r = combine(r, part[i]);
  }
  return r;
}

// pass 1: each block reduces a grid-strided slice of x (NaNs skipped)
__global__ __launch_bounds__(256) void col_moments_p1(const double* __restrict__ x, long long n,
                                                      Mom* __restrict__ partial) {
  Mom m = {0, 0, 0, INFINITY, -INFINITY, 0};
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const double v = x[i];
    if (v != v) continue;
    Mom one = {1, v, 0, v, v, v == 0.0 ? 1.0 : 0.0};
    m = combine(m, one);
  }
  Mom r = block_reduce(m);
  if (threadIdx.x == 0) partial[blockIdx.x] = r;
}

__global__ __launch_bounds__(256) void col_moments_p2(const Mom* __restrict__ partial, int np,
                                                      double* __restrict__ out) {
  Mom m = {0, 0, 0, INFINITY, -INFINITY, 0};
  for (int i = threadIdx.x; i < np; i += 256) m = combine(m, partial[i]);  // fixed order per thread
  Mom r = block_reduce(m);
  if (threadIdx.x == 0) {
    out[0] = r.n;
    out[1] = r.mean;
    out[2] = r.n > 0 ? r.m2 / r.n : 0.0;  // population variance (tft.var)
    out[3] = r.mn;
    out[4] = r.mx;
    out[5] = r.zeros;
  }
}

// bucket index = number of boundaries <= x  (tf.raw_ops.Bucketize / tft.apply_buckets)
__global__ __launch_bounds__(256) void bucketize_k(const double* __restrict__ x, long long n,
                                                   const double* __restrict__ bnd, int nb,
                                                   long long* __restrict__ out) {
  __shared__ double b[1024];
  for (int i = threadIdx.x; i < nb; i += 256) b[i] = bnd[i];
  __syncthreads();
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const double v = x[i];
    int lo = 0, hi = nb;
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      const bool le = b[mid] <= v;
      lo = le ? mid + 1 : lo;
      hi = le ? hi : mid;
    }
    out[i] = lo;
  }
}

// per-slice sums + label-split prediction histograms; NS*NB*2 bins in global, LDS staging when it fits
__global__ __launch_bounds__(256) void segment_hist_k(const int* __restrict__ seg, const float* __restrict__ label,
                                                      const float* __restrict__ prob, long long n, int ns, int nb,
                                                      double* __restrict__ sums /*[ns][5]*/,
                                                      unsigned int* __restrict__ hist /*[ns][nb][2]*/) {
  extern __shared__ unsigned int lhist[];
  const int nbins = ns * nb * 2;
  const bool use_lds = nbins <= 32768;
  if (use_lds) {
    for (int i = threadIdx.x; i < nbins; i += 256) lhist[i] = 0;
    __syncthreads();
  }
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const int s = seg[i];
    if (s < 0 || s >= ns) continue;
    const float y = label[i];
    const float p = fminf(fmaxf(prob[i], 1e-7f), 1.f - 1e-7f);
    const int yb = y > 0.5f ? 1 : 0;
    int b = (int)((double)p * nb);  // fp64 product: bucket edges must match the host definition
    b = b >= nb ? nb - 1 : b;
    const int bin = (s * nb + b) * 2 + yb;
    if (use_lds) atomicAdd(&lhist[bin], 1u);
    else atomicAdd(&hist[bin], 1u);
    const double loss = -(y * log((double)p) + (1.0 - y) * log(1.0 - (double)p));
    atomicAdd(&sums[s * 5 + 0], 1.0);
    atomicAdd(&sums[s * 5 + 1], (double)y);
    atomicAdd(&sums[s * 5 + 2], (double)p);
    atomicAdd(&sums[s * 5 + 3], loss);
    atomicAdd(&sums[s * 5 + 4], ((p > 0.5f) == (y > 0.5f)) ? 1.0 : 0.0);
  }
  if (use_lds) {
    __syncthreads();
    for (int i = threadIdx.x; i < nbins; i += 256)
      if (lhist[i]) atomicAdd(&hist[i], lhist[i]);
  }
}

// ---- histograms (TFDV equal-width histograms, integer value counts, quantile narrowing)
// mode 0 (edges): bin = searchsorted(edges, x, right) - 1 over nb + 1 sorted edges, the last bin closed --
//   np.histogram's binning exactly (values outside [e0, e_nb] dropped); nb <= 4096.
// mode 1 (uniform): bin = floor((x - lo) * inv), values with bin outside [0, nb) dropped; monotone in x (IEEE
//   subtraction / multiplication by a positive constant), which is all the exact quantile selection needs;
//   integer unit bins (inv = 1) are exact for integer-valued doubles.
// Counts in LDS (ds_add) when nb <= 16384, one global atomic per non-zero bin per block; global atomics beyond.
constexpr int HIST_LDS_BINS = 16384;

__global__ __launch_bounds__(256) void hist_k(const double* __restrict__ x, long long n, int mode,
                                              const double* __restrict__ edges, double lo, double inv, int nb,
                                              unsigned long long* __restrict__ counts) {
  extern __shared__ unsigned int lh[];
  __shared__ double se[4097];
  const bool use_lds = nb <= HIST_LDS_BINS;
  if (use_lds)
    for (int i = threadIdx.x; i < nb; i += 256) lh[i] = 0;
  if (mode == 0)
    for (int i = threadIdx.x; i <= nb; i += 256) se[i] = edges[i];
  __syncthreads();
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const double v = x[i];
    if (v != v) continue;
    int b;
    if (mode == 0) {
      if (v < se[0] || v > se[nb]) continue;
      int l = 0, h = nb + 1;  // number of edges <= v
      while (l < h) {
        const int mid = (l + h) >> 1;
        const bool le = se[mid] <= v;
        l = le ? mid + 1 : l;
        h = le ? h : mid;
      }
      b = l - 1;
      if (b >= nb) b = nb - 1;  // v == last edge: the closed last bin
    } else {
      const double f = (v - lo) * inv;
      if (!(f >= 0.0) || f >= (double)nb) continue;
      b = (int)f;
    }
    if (use_lds)
      atomicAdd(&lh[b], 1u);
    else
      atomicAdd(&counts[b], 1ull);
  }
  if (use_lds) {
    __syncthreads();
    for (int i = threadIdx.x; i < nb; i += 256)
      if (lh[i]) atomicAdd(&counts[i], (unsigned long long)lh[i]);
  }
}

// candidate gather of the exact quantile selection: values whose uniform bin b has slot[b] >= 0 are appended to
// out[slot * cap + pos] (pos from a per-slot counter; counts past cap are still counted, the host then narrows)
__global__ __launch_bounds__(256) void select_k(const double* __restrict__ x, long long n, double lo, double inv,
                                                int nb, const int* __restrict__ slot, int cap,
                                                unsigned int* __restrict__ cnt, double* __restrict__ out) {
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const double v = x[i];
    if (v != v) continue;
    const double f = (v - lo) * inv;
    if (!(f >= 0.0) || f >= (double)nb) continue;
    const int s = slot[(int)f];
    if (s < 0) continue;
    const unsigned int p = atomicAdd(&cnt[s], 1u);
    if (p < (unsigned int)cap) out[(size_t)s * cap + p] = v;
  }
}

}  // namespace

extern "C" {

int mifx_an_histogram(const double* x, long long n, int mode, const double* edges, double lo, double inv, int nb,
                      unsigned long long* counts, hipStream_t st) {
  if (nb <= 0 || (mode == 0 && (edges == nullptr || nb > 4096)) || mode < 0 || mode > 1) return -1;
  const long long blocks = (n + 1023) / 1024;
  const int grid = (int)(blocks < 1024 ? (blocks > 0 ? blocks : 1) : 1024);
  const size_t lds = nb <= HIST_LDS_BINS ? (size_t)nb * 4 : 0;
  if (lds > 32768) (void)hipFuncSetAttribute((const void*)hist_k, hipFuncAttributeMaxDynamicSharedMemorySize, 65536);
  hipLaunchKernelGGL(hist_k, dim3(grid), dim3(256), lds, st, x, n, mode, edges, lo, inv, nb, counts);
  return (int)hipGetLastError();
}

int mifx_an_select(const double* x, long long n, double lo, double inv, int nb, const int* slot, int cap,
                   unsigned int* cnt, double* out, hipStream_t st) {
  if (nb <= 0 || cap <= 0) return -1;
  const long long blocks = (n + 1023) / 1024;
  const int grid = (int)(blocks < 1024 ? (blocks > 0 ? blocks : 1) : 1024);
  hipLaunchKernelGGL(select_k, dim3(grid), dim3(256), 0, st, x, n, lo, inv, nb, slot, cap, cnt, out);
  return (int)hipGetLastError();
}


int mifx_an_moments(const double* x, long long n, void* partial, int grid, double* out, hipStream_t st) {
  if (grid <= 0 || grid > 4096) return -1;
  hipLaunchKernelGGL(col_moments_p1, dim3(grid), dim3(256), 0, st, x, n, (Mom*)partial);
  hipLaunchKernelGGL(col_moments_p2, dim3(1), dim3(256), 0, st, (const Mom*)partial, grid, out);
  return (int)hipGetLastError();
}

int mifx_an_moments_partial_bytes() { return (int)sizeof(Mom); }

int mifx_an_bucketize(const double* x, long long n, const double* bnd, int nb, long long* out, hipStream_t st) {
  if (nb < 0 || nb > 1024) return -1;
  const long long blocks = (n + 255) / 256;
  const int grid = (int)(blocks < 4096 ? (blocks > 0 ? blocks : 1) : 4096);
  hipLaunchKernelGGL(bucketize_k, dim3(grid), dim3(256), 0, st, x, n, bnd, nb, out);
  return (int)hipGetLastError();
}

int mifx_an_segment_hist(const int* seg, const float* label, const float* prob, long long n, int ns, int nb,
                         double* sums, unsigned int* hist, hipStream_t st) {
  if (ns <= 0 || nb <= 0) return -1;
  const long long blocks = (n + 255) / 256;
  const int grid = (int)(blocks < 1024 ? (blocks > 0 ? blocks : 1) : 1024);
  const int nbins = ns * nb * 2;
  const size_t lds = nbins <= 32768 ? (size_t)nbins * 4 : 0;
  if (lds > 65536) (void)hipFuncSetAttribute((const void*)segment_hist_k,
                                             hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
  hipLaunchKernelGGL(segment_hist_k, dim3(grid), dim3(256), lds, st, seg, label, prob, n, ns, nb, sums, hist);
  return (int)hipGetLastError();
}

}  // extern "C"
