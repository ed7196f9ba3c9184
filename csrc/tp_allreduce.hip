// Two-shot all-reduce of bf16 activations over xGMI peer memory, for tensor parallelism (BERT, BASELINE config 4).
//
// Megatron-style TP reduces a [tokens, hidden] activation after every row-parallel projection (attention out, FFN
// out) and every column-parallel input gradient: 2 + 2 per transformer block per step, 6.3 MB each at B = 32,
// S = 128. Issued through torch.distributed they are host-side collectives between kernels (no hipGraph capture of
// the TP step, a host round trip each). Here each rank's partial is exchanged through IPC-mapped HBM with device-side
// epoch flags, in three stream-ordered kernels that capture into a graph:
//
//   A  tpar_publish   (one workgroup per 8 KB chunk): copy the partial into this rank's IPC buffer half (epoch & 1)
//                     with system-scope stores, then stamp flag[0][chunk][rank] = epoch in every peer;
//   B  tpar_reduce    (chunks c with c % world == rank): wait for every peer's stamp of c, sum the world partials
//                     of c in rank order in fp32 (identical bits on every rank), round to bf16 into this rank's
//                     reduced buffer half, stamp flag[1][c][rank] in every peer (the reduce-scatter);
//   C  tpar_gather    (every chunk): wait for the owner's phase-1 stamp, copy its reduced chunk into the output (the
//                     all-gather); the last workgroup advances the epoch counter.
//
// Bytes over xGMI per rank: (world - 1) / world of the tensor twice (the two shots), instead of (world - 1) x the
// tensor for a one-shot sum; point-to-point links to every peer at once (xGMI full mesh, no ring hops).
// Double buffering by epoch parity makes one flag per chunk and phase enough (a rank rewrites half (e & 1) only in
// epoch e + 2, after every peer's epoch e + 1 kernel A stamp, which that peer issued after its epoch e kernels B and
// C had read the half). Waits run in one-wave workgroups and are bounded by wall-clock time: a peer that never
// arrives sets the sticky err flag; every later kernel of this group then does nothing (the host raises at its
// next check) instead of hanging the GPU. Data moves as 8-byte system-scope accesses (write-through stores, L2-
// bypassing loads), so no cache maintenance is needed anywhere.
//
// Split waits (mifx_tpar_allreduce2 with waiters = 1): kernels B and C above spin inside their data-moving workgroups,
// one per chunk -- thousands of waves that can hold every CU while a peer is late. A kernel that needs whole CUs
// (csrc/gemm8.hip's 8-wave workgroups: the deferred weight-gradient flush) then cannot start, on another rank's stream
// sharing the GPU or on this rank's own compute stream while the exchange runs on a side stream (data parallelism).
// With split waits NO data-moving workgroup ever waits: each data kernel's last-arriving workgroup (an arrival
// counter, no spinning) stamps ONE per-rank flag in every peer, and the waiting is done by a separate one-wave kernel
// (tpar_wait: lane p polls peer p's stamp with s_sleep backoff, bounded by the same timeout) between the data kernels:
//   publish -> wait(phase 0) -> reduce -> wait(phase 1) -> gather.
// Two more launches per all-reduce, a footprint of one wave while waiting. The per-rank stamps reuse the chunk-0
// flag slots; the double-buffering argument is unchanged (every data kernel of epoch e + 1 runs after a wait that saw
// all peers' epoch e + 1 stamps, issued after their epoch e reads).
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

constexpr int MAXW = 8;
constexpr int CHUNK = 4096;          // bf16 elements per chunk (8 KB)
constexpr int WG = 64;               // one wave per workgroup
constexpr int PER_LANE = CHUNK / 4 / WG;  // uint64 (4 x bf16) per lane per chunk = 16
constexpr long long TIMEOUT_TICKS = 12000ll * 1000 * 1000;  // 120 s at the 100 MHz real-time clock (8 ranks time-sharing one
// GPU in the rehearsals: a rank held up on the host for seconds must not trip it)

struct Peers {
  uint64_t* buf[MAXW];     // peer p's partial buffer [2][npad / 4] (uint64 = 4 bf16)
  uint64_t* red[MAXW];     // peer p's reduced buffer [2][npad / 4]
  unsigned int* flag[MAXW];  // peer p's flags [2][nchunks][MAXW] (uncached)
};

__device__ __forceinline__ void st_sys64(uint64_t* p, uint64_t v) {
  __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ uint64_t ld_sys64(const uint64_t* p) {
  return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
}
__device__ __forceinline__ bool failed(const int* err) {
  return __hip_atomic_load(err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) != 0;
}
__device__ __forceinline__ void publish(unsigned int* f, unsigned int e) {
  __hip_atomic_store(f, e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
}
// wait until *f reaches epoch e (wrapping compare); false on timeout or an earlier failure
__device__ __forceinline__ bool wait_flag(const unsigned int* f, unsigned int e, int* err) {
  const long long t0 = wall_clock64();
  while ((int)(__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) - e) < 0) {
    __builtin_amdgcn_s_sleep(2);
    if (failed(err)) return false;
    if (wall_clock64() - t0 > TIMEOUT_TICKS) {
      __hip_atomic_store(err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
      return false;
    }
  }
  return true;
}

__device__ __forceinline__ float2 bf2f(uint32_t u) {
  return make_float2(__uint_as_float(u << 16), __uint_as_float(u & 0xffff0000u));
}
__device__ __forceinline__ uint32_t f2bf(float a, float b) {  // round to nearest even, NaN kept a NaN
  typedef __bf16 v2bf __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(uint32_t, (v2bf){(__bf16)a, (__bf16)b});
}

// DP gradient buckets (mifx.parallel.ddp exchange="ipc") take the same three kernels over fp32 data: F32 = the
// 8-byte words hold 2 fp32 instead of 4 bf16, the rank-order sum stays fp32 and is scaled once (the 1 / world average)
// before it is stored -- every rank gets the same bits, and the captured backward carries the exchange on a side stream.

// A: partial -> own buffer half, stamp phase 0
__global__ __launch_bounds__(WG) void tpar_publish(const uint64_t* __restrict__ x, long long n4, Peers pe, int world,
                                                   int rank, long long npad4, const long long* __restrict__ ep,
                                                   const int* __restrict__ err, int nchunks) {
  if (failed(err)) return;  // one wave: a uniform exit
  const long long e = ep[0] + 1;
  const int c = blockIdx.x;
  uint64_t* dst = pe.buf[rank] + (size_t)(e & 1) * npad4 + (size_t)c * (CHUNK / 4);
  const long long base = (long long)c * (CHUNK / 4);
#pragma unroll
  for (int i = 0; i < PER_LANE; ++i) {
    const long long q = base + i * WG + threadIdx.x;
    st_sys64(dst + i * WG + threadIdx.x, q < n4 ? x[q] : 0ull);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every store of this wave acknowledged before the stamps
  if (threadIdx.x < world)
    publish(pe.flag[threadIdx.x] + ((size_t)0 * nchunks + c) * MAXW + rank, (unsigned int)e);
}

// B: reduce-scatter of the chunks this rank owns (c = rank + world k)
template <bool F32>
__global__ __launch_bounds__(WG) void tpar_reduce(Peers pe, int world, int rank, long long npad4,
                                                  const long long* __restrict__ ep, int* __restrict__ err,
                                                  int nchunks, int nch, float scale) {
  if (failed(err)) return;
  const int c = rank + world * blockIdx.x;
  if (c >= nch) return;  // (nch: chunks holding data; nchunks: the flag array's chunk dimension)
  const long long e = ep[0] + 1;
  const unsigned int* my = pe.flag[rank];
  bool ok = true;
  if (threadIdx.x < world) ok = wait_flag(my + ((size_t)0 * nchunks + c) * MAXW + threadIdx.x, (unsigned int)e, err);
  if (__ballot(!ok) != 0ull) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");  // the peers' partials were stored before their stamps
  const size_t off = (size_t)(e & 1) * npad4 + (size_t)c * (CHUNK / 4);
  uint64_t* dst = pe.red[rank] + off;
#pragma unroll 4
  for (int i = 0; i < PER_LANE; ++i) {
    const int q = i * WG + threadIdx.x;
    uint64_t v[MAXW];
#pragma unroll
    for (int p = 0; p < MAXW; ++p) v[p] = p < world ? ld_sys64(pe.buf[p] + off + q) : 0ull;
    if constexpr (F32) {
      float s0 = 0.f, s1 = 0.f;
#pragma unroll
      for (int p = 0; p < MAXW; ++p)  // rank order: the same fp32 sum on every rank
        if (p < world) {
          s0 += __uint_as_float((uint32_t)v[p]);
          s1 += __uint_as_float((uint32_t)(v[p] >> 32));
        }
      st_sys64(dst + q, (uint64_t)__float_as_uint(s0 * scale) | ((uint64_t)__float_as_uint(s1 * scale) << 32));
    } else {
      float s[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int p = 0; p < MAXW; ++p)  // rank order: the same fp32 sum on every rank
        if (p < world) {
          const float2 a = bf2f((uint32_t)v[p]), b = bf2f((uint32_t)(v[p] >> 32));
          s[0] += a.x;
          s[1] += a.y;
          s[2] += b.x;
          s[3] += b.y;
        }
      st_sys64(dst + q, (uint64_t)f2bf(s[0], s[1]) | ((uint64_t)f2bf(s[2], s[3]) << 32));
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (threadIdx.x < world)
    publish(pe.flag[threadIdx.x] + ((size_t)1 * nchunks + c) * MAXW + rank, (unsigned int)e);
}

// C: all-gather of the reduced chunks into the output; the last workgroup advances the epoch
// A failed group (sticky err) writes NaN into the output chunk instead of leaving it uninitialised: whatever consumes
// the activation goes non-finite (the loss shows it) even before the host's next check() raises.
__device__ __forceinline__ void poison(uint64_t* __restrict__ y, long long n4, int c, bool f32) {
  const long long base = (long long)c * (CHUNK / 4);
#pragma unroll
  for (int i = 0; i < PER_LANE; ++i) {
    const long long q = base + i * WG + threadIdx.x;
    if (q < n4) y[q] = f32 ? 0x7FC000007FC00000ull : 0x7FC07FC07FC07FC0ull;  // fp32 / bf16 quiet NaNs
  }
}

__global__ __launch_bounds__(WG) void tpar_gather(uint64_t* __restrict__ y, long long n4, Peers pe, int world, int rank,
                                                  long long npad4, long long* __restrict__ ep, int* __restrict__ err,
                                                  int nchunks, unsigned int* __restrict__ done, int f32) {
  const int c = blockIdx.x, owner = c % world;
  if (failed(err)) {
    poison(y, n4, c, f32);
    return;
  }
  const long long e = ep[0] + 1;
  bool ok = true;
  if (threadIdx.x == 0)  // (own chunks too: uniform code; their stamp is already there)
    ok = wait_flag(pe.flag[rank] + ((size_t)1 * nchunks + c) * MAXW + owner, (unsigned int)e, err);
  if (__ballot(!ok) != 0ull) {  // no epoch advance: the error is sticky, the host raises
    poison(y, n4, c, f32);
    return;
  }
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  const uint64_t* src = pe.red[owner] + (size_t)(e & 1) * npad4 + (size_t)c * (CHUNK / 4);
  const long long base = (long long)c * (CHUNK / 4);
#pragma unroll
  for (int i = 0; i < PER_LANE; ++i) {
    const long long q = base + i * WG + threadIdx.x;
    const uint64_t v = ld_sys64(src + i * WG + threadIdx.x);
    if (q < n4) y[q] = v;
  }
  // every workgroup read ep before its arrival: the last one to arrive advances it for the next call
  if (threadIdx.x == 0) {
    const unsigned int old = __hip_atomic_fetch_add(done, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (old == (unsigned int)gridDim.x - 1) {
      __hip_atomic_store(done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      ep[0] = e;
    }
  }
}

// ---- split waits (see the header): data kernels that never wait, and the one-wave waiter

// the last of `n` arriving workgroups (counter reset for the next call) stamps epoch e as flag[phase][0][rank] in every
// peer; every workgroup's own stores were acknowledged before its arrival
__device__ __forceinline__ void arrive_and_stamp(unsigned int* cnt, unsigned int n, const Peers& pe, int world, int rank,
                                                 int nchunks, int phase, unsigned int e) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  unsigned int old = 0;
  if (threadIdx.x == 0) old = __hip_atomic_fetch_add(cnt, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  old = __shfl(old, 0);
  if (old != n - 1) return;
  if (threadIdx.x == 0) __hip_atomic_store(cnt, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (threadIdx.x < world) publish(pe.flag[threadIdx.x] + ((size_t)phase * nchunks + 0) * MAXW + rank, e);
}

__global__ __launch_bounds__(WG) void tpar_publish_s(const uint64_t* __restrict__ x, long long n4, Peers pe, int world,
                                                     int rank, long long npad4, const long long* __restrict__ ep,
                                                     const int* __restrict__ err, int nchunks,
                                                     unsigned int* __restrict__ cnt) {
  if (failed(err)) return;
  const long long e = ep[0] + 1;
  const int c = blockIdx.x;
  uint64_t* dst = pe.buf[rank] + (size_t)(e & 1) * npad4 + (size_t)c * (CHUNK / 4);
  const long long base = (long long)c * (CHUNK / 4);
#pragma unroll
  for (int i = 0; i < PER_LANE; ++i) {
    const long long q = base + i * WG + threadIdx.x;
    st_sys64(dst + i * WG + threadIdx.x, q < n4 ? x[q] : 0ull);
  }
  arrive_and_stamp(cnt, gridDim.x, pe, world, rank, nchunks, 0, (unsigned int)e);
}

// one wave: lane p < world waits for peer p's stamp of `phase`; a timeout (or an earlier failure) leaves err set and
// every later kernel of the group a no-op
__global__ __launch_bounds__(WG) void tpar_wait(Peers pe, int world, int rank, const long long* __restrict__ ep,
                                                int* __restrict__ err, int nchunks, int phase) {
  if (failed(err)) return;
  const unsigned int e = (unsigned int)(ep[0] + 1);
  if (threadIdx.x < world) wait_flag(pe.flag[rank] + ((size_t)phase * nchunks + 0) * MAXW + threadIdx.x, e, err);
}

template <bool F32>
__global__ __launch_bounds__(WG) void tpar_reduce_s(Peers pe, int world, int rank, long long npad4,
                                                    const long long* __restrict__ ep, int* __restrict__ err,
                                                    int nchunks, int nch, float scale, unsigned int* __restrict__ cnt) {
  if (failed(err)) return;
  const long long e = ep[0] + 1;
  const int c = rank + world * blockIdx.x;
  if (c < nch) {
    const size_t off = (size_t)(e & 1) * npad4 + (size_t)c * (CHUNK / 4);
    uint64_t* dst = pe.red[rank] + off;
#pragma unroll 4
    for (int i = 0; i < PER_LANE; ++i) {
      const int q = i * WG + threadIdx.x;
      uint64_t v[MAXW];
#pragma unroll
      for (int p = 0; p < MAXW; ++p) v[p] = p < world ? ld_sys64(pe.buf[p] + off + q) : 0ull;
      if constexpr (F32) {
        float s0 = 0.f, s1 = 0.f;
#pragma unroll
        for (int p = 0; p < MAXW; ++p)  // rank order: the same fp32 sum on every rank
          if (p < world) {
            s0 += __uint_as_float((uint32_t)v[p]);
            s1 += __uint_as_float((uint32_t)(v[p] >> 32));
          }
        st_sys64(dst + q, (uint64_t)__float_as_uint(s0 * scale) | ((uint64_t)__float_as_uint(s1 * scale) << 32));
      } else {
        float sm[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int p = 0; p < MAXW; ++p)
          if (p < world) {
            const float2 a = bf2f((uint32_t)v[p]), b = bf2f((uint32_t)(v[p] >> 32));
            sm[0] += a.x;
            sm[1] += a.y;
            sm[2] += b.x;
            sm[3] += b.y;
          }
        st_sys64(dst + q, (uint64_t)f2bf(sm[0], sm[1]) | ((uint64_t)f2bf(sm[2], sm[3]) << 32));
      }
    }
  }
  arrive_and_stamp(cnt, gridDim.x, pe, world, rank, nchunks, 1, (unsigned int)e);
}

__global__ __launch_bounds__(WG) void tpar_gather_s(uint64_t* __restrict__ y, long long n4, Peers pe, int world,
                                                    int rank, long long npad4, long long* __restrict__ ep,
                                                    int* __restrict__ err, unsigned int* __restrict__ done, int f32) {
  const int c = blockIdx.x, owner = c % world;
  if (failed(err)) {
    poison(y, n4, c, f32);
    return;
  }
  const long long e = ep[0] + 1;
  const uint64_t* src = pe.red[owner] + (size_t)(e & 1) * npad4 + (size_t)c * (CHUNK / 4);
  const long long base = (long long)c * (CHUNK / 4);
#pragma unroll
  for (int i = 0; i < PER_LANE; ++i) {
    const long long q = base + i * WG + threadIdx.x;
    const uint64_t v = ld_sys64(src + i * WG + threadIdx.x);
    if (q < n4) y[q] = v;
  }
  if (threadIdx.x == 0) {
    const unsigned int old = __hip_atomic_fetch_add(done, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (old == (unsigned int)gridDim.x - 1) {
      __hip_atomic_store(done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      ep[0] = e;
    }
  }
}

// ---- sequence parallelism (Megatron-SP): reduce-scatter / all-gather of a token-major [T, H] bf16 activation whose
// T / world-token shards are contiguous: rank r owns elements [r m, (r + 1) m), m = n / world, m % CHUNK == 0 (so a
// chunk has one owner: chunk c belongs to rank c / (m / CHUNK)). Both reuse the publish kernels above (the whole
// partial for a reduce-scatter; for an all-gather only the own shard's chunks, tpar_publish_range) and take one epoch
// each, like an all-reduce; the double-buffering argument is the all-reduce's (every waiting kernel of epoch e + 1
// sees at least one stamp from every peer, issued after that peer's epoch-e reads).

// publish chunks [c0, c0 + gridDim) of x (element offset c0 CHUNK of the tensor) into the own buffer half; per-chunk
// stamps (fused waits) or one arrival-counted stamp (split waits, cnt != null)
__global__ __launch_bounds__(WG) void tpar_publish_range(const uint64_t* __restrict__ x, int c0, Peers pe, int world,
                                                         int rank, long long npad4, const long long* __restrict__ ep,
                                                         const int* __restrict__ err, int nchunks,
                                                         unsigned int* __restrict__ cnt) {
  if (failed(err)) return;
  const long long e = ep[0] + 1;
  const int c = c0 + blockIdx.x;
  uint64_t* dst = pe.buf[rank] + (size_t)(e & 1) * npad4 + (size_t)c * (CHUNK / 4);
  const uint64_t* src = x + (size_t)blockIdx.x * (CHUNK / 4);
#pragma unroll
  for (int i = 0; i < PER_LANE; ++i) st_sys64(dst + i * WG + threadIdx.x, src[i * WG + threadIdx.x]);
  if (cnt != nullptr) {
    arrive_and_stamp(cnt, gridDim.x, pe, world, rank, nchunks, 0, (unsigned int)e);
    return;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  if (threadIdx.x < world) publish(pe.flag[threadIdx.x] + ((size_t)0 * nchunks + c) * MAXW + rank, (unsigned int)e);
}

// the last arriving workgroup of the epoch's final kernel advances the epoch counter
__device__ __forceinline__ void finish_epoch(long long* ep, unsigned int* done, long long e) {
  if (threadIdx.x == 0) {
    const unsigned int old = __hip_atomic_fetch_add(done, 1u, __ATOMIC_ACQ_REL, __HIP_MEMORY_SCOPE_AGENT);
    if (old == (unsigned int)gridDim.x - 1) {
      __hip_atomic_store(done, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      ep[0] = e;
    }
  }
}

// reduce-scatter, second kernel: chunk c = rank * cps + blockIdx of the own shard, rank-order fp32 sum of every peer's
// published partial rounded once to bf16 into y (the shard, local). WAIT: per-chunk waits inside (fused form)
template <bool WAIT>
__global__ __launch_bounds__(WG) void tpar_rs_own(uint64_t* __restrict__ y, Peers pe, int world, int rank, int cps,
                                                  long long npad4, long long* __restrict__ ep, int* __restrict__ err,
                                                  int nchunks, unsigned int* __restrict__ done) {
  const int c = rank * cps + blockIdx.x;
  uint64_t* dst = y + (size_t)blockIdx.x * (CHUNK / 4);
  if (failed(err)) {
#pragma unroll
    for (int i = 0; i < PER_LANE; ++i) dst[i * WG + threadIdx.x] = 0x7FC07FC07FC07FC0ull;  // bf16 NaNs
    return;
  }
  const long long e = ep[0] + 1;
  if constexpr (WAIT) {
    bool ok = true;
    if (threadIdx.x < world) ok = wait_flag(pe.flag[rank] + ((size_t)0 * nchunks + c) * MAXW + threadIdx.x,
                                            (unsigned int)e, err);
    if (__ballot(!ok) != 0ull) {
#pragma unroll
      for (int i = 0; i < PER_LANE; ++i) dst[i * WG + threadIdx.x] = 0x7FC07FC07FC07FC0ull;
      return;
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  }
  const size_t off = (size_t)(e & 1) * npad4 + (size_t)c * (CHUNK / 4);
#pragma unroll 4
  for (int i = 0; i < PER_LANE; ++i) {
    const int q = i * WG + threadIdx.x;
    uint64_t v[MAXW];
#pragma unroll
    for (int p = 0; p < MAXW; ++p) v[p] = p < world ? ld_sys64(pe.buf[p] + off + q) : 0ull;
    float sm[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int p = 0; p < MAXW; ++p)
      if (p < world) {
        const float2 a = bf2f((uint32_t)v[p]), b = bf2f((uint32_t)(v[p] >> 32));
        sm[0] += a.x;
        sm[1] += a.y;
        sm[2] += b.x;
        sm[3] += b.y;
      }
    dst[q] = (uint64_t)f2bf(sm[0], sm[1]) | ((uint64_t)f2bf(sm[2], sm[3]) << 32);
  }
  finish_epoch(ep, done, e);
}

// all-gather, second kernel: every chunk of y from its owner's published shard (own chunks from the own buffer too)
template <bool WAIT>
__global__ __launch_bounds__(WG) void tpar_ag_gather(uint64_t* __restrict__ y, Peers pe, int world, int rank, int cps,
                                                     long long npad4, long long* __restrict__ ep,
                                                     int* __restrict__ err, int nchunks,
                                                     unsigned int* __restrict__ done) {
  const int c = blockIdx.x, owner = c / cps;
  uint64_t* dst = y + (size_t)c * (CHUNK / 4);
  if (failed(err)) {
#pragma unroll
    for (int i = 0; i < PER_LANE; ++i) dst[i * WG + threadIdx.x] = 0x7FC07FC07FC07FC0ull;
    return;
  }
  const long long e = ep[0] + 1;
  if constexpr (WAIT) {
    bool ok = true;
    if (threadIdx.x == 0)
      ok = wait_flag(pe.flag[rank] + ((size_t)0 * nchunks + c) * MAXW + owner, (unsigned int)e, err);
    if (__ballot(!ok) != 0ull) {
#pragma unroll
      for (int i = 0; i < PER_LANE; ++i) dst[i * WG + threadIdx.x] = 0x7FC07FC07FC07FC0ull;
      return;
    }
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "");
  }
  const uint64_t* src = pe.buf[owner] + (size_t)(e & 1) * npad4 + (size_t)c * (CHUNK / 4);
#pragma unroll
  for (int i = 0; i < PER_LANE; ++i) dst[i * WG + threadIdx.x] = ld_sys64(src + i * WG + threadIdx.x);
  finish_epoch(ep, done, e);
}

}  // namespace

extern "C" {

int mifx_tpar_chunk() { return CHUNK; }

// x, y: bf16 [n] (n % 4 == 0, 8-byte aligned; y may equal x); bufs / reds / flags: host arrays of `world` device
// pointers (IPC-opened peer buffers, [rank] = own): bufs / reds [2][npad] bf16 with npad = nchunks * CHUNK >= n,
// flags [2][nchunks][8] uint32 (uncached). ep: int64 epoch counter (device), done: uint32 arrival counter (device,
// zero), err: sticky int flag (device). Three kernels on `stream`.
static int tpar_allreduce(const void* x, void* y, long long n, void* const* bufs, void* const* reds,
                          void* const* flags, int world, int rank, long long npad, long long* ep, unsigned int* done,
                          int* err, bool f32, float scale, bool waiters, hipStream_t stream) {
  if (world < 1 || world > MAXW || rank < 0 || rank >= world || n <= 0 || n % 4 != 0 || npad % CHUNK != 0 ||
      n > npad || x == nullptr || y == nullptr || ep == nullptr || done == nullptr || err == nullptr)
    return -1;
  if ((uintptr_t)x % 8 != 0 || (uintptr_t)y % 8 != 0) return -1;
  Peers pe{};
  for (int p = 0; p < world; ++p) {
    if (bufs[p] == nullptr || reds[p] == nullptr || flags[p] == nullptr) return -1;
    pe.buf[p] = (uint64_t*)bufs[p];
    pe.red[p] = (uint64_t*)reds[p];
    pe.flag[p] = (unsigned int*)flags[p];
  }
  const int nchunks = (int)((n + CHUNK - 1) / CHUNK);
  const int nchunks_all = (int)(npad / CHUNK);  // the flag array's chunk dimension
  const long long n4 = n / 4, npad4 = npad / 4;
  if (waiters) {  // done: [0] gather arrivals, [1] publish arrivals, [2] reduce arrivals
    const int rgrid = (nchunks + world - 1) / world;
    hipLaunchKernelGGL(tpar_publish_s, dim3(nchunks), dim3(WG), 0, stream, (const uint64_t*)x, n4, pe, world, rank,
                       npad4, ep, err, nchunks_all, done + 1);
    hipLaunchKernelGGL(tpar_wait, dim3(1), dim3(WG), 0, stream, pe, world, rank, ep, err, nchunks_all, 0);
    if (f32)
      hipLaunchKernelGGL(tpar_reduce_s<true>, dim3(rgrid), dim3(WG), 0, stream, pe, world, rank, npad4, ep, err,
                         nchunks_all, nchunks, scale, done + 2);
    else
      hipLaunchKernelGGL(tpar_reduce_s<false>, dim3(rgrid), dim3(WG), 0, stream, pe, world, rank, npad4, ep, err,
                         nchunks_all, nchunks, 1.f, done + 2);
    hipLaunchKernelGGL(tpar_wait, dim3(1), dim3(WG), 0, stream, pe, world, rank, ep, err, nchunks_all, 1);
    hipLaunchKernelGGL(tpar_gather_s, dim3(nchunks), dim3(WG), 0, stream, (uint64_t*)y, n4, pe, world, rank, npad4,
                       ep, err, done, (int)f32);
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL(tpar_publish, dim3(nchunks), dim3(WG), 0, stream, (const uint64_t*)x, n4, pe, world, rank, npad4,
                     ep, err, nchunks_all);
  if (f32)
    hipLaunchKernelGGL(tpar_reduce<true>, dim3((nchunks + world - 1) / world), dim3(WG), 0, stream, pe, world, rank,
                       npad4, ep, err, nchunks_all, nchunks, scale);
  else
    hipLaunchKernelGGL(tpar_reduce<false>, dim3((nchunks + world - 1) / world), dim3(WG), 0, stream, pe, world, rank,
                       npad4, ep, err, nchunks_all, nchunks, 1.f);
  hipLaunchKernelGGL(tpar_gather, dim3(nchunks), dim3(WG), 0, stream, (uint64_t*)y, n4, pe, world, rank, npad4, ep,
                     err, nchunks_all, done, (int)f32);
  return (int)hipGetLastError();
}

int mifx_tpar_allreduce(const void* x, void* y, long long n, void* const* bufs, void* const* reds, void* const* flags,
                        int world, int rank, long long npad, long long* ep, unsigned int* done, int* err,
                        hipStream_t stream) {
  return tpar_allreduce(x, y, n, bufs, reds, flags, world, rank, npad, ep, done, err, false, 1.f, false, stream);
}

// fp32 variant (DP gradient buckets): n = fp32 elements (even), npad = the buffers' capacity in bf16-element units
// as above (i.e. 2 x the fp32 capacity); the rank-order sum is multiplied by `scale` before it is stored.
int mifx_tpar_allreduce_f32(const void* x, void* y, long long n, void* const* bufs, void* const* reds,
                            void* const* flags, int world, int rank, long long npad, long long* ep, unsigned int* done,
                            int* err, float scale, hipStream_t stream) {
  if (n <= 0 || n % 2 != 0) return -1;
  return tpar_allreduce(x, y, 2 * n, bufs, reds, flags, world, rank, npad, ep, done, err, true, scale, false, stream);
}

// Either dtype (f32: n = fp32 elements, even; else bf16, n % 4 == 0) and either wait placement: waiters = 1 runs the
// split-wait sequence (publish / wait / reduce / wait / gather: no data-moving workgroup ever spins), 0 the three
// kernels with the waits inside. done: uint32 [3] arrival counters (zero). scale: fp32 only.
int mifx_tpar_allreduce2(const void* x, void* y, long long n, void* const* bufs, void* const* reds, void* const* flags,
                         int world, int rank, long long npad, long long* ep, unsigned int* done, int* err, int f32,
                         float scale, int waiters, hipStream_t stream) {
  if (f32) {
    if (n <= 0 || n % 2 != 0) return -1;
    n *= 2;
  } else if (scale != 1.f) {
    return -1;
  }
  return tpar_allreduce(x, y, n, bufs, reds, flags, world, rank, npad, ep, done, err, f32 != 0, scale, waiters != 0,
                        stream);
}

}  // extern "C"

extern "C" {

// Sequence-parallel reduce-scatter of a bf16 [n] partial: y (n / world elements, this rank's contiguous shard) = rank-
// order sum over the ranks of x's shard, rounded once to bf16. all-gather: y [n] = the ranks' shards x [n / world] in
// rank order. n % (world * CHUNK) == 0 (whole chunks per shard). waiters: split waits as mifx_tpar_allreduce2.
int mifx_tpar_reduce_scatter(const void* x, void* y, long long n, void* const* bufs, void* const* flags, int world,
                             int rank, long long npad, long long* ep, unsigned int* done, int* err, int waiters,
                             hipStream_t stream) {
  if (world < 1 || world > MAXW || rank < 0 || rank >= world || n <= 0 || n % ((long long)world * CHUNK) != 0 ||
      n > npad || npad % CHUNK != 0 || x == nullptr || y == nullptr || ep == nullptr || done == nullptr ||
      err == nullptr || (uintptr_t)x % 8 != 0 || (uintptr_t)y % 8 != 0)
    return -1;
  Peers pe{};
  for (int p = 0; p < world; ++p) {
    if (bufs[p] == nullptr || flags[p] == nullptr) return -1;
    pe.buf[p] = (uint64_t*)bufs[p];
    pe.flag[p] = (unsigned int*)flags[p];
  }
  const int nchunks = (int)(n / CHUNK), nchunks_all = (int)(npad / CHUNK), cps = nchunks / world;
  const long long npad4 = npad / 4;
  hipLaunchKernelGGL(tpar_publish_range, dim3(nchunks), dim3(WG), 0, stream, (const uint64_t*)x, 0, pe, world, rank,
                     npad4, ep, err, nchunks_all, waiters ? done + 1 : nullptr);
  if (waiters) {
    hipLaunchKernelGGL(tpar_wait, dim3(1), dim3(WG), 0, stream, pe, world, rank, ep, err, nchunks_all, 0);
    hipLaunchKernelGGL(tpar_rs_own<false>, dim3(cps), dim3(WG), 0, stream, (uint64_t*)y, pe, world, rank, cps, npad4,
                       ep, err, nchunks_all, done);
  } else {
    hipLaunchKernelGGL(tpar_rs_own<true>, dim3(cps), dim3(WG), 0, stream, (uint64_t*)y, pe, world, rank, cps, npad4,
                       ep, err, nchunks_all, done);
  }
  return (int)hipGetLastError();
}

int mifx_tpar_all_gather(const void* x, void* y, long long n, void* const* bufs, void* const* flags, int world,
                         int rank, long long npad, long long* ep, unsigned int* done, int* err, int waiters,
                         hipStream_t stream) {
  if (world < 1 || world > MAXW || rank < 0 || rank >= world || n <= 0 || n % ((long long)world * CHUNK) != 0 ||
      n > npad || npad % CHUNK != 0 || x == nullptr || y == nullptr || ep == nullptr || done == nullptr ||
      err == nullptr || (uintptr_t)x % 8 != 0 || (uintptr_t)y % 8 != 0)
    return -1;
  Peers pe{};
  for (int p = 0; p < world; ++p) {
    if (bufs[p] == nullptr || flags[p] == nullptr) return -1;
    pe.buf[p] = (uint64_t*)bufs[p];
    pe.flag[p] = (unsigned int*)flags[p];
  }
  const int nchunks = (int)(n / CHUNK), nchunks_all = (int)(npad / CHUNK), cps = nchunks / world;
  const long long npad4 = npad / 4;
  hipLaunchKernelGGL(tpar_publish_range, dim3(cps), dim3(WG), 0, stream, (const uint64_t*)x, rank * cps, pe, world,
                     rank, npad4, ep, err, nchunks_all, waiters ? done + 1 : nullptr);
  if (waiters) {
    hipLaunchKernelGGL(tpar_wait, dim3(1), dim3(WG), 0, stream, pe, world, rank, ep, err, nchunks_all, 0);
    hipLaunchKernelGGL(tpar_ag_gather<false>, dim3(nchunks), dim3(WG), 0, stream, (uint64_t*)y, pe, world, rank, cps,
                       npad4, ep, err, nchunks_all, done);
  } else {
    hipLaunchKernelGGL(tpar_ag_gather<true>, dim3(nchunks), dim3(WG), 0, stream, (uint64_t*)y, pe, world, rank, cps,
                       npad4, ep, err, nchunks_all, done);
  }
  return (int)hipGetLastError();
}

}  // extern "C"
