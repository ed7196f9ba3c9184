// String-vocabulary analyzer + mapper kernels for gfx950 (Transform: tft.compute_and_apply_vocabulary,
// tft.string_to_int, tft.hash_strings).
//
// Reference ops: vocabulary over `payment_type` / `company` with top_k=1000 and 10 OOV
// buckets (`airflow-dags/taxi_utils.py:121-126`), `transform.string_to_int` over 6 features
// (`kubeflow-pipelines/taxi/preprocessing.py:77-85`).
//
// Strings arrive as one packed byte buffer + int64 offsets (n+1). Design:
//  * str_hash: one lane per string, 64-bit FNV-1a over its bytes (identical to the host
//    `mifx.transform.api.fingerprint64`, so OOV buckets agree with the CPU path bit-for-bit).
//  * vocab_count_lds: open-addressing hash table in global memory (power-of-two capacity, linear
//    probing), fed by per-block LDS pre-aggregation. Keys are inserted with a 64-bit atomicCAS;
//    occurrences counted with atomicAdd; each slot keeps the smallest row index that produced it
//    (atomicMin) as its representative, so the result is independent of scheduling.
//  * vocab_verify: every row compares its bytes with its slot's representative; a genuine 64-bit
//    hash collision between distinct strings raises a flag and the host redoes the column on the
//    exact CPU path. (The host sorts the few unique (count, token) pairs: frequency desc, token desc.)
//  * vocab_lookup: apply phase. The vocabulary (hash -> index table + packed vocab bytes) is
//    device-resident; each lane probes, confirms the bytes, else maps to n_vocab + h % n_oov or the
//    default value.
// The table is sized by the host to >= 2x the key count, so probes stay short; every probe loop is
// bounded by the capacity, so a full table cannot spin forever.
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace {

constexpr unsigned long long kEmpty = 0ull;
constexpr unsigned long long kFnvOff = 0xCBF29CE484222325ull;
constexpr unsigned long long kFnvPrime = 0x100000001B3ull;

__device__ __forceinline__ unsigned long long fnv1a(const uint8_t* p, long long len) {
  unsigned long long h = kFnvOff;
  for (long long i = 0; i < len; ++i) h = (h ^ p[i]) * kFnvPrime;
  return h;
}

// key 0 marks an empty slot; the (astronomically rare) hash 0 is stored as 1 -- any string pair
// that aliases through this remap is caught by the byte verification like any other collision.
__device__ __forceinline__ unsigned long long as_key(unsigned long long h) { return h == kEmpty ? 1ull : h; }

__device__ __forceinline__ unsigned int slot0(unsigned long long key, unsigned int mask) {
  return (unsigned int)((key ^ (key >> 29)) * 0x9E3779B97F4A7C15ull >> 32) & mask;
}

__device__ __forceinline__ bool bytes_eq(const uint8_t* a, long long la, const uint8_t* b, long long lb) {
  if (la != lb) return false;
  for (long long i = 0; i < la; ++i)
    if (a[i] != b[i]) return false;
  return true;
}

__global__ __launch_bounds__(256) void str_hash(const uint8_t* __restrict__ buf, const long long* __restrict__ offs,
                                                long long n, unsigned long long* __restrict__ out) {
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const long long b = offs[i], e = offs[i + 1];
    out[i] = fnv1a(buf + b, e - b);
  }
}

// Zipf-distributed columns (a few tokens carry most rows) make one global counter per hot token a
// serialisation point: 1M rows spent 3 ms in vocab_count (profiles/archive/analyzers_kernels_s2.md). Each
// block therefore pre-aggregates its rows in an LDS hash table (count + smallest row per key, LDS
// atomics) and flushes one global insert per distinct key it saw; rows whose key finds no LDS slot
// within kLdsProbe probes go straight to the global table.
constexpr int kLdsSlots = 2048;
constexpr int kLdsProbe = 32;

__device__ __forceinline__ void global_insert(unsigned long long k, unsigned int cnt, int row,
                                              unsigned long long* keys, unsigned int* counts, int* rep,
                                              unsigned int mask, int* overflow) {
  unsigned int s = slot0(k, mask);
  for (unsigned int probe = 0; probe <= mask; ++probe) {
    const unsigned long long prev = atomicCAS(&keys[s], kEmpty, k);
    if (prev == kEmpty || prev == k) {
      atomicAdd(&counts[s], cnt);
      atomicMin(&rep[s], row);
      return;
    }
    s = (s + 1) & mask;
  }
  atomicOr(overflow, 1);
}

__global__ __launch_bounds__(256) void vocab_count_lds(const unsigned long long* __restrict__ hash, long long n,
                                                       unsigned long long* __restrict__ keys,
                                                       unsigned int* __restrict__ counts, int* __restrict__ rep,
                                                       unsigned int mask, int* __restrict__ overflow) {
  __shared__ unsigned long long lk[kLdsSlots];
  __shared__ unsigned int lc[kLdsSlots];
  __shared__ int lr[kLdsSlots];
  for (int s = threadIdx.x; s < kLdsSlots; s += 256) {
    lk[s] = kEmpty;
    lc[s] = 0u;
    lr[s] = 0x7fffffff;
  }
  __syncthreads();
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const unsigned long long k = as_key(hash[i]);
    unsigned int s = slot0(k, kLdsSlots - 1);
    bool done = false;
    for (int probe = 0; probe < kLdsProbe; ++probe) {
      const unsigned long long prev = atomicCAS(&lk[s], kEmpty, k);
      if (prev == kEmpty || prev == k) {
        atomicAdd(&lc[s], 1u);
        if (lr[s] > (int)i) atomicMin(&lr[s], (int)i);  // racy pre-check only skips useless atomics
        done = true;
        break;
      }
      s = (s + 1) & (kLdsSlots - 1);
    }
    if (!done) global_insert(k, 1u, (int)i, keys, counts, rep, mask, overflow);
  }
  __syncthreads();
  for (int s = threadIdx.x; s < kLdsSlots; s += 256)
    if (lc[s] != 0u) global_insert(lk[s], lc[s], lr[s], keys, counts, rep, mask, overflow);
}

__device__ __forceinline__ int find_slot(const unsigned long long* keys, unsigned long long k, unsigned int mask) {
  unsigned int s = slot0(k, mask);
  for (unsigned int probe = 0; probe <= mask; ++probe) {
    const unsigned long long v = keys[s];
    if (v == k) return (int)s;
    if (v == kEmpty) return -1;
    s = (s + 1) & mask;
  }
  return -1;
}

__global__ __launch_bounds__(256) void vocab_verify(const uint8_t* __restrict__ buf, const long long* __restrict__ offs,
                                                    const unsigned long long* __restrict__ hash, long long n,
                                                    const unsigned long long* __restrict__ keys,
                                                    const int* __restrict__ rep, unsigned int mask,
                                                    int* __restrict__ collision) {
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const int s = find_slot(keys, as_key(hash[i]), mask);
    if (s < 0) {
      atomicOr(collision, 2);
      continue;
    }
    const long long r = rep[s];
    if (r == i) continue;
    if (!bytes_eq(buf + offs[i], offs[i + 1] - offs[i], buf + offs[r], offs[r + 1] - offs[r])) atomicOr(collision, 1);
  }
}

__global__ __launch_bounds__(256) void vocab_lookup(const uint8_t* __restrict__ buf, const long long* __restrict__ offs,
                                                    long long n, const unsigned long long* __restrict__ keys,
                                                    const int* __restrict__ vals, unsigned int mask,
                                                    const uint8_t* __restrict__ vbuf,
                                                    const long long* __restrict__ voffs, int n_vocab, int n_oov,
                                                    long long default_value, long long* __restrict__ out) {
  for (long long i = blockIdx.x * 256LL + threadIdx.x; i < n; i += (long long)gridDim.x * 256) {
    const long long b = offs[i], e = offs[i + 1];
    const unsigned long long h = fnv1a(buf + b, e - b);
    const int s = find_slot(keys, as_key(h), mask);
    long long id = -1;
    if (s >= 0) {
      const int v = vals[s];
      if (bytes_eq(buf + b, e - b, vbuf + voffs[v], voffs[v + 1] - voffs[v])) id = v;
    }
    if (id < 0) id = n_oov > 0 ? (long long)n_vocab + (long long)(h % (unsigned long long)n_oov) : default_value;
    out[i] = id;
  }
}

// apply-phase table build: vocab entry v -> slot; a duplicate key (two vocab strings with one hash)
// or a full table sets *flag and the host maps the column on the CPU instead.
__global__ __launch_bounds__(256) void vocab_insert(const uint8_t* __restrict__ vbuf, const long long* __restrict__ voffs,
                                                    int n_vocab, unsigned long long* __restrict__ keys,
                                                    int* __restrict__ vals, unsigned int mask, int* __restrict__ flag) {
  for (int v = blockIdx.x * 256 + threadIdx.x; v < n_vocab; v += gridDim.x * 256) {
    const unsigned long long k = as_key(fnv1a(vbuf + voffs[v], voffs[v + 1] - voffs[v]));
    unsigned int s = slot0(k, mask);
    bool done = false;
    for (unsigned int probe = 0; probe <= mask; ++probe) {
      const unsigned long long prev = atomicCAS(&keys[s], kEmpty, k);
      if (prev == kEmpty) {
        vals[s] = v;
        done = true;
        break;
      }
      if (prev == k) break;
      s = (s + 1) & mask;
    }
    if (!done) atomicOr(flag, 1);
  }
}

int grid_for(long long n) {
  const long long blocks = (n + 255) / 256;
  return (int)(blocks < 2048 ? (blocks > 0 ? blocks : 1) : 2048);
}

bool pow2_mask(long long cap, unsigned int* mask) {
  if (cap <= 0 || cap > (1ll << 30) || (cap & (cap - 1)) != 0) return false;
  *mask = (unsigned int)(cap - 1);
  return true;
}

}  // namespace

extern "C" {

int mifx_vocab_hash(const uint8_t* buf, const long long* offs, long long n, unsigned long long* out, hipStream_t st) {
  if (n < 0) return -1;
  if (n == 0) return 0;
  hipLaunchKernelGGL(str_hash, dim3(grid_for(n)), dim3(256), 0, st, buf, offs, n, out);
  return (int)hipGetLastError();
}

// keys/counts zeroed and rep filled with INT_MAX by the caller; flags[0] = overflow, flags[1] = collision
int mifx_vocab_count(const uint8_t* buf, const long long* offs, long long n, unsigned long long* hash,
                     unsigned long long* keys, unsigned int* counts, int* rep, long long cap, int* flags,
                     hipStream_t st) {
  unsigned int mask;
  if (n < 0 || !pow2_mask(cap, &mask)) return -1;
  if (n == 0) return 0;
  const int g = grid_for(n);
  hipLaunchKernelGGL(str_hash, dim3(g), dim3(256), 0, st, buf, offs, n, hash);
  // ~2K rows per block for the LDS pre-aggregation (flush cost is per block), at least one block per CU
  const long long cb = (n + 2047) / 2048;
  const int gc = (int)(cb < 256 ? 256 : (cb > 4096 ? 4096 : cb));
  hipLaunchKernelGGL(vocab_count_lds, dim3(gc), dim3(256), 0, st, hash, n, keys, counts, rep, mask, flags);
  hipLaunchKernelGGL(vocab_verify, dim3(g), dim3(256), 0, st, buf, offs, hash, n, keys, rep, mask, flags + 1);
  return (int)hipGetLastError();
}

// keys zeroed by the caller; *flag != 0 afterwards means the table is unusable
int mifx_vocab_build(const uint8_t* vbuf, const long long* voffs, int n_vocab, unsigned long long* keys, int* vals,
                     long long cap, int* flag, hipStream_t st) {
  unsigned int mask;
  if (n_vocab < 0 || !pow2_mask(cap, &mask) || cap < n_vocab) return -1;
  if (n_vocab == 0) return 0;
  hipLaunchKernelGGL(vocab_insert, dim3(grid_for(n_vocab)), dim3(256), 0, st, vbuf, voffs, n_vocab, keys, vals, mask,
                     flag);
  return (int)hipGetLastError();
}

int mifx_vocab_lookup(const uint8_t* buf, const long long* offs, long long n, const unsigned long long* keys,
                      const int* vals, long long cap, const uint8_t* vbuf, const long long* voffs, int n_vocab,
                      int n_oov, long long default_value, long long* out, hipStream_t st) {
  unsigned int mask;
  if (n < 0 || !pow2_mask(cap, &mask) || n_vocab < 0 || n_oov < 0) return -1;
  if (n == 0) return 0;
  hipLaunchKernelGGL(vocab_lookup, dim3(grid_for(n)), dim3(256), 0, st, buf, offs, n, keys, vals, mask, vbuf, voffs,
                     n_vocab, n_oov, default_value, out);
  return (int)hipGetLastError();
}

}  // extern "C"
