// Record feed of the fused Wide&Deep training kernels: which resident record a batch row trains on.
//
// The reference reads its training files through `read_batch_features(..., randomize_input=True)`
// (`airflow-dags/taxi_utils.py:275-276`): a fresh shuffle of the records every epoch. Here the records stay
// resident in HBM and the shuffle is a pseudo-random PERMUTATION of [0, n) per epoch, evaluated per record in the
// kernel's own fetch (no index array, no host work, nothing re-uploaded between epochs):
//
//   position p = step * gstride + goff + row          (the global stream: a data-parallel rank r with per-replica
//                                                      batch B and world W uses gstride = W B, goff = r B, so the
//                                                      ranks read disjoint rows of ONE global stream and the job
//                                                      equals one process at batch W B)
//   epoch e = p / n,  i = p mod n
//   record  = key == 0 ? i : feistel_perm(i, n, epoch_key(key, e))
//
// The permutation moves GROUPS of 2^MIFX_SHUFFLE_GLOG2 = 4 consecutive records (one 128-byte cache line of 32-byte
// records): a fresh random order of the record groups every epoch, records inside a group kept together (the
// n mod 4 records past the last whole group keep their place). A batch of B rows then reads B / 4 random lines
// instead of B random half-lines: the per-record shuffle cost 1.4 us of a 35 us step at B = 65536 (the wave's 16
// distinct records per load instruction each a separate line), this one ~0 (profiles/wd_shuffle_ab_r4.txt).
//
// feistel_perm: a 4-round balanced Feistel network on [0, 2^(2h)) (2^(2h) >= n, h >= 1) with cycle walking down to
// [0, n) -- a bijection of [0, n) for every n and key (each walk follows the permutation's cycle from i until it
// re-enters [0, n), which it must: at the latest back at i). Expected walk length < 4 (2^(2h) < 4n).
// mifx/data/shuffle.py is the bit-exact host implementation (tests and the CPU trainer).
#pragma once
#include <stdint.h>

#ifndef MIFX_SHUFFLE_GLOG2
#define MIFX_SHUFFLE_GLOG2 2
#endif

#ifdef __HIPCC__
#define MIFX_HD __host__ __device__ __forceinline__
#else
#define MIFX_HD inline
#endif

MIFX_HD uint32_t mifx_mix32(uint32_t x) {  // "lowbias32" integer hash
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

MIFX_HD uint64_t mifx_epoch_key(uint64_t key, uint64_t epoch) {
  const uint32_t a = mifx_mix32((uint32_t)key ^ mifx_mix32((uint32_t)epoch + 0x9e3779b9u));
  const uint32_t b = mifx_mix32((uint32_t)(key >> 32) ^ mifx_mix32((uint32_t)(epoch >> 32) + 0x85ebca6bu) ^ a);
  return ((uint64_t)b << 32) | a;
}

// half width h (bits) of the Feistel domain for n records: the smallest h >= 1 with 4^h >= n
MIFX_HD int mifx_feistel_half(uint64_t n) {
  if (n <= 4) return 1;
#if defined(__HIP_DEVICE_COMPILE__)
  const int b = 64 - __clzll((long long)(n - 1));  // bits of n - 1
#else
  const int b = 64 - __builtin_clzll(n - 1);
#endif
  return (b + 1) >> 1;  // the smallest h with 4^h >= n
}

// the same network in 32-bit arithmetic (n <= 2^32, h <= 16): identical values, half the instructions
MIFX_HD uint32_t mifx_feistel_perm32(uint32_t i, uint64_t n, uint64_t ekey, int h) {
  const uint32_t mask = (1u << h) - 1u;
  const uint32_t k0 = (uint32_t)ekey, k1 = (uint32_t)(ekey >> 32);
  const uint32_t rk[4] = {k0, k1, k0 ^ 0x68e31da4u, k1 ^ 0xb5297a4du};
  uint32_t x = i;
  do {
    uint32_t L = x >> h, R = x & mask;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const uint32_t t = L ^ (mifx_mix32(R ^ rk[r]) & mask);
      L = R;
      R = t;
    }
    x = (L << h) | R;
  } while ((uint64_t)x >= n);
  return x;
}

MIFX_HD uint64_t mifx_feistel_perm(uint64_t i, uint64_t n, uint64_t ekey, int h) {
  const uint64_t mask = (uint64_t(1) << h) - 1;
  const uint32_t k0 = (uint32_t)ekey, k1 = (uint32_t)(ekey >> 32);
  const uint32_t rk[4] = {k0, k1, k0 ^ 0x68e31da4u, k1 ^ 0xb5297a4du};
  uint64_t x = i;
  do {
    uint64_t L = x >> h, R = x & mask;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const uint64_t t = L ^ ((uint64_t)mifx_mix32((uint32_t)R ^ rk[r] ^ (uint32_t)(R >> 32)) & mask);
      L = R;
      R = t;
    }
    x = (L << h) | R;
  } while (x >= n);
  return x;
}

struct MifxFeed {
  long long gstride;   // stream positions per training step (the global batch)
  long long goff;      // this replica's offset inside the global batch
  unsigned long long key;  // 0: no shuffle (records in stored order); else the shuffle seed
};

// per step: the epoch and in-epoch index of this replica's first row, the group count and Feistel half width, and
// the epoch keys of the step's epoch and the next (a batch spans at most one epoch boundary)
struct MifxFeedStep {
  long long e0, i0;
  long long ng;
  int h;
  uint64_t ek0, ek1;
};
MIFX_HD MifxFeedStep mifx_feed_step(const MifxFeed& f, long long step, long long n) {
  const long long p = step * f.gstride + f.goff;
  MifxFeedStep s;
  // p / n through a double quotient (exact to +-1 below 2^53) and an integer correction: no 64-bit divide
  long long e = (long long)((double)p / (double)n);
  long long i = p - e * n;
  while (i < 0) {
    i += n;
    --e;
  }
  while (i >= n) {
    i -= n;
    ++e;
  }
  s.e0 = e;
  s.i0 = i;
  s.ng = n >> MIFX_SHUFFLE_GLOG2;
  s.h = mifx_feistel_half((uint64_t)(s.ng > 0 ? s.ng : 1));
  s.ek0 = f.key ? mifx_epoch_key(f.key, (uint64_t)e) : 0;
  s.ek1 = f.key ? mifx_epoch_key(f.key, (uint64_t)e + 1) : 0;
  return s;
}
// record of batch row `row` (0 <= row < batch <= n)
MIFX_HD long long mifx_feed_record(const MifxFeed& f, const MifxFeedStep& s, long long row, long long n) {
  long long i = s.i0 + row, e = s.e0;
  if (i >= n) {
    i -= n;
    e += 1;
  }
  if (f.key == 0) return i;
  constexpr int GL = MIFX_SHUFFLE_GLOG2;
  if (i >= (s.ng << GL)) return i;  // the records past the last whole group
  const uint64_t ek = e == s.e0 ? s.ek0 : s.ek1;
  const long long g = i >> GL, in = i & ((1ll << GL) - 1);
  const long long pg = s.h <= 16 ? (long long)mifx_feistel_perm32((uint32_t)g, (uint64_t)s.ng, ek, s.h)
                                 : (long long)mifx_feistel_perm((uint64_t)g, (uint64_t)s.ng, ek, s.h);
  return (pg << GL) | in;
}
