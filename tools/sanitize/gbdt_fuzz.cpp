// Host sanitizer harness for csrc/gbdt.cpp (the multithreaded histogram tree learner behind mifx.gbdt).
// Built twice by tests/test_sanitizers.py: AddressSanitizer + UBSan, and ThreadSanitizer (the learner splits
// features over std::threads in mifx_gbdt_bin / mifx_gbdt_grow and rows over threads in mifx_gbdt_predict).
//
// Per trial: a random matrix (NaNs, duplicated values, constant and all-NaN columns, n from 1 to ~3000 with 1-12
// features, or 20k-40k rows x 10-12 features so the threaded paths run) is binned with per-feature cuts, then trees are grown with 1, 2, 3 and 8 threads -- every thread count
// must produce the SAME tree bit for bit (the learner's determinism contract) -- and predicted with the raw values,
// which must land every training row in the leaf the learner recorded for it. Exact-size heap buffers everywhere, so
// any over-read / over-write is an ASan report; edge cases: max_nodes too small (-1), invalid max_bins (-1).
//   g++ -O1 -g -fsanitize=address,undefined -std=c++17 -pthread tools/sanitize/gbdt_fuzz.cpp csrc/gbdt.cpp
//   g++ -O1 -g -fsanitize=thread -std=c++17 -pthread tools/sanitize/gbdt_fuzz.cpp csrc/gbdt.cpp
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <limits>
#include <random>
#include <vector>

extern "C" {
int mifx_gbdt_cuts(const double* x, long n, long stride, int max_bins, double* cuts);
int mifx_gbdt_bin(const double* X, long n, int f, const double* cuts, const int* cut_off, const int* ncut,
                  uint16_t* bins, int threads);
int mifx_gbdt_grow(const uint16_t* bins, long n, int f, const int* nbins, const float* g, const float* h,
                   int max_depth, double min_child_weight, double lambda, double gamma, double eta, int threads,
                   int max_nodes, int* feature, int* split_bin, uint8_t* default_left, int* left, int* right,
                   double* value, int* leaf_of_row);
int mifx_gbdt_predict(const double* X, long n, int f, int n_trees, const int* tree_off, const int* feature,
                      const double* thr, const uint8_t* default_left, const int* left, const int* right,
                      const double* value, double base, double* out, int threads);
}

struct Tree {
  std::vector<int> feature, split_bin, left, right, leaf;
  std::vector<uint8_t> dl;
  std::vector<double> value;
  int count = 0;
};

static Tree grow(const std::vector<uint16_t>& bins, long n, int f, const std::vector<int>& nbins,
                 const std::vector<float>& g, const std::vector<float>& h, int depth, int threads, int max_nodes) {
  Tree t;
  t.feature.resize(max_nodes);
  t.split_bin.resize(max_nodes);
  t.left.resize(max_nodes);
  t.right.resize(max_nodes);
  t.dl.resize(max_nodes);
  t.value.resize(max_nodes);
  t.leaf.resize(n);
  t.count = mifx_gbdt_grow(bins.data(), n, f, nbins.data(), g.data(), h.data(), depth, 1.0, 1.0, 0.0, 0.3, threads,
                           max_nodes, t.feature.data(), t.split_bin.data(), t.dl.data(), t.left.data(),
                           t.right.data(), t.value.data(), t.leaf.data());
  return t;
}

static bool same(const Tree& a, const Tree& b, long n) {
  if (a.count != b.count) return false;
  for (int k = 0; k < a.count; ++k)
    if (a.feature[k] != b.feature[k] || a.split_bin[k] != b.split_bin[k] || a.left[k] != b.left[k] ||
        a.right[k] != b.right[k] || a.dl[k] != b.dl[k] || std::memcmp(&a.value[k], &b.value[k], sizeof(double)))
      return false;
  for (long i = 0; i < n; ++i)
    if (a.leaf[i] != b.leaf[i]) return false;
  return true;
}

int main() {
  std::mt19937_64 rng(20251018);
  int failures = 0, trees = 0;
  if (mifx_gbdt_cuts(nullptr, 0, 1, 1, nullptr) != -1 || mifx_gbdt_cuts(nullptr, 0, 1, 70000, nullptr) != -1) {
    std::printf("invalid max_bins accepted\n");
    ++failures;
  }
  for (int trial = 0; trial < 60; ++trial) {
    // every 6th trial is large enough (n * f > 200000) for the learner to split features over threads and for
    // predict to split rows (n > 4096): the paths ThreadSanitizer must see
    const bool big = trial % 6 == 5;
    const long n = trial < 4 ? 1 + trial : big ? 20000 + (long)(rng() % 20000) : 1 + (long)(rng() % 3000);
    const int f = big ? 10 + (int)(rng() % 3) : 1 + (int)(rng() % 12);
    const int max_bins = 2 + (int)(rng() % 300);
    std::vector<double> X((size_t)n * f);
    for (int j = 0; j < f; ++j) {
      const int kind = (int)(rng() % 5);  // 0 continuous, 1 few distinct, 2 constant, 3 all NaN, 4 mixed NaN
      for (long i = 0; i < n; ++i) {
        double v;
        std::uniform_real_distribution<double> u(-3.0, 3.0);
        if (kind == 0) v = u(rng);
        else if (kind == 1) v = (double)(rng() % 7);
        else if (kind == 2) v = 1.25;
        else if (kind == 3) v = std::numeric_limits<double>::quiet_NaN();
        else v = (rng() % 4 == 0) ? std::numeric_limits<double>::quiet_NaN() : u(rng);
        X[(size_t)i * f + j] = v;
      }
    }
    // cuts per feature, exact-size storage
    std::vector<int> ncut(f), cut_off(f + 1, 0), nbins(f);
    std::vector<std::vector<double>> cj(f);
    for (int j = 0; j < f; ++j) {
      std::vector<double> tmp(max_bins - 1);
      const int c = mifx_gbdt_cuts(X.data() + j, n, f, max_bins, tmp.data());
      if (c < 0 || c > max_bins - 1) {
        std::printf("cuts: bad count %d\n", c);
        ++failures;
        continue;
      }
      for (int k = 1; k < c; ++k)
        if (!(tmp[k - 1] < tmp[k])) ++failures;  // strictly ascending
      cj[j].assign(tmp.begin(), tmp.begin() + c);
      ncut[j] = c;
      nbins[j] = c + 1;
      cut_off[j + 1] = cut_off[j] + c;
    }
    std::vector<double> cuts(std::max(1, cut_off[f]));
    for (int j = 0; j < f; ++j) std::copy(cj[j].begin(), cj[j].end(), cuts.begin() + cut_off[j]);
    std::vector<uint16_t> bins((size_t)n * f);
    mifx_gbdt_bin(X.data(), n, f, cuts.data(), cut_off.data(), ncut.data(), bins.data(), 4);
    // gradients of a squared loss toward a random target
    std::vector<float> g(n), h(n, 1.0f);
    std::normal_distribution<float> nd(0.f, 1.f);
    for (long i = 0; i < n; ++i) g[i] = nd(rng);
    const int depth = 1 + (int)(rng() % 6);
    const int max_nodes = (1 << (depth + 1)) - 1;
    Tree t1 = grow(bins, n, f, nbins, g, h, depth, 1, max_nodes);
    ++trees;
    if (t1.count <= 0) {
      std::printf("grow failed: %d\n", t1.count);
      ++failures;
      continue;
    }
    for (int th : {2, 3, 8}) {
      Tree tt = grow(bins, n, f, nbins, g, h, depth, th, max_nodes);
      ++trees;
      if (!same(t1, tt, n)) {
        std::printf("trial %d: %d threads grew a different tree\n", trial, th);
        ++failures;
      }
    }
    if (t1.count > 1) {  // a split tree does not fit a 1-node budget
      Tree small = grow(bins, n, f, nbins, g, h, depth, 2, 1);
      if (small.count != -1) ++failures;
    }
    // prediction with raw values: thr = the cut after the split bin
    std::vector<double> thr(t1.count, 0.0);
    for (int k = 0; k < t1.count; ++k)
      if (t1.feature[k] >= 0) thr[k] = cj[t1.feature[k]][t1.split_bin[k]];
    std::vector<int> off = {0};
    std::vector<double> out(n);
    mifx_gbdt_predict(X.data(), n, f, 1, off.data(), t1.feature.data(), thr.data(), t1.dl.data(), t1.left.data(),
                      t1.right.data(), t1.value.data(), 0.5, out.data(), 4);
    for (long i = 0; i < n; ++i)
      if (out[i] != 0.5 + t1.value[t1.leaf[i]]) {
        std::printf("trial %d row %ld: predict %.17g vs leaf %.17g\n", trial, i, out[i], 0.5 + t1.value[t1.leaf[i]]);
        ++failures;
        break;
      }
  }
  std::printf("%d trees, %d failures\n", trees, failures);
  return failures != 0;
}
