// Histogram gradient-boosted trees (host C++): the tree learner behind mifx.gbdt's XGBRegressor / XGBClassifier.
//
// Reference workload: the fairing XGBoost sample (`kubeflow-pipelines/fairing/fairing_xgboost.py:69-87`: 1000
// estimators, learning rate 0.1, early stopping 50 on an eval set) and notebook N12 (CPU scope, the
// Ames housing table is ~1.5k rows x 37 numeric columns -- far below the size where a GPU launch pays). The learner
// is XGBoost's second-order one on quantised features:
//  * binning: per feature, the sorted distinct values give the cut points (value < cut goes left); more than
//    max_bins distinct values are thinned to count quantiles. NaN is "missing" (bin 0xFFFF) and each split learns
//    the direction missing values take (both tried, the better kept), as XGBoost's sparsity-aware split does.
//  * growth: depth-wise to max_depth; a node's histogram of (sum g, sum h) per bin is built for the smaller child
//    only and the larger one is the parent's minus it; the best split maximises
//    G_L^2 / (H_L + lambda) + G_R^2 / (H_R + lambda) - G^2 / (H + lambda) (halved, minus gamma) subject to
//    H_L, H_R >= min_child_weight; leaves take -eta G / (H + lambda).
//  * determinism: ties go to the lowest feature, then the lowest cut; histograms are summed in row order, so a
//    model is bit-reproducible for any thread count (threads split the features, never the rows of one feature).
// Rows of a node are a contiguous range of one permutation array, partitioned in place after each split.
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <thread>
#include <vector>

namespace {

constexpr uint16_t kMissing = 0xFFFF;

struct Hist {
  double g, h;
};

struct Split {
  double gain = 0.0;
  int feature = -1;
  int bin = -1;  // rows with bin <= this go left
  bool default_left = false;
  double gl = 0, hl = 0, gr = 0, hr = 0;
};

struct Node {
  int begin, end, depth, id;
  double g, h;
  std::vector<Hist> hist;  // [features][nbins + 1], the last slot is "missing"
};

template <class F>
void parallel_for(int n, int threads, F&& fn) {
  if (threads <= 1 || n <= 1) {
    for (int i = 0; i < n; ++i) fn(i);
    return;
  }
  threads = std::min(threads, n);
  std::vector<std::thread> pool;
  pool.reserve(threads);
  for (int t = 0; t < threads; ++t)
    pool.emplace_back([&, t] {
      for (int i = t; i < n; i += threads) fn(i);
    });
  for (auto& th : pool) th.join();
}

}  // namespace

extern "C" {

// Cut points of one feature column (n values, stride `stride` doubles apart): writes up to max_bins - 1 ascending
// cuts into `cuts` and returns their count.
int mifx_gbdt_cuts(const double* x, long n, long stride, int max_bins, double* cuts) {
  if (max_bins < 2 || max_bins > 65535) return -1;
  std::vector<double> v;
  v.reserve(n);
  for (long i = 0; i < n; ++i) {
    const double a = x[i * stride];
    if (!std::isnan(a)) v.push_back(a);
  }
  if (v.empty()) return 0;
  std::sort(v.begin(), v.end());
  // distinct values with their counts
  std::vector<double> u;
  std::vector<long> cnt;
  for (size_t i = 0; i < v.size(); ++i) {
    if (u.empty() || v[i] != u.back()) {
      u.push_back(v[i]);
      cnt.push_back(1);
    } else {
      ++cnt.back();
    }
  }
  int nc = 0;
  if ((long)u.size() <= max_bins) {
    for (size_t i = 1; i < u.size(); ++i) cuts[nc++] = u[i];  // one bin per distinct value
    return nc;
  }
  // count quantiles: a cut before the distinct value at which the running count crosses k n / max_bins
  const double total = (double)v.size();
  long run = 0;
  int k = 1;
  for (size_t i = 0; i < u.size() && nc < max_bins - 1; ++i) {
    if (i > 0 && (double)run >= k * total / max_bins) {
      cuts[nc++] = u[i];
      while (k * total / max_bins <= (double)run) ++k;
    }
    run += cnt[i];
  }
  return nc;
}

// Bin a row-major [n, f] matrix into a column-major [f, n] uint16 matrix with the per-feature cuts
// (cuts + cut_off[j], ncut[j] of them): bin = number of cuts <= x, NaN -> 0xFFFF.
int mifx_gbdt_bin(const double* X, long n, int f, const double* cuts, const int* cut_off, const int* ncut,
                  uint16_t* bins, int threads) {
  parallel_for(f, n * (long)f > 200000 ? threads : 1, [&](int j) {
    const double* c = cuts + cut_off[j];
    const int m = ncut[j];
    uint16_t* out = bins + (size_t)j * n;
    for (long i = 0; i < n; ++i) {
      const double a = X[(size_t)i * f + j];
      out[i] = std::isnan(a) ? kMissing : (uint16_t)(std::upper_bound(c, c + m, a) - c);
    }
  });
  return 0;
}

// Grow one tree on binned features. nbins[j] = ncut[j] + 1. g / h: per-row gradients and hessians. The tree is
// written as parallel arrays of at most max_nodes entries: feature (-1 = leaf), split bin, default_left, left,
// right, value (leaf output, eta applied). leaf_of_row[i] receives the leaf id of row i (for the caller's
// prediction update). Returns the node count, or -1 if max_nodes is too small.
int mifx_gbdt_grow(const uint16_t* bins, long n, int f, const int* nbins, const float* g, const float* h,
                   int max_depth, double min_child_weight, double lambda, double gamma, double eta, int threads,
                   int max_nodes, int* feature, int* split_bin, uint8_t* default_left, int* left, int* right,
                   double* value, int* leaf_of_row) {
  std::vector<int> off(f + 1, 0);
  for (int j = 0; j < f; ++j) off[j + 1] = off[j] + nbins[j] + 1;
  const int hsize = off[f];
  std::vector<int> rows(n);
  for (long i = 0; i < n; ++i) rows[i] = (int)i;
  const int th = n * (long)f > 200000 ? threads : 1;

  auto build = [&](Node& nd) {
    nd.hist.assign(hsize, Hist{0.0, 0.0});
    parallel_for(f, th, [&](int j) {
      Hist* hj = nd.hist.data() + off[j];
      const uint16_t* bj = bins + (size_t)j * n;
      const int nb = nbins[j];
      for (int k = nd.begin; k < nd.end; ++k) {
        const int r = rows[k];
        const uint16_t b = bj[r];
        Hist& e = hj[b == kMissing ? nb : b];
        e.g += g[r];
        e.h += h[r];
      }
    });
  };
  auto score = [&](double G, double H) { return G * G / (H + lambda); };
  auto best_split = [&](const Node& nd) {
    std::vector<Split> per(f);
    const double parent = score(nd.g, nd.h);
    parallel_for(f, th, [&](int j) {
      const Hist* hj = nd.hist.data() + off[j];
      const int nb = nbins[j];
      const double gm = hj[nb].g, hm = hj[nb].h;
      Split bs;
      double gl = 0, hl = 0;
      for (int b = 0; b + 1 < nb; ++b) {  // cut after bin b
        gl += hj[b].g;
        hl += hj[b].h;
        for (int dir = 0; dir < 2; ++dir) {  // dir 0: missing right, 1: missing left
          if (dir == 1 && hm == 0.0 && gm == 0.0) break;
          const double GL = gl + (dir ? gm : 0.0), HL = hl + (dir ? hm : 0.0);
          const double GR = nd.g - GL, HR = nd.h - HL;
          if (HL < min_child_weight || HR < min_child_weight) continue;
          const double gain = 0.5 * (score(GL, HL) + score(GR, HR) - parent) - gamma;
          if (gain > bs.gain) {
            bs.gain = gain;
            bs.feature = j;
            bs.bin = b;
            bs.default_left = dir == 1;
            bs.gl = GL, bs.hl = HL, bs.gr = GR, bs.hr = HR;
          }
        }
      }
      per[j] = bs;
    });
    Split best;
    for (int j = 0; j < f; ++j)
      if (per[j].feature >= 0 && per[j].gain > best.gain + 1e-12 * std::fabs(best.gain)) best = per[j];
    return best;
  };

  int count = 0;
  auto new_node = [&]() -> int {
    if (count >= max_nodes) return -1;
    feature[count] = -1;
    split_bin[count] = -1;
    default_left[count] = 0;
    left[count] = right[count] = -1;
    value[count] = 0.0;
    return count++;
  };
  Node root{0, (int)n, 0, new_node(), 0.0, 0.0, {}};
  if (root.id < 0) return -1;
  for (long i = 0; i < n; ++i) {
    root.g += g[i];
    root.h += h[i];
  }
  build(root);
  std::vector<Node> level;
  level.push_back(std::move(root));
  auto make_leaf = [&](const Node& nd) {
    value[nd.id] = -eta * nd.g / (nd.h + lambda);
    for (int k = nd.begin; k < nd.end; ++k) leaf_of_row[rows[k]] = nd.id;
  };
  while (!level.empty()) {
    std::vector<Node> next;
    for (Node& nd : level) {
      Split s;
      if (nd.depth < max_depth && nd.end - nd.begin >= 2) s = best_split(nd);
      if (s.feature < 0 || s.gain <= 1e-6) {
        make_leaf(nd);
        continue;
      }
      // partition rows: left = bin <= s.bin (or missing with default_left)
      const uint16_t* bj = bins + (size_t)s.feature * n;
      auto goes_left = [&](int r) {
        const uint16_t b = bj[r];
        return b == kMissing ? s.default_left : (int)b <= s.bin;
      };
      const int mid = (int)(std::stable_partition(rows.begin() + nd.begin, rows.begin() + nd.end, goes_left) -
                            rows.begin());
      const int li = new_node(), ri = new_node();
      if (li < 0 || ri < 0) return -1;
      feature[nd.id] = s.feature;
      split_bin[nd.id] = s.bin;
      default_left[nd.id] = s.default_left;
      left[nd.id] = li;
      right[nd.id] = ri;
      Node L{nd.begin, mid, nd.depth + 1, li, s.gl, s.hl, {}};
      Node R{mid, nd.end, nd.depth + 1, ri, s.gr, s.hr, {}};
      const bool grow_more = nd.depth + 1 < max_depth;
      if (grow_more) {  // smaller child built, larger = parent - smaller
        Node& small = (L.end - L.begin) <= (R.end - R.begin) ? L : R;
        Node& large = &small == &L ? R : L;
        build(small);
        large.hist = std::move(nd.hist);
        for (int k = 0; k < hsize; ++k) {
          large.hist[k].g -= small.hist[k].g;
          large.hist[k].h -= small.hist[k].h;
        }
      }
      next.push_back(std::move(L));
      next.push_back(std::move(R));
    }
    level = std::move(next);
  }
  return count;
}

// Sum of the first n_trees trees' outputs for each row of a row-major [n, f] matrix of raw values. Trees are
// concatenated: tree t's nodes are [tree_off[t], tree_off[t + 1]) with child indices local to the tree; thr is
// the split's cut value (go left iff x < thr, NaN follows default_left).
int mifx_gbdt_predict(const double* X, long n, int f, int n_trees, const int* tree_off, const int* feature,
                      const double* thr, const uint8_t* default_left, const int* left, const int* right,
                      const double* value, double base, double* out, int threads) {
  const int chunks = n > 4096 ? std::max(1, threads) : 1;
  parallel_for(chunks, chunks, [&](int c) {
    const long lo = n * c / chunks, hi = n * (c + 1) / chunks;
    for (long i = lo; i < hi; ++i) {
      const double* xi = X + (size_t)i * f;
      double s = base;
      for (int t = 0; t < n_trees; ++t) {
        const int o = tree_off[t];
        int k = 0;
        while (feature[o + k] >= 0) {
          const double a = xi[feature[o + k]];
          const bool l = std::isnan(a) ? default_left[o + k] != 0 : a < thr[o + k];
          k = l ? left[o + k] : right[o + k];
        }
        s += value[o + k];
      }
      out[i] = s;
    }
  });
  return 0;
}

}  // extern "C"
