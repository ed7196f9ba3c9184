"""PATE-2017 privacy analysis: the data-dependent moments accountant of the Laplace noisy-max aggregator.

Papernot et al., "Semi-supervised Knowledge Transfer for Deep Learning from Private Training Data" (ICLR 2017),
Theorems 2-3 and Appendix C. The aggregator answers a query by argmax_j (n_j + Lap(1/gamma)) over the teachers'
vote counts n; changing one teacher moves one count up and one down, so one answer is (2 gamma)-DP.

* The probability that the noisy answer differs from the plurality j* is at most
      q <= sum_{j != j*} (2 + gamma D_j) / (4 exp(gamma D_j)),   D_j = n_{j*} - n_j          (Thm 3)
  (the tail of a difference of two Laplace variables), capped at 1 - 1/C.
* The l-th log moment of one answer of an (2 gamma)-DP mechanism whose outcome is j* with probability 1 - q is
      alpha(l) <= min( 2 gamma^2 l (l + 1),                                 (data-independent, Thm 2)
                       log((1-q) ((1-q) / (1 - e^{2 gamma} q))^l + q e^{2 gamma l}),   (q < 1/2)
                       2 gamma l )
  and moments compose additively; eps = min_l (sum alpha(l) + log(1/delta)) / l.
* Releasing the data-dependent eps needs its smooth sensitivity (Appendix C): the local sensitivity of alpha at
  distance k is the change of alpha when one more vote moves from the plurality class to the runner-up, after k
  such moves; the beta-smooth bound is max_k e^{-beta k} LS(k), and the release costs eps_ss = 2 beta log(1/delta).

Reference driver and report: `research/pate_2017/analysis.py:70-304`. One deliberate difference: the reference's
distance-k check compares the UNSORTED input's first two counts (its `counts[0] < counts[1] + k` after sorting a
copy); here every step uses the plurality and runner-up of the sorted counts, as the analysis defines them (equal
results for count vectors already sorted in decreasing order)."""
from __future__ import annotations

import math

import numpy as np


def noisy_max_q(counts, gamma: float) -> np.ndarray:
    """Thm 3 bound on Pr[noisy argmax != plurality], for one count vector [C] or a batch [N, C]."""
    c = np.atleast_2d(np.asarray(counts, dtype=np.float64))
    gaps = gamma * (c.max(axis=1, keepdims=True) - c)  # D_j gamma >= 0; the plurality itself has gap 0
    terms = (gaps + 2.0) / (4.0 * np.exp(gaps))
    top = np.argmax(c, axis=1)
    terms[np.arange(c.shape[0]), top] = 0.0  # j != j* (only the first plurality class is excluded)
    q = np.minimum(terms.sum(axis=1), 1.0 - 1.0 / c.shape[1])
    return q if np.ndim(counts) > 1 else q[0]


def compute_q_noisy_max(counts, noise_eps: float) -> float:
    return float(noisy_max_q(counts, noise_eps))


def compute_q_noisy_max_approx(counts, noise_eps: float) -> float:
    """The cheaper bound with every class at the runner-up's gap: (C - 1) (2 + g) / (4 e^g)."""
    c = np.asarray(counts, dtype=np.float64)
    srt = np.sort(c)[::-1]
    g = noise_eps * (srt[0] - srt[1])
    return float(min((len(c) - 1) * (g + 2.0) / (4.0 * math.exp(g)), 1.0 - 1.0 / len(c)))


def log_moment(q: float, eps: float, l: float) -> float:
    """Thm 2 bound on the l-th log moment of an eps-DP answer that is the plurality w.p. 1 - q."""
    bounds = [0.5 * eps * eps * l * (l + 1), eps * l]
    if q < 0.5:
        t = (1.0 - q) * ((1.0 - q) / (1.0 - math.exp(eps) * q)) ** l + q * math.exp(eps * l)
        if t > 0:
            bounds.append(math.log(t))
    return min(bounds)


def logmgf_exact(q: float, priv_eps: float, l: float) -> float:
    return log_moment(q, priv_eps, l)


def logmgf_from_counts(counts, noise_eps: float, l: float) -> float:
    """alpha(l) of one noisy-max answer with Lap(1/noise_eps) noise: a (2 noise_eps)-DP mechanism."""
    return log_moment(compute_q_noisy_max(counts, noise_eps), 2.0 * noise_eps, l)


def _moved(srt: np.ndarray, k: int) -> np.ndarray:
    """The sorted counts after k votes moved from the plurality class to the runner-up."""
    v = srt.copy()
    v[0] -= k
    v[1] += k
    return v


def local_sensitivity(counts, noise_eps: float, l: float, k: int) -> float:
    """LS of alpha(l) at distance k (Appendix C); 0 once the runner-up could overtake (the bound is then the
    data-independent one) or when 2 gamma l / 2 > 1 (outside the range the analysis covers)."""
    if 0.5 * noise_eps * l > 1:
        return 0.0
    srt = np.sort(np.asarray(counts, dtype=np.float64))[::-1]
    if srt[0] < srt[1] + k:
        return 0.0
    return logmgf_from_counts(_moved(srt, k + 1), noise_eps, l) - logmgf_from_counts(_moved(srt, k), noise_eps, l)


sens_at_k = local_sensitivity


def smoothed_sens(counts, noise_eps: float, l: float, beta: float) -> float:
    """beta-smooth upper bound max_k e^{-beta k} LS(k), scanning k until LS vanishes (or k exceeds the votes)."""
    best = local_sensitivity(counts, noise_eps, l, 0)
    kmax = int(np.max(counts))
    for k in range(1, kmax + 1):
        s = local_sensitivity(counts, noise_eps, l, k)
        best = max(best, math.exp(-beta * k) * s)
        if s == 0.0:
            break
    return best


def votes_to_counts(teacher_labels: np.ndarray, num_classes: int = 10) -> np.ndarray:
    """[T, N] teacher labels -> [N, C] vote counts."""
    lab = np.asarray(teacher_labels, dtype=np.int64)
    T, N = lab.shape
    flat = (np.arange(N)[None, :] * num_classes + lab).ravel()
    return np.bincount(flat, minlength=N * num_classes).reshape(N, num_classes)


def analyze(counts_mat: np.ndarray, noise_eps: float = 0.1, delta: float = 1e-5, moments: int = 8,
            beta: float = 0.09, indices=None, max_examples: int = 1000) -> dict:
    """The privacy report for the first `max_examples` answered queries: the data-dependent eps (best moment), the
    per-moment smooth sensitivity and the cost / noise scale of releasing it, and the data-independent eps."""
    counts_mat = np.asarray(counts_mat)
    num = min(counts_mat.shape[0], max_examples)
    idx = np.arange(num) if indices is None else np.asarray(indices)[:num]
    ls = np.arange(1, moments + 1, dtype=np.float64)
    qs = noisy_max_q(counts_mat[idx], noise_eps)
    tot_mgf = np.array([sum(log_moment(float(q), 2.0 * noise_eps, l) for q in qs) for l in ls])
    tot_ss = np.array([sum(smoothed_sens(counts_mat[i], noise_eps, l, beta) for i in idx) for l in ls])
    eps_list = (tot_mgf - math.log(delta)) / ls
    ss_eps = 2.0 * beta * math.log(1 / delta)
    data_ind = num * np.array([log_moment(1.0, 2.0 * noise_eps, l) for l in ls])
    return {"eps_list": eps_list, "eps": float(eps_list.min()), "smoothed_sens": tot_ss / ls, "ss_eps": ss_eps,
            "ss_scale": 2.0 / ss_eps, "data_independent_eps": float(((data_ind - math.log(delta)) / ls).min()),
            "enough_moments": bool(eps_list.min() != eps_list[-1])}
