"""PATE-2017 data-dependent moments accountant for the Laplace noisy-max (with smooth sensitivity).

Reference: `research/pate_2017/analysis.py:70-304` (compute_q_noisy_max, logmgf_exact,
logmgf_from_counts, sens_at_k, smoothed_sens, and the epsilon report of `main`)."""
from __future__ import annotations

import math

import numpy as np


def compute_q_noisy_max(counts, noise_eps: float) -> float:
    """Upper bound on Pr[noisy argmax != true argmax]."""
    c = np.asarray(counts, dtype=np.float64)
    w = int(np.argmax(c))
    gaps = -noise_eps * (np.delete(c, w) - c[w])
    q = float(np.sum((gaps + 2.0) / (4.0 * np.exp(gaps))))
    return min(q, 1.0 - 1.0 / len(c))


def compute_q_noisy_max_approx(counts, noise_eps: float) -> float:
    c = np.asarray(counts, dtype=np.float64)
    w = int(np.argmax(c))
    gap = -float(np.max(noise_eps * (np.delete(c, w) - c[w])))
    q = (len(c) - 1) * (gap + 2.0) / (4.0 * math.exp(gap))
    return min(q, 1.0 - 1.0 / len(c))


def logmgf_exact(q: float, priv_eps: float, l: float) -> float:
    """min of three bounds on the log moment generating function at moment l."""
    if q < 0.5:
        t = (1 - q) * math.pow((1 - q) / (1 - math.exp(priv_eps) * q), l) + q * math.exp(priv_eps * l)
        log_t = math.log(t) if t > 0 else priv_eps * l
    else:
        log_t = priv_eps * l
    return min(0.5 * priv_eps * priv_eps * l * (l + 1), log_t, priv_eps * l)


def logmgf_from_counts(counts, noise_eps: float, l: float) -> float:
    """ReportNoisyMax with Lap(1/noise_eps) is 2*noise_eps-DP (one count up, one down)."""
    return logmgf_exact(compute_q_noisy_max(counts, noise_eps), 2.0 * noise_eps, l)


def sens_at_k(counts, noise_eps: float, l: float, k: int) -> float:
    c = sorted(counts, reverse=True)
    if 0.5 * noise_eps * l > 1:
        return 0.0
    if counts[0] < counts[1] + k:
        return 0.0
    c[0] -= k
    c[1] += k
    base = logmgf_from_counts(c, noise_eps, l)
    c[0] -= 1
    c[1] += 1
    return logmgf_from_counts(c, noise_eps, l) - base


def smoothed_sens(counts, noise_eps: float, l: float, beta: float) -> float:
    k = 0
    best = sens_at_k(counts, noise_eps, l, k)
    while k < max(counts):
        k += 1
        s = sens_at_k(counts, noise_eps, l, k)
        best = max(best, math.exp(-beta * k) * s)
        if s == 0.0:
            break
    return best


def votes_to_counts(teacher_labels: np.ndarray, num_classes: int = 10) -> np.ndarray:
    """[T, N] teacher labels -> [N, C] vote counts."""
    T, N = teacher_labels.shape
    counts = np.zeros((N, num_classes), np.int64)
    for t in range(T):
        np.add.at(counts, (np.arange(N), teacher_labels[t].astype(np.int64)), 1)
    return counts


def analyze(counts_mat: np.ndarray, noise_eps: float = 0.1, delta: float = 1e-5, moments: int = 8,
            beta: float = 0.09, indices=None, max_examples: int = 1000) -> dict:
    """The reference's epsilon report: data-dependent eps, smooth-sensitivity scale, data-independent eps."""
    n = counts_mat.shape[0]
    num = min(n, max_examples)
    idx = np.arange(num) if indices is None else np.asarray(indices)[:num]
    ls = 1.0 + np.arange(moments)
    tot_mgf = np.zeros(moments)
    tot_ss = np.zeros(moments)
    for i in idx:
        tot_mgf += [logmgf_from_counts(counts_mat[i], noise_eps, l) for l in ls]
        tot_ss += [smoothed_sens(list(counts_mat[i]), noise_eps, l, beta) for l in ls]
    eps_list = (tot_mgf - math.log(delta)) / ls
    ss_eps = 2.0 * beta * math.log(1 / delta)
    data_ind = num * np.array([logmgf_exact(1.0, 2.0 * noise_eps, l) for l in ls])
    return {"eps_list": eps_list, "eps": float(eps_list.min()), "smoothed_sens": tot_ss / ls, "ss_eps": ss_eps,
            "ss_scale": 2.0 / ss_eps, "data_independent_eps": float(((data_ind - math.log(delta)) / ls).min()),
            "enough_moments": bool(eps_list.min() != eps_list[-1])}
