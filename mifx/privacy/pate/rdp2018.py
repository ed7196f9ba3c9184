"""PATE-2018 ("Scalable Private Learning with PATE") RDP analysis of GNMax / threshold / LNMax.

Reference: `research/pate_2018/core.py:27-370` — compute_eps_from_delta, compute_logq_gaussian
(Prop. 7), rdp_data_independent_gaussian (Prop. 8), rdp_gaussian (Thm. 6), the threshold
mechanism, compute_logq_laplace and rdp_pure_eps (PATE-2017 Thm. 3 in RDP form)."""
from __future__ import annotations

import math

import numpy as np
import scipy.stats


def _logsumexp(x) -> float:
    x = np.asarray(x, dtype=np.float64)
    m = x.max()
    return float(m + math.log(np.exp(x - m).sum()))


def log1mexp(x: float) -> float:
    """log(1 - exp(x)) for x <= 0, stable."""
    if x < -1:
        return math.log1p(-math.exp(x))
    if x < 0:
        return math.log(-math.expm1(x))
    if x == 0:
        return -math.inf
    raise ValueError("Argument must be non-positive.")


def compute_eps_from_delta(orders, rdp, delta: float):
    if len(orders) != len(rdp):
        raise ValueError("Input lists must have the same length.")
    eps = np.asarray(rdp, dtype=np.float64) - math.log(delta) / (np.asarray(orders, dtype=np.float64) - 1)
    i = int(np.argmin(eps))
    return float(eps[i]), orders[i]


def compute_logq_gaussian(counts, sigma: float) -> float:
    """Upper bound on ln Pr[GNMax outcome != argmax] (Proposition 7)."""
    c = np.asarray(counts, dtype=np.float64)
    n = len(c)
    top = int(np.argmax(c))
    gaps = (c[top] - c)[np.arange(n) != top]
    logq = _logsumexp(scipy.stats.norm.logsf(gaps, scale=math.sqrt(2 * sigma ** 2)))
    return min(logq, math.log(1 - 1 / n))


def rdp_data_independent_gaussian(sigma: float, orders):
    if sigma < 0 or np.any(np.asarray(orders) <= 1):
        raise ValueError("Inputs are malformed.")
    return orders / sigma ** 2 if np.isscalar(orders) else np.atleast_1d(orders) / sigma ** 2


def rdp_gaussian(logq: float, sigma: float, orders):
    """Data-dependent RDP of GNMax given logq (Theorem 6); falls back to the data-independent bound."""
    if logq > 0 or sigma < 0 or np.any(np.asarray(orders) <= 1):
        raise ValueError("Inputs are malformed.")
    scalar = np.isscalar(orders)
    if np.isneginf(logq):
        return 0.0 if scalar else np.zeros(len(np.atleast_1d(orders)))
    var = sigma ** 2
    mu2 = math.sqrt(var * -logq)
    mu1 = mu2 + 1
    ov = np.atleast_1d(np.asarray(orders, dtype=np.float64))
    ret = ov / var
    mask = np.logical_and(mu1 > ov, mu2 > 1)
    eps1, eps2 = mu1 / var, mu2 / var
    log_a2 = (mu2 - 1) * eps2
    if (np.any(mask) and logq <= log_a2 - mu2 * (math.log(1 + 1 / (mu1 - 1)) + math.log(1 + 1 / (mu2 - 1)))
            and -logq > eps2):
        log1q = log1mexp(logq)
        log_a = (ov - 1) * (log1q - log1mexp((logq + eps2) * (1 - 1 / mu2)))
        log_b = (ov - 1) * (eps1 - logq / (mu1 - 1))
        log_s = np.logaddexp(log1q + log_a, logq + log_b)
        ret[mask] = np.minimum(ret, log_s / (ov - 1))[mask]
    assert np.all(ret >= 0)
    return float(ret[0]) if scalar else ret


def is_data_independent_always_opt_gaussian(num_teachers: int, num_classes: int, sigma: float, orders):
    unanimous = np.array([num_teachers] + [0] * (num_classes - 1))
    return np.isclose(rdp_gaussian(compute_logq_gaussian(unanimous, sigma), sigma, orders),
                      rdp_data_independent_gaussian(sigma, orders))


def compute_logpr_answered(t: float, sigma: float, counts) -> float:
    """ln Pr[max vote + N(0, sigma^2) >= t]."""
    return float(scipy.stats.norm.logsf(t - round(max(counts)), scale=sigma))


def compute_rdp_data_independent_threshold(sigma: float, orders):
    return rdp_data_independent_gaussian(2 ** 0.5 * sigma, orders)


def compute_rdp_threshold(log_pr_answered: float, sigma: float, orders):
    logq = min(log_pr_answered, log1mexp(log_pr_answered))
    return rdp_gaussian(logq, 2 ** 0.5 * sigma, orders)


def is_data_independent_always_opt_threshold(num_teachers: int, threshold: float, sigma: float, orders):
    ind = compute_rdp_data_independent_threshold(sigma, orders)
    d1 = compute_rdp_threshold(compute_logpr_answered(threshold, sigma, [0]), sigma, orders)
    d2 = compute_rdp_threshold(compute_logpr_answered(threshold, sigma, [num_teachers]), sigma, orders)
    return np.isclose(d1, ind) and np.isclose(d2, ind)


def compute_logq_laplace(counts, lmbd: float) -> float:
    """Upper bound on ln Pr[LNMax outcome != argmax] with Laplace(lmbd) noise."""
    c = np.asarray(counts, dtype=np.float64)
    top = int(np.argmax(c))
    rest = np.delete((c - c[top]) / lmbd, top)
    logq = _logsumexp(np.log(2 - rest) + math.log(0.25) + rest)
    return min(logq, math.log(1 - 1 / len(c)))


def rdp_pure_eps(logq: float, pure_eps: float, orders):
    ov = np.atleast_1d(np.asarray(orders, dtype=np.float64))
    q = math.exp(logq)
    log_t = np.full_like(ov, np.inf)
    if q <= 1 / (math.exp(pure_eps) + 1):
        t1 = math.log1p(-q) + (math.log1p(-q) - log1mexp(pure_eps + logq)) * (ov - 1)
        t2 = logq + pure_eps * (ov - 1)
        log_t = np.logaddexp(t1, t2)
    ret = np.minimum(np.minimum(0.5 * pure_eps * pure_eps * ov, log_t / (ov - 1)), pure_eps)
    return float(ret[0]) if np.isscalar(orders) else ret
