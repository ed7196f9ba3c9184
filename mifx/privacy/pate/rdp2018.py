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
    """Data-dependent RDP of GNMax (Papernot et al. 2018, Theorem 6), the data-independent lambda / sigma^2
    wherever the theorem gives nothing better.

    Derivation used here. GNMax with noise N(0, sigma^2) is (lambda, lambda / sigma^2)-RDP for every order. Let
    q >= Pr[GNMax(D) != the plurality class] (logq = ln q, Proposition 7). Theorem 6 picks two higher orders
    mu1 = mu2 + 1 > lambda with eps_i = mu_i / sigma^2 and bounds, for lambda < mu1,

        RDP(lambda) <= 1 / (lambda - 1) * ln[(1 - q) A^(lambda - 1) + q B^(lambda - 1)],
        A = (1 - q) / (1 - (q e^eps2)^((mu2 - 1) / mu2)),      B = e^eps1 / q^(1 / (mu1 - 1)),

    valid when q <= e^((mu2 - 1) eps2) / [(mu1 / (mu1 - 1)) (mu2 / (mu2 - 1))]^mu2 and q e^eps2 < 1. The free
    parameter mu2 is set to sqrt(sigma^2 ln(1/q)) (the choice that minimises the bound to first order). Everything
    is evaluated in log space (q can be ~1e-300), and the minimum with the data-independent bound is taken."""
    if logq > 0 or sigma < 0 or np.any(np.asarray(orders) <= 1):
        raise ValueError("Inputs are malformed.")
    lam = np.atleast_1d(np.asarray(orders, dtype=np.float64))
    data_ind = lam / sigma ** 2
    if np.isneginf(logq):  # q = 0: the answer never changes
        out = np.zeros_like(lam)
        return float(out[0]) if np.isscalar(orders) else out
    mu2 = math.sqrt(sigma ** 2 * -logq)
    mu1 = mu2 + 1.0
    eps1, eps2 = mu1 / sigma ** 2, mu2 / sigma ** 2
    applicable = (lam < mu1) & (mu2 > 1)
    # the theorem's conditions on q, in log form: ln q <= (mu2 - 1) eps2 - mu2 ln[(mu1/(mu1-1)) (mu2/(mu2-1))]
    # and ln q + eps2 < 0
    q_small_enough = logq <= (mu2 - 1) * eps2 - mu2 * (math.log(mu1 / (mu1 - 1)) + math.log(mu2 / (mu2 - 1)))
    bound = data_ind.copy()
    if applicable.any() and q_small_enough and logq + eps2 < 0:
        log_1mq = log1mexp(logq)                                        # ln(1 - q)
        log_A = log_1mq - log1mexp((logq + eps2) * (mu2 - 1) / mu2)     # ln A
        log_B = eps1 - logq / (mu1 - 1)                                  # ln B
        log_mix = np.logaddexp(log_1mq + (lam - 1) * log_A, logq + (lam - 1) * log_B)
        dep = log_mix / (lam - 1)
        bound = np.where(applicable, np.minimum(data_ind, dep), data_ind)
    assert np.all(bound >= 0)
    return float(bound[0]) if np.isscalar(orders) else bound


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
