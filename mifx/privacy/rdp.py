"""Rényi-DP accountant for the Sampled Gaussian Mechanism (DP-SGD).

Reference: `notebooks/privacy/privacy/analysis/rdp_accountant.py:40-301` (public API
`compute_rdp(q, noise_multiplier, steps, orders)` and
`get_privacy_spent(orders, rdp, target_eps=None, target_delta=None)`), pinned by
`rdp_accountant_test.py` goldens (0.07737; 1.258575 @ order 20; 8.509656 @ order 2.5) and an
mpmath quadrature oracle for log A_alpha.

log A_alpha = log E_{z~N(0,s^2)} [((1-q) + q exp((2z-1)/(2 s^2)))^alpha]:
* integer alpha — binomial expansion, summed in log space;
* fractional alpha — the two-sided series split at z0 = s^2 log(1/q - 1) + 1/2 with erfc tails,
  iterated until both terms fall below e^-30.
RDP(alpha) = log A_alpha / (alpha - 1); (eps, delta) via eps = rdp - log(delta)/(alpha - 1)."""
from __future__ import annotations

import math

import numpy as np
from scipy import special

DEFAULT_ORDERS = tuple([1 + x / 10.0 for x in range(1, 100)] + list(range(12, 64)) + [128, 256, 512])


def _logsumexp2(a: float, b: float) -> float:
    lo, hi = (a, b) if a < b else (b, a)
    if lo == -math.inf:
        return hi
    return hi + math.log1p(math.exp(lo - hi))


def _logdiffexp(a: float, b: float) -> float:
    """log(exp(a) - exp(b)), a >= b."""
    if a < b:
        raise ValueError("log-space subtraction would be negative")
    if b == -math.inf:
        return a
    if a == b:
        return -math.inf
    try:
        return a + math.log(-math.expm1(b - a))
    except (OverflowError, ValueError):
        return a


def _log_erfc(x: float) -> float:
    return math.log(2.0) + special.log_ndtr(-x * math.sqrt(2.0))


def _log_a_integer(q: float, sigma: float, alpha: int) -> float:
    lq, l1q = math.log(q), math.log1p(-q)
    terms = np.array([special.gammaln(alpha + 1) - special.gammaln(i + 1) - special.gammaln(alpha - i + 1)
                      + i * lq + (alpha - i) * l1q + (i * i - i) / (2.0 * sigma * sigma)
                      for i in range(alpha + 1)])
    m = terms.max()
    return float(m + math.log(np.exp(terms - m).sum()))


def _log_a_fractional(q: float, sigma: float, alpha: float) -> float:
    neg_inf = -math.inf
    acc0, acc1 = neg_inf, neg_inf
    z0 = sigma * sigma * math.log(1.0 / q - 1.0) + 0.5
    lq, l1q = math.log(q), math.log1p(-q)
    i = 0
    while True:
        coef = special.binom(alpha, i)
        lc = math.log(abs(coef))
        j = alpha - i
        s0 = lc + i * lq + j * l1q + (i * i - i) / (2 * sigma * sigma) + \
            math.log(0.5) + _log_erfc((i - z0) / (math.sqrt(2) * sigma))
        s1 = lc + j * lq + i * l1q + (j * j - j) / (2 * sigma * sigma) + \
            math.log(0.5) + _log_erfc((z0 - j) / (math.sqrt(2) * sigma))
        if coef > 0:
            acc0, acc1 = _logsumexp2(acc0, s0), _logsumexp2(acc1, s1)
        else:
            acc0, acc1 = _logdiffexp(acc0, s0), _logdiffexp(acc1, s1)
        i += 1
        if max(s0, s1) < -30:
            return _logsumexp2(acc0, acc1)


def log_a(q: float, sigma: float, alpha: float) -> float:
    """log A_alpha of the sampled Gaussian mechanism, 0 < q < 1."""
    if float(alpha).is_integer():
        return _log_a_integer(q, sigma, int(alpha))
    return _log_a_fractional(q, sigma, float(alpha))


def _rdp_one(q: float, sigma: float, alpha: float) -> float:
    if q == 0:
        return 0.0
    if q == 1.0:
        return alpha / (2 * sigma ** 2)
    if np.isinf(alpha):
        return np.inf
    return log_a(q, sigma, alpha) / (alpha - 1)


def compute_rdp(q: float, noise_multiplier: float, steps: int, orders):
    """RDP of `steps` compositions of the SGM with sampling rate q, at each order."""
    if np.isscalar(orders):
        return _rdp_one(q, noise_multiplier, orders) * steps
    return np.array([_rdp_one(q, noise_multiplier, a) for a in orders]) * steps


def get_privacy_spent(orders, rdp, target_eps=None, target_delta=None):
    """(eps, delta, optimal_order) for a given delta (or eps)."""
    if (target_eps is None) == (target_delta is None):
        raise ValueError("Exactly one out of eps and delta must be None.")
    orders_v, rdp_v = np.atleast_1d(orders).astype(float), np.atleast_1d(rdp).astype(float)
    if len(orders_v) != len(rdp_v):
        raise ValueError("Input lists must have the same length.")
    if target_eps is not None:
        deltas = np.exp((rdp_v - target_eps) * (orders_v - 1))
        i = int(np.argmin(deltas))
        return target_eps, min(float(deltas[i]), 1.0), np.atleast_1d(orders)[i]
    eps = rdp_v - math.log(target_delta) / (orders_v - 1)
    i = int(np.nanargmin(eps))
    return float(eps[i]), target_delta, np.atleast_1d(orders)[i]


def compute_dp_sgd_privacy(n: int, batch_size: int, noise_multiplier: float, epochs: float, delta: float = 1e-5,
                           orders=DEFAULT_ORDERS):
    """eps of DP-SGD with Poisson rate batch/n for epochs*n/batch steps (the tutorial's `compute_epsilon`,
    `tutorials/mnist_dpsgd_tutorial.py:87-98`)."""
    q = batch_size / n
    steps = int(math.ceil(epochs * n / batch_size))
    rdp = compute_rdp(q, noise_multiplier, steps, orders)
    eps, _, order = get_privacy_spent(orders, rdp, target_delta=delta)
    return eps, order


class RdpAccountant:
    """Stateful composition over heterogeneous SGM steps (e.g. changing batch size / noise)."""

    def __init__(self, orders=DEFAULT_ORDERS):
        self.orders = tuple(orders)
        self.rdp = np.zeros(len(self.orders))

    def step(self, q: float, noise_multiplier: float, steps: int = 1) -> None:
        self.rdp = self.rdp + compute_rdp(q, noise_multiplier, steps, self.orders)

    def epsilon(self, delta: float) -> float:
        return get_privacy_spent(self.orders, self.rdp, target_delta=delta)[0]
