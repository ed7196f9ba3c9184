"""Smooth sensitivity of the PATE-2018 data-dependent RDP (GNMax and threshold mechanisms).

Reference: `research/pate_2018/smooth_sensitivity.py:27-419` — logq0 (where the data-dependent
bound meets the data-independent one, by Brent root finding), local-sensitivity bounds at every
distance in O(teachers * classes), discounted max, RDP of the smooth-sensitivity release
(Thm. 23), and the symbolic monotonicity checks (Conditions 5/6) done with sympy."""
from __future__ import annotations

import functools
import math

import numpy as np
import scipy.optimize
import scipy.special
import scipy.stats

from . import rdp2018 as core


def _mu(sigma: float, logq: float):
    mu2 = sigma * math.sqrt(-logq)
    return mu2 + 1, mu2


def _data_dep_bound(sigma: float, logq: float, order: float) -> float:
    var = sigma ** 2
    mu1, mu2 = _mu(sigma, logq)
    eps1, eps2 = mu1 / var, mu2 / var
    log1q = np.log1p(-math.exp(logq))
    log_a = (order - 1) * (log1q - np.log1p(-math.exp((logq + eps2) * (1 - 1 / mu2))))
    log_b = (order - 1) * (eps1 - logq / (mu1 - 1))
    return float(np.logaddexp(log1q + log_a, logq + log_b) / (order - 1))


def compute_logq0_gnmax(sigma: float, order: float) -> float:
    """logq above which the data-independent bound is the better one."""
    def valid(logq):
        mu1, mu2 = _mu(sigma, logq)
        if mu1 < order:
            return False
        eps2 = mu2 / sigma ** 2
        return logq <= (mu2 - 1) * eps2 - mu2 * math.log(mu1 / (mu1 - 1) * mu2 / (mu2 - 1))

    def gap(logq):
        return _data_dep_bound(sigma, logq, order) - core.rdp_data_independent_gaussian(sigma, order)

    hi = min(-(1 + 1.0 / sigma) ** 2, -((order - 0.99) / sigma) ** 2, -1 / sigma ** 2)
    assert valid(hi)
    if gap(hi) < 0:
        return hi
    lo = 2 * hi
    while gap(lo) > 0:
        assert lo > -10000, "The lower bound on q0 is way too low."
        lo *= 1.5
    root, r = scipy.optimize.brentq(gap, lo, hi, full_output=True)
    assert r.converged and valid(root)
    return root


@functools.lru_cache(maxsize=None)
def _logq0(sigma: float, order: float) -> float:
    return compute_logq0_gnmax(sigma, order)


def _bl(q: float, sigma: float, m: int) -> float:
    return (m - 1) / 2 * scipy.special.erfc(1 / sigma + scipy.special.erfcinv(2 * q / (m - 1)))


def _bu(q: float, sigma: float, m: int) -> float:
    return min(1, (m - 1) / 2 * scipy.special.erfc(-1 / sigma + scipy.special.erfcinv(2 * q / (m - 1))))


@functools.lru_cache(maxsize=None)
def _logq1(sigma: float, order: float, m: int) -> float:
    lq0 = _logq0(sigma, order)
    lq1 = math.log(_bl(math.exp(lq0), sigma, m))
    assert lq1 <= lq0
    return lq1


def _rdp_gnmax(sigma: float, logq: float, order: float) -> float:
    if logq >= _logq0(sigma, order):
        return core.rdp_data_independent_gaussian(sigma, order)
    return _data_dep_bound(sigma, logq, order)


def _local_sens(logq: float, sigma: float, m: int, order: float) -> float:
    lq0, lq1 = _logq0(sigma, order), _logq1(sigma, order, m)
    if lq1 <= logq <= lq0:
        logq = lq1
    beta = _rdp_gnmax(sigma, logq, order)
    up = _rdp_gnmax(sigma, math.log(_bu(math.exp(logq), sigma, m)), order)
    down = _rdp_gnmax(sigma, math.log(_bl(math.exp(logq), sigma, m)), order)
    return max(up - beta, beta - down)


def compute_local_sensitivity_bounds_gnmax(votes, num_teachers: int, sigma: float, order: float) -> np.ndarray:
    """Local sensitivity of GNMax's data-dependent RDP at distances 0..num_teachers-1."""
    m = len(votes)
    lq0, lq1 = _logq0(sigma, order), _logq1(sigma, order, m)
    logq = core.compute_logq_gaussian(votes, sigma)
    res = np.full(num_teachers, _local_sens(lq1, sigma, m, order))
    if lq1 <= logq <= lq0:
        return res
    v = sorted(votes, reverse=True)
    res[0] = _local_sens(logq, sigma, m, order)
    d = 0
    left = logq > lq0  # otherwise logq < lq1: move right
    while (left and logq > lq0 and v[1] > 0) or (not left and logq < lq1):
        d += 1
        if left:  # make the top class stronger
            v[0] += 1
            v[1] -= 1
            i = 1
            while i < len(v) - 1 and v[i] < v[i + 1]:
                v[i], v[i + 1] = v[i + 1], v[i]
                i += 1
        else:
            v[0] -= 1
            v[1] += 1
        logq = core.compute_logq_gaussian(v, sigma)
        res[d] = _local_sens(logq, sigma, m, order)
    return res


@functools.lru_cache(maxsize=None)
def _rdp_threshold_table(num_teachers: int, threshold: float, sigma: float, order: float) -> tuple:
    return tuple(core.compute_rdp_threshold(float(scipy.stats.norm.logsf(threshold - v, scale=sigma)), sigma, order)
                 for v in range(num_teachers + 1))


def compute_local_sensitivity_bounds_threshold(counts, num_teachers: int, threshold: float, sigma: float,
                                               order: float) -> np.ndarray:
    rdp = _rdp_threshold_table(num_teachers, threshold, sigma, order)

    def ls_at(v):
        cands = []
        if v > 0:
            cands.append(abs(rdp[v - 1] - rdp[v]))
        if v < num_teachers:
            cands.append(abs(rdp[v + 1] - rdp[v]))
        return max(cands)

    cur = int(round(max(counts)))
    out = np.zeros(num_teachers)
    for d in range(max(cur, num_teachers - cur)):
        cands = []
        if cur + d <= num_teachers:
            cands.append(ls_at(cur + d))
        if cur - d >= 0:
            cands.append(ls_at(cur - d))
        out[d] = max(cands)
    return out


def compute_discounted_max(beta: float, a) -> float:
    a = np.asarray(a)
    return float(np.max(a * np.exp(-beta * np.arange(len(a)))))


def compute_smooth_sensitivity_gnmax(beta: float, counts, num_teachers: int, sigma: float, order: float) -> float:
    return compute_discounted_max(beta, compute_local_sensitivity_bounds_gnmax(counts, num_teachers, sigma, order))


def compute_rdp_of_smooth_sensitivity_gaussian(beta: float, sigma: float, order: float) -> float:
    """RDP of releasing smooth sensitivity with Gaussian noise (Theorem 23)."""
    if beta > 0 and not 1 < order < 1 / (2 * beta):
        raise ValueError("Order outside the (1, 1/(2*beta)) range.")
    return order * math.exp(2 * beta) / sigma ** 2 + (-0.5 * math.log(1 - 2 * order * beta) + beta * order) / (order - 1)


def compute_params_for_ss_release(eps: float, delta: float):
    a = scipy.special.ndtri(1 - delta / 2)
    return math.sqrt(a ** 2 + eps / 2) - a, eps / (2 * scipy.special.chdtri(1, delta / 2))


def _symbolic_beta(q, sigma, order):
    import sympy as sp

    mu2 = sigma * sp.sqrt(sp.log(1 / q))
    mu1 = mu2 + 1
    eps1, eps2 = mu1 / sigma ** 2, mu2 / sigma ** 2
    a = (1 - q) / (1 - (q * sp.exp(eps2)) ** (1 - 1 / mu2))
    b = sp.exp(eps1) / q ** (1 / (mu1 - 1))
    return (1 / (order - 1)) * sp.log((1 - q) * a ** (order - 1) + q * b ** (order - 1))


def _non_decreasing(fn, q, bounds) -> bool:
    import sympy as sp

    d = sp.lambdify(q, sp.diff(fn, q), modules=["numpy", {"erfc": scipy.special.erfc,
                                                          "erfcinv": scipy.special.erfcinv}])
    r = scipy.optimize.minimize_scalar(d, bounds=bounds, method="bounded")
    assert r.success
    return bool(r.fun >= 0)


def check_conditions(sigma: float, m: int, order: float):
    """(Condition 5, Condition 6) of the smooth-sensitivity analysis, checked symbolically."""
    import sympy as sp

    q = sp.symbols("q", positive=True, real=True)
    beta = _symbolic_beta(q, sigma, order)
    q0 = math.exp(compute_logq0_gnmax(sigma, order))
    c5 = _non_decreasing(beta, q, (0, q0))
    if not c5:
        return c5, False
    bu = (m - 1) / 2 * sp.erfc(sp.erfcinv(2 * q / (m - 1)) - 1 / sigma)
    c6 = _non_decreasing(beta.subs(q, bu) - beta, q, (0, _bl(q0, sigma, m)))
    return c5, c6
