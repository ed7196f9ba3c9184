"""Smooth sensitivity of the PATE-2018 data-dependent privacy cost (GNMax and the threshold check).

Papernot et al., "Scalable Private Learning with PATE" (ICLR 2018), Appendix B-C. Releasing a DATA-DEPENDENT
RDP cost leaks the votes, so the paper releases it with noise scaled to a beta-smooth upper bound on its local
sensitivity, SS_beta = max_d e^{-beta d} LS(d), where LS(d) bounds how much the cost can change between any two
neighbouring vote histograms at distance d from the actual one.

GNMax (Gaussian noisy max, noise sigma, m classes). With q = Pr[answer != plurality] (bounded from the votes),
the data-dependent RDP at order lambda (Prop. 10) is
    beta(q) = log((1-q) A^{lambda-1} + q B^{lambda-1}) / (lambda - 1),
    mu2 = sigma sqrt(log 1/q), mu1 = mu2 + 1, eps_i = mu_i / sigma^2,
    A = (1-q) / (1 - (q e^{eps2})^{1 - 1/mu2}),  B = e^{eps1} / q^{1/(mu1-1)},
valid (and better than the data-independent lambda / sigma^2) for q below a threshold q0 (found here by root
finding where the two bounds meet). One teacher changing its vote moves q inside [B_l(q), B_u(q)] with
    B_{l,u}(q) = (m-1)/2 erfc(erfc^{-1}(2q / (m-1)) +- 1/sigma),
so LS at the current histogram is max(beta(B_u(q)) - beta(q), beta(q) - beta(B_l(q))). Because beta is
non-decreasing in q below q0 (Condition 5, checked symbolically by check_conditions), the cost is flat above q0
and LS is constant once q is pushed into [q1, q0] (q1 = B_l(q0)). LS(d) follows the histogram as d votes move:
from the plurality to the runner-up while q < q1 ("right", q grows), or towards the plurality while q > q0 ("left").

Threshold check (Gaussian noise sigma on the plurality count v vs a threshold T): the RDP of the check is a
function of v alone (rdp2018.compute_rdp_threshold of log Pr[v + N(0, sigma^2) >= T]); LS at distance d is the
largest one-vote change of that table at the vote counts d away from the current plurality.

Reference: `research/pate_2018/smooth_sensitivity.py:43-412`; its numeric goldens are pinned in
tests/test_privacy.py (`smooth_sensitivity_test.py:28-126`)."""
from __future__ import annotations

import functools
import math
from dataclasses import dataclass

import numpy as np
import scipy.optimize
import scipy.special
import scipy.stats

from . import rdp2018 as core


# ------------------------------------------------------------------------------------------- GNMax
@dataclass(frozen=True)
class GNMaxCost:
    """The data-dependent RDP of one GNMax answer as a function of log q, at noise sigma and order lambda."""

    sigma: float
    order: float

    def _mu(self, logq: float) -> tuple[float, float]:
        mu2 = self.sigma * math.sqrt(-logq)
        return mu2 + 1.0, mu2

    def dependent(self, logq: float) -> float:
        """Prop. 10's bound, evaluated in log space (log1p for the 1 - q factors)."""
        lam, var = self.order, self.sigma ** 2
        mu1, mu2 = self._mu(logq)
        eps1, eps2 = mu1 / var, mu2 / var
        log_1mq = math.log1p(-math.exp(logq))
        log_a = (lam - 1) * (log_1mq - math.log1p(-math.exp((logq + eps2) * (1 - 1 / mu2))))
        log_b = (lam - 1) * (eps1 - logq / (mu1 - 1))
        return float(np.logaddexp(log_1mq + log_a, logq + log_b)) / (lam - 1)

    def independent(self) -> float:
        return core.rdp_data_independent_gaussian(self.sigma, self.order)

    def _valid(self, logq: float) -> bool:
        """Prop. 10's preconditions: mu1 >= lambda and q <= e^{(mu2-1) eps2} / (mu1/(mu1-1) mu2/(mu2-1))^{mu2}."""
        mu1, mu2 = self._mu(logq)
        if mu1 < self.order:
            return False
        eps2 = mu2 / self.sigma ** 2
        return logq <= (mu2 - 1) * eps2 - mu2 * math.log(mu1 / (mu1 - 1) * mu2 / (mu2 - 1))

    @functools.cached_property
    def logq0(self) -> float:
        """log q0: where the data-dependent bound rises to the data-independent one (the cost is flat above)."""
        s, lam = self.sigma, self.order
        # the largest logq that meets the preconditions with margin: mu2 > 1 and mu2 >= lambda - 0.99,
        # and mu2 >= 1 + sigma (so that the (mu2 - 1) eps2 term of the validity test is positive)
        top = -max((1 + 1 / s) ** 2, ((lam - 0.99) / s) ** 2, 1 / s ** 2)
        if not self._valid(top):
            raise AssertionError("GNMax bound not valid at the search start")

        def excess(lq):
            return self.dependent(lq) - self.independent()

        if excess(top) < 0:  # still below the data-independent cost at the validity edge
            return top
        bottom = 2 * top
        while excess(bottom) > 0:  # geometric search down for a sign change
            if bottom <= -10000:
                raise AssertionError("no sign change of the bound excess above log q = -10000")
            bottom *= 1.5
        root, res = scipy.optimize.brentq(excess, bottom, top, full_output=True)
        if not (res.converged and self._valid(root)):
            raise AssertionError("q0 root finding failed")
        return root

    def rdp(self, logq: float) -> float:
        return self.independent() if logq >= self.logq0 else self.dependent(logq)


def _q_bound(q: float, sigma: float, m: int, sign: float) -> float:
    return (m - 1) / 2 * scipy.special.erfc(scipy.special.erfcinv(2 * q / (m - 1)) + sign / sigma)


def q_lower(q: float, sigma: float, m: int) -> float:
    """B_l: the smallest q of a histogram one vote away."""
    return _q_bound(q, sigma, m, 1.0)


def q_upper(q: float, sigma: float, m: int) -> float:
    """B_u: the largest q of a histogram one vote away (a probability: at most 1)."""
    return min(1.0, _q_bound(q, sigma, m, -1.0))


@functools.lru_cache(maxsize=None)
def gnmax_cost(sigma: float, order: float) -> GNMaxCost:
    return GNMaxCost(float(sigma), float(order))


@functools.lru_cache(maxsize=None)
def gnmax_logq1(sigma: float, order: float, m: int) -> float:
    """log q1 = log B_l(q0): from q1 upward one vote can reach the flat region."""
    lq0 = gnmax_cost(sigma, order).logq0
    lq1 = math.log(q_lower(math.exp(lq0), sigma, m))
    if lq1 > lq0:
        raise AssertionError("q1 above q0")
    return lq1


def compute_logq0_gnmax(sigma: float, order: float) -> float:
    return gnmax_cost(sigma, order).logq0


def gnmax_local_sensitivity(logq: float, sigma: float, m: int, order: float) -> float:
    """LS of GNMax's data-dependent RDP at a histogram with log q = logq (inside [q1, q0] the worst case q1)."""
    cost = gnmax_cost(sigma, order)
    lq1 = gnmax_logq1(sigma, order, m)
    if lq1 <= logq <= cost.logq0:
        logq = lq1
    q = math.exp(logq)
    here = cost.rdp(logq)
    return max(cost.rdp(math.log(q_upper(q, sigma, m))) - here, here - cost.rdp(math.log(q_lower(q, sigma, m))))


def _gnmax_walk(votes, sigma: float, lq0: float, lq1: float):
    """log q of the histograms the worst-case walk visits at distances 1, 2, ...: votes move from the plurality to
    the runner-up while q < q1, or from the runner-up (kept the largest non-plurality count) to the plurality while
    q > q0; stops once q enters [q1, q0] (or the runner-up runs out of votes)."""
    v = sorted(votes, reverse=True)
    logq = core.compute_logq_gaussian(v, sigma)
    left = logq > lq0
    while (logq > lq0 and v[1] > 0) if left else (logq < lq1):
        if left:
            v[0] += 1
            v[1] -= 1
            j = 1  # restore the decreasing order of the non-plurality counts
            while j + 1 < len(v) and v[j] < v[j + 1]:
                v[j], v[j + 1] = v[j + 1], v[j]
                j += 1
        else:
            v[0] -= 1
            v[1] += 1
        logq = core.compute_logq_gaussian(v, sigma)
        yield logq


def compute_local_sensitivity_bounds_gnmax(votes, num_teachers: int, sigma: float, order: float) -> np.ndarray:
    """LS(d) of GNMax's data-dependent RDP for d = 0 .. num_teachers - 1."""
    m = len(votes)
    cost = gnmax_cost(sigma, order)
    lq0, lq1 = cost.logq0, gnmax_logq1(sigma, order, m)
    plateau = gnmax_local_sensitivity(lq1, sigma, m, order)
    out = np.full(num_teachers, plateau)
    logq = core.compute_logq_gaussian(votes, sigma)
    if lq1 <= logq <= lq0:
        return out
    out[0] = gnmax_local_sensitivity(logq, sigma, m, order)
    for d, lq in enumerate(_gnmax_walk(votes, sigma, lq0, lq1), start=1):
        out[d] = gnmax_local_sensitivity(lq, sigma, m, order)
    return out


# --------------------------------------------------------------------------------- threshold check
@functools.lru_cache(maxsize=None)
def _threshold_cost_table(num_teachers: int, threshold: float, sigma: float, order: float) -> np.ndarray:
    """RDP of the threshold check for every plurality count v = 0 .. num_teachers."""
    v = np.arange(num_teachers + 1)
    logpr = scipy.stats.norm.logsf(threshold - v, scale=sigma)
    return np.array([core.compute_rdp_threshold(float(lp), sigma, order) for lp in logpr])


def compute_local_sensitivity_bounds_threshold(counts, num_teachers: int, threshold: float, sigma: float,
                                               order: float) -> np.ndarray:
    """LS(d) of the threshold check's RDP: the largest one-vote change of the cost table at the plurality counts
    d away from the current (rounded) plurality, for d = 0 .. num_teachers - 1."""
    table = _threshold_cost_table(num_teachers, threshold, sigma, order)
    step = np.abs(np.diff(table))  # step[v] = |cost(v + 1) - cost(v)|
    # one-vote sensitivity at each count: the larger of its two steps (one step at the ends)
    at = np.zeros(num_teachers + 1)
    at[:-1] = step
    at[1:] = np.maximum(at[1:], step)
    cur = int(round(max(counts)))
    out = np.zeros(num_teachers)
    for d in range(max(cur, num_teachers - cur)):
        reach = [v for v in (cur + d, cur - d) if 0 <= v <= num_teachers]
        out[d] = max(at[v] for v in reach)
    return out


# ------------------------------------------------------------------------------- smooth sensitivity
def compute_discounted_max(beta: float, a) -> float:
    """max_d e^{-beta d} a[d]."""
    a = np.asarray(a)
    return float(np.max(a * np.exp(-beta * np.arange(len(a)))))


def compute_smooth_sensitivity_gnmax(beta: float, counts, num_teachers: int, sigma: float, order: float) -> float:
    return compute_discounted_max(beta, compute_local_sensitivity_bounds_gnmax(counts, num_teachers, sigma, order))


def compute_rdp_of_smooth_sensitivity_gaussian(beta: float, sigma: float, order: float) -> float:
    """RDP at `order` of releasing the cost plus Gaussian noise scaled by its beta-smooth sensitivity (Thm. 23):
    order e^{2 beta} / sigma^2 + (beta order - log(1 - 2 order beta) / 2) / (order - 1), for 1 < order < 1/(2 beta)."""
    if beta > 0 and not 1 < order < 1 / (2 * beta):
        raise ValueError("Order outside the (1, 1/(2*beta)) range.")
    return order * math.exp(2 * beta) / sigma ** 2 + (beta * order - 0.5 * math.log(1 - 2 * order * beta)) / (order - 1)


def compute_params_for_ss_release(eps: float, delta: float):
    """(beta, sigma multiplier) for an (eps, delta) smooth-sensitivity release (the paper's Gaussian recipe)."""
    a = scipy.special.ndtri(1 - delta / 2)
    return math.sqrt(a ** 2 + eps / 2) - a, eps / (2 * scipy.special.chdtri(1, delta / 2))


# ------------------------------------------------------------------------------ symbolic conditions
def _beta_expr(q, sigma: float, order: float):
    """Prop. 10's bound as a sympy expression of q (same formula as GNMaxCost.dependent)."""
    import sympy as sp

    mu2 = sigma * sp.sqrt(sp.log(1 / q))
    mu1 = mu2 + 1
    eps1, eps2 = mu1 / sigma ** 2, mu2 / sigma ** 2
    a = (1 - q) / (1 - (q * sp.exp(eps2)) ** (1 - 1 / mu2))
    b = sp.exp(eps1) / q ** (1 / (mu1 - 1))
    return sp.log((1 - q) * a ** (order - 1) + q * b ** (order - 1)) / (order - 1)


def _derivative_nonnegative(expr, q, interval) -> bool:
    """min over the interval of d expr / dq >= 0 (numeric minimisation of the symbolic derivative)."""
    import sympy as sp

    f = sp.lambdify(q, sp.diff(expr, q),
                    modules=["numpy", {"erfc": scipy.special.erfc, "erfcinv": scipy.special.erfcinv}])
    r = scipy.optimize.minimize_scalar(f, bounds=interval, method="bounded")
    if not r.success:
        raise RuntimeError("derivative minimisation failed")
    return bool(r.fun >= 0)


def check_conditions(sigma: float, m: int, order: float):
    """(Condition 5: beta non-decreasing on (0, q0); Condition 6: beta(B_u(q)) - beta(q) non-decreasing on
    (0, q1)) for GNMax with m classes. Condition 6 is only checked when 5 holds."""
    import sympy as sp

    q = sp.symbols("q", positive=True, real=True)
    beta = _beta_expr(q, sigma, order)
    q0 = math.exp(compute_logq0_gnmax(sigma, order))
    if not _derivative_nonnegative(beta, q, (0, q0)):
        return False, False
    bu = (m - 1) / 2 * sp.erfc(sp.erfcinv(2 * q / (m - 1)) - 1 / sigma)
    return True, _derivative_nonnegative(beta.subs(q, bu) - beta, q, (0, q_lower(q0, sigma, m)))


# names the ICLR'18 scripts use
def rdp_gnmax(sigma: float, logq: float, order: float) -> float:
    return gnmax_cost(sigma, order).rdp(logq)
