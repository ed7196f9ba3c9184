"""Privacy analysis driver of "Scalable Private Learning with PATE" (ICLR 2018) — the Table 2
pipeline (reference `research/pate_2018/ICLR2018/smooth_sensitivity_table.py`,
`generate_table.sh`): for a matrix of teacher vote counts [queries, classes],

 1. accumulate the data-dependent RDP of Confident GNMax (threshold step with sigma1, GNMax step
    with sigma2, answered with probability Pr[max vote + N(0, sigma1^2) >= T]) over all orders,
    reporting E[answered], E[eps] and its std every 1000 queries, and pick the optimal order;
 2. if the analysis is not data-independent at that order, verify conditions C5/C6 symbolically
    and search the smooth-sensitivity parameters (beta, sigma_SS) minimising
    eps + cost(SS release) + 2 std (only for analysis: uses the sensitive votes).

Plain GNMax is analysed when `threshold`/`sigma1` are absent; interactive GNMax when a baseline
matrix is given. `generate_table` runs the paper's MNIST / SVHN / Adult rows on vote matrices
with those datasets' shapes (the reference downloads the real ones; offline they are synthesised
with a controllable teacher agreement)."""
from __future__ import annotations

import argparse
import math
import os

import numpy as np

from . import rdp2018 as pate
from . import smooth_sensitivity as pate_ss

DEFAULT_ORDERS = np.concatenate((np.arange(2, 100 + 1, .5), np.logspace(np.log10(100), np.log10(500), num=100)))

# (dataset, teachers, classes, threshold, sigma1, sigma2, queries, delta) -- generate_table.sh
TABLE2 = [("mnist", 250, 10, 200.0, 150.0, 40.0, 640, 1e-5),
          ("svhn", 250, 10, 300.0, 200.0, 40.0, 8500, 1e-6),
          ("adult", 250, 2, 300.0, 200.0, 40.0, 1500, 1e-5)]


def load_votes(counts_file: str, baseline_file: str | None = None, queries: int | None = None):
    votes = np.load(os.path.expanduser(counts_file), allow_pickle=False)
    baseline = np.load(os.path.expanduser(baseline_file), allow_pickle=False) if baseline_file else \
        np.zeros_like(votes)
    if votes.shape != baseline.shape:
        raise ValueError(f"counts and baseline shapes differ: {votes.shape} vs {baseline.shape}")
    if queries is not None:
        if votes.shape[0] < queries:
            raise ValueError(f"expected {queries} rows, got {votes.shape[0]} in {counts_file}")
        votes, baseline = votes[:queries], baseline[:queries]
    return votes, baseline


def count_teachers(votes: np.ndarray) -> int:
    s = votes.sum(axis=1)
    if s.min() != s.max():
        raise ValueError("malformed votes: the number of votes differs across rows")
    return int(s.max())


def synthetic_votes(queries: int, teachers: int, classes: int, agreement: float = 0.9, seed: int = 0) -> np.ndarray:
    """Vote histograms where each query's plurality class gets ~`agreement` of the teachers (varying
    per query, like real ensembles: most queries near-unanimous, a tail of contested ones)."""
    rng = np.random.default_rng(seed)
    out = np.zeros((queries, classes), dtype=np.int64)
    agree = np.clip(rng.beta(agreement * 20, (1 - agreement) * 20, size=queries), 1.0 / classes, 1.0)
    top = rng.integers(0, classes, size=queries)
    for i in range(queries):
        k = int(round(agree[i] * teachers))
        out[i, top[i]] = k
        rest = rng.multinomial(teachers - k, np.full(classes, 1.0 / classes))
        out[i] += rest
    return out


def compute_rdp(votes, baseline, threshold, sigma1, sigma2, delta, orders=DEFAULT_ORDERS, data_ind=False,
                log=print, every: int = 1000) -> dict:
    orders = np.asarray(orders, dtype=float)
    rdp_cum = np.zeros(len(orders))
    rdp_sqrd_cum = np.zeros(len(orders))
    answered = 0.0
    rows = []
    for i, v in enumerate(votes):
        if threshold is None:
            logq1, rdp1 = 0.0, np.zeros(len(orders))
        else:
            logq1 = pate.compute_logpr_answered(threshold, sigma1, v - baseline[i])
            rdp1 = (pate.compute_rdp_data_independent_threshold(sigma1, orders) if data_ind
                    else pate.compute_rdp_threshold(logq1, sigma1, orders))
        rdp2 = (pate.rdp_data_independent_gaussian(sigma2, orders) if data_ind
                else pate.rdp_gaussian(pate.compute_logq_gaussian(v, sigma2), sigma2, orders))
        q1 = math.exp(logq1)
        rdp_cum += rdp1 + rdp2 * q1
        rdp_sqrd_cum += rdp1 ** 2 + 2 * rdp1 * q1 * rdp2 + q1 * rdp2 ** 2  # E[(c1 + Bern(q1) c2)^2]
        answered += q1
        if (i + 1) % every == 0 or i == len(votes) - 1:
            n = max(i, 1)
            var = rdp_sqrd_cum / n - (rdp_cum / n) ** 2
            eps, order_opt = pate.compute_eps_from_delta(orders, rdp_cum, delta)
            idx = min(int(np.searchsorted(orders, order_opt)), len(orders) - 1)
            row = {"queries": i + 1, "answered": answered, "eps": float(eps),
                   "eps_std": float(((i + 1) * max(var[idx], 0.0)) ** .5), "order": float(order_opt),
                   "delta_contribution": -math.log(delta) / (order_opt - 1)}
            rows.append(row)
            if log:
                log("queries = {queries}, E[answered] = {answered:.2f}, E[eps] = {eps:.3f} (std = {eps_std:.5f}) "
                    "at order = {order:.2f} (contribution from delta = {delta_contribution:.3f})".format(**row))
    eps, order_opt = pate.compute_eps_from_delta(orders, rdp_cum, delta)
    return {"order": float(order_opt), "eps": float(eps), "answered": answered, "rows": rows}


def is_data_ind_step1(num_teachers, threshold, sigma1, orders) -> bool:
    return threshold is None or bool(np.all(pate.is_data_independent_always_opt_threshold(
        num_teachers, threshold, sigma1, np.atleast_1d(orders))))


def is_data_ind_step2(num_teachers, num_classes, sigma, orders) -> bool:
    return bool(np.all(pate.is_data_independent_always_opt_gaussian(num_teachers, num_classes, sigma,
                                                                     np.atleast_1d(orders))))


def find_optimal_smooth_sensitivity_parameters(votes, baseline, num_teachers, threshold, sigma1, sigma2, delta,
                                               ind_step1, ind_step2, order, log=print, every: int = 100) -> dict:
    rdp_cum = answered_cum = 0.0
    ls_cum = 0.0
    betas = np.arange(.3 / order, .495 / order, .01 / order)
    cost_delta = math.log(1 / delta) / (order - 1)
    best = {}
    for i, v in enumerate(votes):
        if threshold is None:
            logpr, rdp1, ls1 = 0.0, 0.0, np.zeros(num_teachers)
        else:
            logpr = pate.compute_logpr_answered(threshold, sigma1, v - baseline[i])
            if ind_step1:
                rdp1, ls1 = float(pate.compute_rdp_data_independent_threshold(sigma1, order)), np.zeros(num_teachers)
            else:
                rdp1 = float(pate.compute_rdp_threshold(logpr, sigma1, order))
                ls1 = pate_ss.compute_local_sensitivity_bounds_threshold(v - baseline[i], num_teachers, threshold,
                                                                         sigma1, order)
        pr = math.exp(logpr)
        answered_cum += pr
        if ind_step2:
            rdp2, ls2 = float(pate.rdp_data_independent_gaussian(sigma2, order)), np.zeros(num_teachers)
        else:
            rdp2 = float(pate.rdp_gaussian(pate.compute_logq_gaussian(v, sigma2), sigma2, order))
            ls2 = pate_ss.compute_local_sensitivity_bounds_gnmax(v, num_teachers, sigma2, order)
        rdp_cum += rdp1 + pr * rdp2
        ls_cum = ls_cum + ls1 + pr * ls2
        if ind_step1 and ind_step2:
            cost_opt, beta_opt, ss_opt, sigma_ss_opt = None, 0.0, 0.0, np.inf
        else:
            cost_opt, beta_opt, ss_opt, sigma_ss_opt = np.inf, None, None, None
            for beta in betas:
                ss = pate_ss.compute_discounted_max(beta, ls_cum)
                sigma_ss = ((order * math.exp(2 * beta)) / ss) ** (1 / 3)  # argmin order e^{2b}/s^2 + 2 ss s
                cost = rdp_cum + pate_ss.compute_rdp_of_smooth_sensitivity_gaussian(beta, sigma_ss, order) + \
                    2 * ss * sigma_ss
                if cost < cost_opt:
                    cost_opt, beta_opt, ss_opt, sigma_ss_opt = cost, beta, ss, sigma_ss
        if (i + 1) % every == 0 or i == len(votes) - 1:
            eps_before = rdp_cum + cost_delta
            eps_with = eps_before + pate_ss.compute_rdp_of_smooth_sensitivity_gaussian(beta_opt, sigma_ss_opt, order)
            best = {"queries": i + 1, "answered": answered_cum, "eps_before_ss": eps_before, "eps_with_ss": eps_with,
                    "noise_std": ss_opt * sigma_ss_opt, "ss": ss_opt, "beta": beta_opt, "sigma_ss": sigma_ss_opt}
            if log:
                log("{queries}: E[answered queries] = {answered:.1f}, RDP goes from {eps_before_ss:.3f} to "
                    "{eps_with_ss:.3f} +/- {noise_std:.3f} (ss = {ss:.4}, beta = {beta:.4f}, sigma_ss = {sigma_ss:.3f})"
                    .format(**best))
    return best


def analyze(votes, baseline=None, threshold=None, sigma1=None, sigma2=None, delta=1e-8, order=None, teachers=None,
            data_independent=False, check_conditions=True, log=print) -> dict:
    if (threshold is None) != (sigma1 is None):
        raise ValueError("threshold and sigma1 must be given together")
    baseline = np.zeros_like(votes) if baseline is None else baseline
    orders = DEFAULT_ORDERS if order is None else np.array([order], float)
    num_teachers = teachers or count_teachers(votes)
    res = compute_rdp(votes, baseline, threshold, sigma1, sigma2, delta, orders, data_independent, log)
    o = res["order"]
    ind1 = is_data_ind_step1(num_teachers, threshold, sigma1, o)
    ind2 = is_data_ind_step2(num_teachers, votes.shape[1], sigma2, o)
    res["data_independent"] = bool(data_independent or (ind1 and ind2))
    if res["data_independent"]:
        if log:
            log("Nothing to do here, all analyses are data-independent.")
        return res
    if check_conditions:
        c5, c6 = pate_ss.check_conditions(sigma2, votes.shape[1], o)
        res["conditions_hold"] = bool(c5 and c6)
        if not res["conditions_hold"]:
            if log:
                log(f"Condition {'C5' if not c5 else 'C6'} does not hold for order = {o}")
            return res
    res["smooth_sensitivity"] = find_optimal_smooth_sensitivity_parameters(
        votes, baseline, num_teachers, threshold, sigma1, sigma2, delta, ind1, ind2, o, log)
    ss = res["smooth_sensitivity"]
    if log:
        log(f"Optimal beta = {ss['beta']:.4f}, E[SS_beta] = {ss['ss']:.4}, sigma_ss = {ss['sigma_ss']:.2f}")
    return res


def generate_table(rows=TABLE2, agreement: float = 0.93, seed: int = 0, log=print) -> list[dict]:
    out = []
    for name, teachers, classes, t, s1, s2, q, delta in rows:
        if log:
            log(f"\n######## {name.upper()} ########")
        votes = synthetic_votes(q, teachers, classes, agreement, seed)
        r = analyze(votes, None, t, s1, s2, delta, log=log)
        out.append({"dataset": name, "queries": q, "answered": r["answered"], "eps": r["eps"], "order": r["order"],
                    "eps_with_ss": (r.get("smooth_sensitivity") or {}).get("eps_with_ss")})
    return out


def main(argv=None):
    ap = argparse.ArgumentParser(prog="python -m mifx.privacy.pate.iclr2018")
    ap.add_argument("--counts_file")
    ap.add_argument("--baseline_file")
    ap.add_argument("--data_independent", action="store_true")
    ap.add_argument("--threshold", type=float)
    ap.add_argument("--sigma1", type=float)
    ap.add_argument("--sigma2", type=float)
    ap.add_argument("--queries", type=int)
    ap.add_argument("--delta", type=float, default=1e-8)
    ap.add_argument("--order", type=float)
    ap.add_argument("--teachers", type=int)
    ap.add_argument("--table", action="store_true", help="reproduce Table 2 rows on synthetic vote matrices")
    a = ap.parse_args(argv)
    if a.table:
        return generate_table()
    if not a.counts_file or a.sigma2 is None:
        ap.error("--counts_file and --sigma2 are required (or --table)")
    votes, baseline = load_votes(a.counts_file, a.baseline_file, a.queries)
    return analyze(votes, baseline, a.threshold, a.sigma1, a.sigma2, a.delta, a.order, a.teachers, a.data_independent)


if __name__ == "__main__":
    main()
