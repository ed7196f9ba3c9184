"""Analyses behind the ICLR-2018 PATE figures ("Scalable Private Learning with PATE").

Reference scripts: `research/pate_2018/ICLR2018/rdp_cumulative.py` (privacy cost per answered query, budget
partition over the run), `rdp_bucketized.py` (answers and cost by teacher-agreement bucket), `plot_ls_q.py`
(local sensitivity of the GNMax RDP bound as a function of q), `plot_partition.py` (where the budget goes:
selection / answering / delta), `utility_queries_answered.py:33-54` (the paper's student accuracy vs queries
answered, hard-coded data). The reference reads a vote-count file produced by teacher ensembles it downloads;
there is no network here, so the CLI analyses either a votes file (`.npy`, no pickles) or synthetic votes
(`iclr2018.synthetic_votes`) and says which in its output.

Design differences: the per-query RDP curves are stacked into one [queries, orders] array and the cumulative
epsilon of every prefix comes from one cumsum + row-wise minimum over orders (the reference re-derives eps
query by query); plotting is optional (matplotlib, Agg backend) and every figure's numbers are also written as
JSON."""
from __future__ import annotations

import argparse
import json
import math
import os

import numpy as np

from . import rdp2018 as core
from . import smooth_sensitivity as ss

# the long order list of the reference's cumulative analysis
ORDERS = np.concatenate((np.arange(2, 100 + 1, 0.5), np.logspace(np.log10(100), np.log10(500), num=100)))

# Paper data (`utility_queries_answered.py:33-54`): student test accuracy (%) after a given number of answered
# queries, MNIST-scale SVHN run of the paper, for LNMax and Confident-GNMax (and the aggressive variant).
UTILITY_QUERIES_ANSWERED = {
    "lnmax": {"answered": [500, 750] + list(range(1000, 12500, 500)),
              "accuracy": [43.3, 52.3, 59.8, 66.7, 68.8, 70.5, 71.6, 72.3, 72.6, 72.9, 73.4, 73.4, 73.7, 73.9,
                           74.2, 74.4, 74.5, 74.7, 74.8, 75, 75.1, 75.1, 75.4, 75.4, 75.4]},
    "gnmax_conf": {"answered": [456, 683, 908, 1353, 1818, 2260, 2702, 3153, 3602, 4055, 4511, 4964, 5422, 5875,
                                6332, 6792, 7244, 7696, 8146, 8599, 9041, 9496, 9945, 10390, 10842],
                   "accuracy": [39.6, 52.2, 59.6, 66.6, 69.6, 70.5, 71.8, 72, 72.7, 72.9, 73.3, 73.4, 73.4, 73.8,
                                74, 74.2, 74.4, 74.5, 74.5, 74.7, 74.8, 75, 75.1, 75.1, 75.4]},
    "gnmax_conf_aggressive": {"answered": [167, 258, 322, 485, 647, 800, 967, 1133, 1282, 1430, 1573, 1728, 1889,
                                           2028, 2190, 2348, 2510, 2668, 2950, 3098, 3265, 3413, 3581, 3730],
                              "accuracy": [17.8, 26.8, 39.3, 48, 55.7, 61, 62.8, 64.8, 65.4, 66.7, 66.2, 68.3, 68.3,
                                           68.7, 69.1, 70, 70.2, 70.5, 70.9, 70.7, 71.3, 71.3, 71.3, 71.8]},
}


def per_query_rdp(votes: np.ndarray, mechanism: str, noise_scale: float, threshold: float | None = None,
                  sigma1: float | None = None, orders=ORDERS) -> dict:
    """RDP curves of every query: {"rdp": [n, len(orders)] expected cost, "rdp_select": selection-step part
    (Confident-GNMax), "rdp_sqrd": E[cost^2] (for the std of the sum), "pr_answered": [n]}.

    lnmax: LNMax, pure-eps Laplace noise of scale noise_scale (eps 2 / scale) with the data-dependent logq;
    gnmax: GNMax with sigma = noise_scale (Theorem 6 bound);
    gnmax_conf: Confident-GNMax -- threshold check with N(0, sigma1^2) (its RDP is paid by every query) and,
    with probability Pr[answered], the GNMax answer."""
    votes = np.asarray(votes)
    n, k = votes.shape[0], len(orders)
    rdp, sq, sel = np.zeros((n, k)), np.zeros((n, k)), np.zeros((n, k))
    pr = np.ones(n)
    for i, v in enumerate(votes):
        if mechanism == "lnmax":
            r = core.rdp_pure_eps(core.compute_logq_laplace(v, noise_scale), 2.0 / noise_scale, orders)
            rdp[i], sq[i] = r, r * r
        elif mechanism == "gnmax":
            r = core.rdp_gaussian(core.compute_logq_gaussian(v, noise_scale), noise_scale, orders)
            rdp[i], sq[i] = r, r * r
        elif mechanism == "gnmax_conf":
            if threshold is None or sigma1 is None:
                raise ValueError("gnmax_conf needs threshold and sigma1")
            lp = core.compute_logpr_answered(threshold, sigma1, v)
            q1 = math.exp(lp)
            s1 = core.rdp_gaussian(min(lp, math.log1p(-q1)) if q1 < 1 else -math.inf, 2 ** 0.5 * sigma1, orders)
            s2 = core.rdp_gaussian(core.compute_logq_gaussian(v, noise_scale), noise_scale, orders)
            rdp[i] = s1 + q1 * s2
            sq[i] = s1 * s1 + 2 * s1 * q1 * s2 + q1 * s2 * s2  # E[(c1 + Bernoulli(q1) c2)^2]
            sel[i] = s1
            pr[i] = q1
        else:
            raise ValueError('mechanism must be one of "lnmax", "gnmax", "gnmax_conf"')
    return {"rdp": rdp, "rdp_sqrd": sq, "rdp_select": sel, "pr_answered": pr}


def cumulative_privacy(votes, mechanism: str, noise_scale: float, threshold=None, sigma1=None, delta: float = 1e-8,
                       orders=ORDERS) -> dict:
    """`rdp_cumulative.py` run_analysis: for every prefix of the query stream the (eps, delta) cost at the best
    order, the expected number of answered queries, and the budget partition [selection, answering, delta]
    (or [answering, delta]) as fractions of eps."""
    orders = np.asarray(orders, dtype=np.float64)
    q = per_query_rdp(votes, mechanism, noise_scale, threshold, sigma1, orders)
    cum = np.cumsum(q["rdp"], axis=0)
    eps_all = cum - math.log(delta) / (orders - 1)
    best = np.argmin(eps_all, axis=1)
    rows = np.arange(cum.shape[0])
    eps = eps_all[rows, best]
    order_opt = orders[best]
    dterm = -math.log(delta) / (order_opt - 1)
    if mechanism == "gnmax_conf":
        sel = np.cumsum(q["rdp_select"], axis=0)[rows, best]
        partition = np.stack([sel, cum[rows, best] - sel, dterm], 1) / eps[:, None]
    else:
        partition = np.stack([cum[rows, best], dterm], 1) / eps[:, None]
    answered = np.cumsum(q["pr_answered"])
    # std of the total cost at the optimal order (variance of the per-query costs, as the reference)
    i = np.maximum(rows, 1)
    var = np.cumsum(q["rdp_sqrd"], axis=0)[rows, best] / i - (cum[rows, best] / i) ** 2
    eps_std = np.sqrt(np.maximum((rows + 1) * var, 0.0))
    return {"eps": eps, "order_opt": order_opt, "answered": answered, "partition": partition, "eps_std": eps_std}


def agreement_bins(votes, bin_num: int) -> np.ndarray:
    """Bucket index of every query by the share of the plurality vote: floor(max(v) * bins / sum(v))."""
    v = np.asarray(votes, dtype=np.float64)
    b = np.floor(v.max(1) * bin_num / v.sum(1)).astype(np.int64)
    if (b < 0).any() or (b >= bin_num).any():  # unanimous queries land in the last bucket
        b = np.minimum(b, bin_num - 1)
    return b


def bucketized(votes, bin_num: int, threshold: float, sigma1: float, sigma2: float | None = None,
               order: float | None = None) -> dict:
    """`rdp_bucketized.py`: per agreement bucket, the number of queries, the expected number answered by the
    threshold check (Confident-GNMax), and (optionally) the mean RDP at `order` of GNMax(sigma2) answers."""
    v = np.asarray(votes)
    b = agreement_bins(v, bin_num)
    counts = np.bincount(b, minlength=bin_num).astype(np.float64)
    pr = np.array([math.exp(core.compute_logpr_answered(threshold, sigma1, x)) for x in v])
    out = {"bins": np.linspace(0, 100, num=bin_num, endpoint=False), "counts": counts,
           "expected_answered": np.bincount(b, weights=pr, minlength=bin_num)}
    if sigma2 is not None and order is not None:
        r = np.array([core.rdp_gaussian(core.compute_logq_gaussian(x, sigma2), sigma2, float(order)) for x in v])
        with np.errstate(invalid="ignore", divide="ignore"):
            out["mean_rdp"] = np.bincount(b, weights=r, minlength=bin_num) / counts
    return out


def ls_of_q(sigma: float = 20.0, order: float = 20.0, num_classes: int = 10, num: int = 1000) -> dict:
    """`plot_ls_q.py`: the local sensitivity (upward change beta(bu(q)) - beta(q)) of GNMax's data-dependent RDP
    bound as a function of q in [0, 0.1], with the q0 / q1 landmarks of the smooth-sensitivity analysis."""
    def beta(q):
        return ss.rdp_gnmax(sigma, math.log(q), order)

    def delta_beta(q):
        if q == 0 or q > 0.8:
            return 0.0
        bq, bu, bl = beta(q), beta(ss.q_upper(q, sigma, num_classes)), beta(ss.q_lower(q, sigma, num_classes))
        assert bl <= bq <= bu
        return bu - bq

    xs = np.linspace(0, 0.1, num=num, endpoint=True)
    return {"q": xs, "ls": np.array([delta_beta(x) for x in xs]),
            "q0": math.exp(ss.compute_logq0_gnmax(sigma, order)), "q1": math.exp(ss.gnmax_logq1(sigma, order, num_classes))}


def _plots(figdir: str, res: dict) -> list[str]:
    try:
        import matplotlib

        matplotlib.use("Agg")
        import matplotlib.pyplot as plt
    except ImportError:
        return []
    out = []

    def save(fig, name):
        p = os.path.join(figdir, name)
        fig.savefig(p, bbox_inches="tight")
        plt.close(fig)
        out.append(p)

    fig, ax = plt.subplots(figsize=(5, 4.7))
    for m, c in (("lnmax", "r"), ("gnmax", "b"), ("gnmax_conf", "g")):
        if m in res["cumulative"]:
            r = res["cumulative"][m]
            ax.plot(r["answered"], r["eps"], color=c, label=m)
    ax.set_xlabel("Number of queries answered")
    ax.set_ylabel(r"Privacy cost $\varepsilon$ at $\delta=10^{-8}$")
    ax.legend()
    save(fig, "cumulative_eps.pdf")
    if "gnmax_conf" in res["cumulative"]:
        p = np.asarray(res["cumulative"]["gnmax_conf"]["partition"])
        fig, ax = plt.subplots(figsize=(5, 4.7))
        ax.stackplot(np.arange(1, len(p) + 1), p.T, labels=["selection", "answering", "delta"])
        ax.set_xlabel("Number of queries")
        ax.set_ylabel("Share of the privacy budget")
        ax.legend(loc="upper right")
        save(fig, "partition.pdf")
    b = res["bucketized"]
    fig, ax = plt.subplots(figsize=(5, 5))
    w = 100 / len(b["bins"])
    ax.bar(b["bins"], b["counts"], w, fill=False, edgecolor="red", linestyle="dotted", align="edge", label="LNMax answers")
    ax.bar(b["bins"], b["expected_answered"], w, color="g", alpha=0.5, align="edge", label="Confident-GNMax answers")
    ax.set_xlabel("Percentage of teachers that agree")
    ax.set_ylabel("Number of queries answered")
    ax.legend(loc=2)
    save(fig, "bucketized.pdf")
    ls = res["ls_of_q"]
    fig, ax = plt.subplots(figsize=(4.7, 4.5))
    ax.plot(ls["q"], ls["ls"], linewidth=3)
    ax.set_xlabel("q")
    ax.set_ylabel("local sensitivity of the RDP bound")
    save(fig, "ls_of_q.pdf")
    u = UTILITY_QUERIES_ANSWERED
    fig, ax = plt.subplots(figsize=(5, 4.7))
    ax.plot(u["lnmax"]["answered"], u["lnmax"]["accuracy"], "r--o", alpha=0.5, label="LNMax")
    ax.plot(u["gnmax_conf"]["answered"], u["gnmax_conf"]["accuracy"], "g-o", alpha=0.5, label="Confident-GNMax")
    ax.set_xlim(0, 6000)
    ax.set_ylim(65, 76)
    ax.set_xlabel("Number of queries answered")
    ax.set_ylabel("Student test accuracy (%)")
    ax.legend(loc=2)
    save(fig, "utility_queries_answered.pdf")
    return out


def main(argv=None) -> int:
    """MNIST settings of the paper's figures: LNMax scale 50, GNMax sigma 40, Confident-GNMax T=200 sigma1=150
    sigma2=40 (generate_table.sh); bucketized with T=3500 sigma1=1500 on 5000-teacher votes when given."""
    from .iclr2018 import load_votes, synthetic_votes

    ap = argparse.ArgumentParser(prog="python -m mifx.privacy.pate.iclr2018_figures")
    ap.add_argument("--counts-file", default=None, help=".npy votes [queries, classes] (allow_pickle=False)")
    ap.add_argument("--queries", type=int, default=2000)
    ap.add_argument("--teachers", type=int, default=250)
    ap.add_argument("--figures-dir", default=".")
    ap.add_argument("--threshold", type=float, default=200.0)
    ap.add_argument("--sigma1", type=float, default=150.0)
    ap.add_argument("--sigma2", type=float, default=40.0)
    ap.add_argument("--lap-scale", type=float, default=50.0)
    a = ap.parse_args(argv)
    if a.counts_file:
        votes, _ = load_votes(a.counts_file, None, a.queries)
        source = os.path.basename(a.counts_file)
    else:
        votes = synthetic_votes(a.queries, a.teachers, 10, seed=0)
        source = f"synthetic votes ({a.queries} queries, {a.teachers} teachers): no network for the paper's data"
    res = {"source": source, "cumulative": {}}
    res["cumulative"]["lnmax"] = cumulative_privacy(votes, "lnmax", a.lap_scale)
    res["cumulative"]["gnmax"] = cumulative_privacy(votes, "gnmax", a.sigma2)
    res["cumulative"]["gnmax_conf"] = cumulative_privacy(votes, "gnmax_conf", a.sigma2, a.threshold, a.sigma1)
    res["bucketized"] = bucketized(votes, 5, a.threshold, a.sigma1, a.sigma2, 50.0)
    res["ls_of_q"] = ls_of_q()
    os.makedirs(a.figures_dir, exist_ok=True)
    figs = _plots(a.figures_dir, res)

    def js(x):
        return x.tolist() if isinstance(x, np.ndarray) else x

    summary = {"source": source, "figures": figs,
               "final": {m: {"eps": float(r["eps"][-1]), "order": float(r["order_opt"][-1]),
                             "answered": float(r["answered"][-1])} for m, r in res["cumulative"].items()},
               "bucketized": {k: js(v) for k, v in res["bucketized"].items()},
               "ls_of_q": {"q0": res["ls_of_q"]["q0"], "q1": res["ls_of_q"]["q1"]}}
    with open(os.path.join(a.figures_dir, "iclr2018_figures.json"), "w") as f:
        json.dump(summary, f)
    print(json.dumps(summary["final"]))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
