"""XGBoost-style gradient-boosted trees: XGBRegressor / XGBClassifier on the native histogram learner of
csrc/gbdt.cpp (second-order split gain, learned missing-value directions, depth-wise growth).

Reference usage: `kubeflow-pipelines/fairing/fairing_xgboost.py:69-87` (XGBRegressor(n_estimators, learning_rate),
fit with `early_stopping_rounds` and `eval_set`, then `best_score`, `best_iteration`, `predict`). Semantics follow
XGBoost's scikit-learn API: the eval metric is RMSE (regression) or logloss (binary classification) on the LAST
eval set; with early stopping, training stops after `early_stopping_rounds` rounds without improvement and
`predict` uses the trees up to `best_iteration` (XGBoost >= 1.4's default `iteration_range`). Defaults are
XGBoost >= 1.0's (learning_rate 0.3, max_depth 6, reg_lambda 1, min_child_weight 1, gamma 0, 256 bins); the
intercept is the training mean (regression) or its log-odds (classification), XGBoost 2's `base_score` estimate.
Binary classification only (the reference has no multi-class GBDT)."""
from __future__ import annotations

import ctypes
import functools
import logging
import os

import numpy as np

_D = ctypes.POINTER(ctypes.c_double)
_F = ctypes.POINTER(ctypes.c_float)
_I = ctypes.POINTER(ctypes.c_int)
_U8 = ctypes.POINTER(ctypes.c_uint8)
_U16 = ctypes.POINTER(ctypes.c_uint16)


@functools.lru_cache(maxsize=None)
def _lib():
    from ..ops import _lib as L

    lib = L.load("gbdt")
    lib.mifx_gbdt_cuts.argtypes = [_D, ctypes.c_long, ctypes.c_long, ctypes.c_int, _D]
    lib.mifx_gbdt_bin.argtypes = [_D, ctypes.c_long, ctypes.c_int, _D, _I, _I, _U16, ctypes.c_int]
    lib.mifx_gbdt_grow.argtypes = [_U16, ctypes.c_long, ctypes.c_int, _I, _F, _F, ctypes.c_int, ctypes.c_double,
                                   ctypes.c_double, ctypes.c_double, ctypes.c_double, ctypes.c_int, ctypes.c_int,
                                   _I, _I, _U8, _I, _I, _D, _I]
    lib.mifx_gbdt_predict.argtypes = [_D, ctypes.c_long, ctypes.c_int, ctypes.c_int, _I, _I, _D, _U8, _I, _I, _D,
                                      ctypes.c_double, _D, ctypes.c_int]
    for f in (lib.mifx_gbdt_cuts, lib.mifx_gbdt_bin, lib.mifx_gbdt_grow, lib.mifx_gbdt_predict):
        f.restype = ctypes.c_int
    return lib


def _p(a: np.ndarray, t):
    return a.ctypes.data_as(t)


def _threads() -> int:
    return max(1, min(16, int(os.environ.get("OMP_NUM_THREADS", os.cpu_count() or 1))))


class _Base:
    _objective = "reg:squarederror"

    def __init__(self, n_estimators: int = 100, learning_rate: float = 0.3, max_depth: int = 6,
                 min_child_weight: float = 1.0, reg_lambda: float = 1.0, gamma: float = 0.0, max_bins: int = 256,
                 base_score: float | None = None, n_jobs: int | None = None, random_state: int = 0,
                 verbosity: int = 0):
        self.n_estimators, self.learning_rate, self.max_depth = n_estimators, learning_rate, max_depth
        self.min_child_weight, self.reg_lambda, self.gamma, self.max_bins = min_child_weight, reg_lambda, gamma, max_bins
        self.base_score, self.n_jobs = base_score, n_jobs
        self.random_state, self.verbosity = random_state, verbosity  # (the learner is deterministic: no sampling)
        self.best_iteration, self.best_score, self.evals_result_ = None, None, {}
        self._trees: list[tuple] = []

    # ---- loss (overridden by the classifier)
    def _base(self, y: np.ndarray) -> float:
        return float(np.mean(y))

    def _grad_hess(self, margin: np.ndarray, y: np.ndarray):
        return (margin - y).astype(np.float32), np.ones(len(y), np.float32)

    def _metric_name(self) -> str:
        return "rmse"

    def _metric(self, margin: np.ndarray, y: np.ndarray) -> float:
        return float(np.sqrt(np.mean((margin - y) ** 2)))

    def _check_y(self, y: np.ndarray) -> np.ndarray:
        return y.astype(np.float64)

    # ---- training
    def _bin_matrix(self, X: np.ndarray):
        lib, (n, f) = _lib(), X.shape
        cuts, offs, ncut = [], [0], []
        buf = np.empty(max(1, self.max_bins), np.float64)
        for j in range(f):
            m = lib.mifx_gbdt_cuts(_p(X[:, j:], _D), n, f, int(self.max_bins), _p(buf, _D))
            if m < 0:
                raise ValueError("max_bins must be in [2, 65535]")
            cuts.append(buf[:m].copy())
            ncut.append(m)
            offs.append(offs[-1] + m)
        self._cuts = cuts
        flat = np.concatenate(cuts) if offs[-1] else np.zeros(1)
        self._cut_flat = np.ascontiguousarray(flat, np.float64)
        self._cut_off = np.asarray(offs[:-1], np.int32)
        self._ncut = np.asarray(ncut, np.int32)
        bins = np.empty((f, n), np.uint16)
        lib.mifx_gbdt_bin(_p(X, _D), n, f, _p(self._cut_flat, _D), _p(self._cut_off, _I), _p(self._ncut, _I),
                          _p(bins, _U16), self._nthreads())
        return bins

    def _nthreads(self) -> int:
        return self.n_jobs if self.n_jobs and self.n_jobs > 0 else _threads()

    def _grow(self, bins, nbins, g, h, leaf_of_row):
        n = bins.shape[1]
        cap = 2 ** (self.max_depth + 1)
        fe, sb, left, right = (np.empty(cap, np.int32) for _ in range(4))
        dl = np.empty(cap, np.uint8)
        val = np.empty(cap, np.float64)
        cnt = _lib().mifx_gbdt_grow(_p(bins, _U16), n, bins.shape[0], _p(nbins, _I), _p(g, _F), _p(h, _F),
                                    int(self.max_depth), float(self.min_child_weight), float(self.reg_lambda),
                                    float(self.gamma), float(self.learning_rate), self._nthreads(), cap, _p(fe, _I),
                                    _p(sb, _I), _p(dl, _U8), _p(left, _I), _p(right, _I), _p(val, _D),
                                    _p(leaf_of_row, _I))
        if cnt < 0:
            raise RuntimeError("tree exceeded its node capacity")
        thr = np.zeros(cnt, np.float64)
        for k in range(cnt):  # the split's cut value: bin <= b  <=>  x < cuts[b]
            if fe[k] >= 0:
                thr[k] = self._cuts[fe[k]][sb[k]]
        return fe[:cnt].copy(), thr, dl[:cnt].copy(), left[:cnt].copy(), right[:cnt].copy(), val[:cnt].copy()

    def fit(self, X, y, eval_set=None, early_stopping_rounds: int | None = None, verbose: bool = False):
        X = np.ascontiguousarray(np.asarray(X, dtype=np.float64))
        y = self._check_y(np.asarray(y).reshape(-1))
        if X.ndim != 2 or len(X) != len(y):
            raise ValueError("X must be [n, features] with one label per row")
        self._nfeat = X.shape[1]
        bins = self._bin_matrix(X)
        nbins = (self._ncut + 1).astype(np.int32)
        self._base_margin = float(self.base_score) if self.base_score is not None else self._base(y)
        if self._objective != "reg:squarederror" and self.base_score is not None:
            self._base_margin = float(np.log(self.base_score / (1 - self.base_score)))
        margin = np.full(len(y), self._base_margin)
        leaf_of_row = np.empty(len(y), np.int32)
        ev = None
        if eval_set:
            ex, ey = eval_set[-1]
            ex = np.ascontiguousarray(np.asarray(ex, dtype=np.float64))
            ey = self._check_y(np.asarray(ey).reshape(-1))
            ev_margin = np.full(len(ey), self._base_margin)
            ev = (ex, ey, ev_margin)
        self._trees = []
        best, best_it, since, hist = None, 0, 0, []
        for it in range(int(self.n_estimators)):
            g, h = self._grad_hess(margin, y)
            tree = self._grow(bins, nbins, g, h, leaf_of_row)
            self._trees.append(tree)
            margin += tree[5][leaf_of_row]
            if ev is not None:
                ev[2][:] += self._predict_trees(ev[0], [tree], 0.0)
                score = self._metric(ev[2], ev[1])
                hist.append(score)
                if verbose:
                    logging.info("[%d]\tvalidation_0-%s:%.5f", it, self._metric_name(), score)
                if best is None or score < best:
                    best, best_it, since = score, it, 0
                else:
                    since += 1
                    if early_stopping_rounds and since >= early_stopping_rounds:
                        break
        self.evals_result_ = {"validation_0": {self._metric_name(): hist}} if ev is not None else {}
        # XGBoost's sklearn API sets best_iteration / best_score only under early stopping; without it predict uses
        # every tree even when an eval_set was given
        self.best_score, self.best_iteration = (best, best_it) if ev is not None and early_stopping_rounds else \
            (None, None)
        return self

    @property
    def n_trees_(self) -> int:
        return len(self._trees)

    # ---- prediction
    def _predict_trees(self, X: np.ndarray, trees, base: float) -> np.ndarray:
        X = np.ascontiguousarray(np.asarray(X, dtype=np.float64))
        if X.ndim != 2 or X.shape[1] != self._nfeat:
            raise ValueError(f"expected [n, {self._nfeat}] features")
        out = np.empty(len(X), np.float64)
        if not trees:
            out[:] = base
            return out
        off = np.cumsum([0] + [len(t[0]) for t in trees[:-1]]).astype(np.int32)
        fe, thr, dl, le, ri, val = (np.ascontiguousarray(np.concatenate([t[k] for t in trees])) for k in range(6))
        _lib().mifx_gbdt_predict(_p(X, _D), len(X), self._nfeat, len(trees), _p(off, _I), _p(fe, _I), _p(thr, _D),
                                 _p(dl, _U8), _p(le, _I), _p(ri, _I), _p(val, _D), float(base), _p(out, _D),
                                 self._nthreads())
        return out

    def _margin(self, X) -> np.ndarray:
        n = len(self._trees) if self.best_iteration is None else self.best_iteration + 1
        return self._predict_trees(X, self._trees[:n], self._base_margin)


class XGBRegressor(_Base):
    """Squared-error regression (objective reg:squarederror)."""

    def predict(self, X) -> np.ndarray:
        return self._margin(X)


class XGBClassifier(_Base):
    """Binary classification (objective binary:logistic); labels are any two values (classes_ sorted)."""
    _objective = "binary:logistic"

    def _check_y(self, y: np.ndarray) -> np.ndarray:
        if not hasattr(self, "classes_") or self._fitting:
            self.classes_ = np.unique(y)
            if len(self.classes_) > 2:
                raise ValueError("XGBClassifier here is binary (binary:logistic)")
        return (np.searchsorted(self.classes_, y) == 1).astype(np.float64) if len(self.classes_) == 2 \
            else np.zeros(len(y))

    def fit(self, X, y, eval_set=None, early_stopping_rounds: int | None = None, verbose: bool = False):
        self._fitting = True
        y = np.asarray(y).reshape(-1)
        self._check_y(y)  # classes from the training labels
        self._fitting = False
        return super().fit(X, y, eval_set, early_stopping_rounds, verbose)

    def _base(self, y: np.ndarray) -> float:
        p = float(np.clip(np.mean(y), 1e-6, 1 - 1e-6))
        return float(np.log(p / (1 - p)))

    def _grad_hess(self, margin: np.ndarray, y: np.ndarray):
        p = 1.0 / (1.0 + np.exp(-margin))
        return (p - y).astype(np.float32), np.maximum(p * (1 - p), 1e-16).astype(np.float32)

    def _metric_name(self) -> str:
        return "logloss"

    def _metric(self, margin: np.ndarray, y: np.ndarray) -> float:
        p = np.clip(1.0 / (1.0 + np.exp(-margin)), 1e-15, 1 - 1e-15)
        return float(-np.mean(y * np.log(p) + (1 - y) * np.log(1 - p)))

    def predict_proba(self, X) -> np.ndarray:
        p1 = 1.0 / (1.0 + np.exp(-self._margin(X)))
        return np.stack([1 - p1, p1], 1)

    def predict(self, X) -> np.ndarray:
        return self.classes_[(self.predict_proba(X)[:, 1] > 0.5).astype(int)]
