"""XGBoost-style estimators on a histogram GBDT (warm-started one tree per round)."""
from __future__ import annotations

import logging

import numpy as np


class _Base:
    _loss = "squared_error"

    def __init__(self, n_estimators: int = 100, learning_rate: float = 0.3, max_depth: int = 6,
                 min_child_weight: float = 1.0, reg_lambda: float = 1.0, max_bins: int = 255, random_state: int = 0,
                 verbosity: int = 0):
        self.n_estimators, self.learning_rate, self.max_depth = n_estimators, learning_rate, max_depth
        self.min_child_weight, self.reg_lambda, self.max_bins = min_child_weight, reg_lambda, max_bins
        self.random_state, self.verbosity = random_state, verbosity
        self.best_iteration, self.best_score, self.evals_result_ = None, None, {}

    def _make(self):
        from sklearn.ensemble import HistGradientBoostingClassifier, HistGradientBoostingRegressor

        cls = HistGradientBoostingRegressor if self._loss == "squared_error" else HistGradientBoostingClassifier
        kw = {"loss": self._loss} if self._loss == "squared_error" else {}
        return cls(learning_rate=self.learning_rate, max_iter=1, max_depth=self.max_depth,
                   min_samples_leaf=max(1, int(self.min_child_weight)), l2_regularization=self.reg_lambda,
                   max_bins=min(255, self.max_bins), early_stopping=False, warm_start=True,
                   random_state=self.random_state, **kw)

    def _metric(self, model, X, y) -> float:
        raise NotImplementedError

    def fit(self, X, y, eval_set=None, early_stopping_rounds: int | None = None, verbose: bool = False):
        X, y = np.asarray(X, dtype=np.float64), np.asarray(y).reshape(-1)
        self._model = self._make()
        best, best_it, since = None, 0, 0
        name = "rmse" if self._loss == "squared_error" else "logloss"
        hist = []
        for it in range(1, self.n_estimators + 1):
            self._model.max_iter = it
            self._model.fit(X, y)
            if eval_set:
                ex, ey = eval_set[0]
                score = self._metric(self._model, np.asarray(ex, dtype=np.float64), np.asarray(ey).reshape(-1))
                hist.append(score)
                if verbose:
                    logging.info("[%d]\tvalidation_0-%s:%.5f", it - 1, name, score)
                if best is None or score < best:
                    best, best_it, since = score, it - 1, 0
                else:
                    since += 1
                    if early_stopping_rounds and since >= early_stopping_rounds:
                        break
        self.evals_result_ = {"validation_0": {name: hist}} if eval_set else {}
        if eval_set:
            self.best_score, self.best_iteration = best, best_it
            if self._model.n_iter_ != best_it + 1:  # refit truncated to the best round (deterministic)
                self._model = self._make()
                self._model.set_params(warm_start=False, max_iter=best_it + 1)
                self._model.fit(X, y)
        return self

    @property
    def n_trees_(self) -> int:
        return int(self._model.n_iter_)


class XGBRegressor(_Base):
    _loss = "squared_error"

    def _metric(self, model, X, y):
        return float(np.sqrt(np.mean((model.predict(X) - y) ** 2)))

    def predict(self, X):
        return self._model.predict(np.asarray(X, dtype=np.float64))


class XGBClassifier(_Base):
    _loss = "log_loss"

    def _metric(self, model, X, y):
        p = np.clip(model.predict_proba(X), 1e-15, 1 - 1e-15)
        return float(-np.mean(np.log(p[np.arange(len(y)), np.searchsorted(model.classes_, y)])))

    def predict(self, X):
        return self._model.predict(np.asarray(X, dtype=np.float64))

    def predict_proba(self, X):
        return self._model.predict_proba(np.asarray(X, dtype=np.float64))
