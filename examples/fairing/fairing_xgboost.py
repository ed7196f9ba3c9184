"""XGBoost-style regressor trained through the fairing config (reference:
`kubeflow-pipelines/fairing/fairing_xgboost.py`). The Ames-housing download is unavailable offline,
so a synthetic table of the same shape (1460 rows, 36 numeric features) is used."""
import logging
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))

import numpy as np  # noqa: E402
from sklearn.metrics import mean_absolute_error  # noqa: E402

from mifx import fairing  # noqa: E402
from mifx.gbdt import XGBRegressor  # noqa: E402

ESTIMATORS, LEARNING_RATE, TEST_FRACTION_SIZE, EARLY_STOPPING_ROUNDS = 1000, 0.1, 0.25, 50


def read_input(test_size=TEST_FRACTION_SIZE):
    rng = np.random.default_rng(0)
    X = rng.normal(size=(1460, 36))
    y = 180000 + 40000 * X[:, 0] + 15000 * np.sin(X[:, 1]) + 8000 * X[:, 2] * X[:, 3] + rng.normal(0, 5000, 1460)
    n = int(len(X) * (1 - test_size))
    return (X[:n], y[:n]), (X[n:], y[n:])


def run_training_and_eval():
    (tx, ty), (vx, vy) = read_input()
    model = XGBRegressor(n_estimators=ESTIMATORS, learning_rate=LEARNING_RATE)
    model.fit(tx, ty, early_stopping_rounds=EARLY_STOPPING_ROUNDS, eval_set=[(vx, vy)])
    logging.info("Best RMSE on eval: %.2f with %d rounds", model.best_score, model.best_iteration + 1)
    mae = mean_absolute_error(model.predict(vx), vy)
    print(f"mean_absolute_error={mae:.2f}")
    return mae


if __name__ == "__main__":
    fairing.config.set_builder("append", base_image="rocm/pytorch:latest", registry="local", push=False)
    fairing.config.set_deployer("local")
    print(fairing.config.fn(run_training_and_eval)())
