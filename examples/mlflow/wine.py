"""ElasticNet on the wine-quality data with experiment tracking (reference: `notebooks/mlflow/mlflow-wine.ipynb`).

Uses the reference's CSV when present (read as text), else a synthetic regression set of the same
shape (11 physico-chemical features -> quality 3..9)."""
import argparse
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))

import numpy as np  # noqa: E402
import pandas as pd  # noqa: E402
from sklearn.linear_model import ElasticNet  # noqa: E402
from sklearn.metrics import mean_absolute_error, mean_squared_error, r2_score  # noqa: E402
from sklearn.model_selection import train_test_split  # noqa: E402

from mifx import tracking  # noqa: E402

REF_CSV = "/root/reference/notebooks/mlflow/wine-quality.csv"


def load(path: str | None):
    if path and os.path.exists(path):
        return pd.read_csv(path)
    rng = np.random.default_rng(40)
    cols = ["fixed acidity", "volatile acidity", "citric acid", "residual sugar", "chlorides", "free sulfur dioxide",
            "total sulfur dioxide", "density", "pH", "sulphates", "alcohol"]
    X = rng.normal(size=(1599, len(cols)))
    q = np.clip(np.round(5.6 + X @ rng.normal(0, 0.3, len(cols)) + rng.normal(0, 0.5, len(X))), 3, 9)
    df = pd.DataFrame(X, columns=cols)
    df["quality"] = q
    return df


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--alpha", type=float, default=0.5)
    ap.add_argument("--l1_ratio", type=float, default=0.5)
    ap.add_argument("--tracking_uri", default="file:///tmp/mifx_experiments")
    ap.add_argument("--data", default=REF_CSV)
    a = ap.parse_args(argv)
    np.random.seed(40)
    tracking.set_tracking_uri(a.tracking_uri)
    tracking.set_experiment("wine")
    data = load(a.data)
    train, test = train_test_split(data, random_state=40)
    tx, ty = train.drop(["quality"], axis=1), train[["quality"]]
    vx, vy = test.drop(["quality"], axis=1), test[["quality"]]
    with tracking.start_run() as run:
        lr = ElasticNet(alpha=a.alpha, l1_ratio=a.l1_ratio, random_state=42).fit(tx, ty)
        pred = lr.predict(vx)
        rmse, mae, r2 = float(np.sqrt(mean_squared_error(vy, pred))), float(mean_absolute_error(vy, pred)), \
            float(r2_score(vy, pred))
        print(f"Elasticnet model (alpha={a.alpha:f}, l1_ratio={a.l1_ratio:f}):\n  RMSE: {rmse}\n  MAE: {mae}\n  R2: {r2}")
        tracking.log_params({"alpha": a.alpha, "l1_ratio": a.l1_ratio})
        tracking.log_metrics({"rmse": rmse, "r2": r2, "mae": mae})
        tracking.log_model(lr, "model")
        return run.info["run_id"], rmse


if __name__ == "__main__":
    main()
