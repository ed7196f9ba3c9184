"""Experiment tracking (MLflow file-store API), XGBoost-style GBDT, fairing-style remote execution."""
import numpy as np
import pytest
import torch

from mifx import fairing, tracking
from mifx.gbdt import XGBClassifier, XGBRegressor


def test_tracking_runs_params_metrics_models(tmp_path):
    tracking.set_tracking_uri(f"file://{tmp_path}")
    eid = tracking.set_experiment("wine")
    assert tracking.set_experiment("wine") == eid
    with tracking.start_run() as run:
        tracking.log_params({"alpha": 0.5, "l1_ratio": 0.5})
        for step, v in enumerate([1.0, 0.8, 0.7]):
            tracking.log_metric("rmse", v, step)
        tracking.set_tag("model", "elasticnet")
        tracking.log_model(torch.nn.Linear(3, 1), "model", module_class="torch.nn:Linear",
                           config={"in_features": 3, "out_features": 1})
        with pytest.raises(ValueError):
            tracking.log_param("alpha", 0.9)
    r = tracking.get_run(run.info["run_id"])
    assert r["info"]["status"] == "FINISHED" and r["data"]["params"] == {"alpha": "0.5", "l1_ratio": "0.5"}
    assert r["data"]["metrics"]["rmse"] == 0.7 and [h["step"] for h in r["data"]["metric_history"]["rmse"]] == [0, 1, 2]
    with tracking.start_run():
        tracking.log_metric("rmse", 0.5)
    runs = tracking.search_runs([eid], order_by="metrics.rmse ASC")
    assert [x["data"]["metrics"]["rmse"] for x in runs] == [0.5, 0.7]
    from mifx.serving.saved_model import load

    lm = load(f"{tmp_path}/{eid}/{run.info['run_id']}/artifacts/model", "cpu")
    assert lm.predict([[1.0, 2.0, 3.0]])["scores"].shape == (1, 1)


def test_wine_example_logs_run(tmp_path):
    import importlib.util
    import os

    p = os.path.join(os.path.dirname(os.path.dirname(__file__)), "examples/mlflow/wine.py")
    spec = importlib.util.spec_from_file_location("wine", p)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    run_id, rmse = mod.main(["--tracking_uri", f"file://{tmp_path}", "--data", ""])
    assert rmse > 0 and tracking.get_run(run_id)["data"]["metrics"]["rmse"] == pytest.approx(rmse)


def test_xgb_regressor_early_stopping():
    r = np.random.default_rng(0)
    X = r.normal(size=(800, 10))
    y = 3 * X[:, 0] + np.sin(X[:, 1]) + r.normal(0, 0.3, 800)
    m = XGBRegressor(n_estimators=500, learning_rate=0.1).fit(X[:600], y[:600], eval_set=[(X[600:], y[600:])],
                                                              early_stopping_rounds=10)
    assert m.best_iteration + 1 == m.n_trees_ < 500
    rmse = float(np.sqrt(np.mean((m.predict(X[600:]) - y[600:]) ** 2)))
    assert rmse == pytest.approx(m.best_score, rel=1e-9) and rmse < 0.6
    assert len(m.evals_result_["validation_0"]["rmse"]) > m.best_iteration


def test_xgb_classifier():
    r = np.random.default_rng(1)
    X = r.normal(size=(600, 5))
    y = (X[:, 0] + X[:, 1] > 0).astype(int)
    m = XGBClassifier(n_estimators=50, learning_rate=0.3).fit(X[:400], y[:400], eval_set=[(X[400:], y[400:])])
    assert (m.predict(X[400:]) == y[400:]).mean() > 0.85 and m.predict_proba(X[:3]).shape == (3, 2)


def _square_sum(n):
    return sum(i * i for i in range(n))


class _Model:
    def train(self):
        return "trained"


def test_fairing_local_and_job_manifest(tmp_path):
    cfg = fairing.Config()
    cfg.set_builder("append", base_image="rocm/pytorch:latest", registry="reg", push=False)
    cfg.set_deployer("local")
    assert cfg.fn(_square_sum)(10) == 285
    cfg.set_model(_Model())
    assert cfg.run() == "trained"
    cfg.set_deployer("job", namespace="ns", gpus=2)
    m = cfg.job_manifest()
    assert m["kind"] == "Job" and m["spec"]["template"]["spec"]["containers"][0]["resources"]["limits"][
        "amd.com/gpu"] == "2"
    d = cfg.build_context(lambda: 1, str(tmp_path / "ctx"))
    assert open(f"{d}/Dockerfile").read().startswith("FROM rocm/pytorch:latest")
