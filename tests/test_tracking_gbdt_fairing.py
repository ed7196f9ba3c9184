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
    # XGBoost semantics: training stops early_stopping_rounds after the best round; predict uses the best round
    assert m.best_iteration + 1 + 10 == m.n_trees_ < 500
    rmse = float(np.sqrt(np.mean((m.predict(X[600:]) - y[600:]) ** 2)))
    assert rmse == pytest.approx(m.best_score, rel=1e-9) and rmse < 0.6
    assert len(m.evals_result_["validation_0"]["rmse"]) > m.best_iteration


def test_xgb_eval_set_without_early_stopping_uses_every_tree():
    """XGBoost's sklearn API: best_iteration / best_score exist only under early stopping; with an eval_set alone
    predict uses all n_estimators trees."""
    r = np.random.default_rng(2)
    X = r.normal(size=(400, 6))
    y = X[:, 0] - 2 * X[:, 2] + r.normal(0, 0.5, 400)
    m = XGBRegressor(n_estimators=60, learning_rate=0.3).fit(X[:300], y[:300], eval_set=[(X[300:], y[300:])])
    assert m.best_iteration is None and m.best_score is None and m.n_trees_ == 60
    hist = m.evals_result_["validation_0"]["rmse"]
    assert len(hist) == 60
    rmse = float(np.sqrt(np.mean((m.predict(X[300:]) - y[300:]) ** 2)))
    assert rmse == pytest.approx(hist[-1], rel=1e-9)  # the last tree's score, not the best one's


def test_xgb_classifier():
    r = np.random.default_rng(1)
    X = r.normal(size=(600, 5))
    y = (X[:, 0] + X[:, 1] > 0).astype(int)
    m = XGBClassifier(n_estimators=50, learning_rate=0.3).fit(X[:400], y[:400], eval_set=[(X[400:], y[400:])])
    assert (m.predict(X[400:]) == y[400:]).mean() > 0.85 and m.predict_proba(X[:3]).shape == (3, 2)


def _ref_tree(X, g, h, depth, lam, mcw, eta):
    """Brute-force second-order tree (every distinct value as a cut, missing rows tried on both sides) -- the
    oracle for csrc/gbdt.cpp on data with at most max_bins distinct values per feature."""
    def leaf(idx):
        return ("leaf", -eta * g[idx].sum() / (h[idx].sum() + lam))

    def grow(idx, d):
        if d == depth or len(idx) < 2:
            return leaf(idx)
        G, H = g[idx].sum(), h[idx].sum()
        best = (1e-6, None)
        for j in range(X.shape[1]):
            col = X[idx, j]
            miss = np.isnan(col)
            for c in np.unique(col[~miss])[1:]:
                lm = (~miss) & (col < c)
                for ml in (False, True):
                    L = lm | (miss & ml)
                    GL, HL = g[idx][L].sum(), h[idx][L].sum()
                    GR, HR = G - GL, H - HL
                    if HL < mcw or HR < mcw:
                        continue
                    gain = 0.5 * (GL ** 2 / (HL + lam) + GR ** 2 / (HR + lam) - G ** 2 / (H + lam))
                    if gain > best[0] + 1e-9:
                        best = (gain, (j, c, ml, L))
        if best[1] is None:
            return leaf(idx)
        j, c, ml, L = best[1]
        return ("split", j, c, ml, grow(idx[L], d + 1), grow(idx[~L], d + 1))

    return grow(np.arange(len(g)), 0)


def _ref_predict(t, x):
    while t[0] == "split":
        _, j, c, ml, lt, rt = t
        t = lt if (ml if np.isnan(x[j]) else x[j] < c) else rt
    return t[1]


def test_gbdt_native_matches_bruteforce_learner():
    """csrc/gbdt.cpp vs an exhaustive Python learner: same trees (hence predictions) for squared error on data with
    missing values, when every distinct value is its own bin."""
    r = np.random.default_rng(3)
    X = np.round(r.normal(size=(300, 4)), 1)  # few distinct values -> one bin each
    X[r.random(X.shape) < 0.1] = np.nan
    y = 2 * np.nan_to_num(X[:, 0]) - np.nan_to_num(X[:, 2]) ** 2 + r.normal(0, 0.1, 300)
    m = XGBRegressor(n_estimators=3, learning_rate=0.5, max_depth=3, max_bins=256, min_child_weight=1.0).fit(X, y)
    margin = np.full(len(y), y.mean())
    trees = []
    for _ in range(3):
        t = _ref_tree(X, margin - y, np.ones(len(y)), 3, 1.0, 1.0, 0.5)
        trees.append(t)
        margin = margin + np.array([_ref_predict(t, x) for x in X])
    Xt = np.round(r.normal(size=(50, 4)), 1)
    Xt[r.random(Xt.shape) < 0.1] = np.nan
    want = y.mean() + np.array([sum(_ref_predict(t, x) for t in trees) for x in Xt])
    np.testing.assert_allclose(m.predict(Xt), want, rtol=1e-6, atol=1e-6)  # (float32 gradients)
    np.testing.assert_allclose(m.predict(X), margin, rtol=1e-6, atol=1e-6)  # (float32 gradients)


def test_gbdt_deterministic_across_threads_and_binned():
    r = np.random.default_rng(5)
    X = r.normal(size=(30000, 12))
    y = X[:, 0] * X[:, 1] + np.abs(X[:, 2]) + r.normal(0, 0.1, 30000)
    a = XGBRegressor(n_estimators=20, max_bins=64, n_jobs=1).fit(X, y)
    b = XGBRegressor(n_estimators=20, max_bins=64, n_jobs=8).fit(X, y)
    assert np.array_equal(a.predict(X[:1000]), b.predict(X[:1000]))  # bit-identical for any thread count
    assert all(len(c) <= 63 for c in a._cuts)  # quantile thinning to max_bins bins
    rmse = float(np.sqrt(np.mean((a.predict(X) - y) ** 2)))
    assert rmse < 0.35 * y.std()


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
