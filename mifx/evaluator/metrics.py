"""Sliced binary-classification metrics (TFMA-equivalent) + result persistence.

Reference: `Evaluator(..., feature_slicing_spec=FeatureSlicingSpec(specs=[SingleSlicingSpec(
column_for_slicing=['trip_start_hour'])]))` (`airflow-dags/taxi_pipeline.py:101-107`) and
`04_TensorFlow_Model_Analysis.ipynb` (overall slice, single column, feature cross, filtered cross
`trip_start_hour == 12`, time series across runs). Metrics per slice: example_count, accuracy,
AUC (rank statistic, tie-corrected), average_loss, precision, recall, label/prediction mean,
calibration. Segmented reductions run on the GPU (mifx.ops.analyzers.segment_metrics) for large
evaluation sets when a device is given.
"""
from __future__ import annotations

import json
import os
from dataclasses import dataclass, field

import numpy as np
import pandas as pd

RESULT_FILE = "eval_result.json"


def _auc(y: np.ndarray, p: np.ndarray) -> float:
    pos = y > 0.5
    npos, nneg = int(pos.sum()), int((~pos).sum())
    if npos == 0 or nneg == 0:
        return float("nan")
    ranks = pd.Series(p).rank(method="average").to_numpy()
    return float((ranks[pos].sum() - npos * (npos + 1) / 2) / (npos * nneg))


def binary_metrics(y: np.ndarray, p: np.ndarray, weights: np.ndarray | None = None) -> dict:
    y = np.asarray(y, np.float64)
    p = np.clip(np.asarray(p, np.float64), 1e-7, 1 - 1e-7)
    n = len(y)
    if n == 0:
        return {"example_count": 0}
    pred = p > 0.5
    tp = float(((y > 0.5) & pred).sum())
    fp = float(((y <= 0.5) & pred).sum())
    fn = float(((y > 0.5) & ~pred).sum())
    loss = -(y * np.log(p) + (1 - y) * np.log(1 - p))
    return {"example_count": n, "accuracy": float((pred == (y > 0.5)).mean()), "auc": _auc(y, p),
            "average_loss": float(loss.mean()), "precision": tp / (tp + fp) if tp + fp else float("nan"),
            "recall": tp / (tp + fn) if tp + fn else float("nan"), "label/mean": float(y.mean()),
            "prediction/mean": float(p.mean()),
            "calibration": float(p.mean() / y.mean()) if y.mean() > 0 else float("nan")}


HIST_BUCKETS = 10000  # TFMA's AUC: confusion matrices at 10000 thresholds (num_buckets of tfma's auc metric)


def binary_metrics_from_hist(sums: np.ndarray, hist: np.ndarray) -> dict:
    """Slice metrics from the GPU segmented reduction (mifx.ops.analyzers.segment_hist): sums = [count, label
    sum, prediction sum, loss sum, correct], hist = [buckets, (neg, pos)] of clipped probabilities. AUC is the
    bucketed (TFMA-style) one; precision / recall count predictions in buckets above one half."""
    from ..ops.analyzers import auc_from_hist

    n = float(sums[0])
    if n == 0:
        return {"example_count": 0}
    nb = hist.shape[0]
    tp, fp = float(hist[nb // 2:, 1].sum()), float(hist[nb // 2:, 0].sum())
    fn = float(hist[:nb // 2, 1].sum())
    ym, pm = sums[1] / n, sums[2] / n
    return {"example_count": int(n), "accuracy": float(sums[4] / n), "auc": auc_from_hist(hist),
            "average_loss": float(sums[3] / n), "precision": tp / (tp + fp) if tp + fp else float("nan"),
            "recall": tp / (tp + fn) if tp + fn else float("nan"), "label/mean": float(ym),
            "prediction/mean": float(pm), "calibration": float(pm / ym) if ym > 0 else float("nan")}


@dataclass
class SliceSpec:
    columns: list = field(default_factory=list)
    feature_values: dict = field(default_factory=dict)

    def key(self) -> str:
        return ",".join(self.columns + [f"{k}={v}" for k, v in sorted(self.feature_values.items())]) or "Overall"


@dataclass
class EvalResult:
    slices: list = field(default_factory=list)  # [{"slice": [[col, value], ...], "spec": str, "metrics": {...}}]
    model_location: str = ""
    data_location: str = ""

    def to_json(self) -> str:
        return json.dumps({"slices": self.slices, "model_location": self.model_location,
                           "data_location": self.data_location}, default=float)

    def overall(self) -> dict:
        for s in self.slices:
            if not s["slice"]:
                return s["metrics"]
        raise KeyError("no overall slice")

    def slice_frame(self, slicing_column: str | None = None) -> pd.DataFrame:
        rows = []
        for s in self.slices:
            cols = [c for c, _ in s["slice"]]
            if slicing_column is None and cols:
                continue
            if slicing_column is not None and cols != [slicing_column]:
                continue
            name = "Overall" if not s["slice"] else ",".join(f"{c}:{v}" for c, v in s["slice"])
            rows.append({"slice": name, **s["metrics"]})
        return pd.DataFrame(rows).set_index("slice") if rows else pd.DataFrame()


def compute_sliced_metrics(labels, preds, features: dict, specs: list[SliceSpec] | None = None,
                           min_slice_size: int = 1, device=None) -> EvalResult:
    """device = a GPU: every slice spec is ONE segmented reduction (csrc/analyzers.hip segment_hist: per-slice
    sums + label-split prediction histograms) instead of a host pass per slice value; AUC is then bucketed."""
    y, p = np.asarray(labels), np.asarray(preds)
    if device is not None and str(device).startswith("cuda"):
        return _sliced_metrics_gpu(y, p, features, specs, min_slice_size, device)
    res = EvalResult()
    specs = specs or [SliceSpec()]
    if not any(not s.columns and not s.feature_values for s in specs):
        specs = [SliceSpec()] + list(specs)
    for spec in specs:
        mask = np.ones(len(y), bool)
        for k, v in spec.feature_values.items():
            mask &= np.asarray([str(x) == str(v) for x in features[k]])
        fixed = [[k, v] for k, v in sorted(spec.feature_values.items())]
        if not spec.columns:
            res.slices.append({"slice": fixed, "spec": spec.key(), "metrics": binary_metrics(y[mask], p[mask])})
            continue
        keys = pd.DataFrame({c: np.asarray(features[c], dtype=object) for c in spec.columns})[mask]
        for vals, grp in keys.groupby(list(spec.columns), dropna=False, sort=True):
            vals = vals if isinstance(vals, tuple) else (vals,)
            rows = grp.index.to_numpy()  # original row positions (RangeIndex before masking)
            if len(rows) < min_slice_size:
                continue
            sl = [[c, (None if (isinstance(v, float) and np.isnan(v)) else v)] for c, v in zip(spec.columns, vals)]
            res.slices.append({"slice": sl + fixed, "spec": spec.key(), "metrics": binary_metrics(y[rows], p[rows])})
    return res


def _sliced_metrics_gpu(y, p, features, specs, min_slice_size, device) -> EvalResult:
    from ..ops.analyzers import segment_hist

    res = EvalResult()
    specs = specs or [SliceSpec()]
    if not any(not s.columns and not s.feature_values for s in specs):
        specs = [SliceSpec()] + list(specs)
    for spec in specs:
        mask = np.ones(len(y), bool)
        for k, v in spec.feature_values.items():
            mask &= np.asarray([str(x) == str(v) for x in features[k]])
        fixed = [[k, v] for k, v in sorted(spec.feature_values.items())]
        if spec.columns:
            keys = pd.DataFrame({c: np.asarray(features[c], dtype=object) for c in spec.columns})
            codes, uniq = pd.MultiIndex.from_frame(keys).factorize(sort=True)
            seg = np.where(mask, codes, -1).astype(np.int32)
            values = list(uniq)
        else:
            seg = np.where(mask, 0, -1).astype(np.int32)
            values = [()]
        sums, hist = segment_hist(seg, y, p, max(1, len(values)), HIST_BUCKETS, device=device)
        for i, vals in enumerate(values):
            if spec.columns and sums[i, 0] < max(1, min_slice_size):
                continue
            vals = vals if isinstance(vals, tuple) else (vals,)
            sl = [[c, (None if (isinstance(v, float) and np.isnan(v)) else v)] for c, v in zip(spec.columns, vals)]
            res.slices.append({"slice": sl + fixed, "spec": spec.key(), "metrics": binary_metrics_from_hist(
                sums[i], hist[i])})
    return res


def save_eval_result(result: EvalResult, uri: str) -> None:
    with open(os.path.join(uri, RESULT_FILE), "w") as f:
        f.write(result.to_json())


def load_eval_result(uri: str) -> EvalResult:
    with open(os.path.join(uri, RESULT_FILE)) as f:
        d = json.load(f)
    return EvalResult(d["slices"], d.get("model_location", ""), d.get("data_location", ""))


def load_eval_results(uris: list[str]) -> pd.DataFrame:
    """Time series of overall metrics across evaluation runs (TFMA `load_eval_results`)."""
    return pd.DataFrame([{"run": u, **load_eval_result(u).overall()} for u in uris]).set_index("run")
