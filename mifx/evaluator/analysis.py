"""TFMA-style entry points over mifx eval exports (reference `04_TensorFlow_Model_Analysis.ipynb`
cells 13-33, `07_Airflow_Model_Analysis.ipynb`; `notebooks/tfx_utils.py:67-83`):

    m = default_eval_shared_model(eval_saved_model_path)
    r = run_model_analysis(m, data_location="eval.csv", slice_spec=[SingleSliceSpec(),
            SingleSliceSpec(columns=["trip_start_hour"]),
            SingleSliceSpec(columns=["trip_start_day", "trip_start_hour"]),
            SingleSliceSpec(columns=["trip_start_day"], features=[("trip_start_hour", 12)])],
            output_path=out_dir)
    r.slice_frame("trip_start_hour");  load_eval_results([out1, out2, out3])  # time series

Predictions run through the exported model (GPU when available); per-slice reductions are the
grouped metrics of :mod:`mifx.evaluator.metrics`."""
from __future__ import annotations

import os
from dataclasses import dataclass, field

import numpy as np

from . import metrics as em


@dataclass
class SingleSliceSpec:
    columns: list = field(default_factory=list)
    features: list = field(default_factory=list)  # [(column, value)] fixed values (filtered slice)

    def to_internal(self) -> em.SliceSpec:
        return em.SliceSpec(columns=list(self.columns), feature_values={k: v for k, v in self.features})


@dataclass
class EvalSharedModel:
    model_path: str
    loaded: object = None


def default_eval_shared_model(eval_saved_model_path: str, device=None) -> EvalSharedModel:
    from ..serving import saved_model

    path = eval_saved_model_path
    if not os.path.exists(os.path.join(path, "saved_model.json")) and os.path.isdir(path):
        path = saved_model.latest_export(path)
    return EvalSharedModel(path, saved_model.load(path, device=device))


def _read_data(data_location: str, file_format: str):
    from ..components.transform import table_to_inputs
    from ..io import dataset

    if file_format == "csv" or data_location.endswith(".csv"):
        from ..data_validation.stats import read_csv_table

        return table_to_inputs(read_csv_table(data_location))
    if file_format == "tfrecords":
        return table_to_inputs(dataset.read_tfrecord_split(data_location))
    return table_to_inputs(dataset.read_split(data_location))


def run_model_analysis(eval_shared_model: EvalSharedModel, data_location: str, file_format: str = "csv",
                       slice_spec: list | None = None, output_path: str | None = None) -> em.EvalResult:
    loaded = eval_shared_model.loaded
    raw = _read_data(data_location, file_format)
    label_key = loaded.meta["receiver"]["label_key"]
    tcols = loaded.transform.transform_raw_features(raw) if loaded.transform else raw
    labels = np.asarray(tcols[label_key], np.float64)
    probs = 1.0 / (1.0 + np.exp(-loaded.wd_logits(raw)))
    specs = [s.to_internal() if isinstance(s, SingleSliceSpec) else s for s in (slice_spec or [SingleSliceSpec()])]
    res = em.compute_sliced_metrics(labels, probs, raw, specs)
    res.model_location, res.data_location = eval_shared_model.model_path, data_location
    if output_path:
        os.makedirs(output_path, exist_ok=True)
        em.save_eval_result(res, output_path)
    return res


load_eval_result = em.load_eval_result
load_eval_results = em.load_eval_results
