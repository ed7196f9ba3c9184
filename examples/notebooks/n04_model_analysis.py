"""Notebook 04 (TensorFlow Model Analysis) with mifx.evaluator (reference
`notebooks/04_TensorFlow_Model_Analysis.ipynb` cells 13-33): evaluate exported taxi models on the
eval CSV with an overall slice, a single-column slice (trip_start_hour), a feature cross
(trip_start_day x trip_start_hour) and a filtered cross (trip_start_day where trip_start_hour == 12),
then follow the overall metrics across three training runs as a time series."""
from __future__ import annotations

import argparse
import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from _data import taxi_csvs  # noqa: E402
from _taxi_run import run_taxi_pipeline  # noqa: E402

import mifx.evaluator as tfma  # noqa: E402
from mifx.components.trainer import EVAL_DIR  # noqa: E402

SLICES = [tfma.SingleSliceSpec(),
          tfma.SingleSliceSpec(columns=["trip_start_hour"]),
          tfma.SingleSliceSpec(columns=["trip_start_day", "trip_start_hour"]),
          tfma.SingleSliceSpec(columns=["trip_start_day"], features=[("trip_start_hour", 12)])]


def main(argv=None) -> dict:
    ap = argparse.ArgumentParser()
    ap.add_argument("--root", default=os.path.join(tempfile.gettempdir(), "mifx_n04"))
    ap.add_argument("--rows", type=int, default=3000)
    ap.add_argument("--steps", type=int, nargs="+", default=[100, 300, 600])
    a = ap.parse_args(argv)
    _, _, runs = run_taxi_pipeline(a.root, a.rows, a.steps)
    _, eval_csv = taxi_csvs(os.path.join(a.root, "csv"), a.rows, a.rows // 2)
    outputs = []
    for i, run in enumerate(runs):
        model_uri = run.components["Trainer"].outputs["output"][0].uri
        shared = tfma.default_eval_shared_model(os.path.join(model_uri, EVAL_DIR))
        out = os.path.join(a.root, "tfma", f"run_{i}")
        res = tfma.run_model_analysis(shared, eval_csv, slice_spec=SLICES, output_path=out)
        outputs.append(out)
        if i == 0:
            print(res.slice_frame().to_string())                       # overall
            print(res.slice_frame("trip_start_hour").head(24).to_string())
            cross = [s for s in res.slices if len(s["slice"]) == 2 and s["spec"] == "trip_start_day,trip_start_hour"]
            print(f"{len(cross)} trip_start_day x trip_start_hour slices")
            filt = [s for s in res.slices if s["spec"] == "trip_start_day,trip_start_hour=12"]
            print(f"{len(filt)} trip_start_day slices with trip_start_hour == 12")
    series = tfma.load_eval_results(outputs)
    print(series[["example_count", "accuracy", "auc", "average_loss"]].to_string())
    return {"outputs": outputs, "series": series}


if __name__ == "__main__":
    main()
