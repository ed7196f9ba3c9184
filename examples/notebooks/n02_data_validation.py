"""Notebook 02 (TensorFlow Data Validation) with mifx.data_validation
(reference `notebooks/02_TensorFlow_Data_Validation.ipynb` cells 9-34):
statistics from CSV -> infer schema -> eval-vs-train statistics -> anomalies -> schema relaxation
(min_domain_mass 0.9, add a domain value) -> TRAINING/SERVING environments -> skew and drift
comparators (L-infinity 0.01 / 0.001) -> freeze schema.pbtxt. Numeric column statistics run on
the GPU reduction kernels when a device is given."""
from __future__ import annotations

import argparse
import os
import sys
import tempfile

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))
sys.path.insert(0, os.path.dirname(__file__))

import pandas as pd  # noqa: E402

import mifx.data_validation as tfdv  # noqa: E402
from _data import taxi_csvs  # noqa: E402


def main(argv=None) -> dict:
    ap = argparse.ArgumentParser()
    ap.add_argument("--workdir", default=os.path.join(tempfile.gettempdir(), "mifx_n02"))
    ap.add_argument("--rows", type=int, default=10000)
    ap.add_argument("--device", default=None)
    a = ap.parse_args(argv)
    train_csv, eval_csv = taxi_csvs(a.workdir, a.rows, a.rows // 2)

    # cell 9: statistics of the training data
    train_stats = tfdv.generate_statistics_from_csv(train_csv, name="train", device=a.device)
    print(tfdv.stats_frame(train_stats).head(20).to_string())
    # cell 13: infer a schema
    schema = tfdv.infer_schema(train_stats, max_string_domain_size=200)  # synthetic data has 150 companies
    print(tfdv.display_schema(schema))
    # cell 15-17: eval statistics and anomalies against the training schema
    eval_stats = tfdv.generate_statistics_from_csv(eval_csv, name="eval", device=a.device)
    tfdv.visualize_statistics(eval_stats, train_stats, "EVAL_DATASET", "TRAIN_DATASET")
    anomalies = tfdv.validate_statistics(eval_stats, schema)
    print(tfdv.display_anomalies(anomalies))
    # cell 19: relax the schema -- accept <10% unseen companies, add the new payment type
    if any(f.name == "company" for f in schema.feature):
        tfdv.get_feature(schema, "company").min_domain_mass = 0.9
    pay = tfdv.get_domain(schema, "payment_type")
    if pay is not None and "Mobile" not in pay.value:
        pay.value.append("Mobile")
    relaxed = tfdv.validate_statistics(eval_stats, schema)
    print("after relaxing:", tfdv.display_anomalies(relaxed))
    # cell 27: environments -- `tips` is the label, absent at serving time
    serving = pd.read_csv(eval_csv).drop(columns=["tips"])
    serving_stats = tfdv.generate_statistics_from_dataframe(serving, name="serving")
    schema.default_environment = ["TRAINING", "SERVING"]
    tfdv.get_feature(schema, "tips").not_in_environment.append("SERVING")
    env_anomalies = tfdv.validate_statistics(serving_stats, schema, environment="SERVING")
    print("serving anomalies:", tfdv.display_anomalies(env_anomalies))
    # cell 31: skew (train vs serving) and drift (train vs previous span) comparators
    tfdv.get_feature(schema, "payment_type").skew_linf_threshold = 0.01
    tfdv.get_feature(schema, "company").drift_linf_threshold = 0.001
    skew_drift = tfdv.validate_statistics(train_stats, schema, previous_statistics=eval_stats,
                                          serving_statistics=serving_stats)
    print("skew/drift:", tfdv.display_anomalies(skew_drift))
    # cell 34: freeze the schema
    out = os.path.join(a.workdir, "schema.pbtxt")
    tfdv.write_schema_text(schema, out)
    print("schema written to", out)
    return {"anomalies": anomalies, "relaxed": relaxed, "serving": env_anomalies, "skew_drift": skew_drift,
            "schema_path": out}


if __name__ == "__main__":
    main()
