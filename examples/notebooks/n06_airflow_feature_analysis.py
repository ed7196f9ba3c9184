"""Notebook 06 (Airflow feature analysis) with mifx (reference
`notebooks/06_Airflow_Feature_Analysis.ipynb` cells 3-11): open the pipeline's ML-Metadata store,
find the SchemaGen artifact, rebuild the raw feature spec from schema.pbtxt, and run the taxi
module's preprocessing_fn over a hand-made raw example (analyze-and-transform on that one row,
as the notebook does) and through the pipeline's own Transform output (full-data constants)."""
from __future__ import annotations

import argparse
import os
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

import numpy as np  # noqa: E402
import pandas as pd  # noqa: E402

from _taxi_run import run_taxi_pipeline  # noqa: E402

import mifx.transform as tft  # noqa: E402
from mifx.data_validation import load_schema_text  # noqa: E402
from mifx.metadata.lineage import TFXArtifactTypes, TFXReadonlyMetadataStore  # noqa: E402

RAW_EXAMPLE = {
    "fare": 100.0, "trip_start_hour": 12, "pickup_census_tract": "abcd", "dropoff_census_tract": 12345.0,
    "company": "taxi inc.", "trip_start_timestamp": 123456, "pickup_longitude": 12.0, "trip_start_month": 5,
    "trip_miles": 8.0, "dropoff_longitude": 12.05, "dropoff_community_area": 123, "pickup_community_area": 123,
    "payment_type": "visa", "trip_seconds": 600.0, "trip_start_day": 12, "tips": 10.0, "pickup_latitude": 80.0,
    "dropoff_latitude": 80.01,
}


def parse_as(value, spec: dict) -> np.ndarray:
    """Coerce a raw value to the schema's dtype; unparseable numerics become missing (None)."""
    if spec["dtype"] in ("string", "bytes", "object"):
        return np.array([str(value)], dtype=object)
    try:
        v = float(value)
    except (TypeError, ValueError):
        return np.array([None], dtype=object)
    return np.array([v], dtype=np.float64)


def main(argv=None) -> dict:
    ap = argparse.ArgumentParser()
    ap.add_argument("--root", default=os.path.join(tempfile.gettempdir(), "mifx_n06"))
    ap.add_argument("--rows", type=int, default=3000)
    ap.add_argument("--steps", type=int, default=200)
    a = ap.parse_args(argv)
    db, _, runs = run_taxi_pipeline(a.root, a.rows, [a.steps])
    print("Pipeline DB:\n" + db)
    store = TFXReadonlyMetadataStore.from_sqlite_db(db)
    schemas = store.get_artifacts_of_type_df(TFXArtifactTypes.SCHEMA)
    assert len(schemas.URI) == 1
    schema_uri = os.path.join(schemas.URI.iloc[0], "schema.pbtxt")
    print("Schema URI:\n" + schema_uri)
    schema = load_schema_text(schema_uri)
    feature_spec = schema.as_feature_spec()
    print("feature spec:", {k: v for k, v in list(feature_spec.items())[:4]}, "...")

    module = tft.import_module_file(os.path.join(HERE, "..", "taxi", "taxi_module.py"))
    cols = {k: parse_as(RAW_EXAMPLE[k], spec) for k, spec in feature_spec.items() if k in RAW_EXAMPLE}
    one_row, _ = tft.analyze(module.preprocessing_fn, cols)
    df_one = pd.DataFrame({k: v for k, v in one_row.items()})
    print(df_one.T.to_string())

    tdir = runs[0].components["Transform"].outputs["transform_output"][0].uri
    full = tft.TransformOutput(tdir).transform_raw_features(cols)
    df_full = pd.DataFrame({k: v for k, v in full.items()})
    print(df_full.T.to_string())
    return {"schema_uri": schema_uri, "one_row": df_one, "pipeline_transform": df_full}


if __name__ == "__main__":
    main()
