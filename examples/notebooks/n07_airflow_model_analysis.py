"""Notebook 07 (Airflow model analysis) with mifx (reference
`notebooks/07_Airflow_Model_Analysis.ipynb`): list the MODEL artifacts of the pipeline's metadata
store, show the sliced evaluation of one model by trip_start_hour, compare two model versions and
plot the model's lineage graph (artifacts <-> executions through MLMD events)."""
from __future__ import annotations

import argparse
import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))

from _taxi_run import run_taxi_pipeline  # noqa: E402

from mifx.metadata.lineage import TFXArtifactTypes, TFXReadonlyMetadataStore  # noqa: E402


def main(argv=None) -> dict:
    ap = argparse.ArgumentParser()
    ap.add_argument("--root", default=os.path.join(tempfile.gettempdir(), "mifx_n07"))
    ap.add_argument("--rows", type=int, default=3000)
    ap.add_argument("--steps", type=int, nargs="+", default=[100, 300])
    a = ap.parse_args(argv)
    db, _, _ = run_taxi_pipeline(a.root, a.rows, a.steps)
    print("Pipeline DB:\n" + db)
    store = TFXReadonlyMetadataStore.from_sqlite_db(db)
    models = store.get_artifacts_of_type_df(TFXArtifactTypes.MODEL)
    print(models.to_string())
    ids = [int(i) for i in models.index] if "id" not in models else [int(i) for i in models["id"]]
    by_hour = store.display_tfma_analysis(ids[-1], slicing_column="trip_start_hour")
    print(by_hour.head(24).to_string())
    comparison = store.compare_tfma_analysis(ids[0], ids[-1]) if len(ids) > 1 else None
    if comparison is not None:
        print(comparison.to_string())
    png = os.path.join(a.root, f"lineage_model_{ids[-1]}.png")
    g = store.plot_artifact_lineage(ids[-1], path=png)
    print("lineage plot:", png)
    return {"models": models, "by_hour": by_hour, "comparison": comparison, "lineage": g, "png": png}


if __name__ == "__main__":
    main()
