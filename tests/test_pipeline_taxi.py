"""End-to-end TFX-style taxi pipeline on LocalDagRunner (BASELINE config 1, CPU plumbing):
9 components, MLMD lineage, caching, sliced evaluation, blessing, push, serving load."""
import csv
import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "examples", "taxi"))

from mifx.data.synthetic import TAXI_COLUMNS, synthetic_taxi_csv_rows  # noqa: E402
from mifx.metadata.lineage import TFXArtifactTypes, TFXReadonlyMetadataStore, TFXExecutionTypes  # noqa: E402
from mifx.orchestration import LocalDagRunner  # noqa: E402


@pytest.fixture(scope="module")
def taxi_run(tmp_path_factory):
    import taxi_pipeline_local as tp

    d = tmp_path_factory.mktemp("taxi")
    data = d / "data"
    data.mkdir()
    with open(data / "data.csv", "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=TAXI_COLUMNS)
        w.writeheader()
        for r in synthetic_taxi_csv_rows(2500, seed=1):
            w.writerow({k: ("" if v is None else v) for k, v in r.items()})
    mk = lambda: tp.create_pipeline("taxi", str(d / "root"), str(data), str(d / "serving"), train_steps=150,  # noqa
                                    eval_steps=10, metadata_db_root=str(d / "md"))
    res1 = LocalDagRunner(max_parallel=2, device="cpu").run(mk())
    res2 = LocalDagRunner(device="cpu").run(mk())
    return d, res1, res2


def test_all_components_ran_then_cached(taxi_run):
    _, r1, r2 = taxi_run
    assert r1.succeeded and len(r1.components) == 9
    assert all(c.state == "complete" for c in r1.components.values())
    assert all(c.state == "cached" for c in r2.components.values())


def test_lineage_model_to_examples(taxi_run):
    d, r1, _ = taxi_run
    md = TFXReadonlyMetadataStore.from_sqlite_db(str(d / "md" / "taxi" / "metadata.db"))
    models = md.store.get_artifacts_by_type(TFXArtifactTypes.MODEL)
    assert len(models) == 1
    ex = md.get_source_artifact_of_type(models[0].id, TFXArtifactTypes.EXAMPLES)
    assert ex is not None and "CsvExampleGen" in ex.uri or "Transform" in ex.uri
    ev = md.get_dest_artifact_of_type(models[0].id, TFXArtifactTypes.MODEL_EVAL)
    assert ev is not None
    assert md.get_execution_for_output_artifact(models[0].id, TFXExecutionTypes.TRAINER) is not None
    frame = md.get_tfma_analysis(models[0].id, "trip_start_hour")
    assert len(frame) >= 20 and "auc" in frame.columns
    g = md.get_artifact_lineage(models[0].id)
    assert g.number_of_nodes() >= 5
    df = md.get_artifacts_of_type_df(TFXArtifactTypes.EXAMPLES)
    assert set(df["split"]) == {"train", "eval"}


def test_model_quality_and_push(taxi_run):
    d, r1, _ = taxi_run
    tr = r1.components["Trainer"].outputs["output"][0]
    m = json.load(open(os.path.join(tr.uri, "metrics.json")))["eval"]
    assert m["auc"] > 0.7 and m["accuracy"] > 0.75
    pushed = os.listdir(d / "serving")
    assert len(pushed) == 1 and pushed[0].isdigit()


def test_serving_load_predicts_raw_rows(taxi_run):
    from mifx.serving import saved_model

    d, _, _ = taxi_run
    path = saved_model.latest_export(str(d / "serving"))
    m = saved_model.load(path, device="cpu")
    rows = synthetic_taxi_csv_rows(20, seed=5)
    for r in rows:
        r.pop("tips")
    out = m.predict(rows)
    p = out["probabilities"]
    assert p.shape == (20, 2) and np.allclose(p.sum(1), 1.0)
    assert set(np.unique(out["class_ids"])) <= {0, 1}
