"""SURVEY §7.3 minimum slice on MI355X: the 9-component taxi pipeline under LocalDagRunner(device="cuda") --
Transform analyzers on the HIP kernels (moments, vocabulary hash-count / lookup, bucketize), the Trainer on the
fused W&D kernel through the Estimator (multi-step hipGraph replays, checkpoints), the Evaluator / ModelValidator
on the segmented-reduction kernel -- against the same pipeline on the CPU (reference: airflow-dags/
taxi_pipeline.py:68-132)."""
import csv
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "examples", "taxi"))

from mifx.data.synthetic import TAXI_COLUMNS, synthetic_taxi_csv_rows  # noqa: E402
from mifx.metadata.lineage import TFXArtifactTypes, TFXExecutionTypes, TFXReadonlyMetadataStore  # noqa: E402
from mifx.orchestration import LocalDagRunner  # noqa: E402


def _loaded_native():
    with open("/proc/self/maps") as f:
        return {os.path.basename(line.split()[-1]) for line in f if "libmifx_" in line}


@pytest.mark.gpu
def test_taxi_pipeline_on_gpu_matches_cpu(tmp_path, monkeypatch):
    import mifx.transform.api as tapi
    import taxi_pipeline_local as tp

    monkeypatch.setattr(tapi, "GPU_MIN_ROWS", 0)  # every analyzer on the GPU, whatever the column size
    data = tmp_path / "data"
    data.mkdir()
    with open(data / "data.csv", "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=TAXI_COLUMNS)
        w.writeheader()
        for r in synthetic_taxi_csv_rows(6000, seed=2):
            w.writerow({k: ("" if v is None else v) for k, v in r.items()})
    out = {}
    for dev in ("cpu", "cuda"):
        p = tp.create_pipeline("taxi", str(tmp_path / dev), str(data), str(tmp_path / f"serving_{dev}"),
                               train_steps=1500, eval_steps=50, metadata_db_root=str(tmp_path / f"md_{dev}"))
        res = LocalDagRunner(device=dev).run(p)
        assert res.succeeded and all(c.state == "complete" for c in res.components.values())
        tr = res.components["Trainer"].outputs["output"][0]
        m = json.load(open(os.path.join(tr.uri, "metrics.json")))
        ev = res.components["Evaluator"].outputs["output"][0]
        out[dev] = (m, ev, res)
    libs = _loaded_native()
    assert {"libmifx_analyzers.so", "libmifx_vocab.so", "libmifx_wd_chain.so", "libmifx_wide_deep.so"} <= libs, libs
    (mc, evc, _), (mg, evg, resg) = out["cpu"], out["cuda"]
    assert abs(mg["eval"]["auc"] - mc["eval"]["auc"]) < 0.01, (mg["eval"], mc["eval"])
    assert abs(mg["eval"]["accuracy"] - mc["eval"]["accuracy"]) < 0.02
    assert abs(evg.custom_properties["auc"] - evc.custom_properties["auc"]) < 0.01
    assert mg["train_examples_per_sec"] > 0 and mg["global_step"] == 1500
    md = TFXReadonlyMetadataStore.from_sqlite_db(str(tmp_path / "md_cuda" / "taxi" / "metadata.db"))
    model = md.store.get_artifacts_by_type(TFXArtifactTypes.MODEL)[0]
    ex = md.get_source_artifact_of_type(model.id, TFXArtifactTypes.EXAMPLES)
    assert ex is not None
    assert md.get_execution_for_output_artifact(model.id, TFXExecutionTypes.TRAINER) is not None
    assert len(md.get_tfma_analysis(model.id, "trip_start_hour")) >= 20
    pushed = os.listdir(tmp_path / "serving_cuda")
    assert len(pushed) == 1
