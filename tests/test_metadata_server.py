"""Metadata service (mifx.metadata.server): MLMD read API, lineage search and the run dashboard over the sqlite
store a pipeline run wrote (fastapi TestClient, no network)."""
import csv
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "examples", "taxi"))

from mifx.data.synthetic import TAXI_COLUMNS, synthetic_taxi_csv_rows  # noqa: E402
from mifx.orchestration import LocalDagRunner  # noqa: E402


@pytest.fixture(scope="module")
def client(tmp_path_factory):
    from fastapi.testclient import TestClient

    import taxi_pipeline_local as tp
    from mifx.metadata.server import create_app

    d = tmp_path_factory.mktemp("md")
    (d / "data").mkdir()
    with open(d / "data" / "data.csv", "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=TAXI_COLUMNS)
        w.writeheader()
        for r in synthetic_taxi_csv_rows(800, seed=1):
            w.writerow({k: ("" if v is None else v) for k, v in r.items()})
    p = tp.create_pipeline("taxi", str(d / "root"), str(d / "data"), str(d / "serving"), train_steps=20,
                           eval_steps=5, metadata_db_root=str(d / "md"))
    assert LocalDagRunner(device="cpu").run(p).succeeded
    return TestClient(create_app(str(d / "md" / "taxi" / "metadata.db")))


def test_types_artifacts_executions(client):
    assert client.get("/healthz").json() == {"status": "ok"}
    names = {t["name"] for t in client.get("/api/v1/artifact_types").json()}
    assert {"ExamplesPath", "ModelExportPath", "SchemaPath"} <= names
    models = client.get("/api/v1/artifacts", params={"type": "ModelExportPath"}).json()
    assert len(models) == 1 and "Trainer" in models[0]["uri"]
    assert client.get(f"/api/v1/artifacts/{models[0]['id']}").json()["id"] == models[0]["id"]
    assert client.get("/api/v1/artifacts/999999").status_code == 404
    ex = client.get("/api/v1/executions", params={"type": "trainer"}).json()
    assert len(ex) == 1
    ev = client.get("/api/v1/events", params={"execution_id": ex[0]["id"]}).json()
    assert any(e["artifact_id"] == models[0]["id"] for e in ev)


def test_lineage_search_and_dashboard(client):
    model = client.get("/api/v1/artifacts", params={"type": "ModelExportPath"}).json()[0]
    src = client.get(f"/api/v1/lineage/{model['id']}", params={"direction": "upstream",
                                                               "type": "ExamplesPath"}).json()
    assert src is not None and src["type"] == "ExamplesPath"
    dst = client.get(f"/api/v1/lineage/{model['id']}", params={"direction": "downstream",
                                                               "type": "ModelEvalPath"}).json()
    assert dst is not None
    g = client.get(f"/api/v1/lineage/{model['id']}").json()
    assert len(g["nodes"]) >= 3 and g["edges"]
    page = client.get("/").text
    assert "Pipeline runs" in page and "ModelExportPath" in page
