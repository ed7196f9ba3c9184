"""Model server (TF-Serving REST semantics), dynamic batching, version policy, tensor store."""
import os
import threading

import numpy as np
import pytest
import torch
from fastapi.testclient import TestClient

from mifx.models.cnn import FashionCNN
from mifx.models.resnet import PREPROCESS_SCRIPT, resnet50_v2
from mifx.serving.saved_model import save_module
from mifx.serving.server import DynamicBatcher, ModelManager, create_app
from mifx.serving.tensorstore import TensorStore


def _export(base, version, seed):
    torch.manual_seed(seed)
    m = FashionCNN()
    save_module(os.path.join(base, str(version)), m, "mifx.models.cnn:FashionCNN", {}, [28, 28],
                class_names=[str(i) for i in range(10)])
    return m


def test_rest_predict_versions_status_metadata(tmp_path):
    base = str(tmp_path / "fashion")
    m1 = _export(base, 1, 1)
    mgr = ModelManager("fashion", base, policy="all", device="cpu", poll_s=0)
    client = TestClient(create_app({"fashion": mgr}))
    x = np.random.default_rng(0).random((3, 28, 28)).astype(np.float32)
    r = client.post("/v1/models/fashion:predict", json={"instances": x.tolist()})
    assert r.status_code == 200
    with torch.no_grad():
        ref = m1(torch.from_numpy(x)).numpy()
    np.testing.assert_allclose(np.array(r.json()["predictions"]), ref, rtol=1e-5, atol=1e-5)
    m2 = _export(base, 2, 2)
    mgr.refresh()
    st = client.get("/v1/models/fashion").json()
    assert [s["version"] for s in st["model_version_status"]] == ["2", "1"]
    r2 = client.post("/v1/models/fashion:predict", json={"instances": x.tolist()}).json()["predictions"]
    with torch.no_grad():
        np.testing.assert_allclose(np.array(r2), m2(torch.from_numpy(x)).numpy(), rtol=1e-5, atol=1e-5)
    r1 = client.post("/v1/models/fashion/versions/1:predict", json={"inputs": x.tolist()}).json()["outputs"]
    np.testing.assert_allclose(np.array(r1), ref, rtol=1e-5, atol=1e-5)
    md = client.get("/v1/models/fashion/metadata").json()
    assert md["model_spec"]["version"] == "2" and "serving_default" in md["metadata"]["signature_def"]
    assert client.post("/v1/models/fashion/versions/7:predict", json={"instances": []}).status_code == 404
    assert client.post("/v1/models/nope:predict", json={"instances": []}).status_code == 404
    cls = client.post("/v1/models/fashion:classify", json={"examples": x.tolist()}).json()["results"]
    assert len(cls) == 3 and len(cls[0]) == 10
    metrics = client.get("/monitoring/prometheus/metrics").text
    assert 'mifx_serving_requests_total{method="predict",model="fashion",status="ok"}' in metrics
    mgr.close()


def test_latest_policy_unloads_old_versions(tmp_path):
    base = str(tmp_path / "m")
    _export(base, 1, 1)
    mgr = ModelManager("m", base, policy="latest", device="cpu", poll_s=0)
    assert list(mgr.servables) == [1]
    _export(base, 5, 5)
    mgr.refresh()
    assert list(mgr.servables) == [5]
    with pytest.raises(KeyError):
        mgr.get(1)
    mgr.close()


def test_dynamic_batcher_merges_concurrent_requests():
    calls = []

    def run(items):
        calls.append(len(items))
        a = np.asarray(items, dtype=np.float32)
        return {"y": a * 2}

    b = DynamicBatcher(run, max_batch_size=64, batch_timeout_s=0.05)
    results = {}

    def worker(i):
        results[i] = b.submit([[float(i)], [float(i) + 0.5]]).result()

    ts = [threading.Thread(target=worker, args=(i,)) for i in range(8)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    b.close()
    for i in range(8):
        np.testing.assert_allclose(results[i]["y"], [[2.0 * i], [2.0 * i + 1.0]])
    assert sum(calls) == 16 and len(calls) < 8  # merged into fewer device launches


def test_tensorstore_resnet_dag():
    ts = TensorStore()
    torch.manual_seed(0)
    m = resnet50_v2()
    ts.modelset("r50", "TORCH", "CPU", model=m)
    ts.scriptset("pp", "CPU", PREPROCESS_SCRIPT)
    img = np.random.default_rng(0).integers(0, 255, (64, 64, 3))
    ts.tensorset("img", "UINT8", [64, 64, 3], values=img)
    ts.dagrun([("SCRIPTRUN", "pp", "pre_process", ["img"], ["x"]), ("MODELRUN", "r50", ["x"], ["y"]),
               ("SCRIPTRUN", "pp", "post_process", ["y"], ["label"])])
    with torch.no_grad():
        ref = m.eval()(torch.from_numpy(img).float().div(255).permute(2, 0, 1)[None]).argmax(1) - 1
    assert ts.tensorget("label")["values"] == ref.tolist()
    assert ts.tensorget("y", "META") == {"dtype": "FLOAT", "shape": [1, 1001]}
    blob = ts.tensorget("img", "BLOB")
    ts.tensorset("img2", "UINT8", [64, 64, 3], blob=blob)
    assert ts.tensorget("img2")["values"][:5] == img.reshape(-1)[:5].tolist()
