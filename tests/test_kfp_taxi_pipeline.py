"""KFP taxi pipeline (8 container steps) compiled and executed on this host by the local executor."""
import csv
import json
import os

import pytest
import yaml

from mifx.data.synthetic import TAXI_COLUMNS, synthetic_taxi_csv_rows

ROOT = os.path.dirname(os.path.dirname(__file__))
REF_TAXI = "/root/reference/kubeflow-pipelines/taxi"


def _write_csv(path, rows):
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        for r in rows:
            w.writerow(["" if r[c] is None else r[c] for c in TAXI_COLUMNS])


def _load_example():
    import importlib.util

    spec = importlib.util.spec_from_file_location("kfp_taxi", os.path.join(ROOT, "examples/kfp/taxi/taxi_pipeline.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_component_specs_roundtrip(tmp_path):
    from mifx import kfp_components

    paths = kfp_components.write_specs(str(tmp_path))
    assert len(paths) == 8
    for n in kfp_components.NAMES:
        op = kfp_components.load(n)
        assert op.component_spec.implementation.container.command[:3] == ["python3", "-m", "mifx.kfp_components.taxi"]


def test_taxi_pipeline_compiles_with_amd_gpu_and_pvc(tmp_path):
    mod = _load_example()
    out = str(tmp_path / "taxi.yaml")
    mod.main(["--output", out])
    wf = yaml.safe_load(open(out))
    t = {x["name"]: x for x in wf["spec"]["templates"]}
    assert set(t) >= {"tfdv", "tft", "dnntrainer", "tfma", "predict", "confusion-matrix", "roc", "deployer"}
    assert t["dnntrainer"]["container"]["resources"]["limits"]["amd.com/gpu"] == "1"
    assert any(v["name"] == "local-storage" for v in wf["spec"]["volumes"])


def _run(tmp_path, data_dir, steps, hidden, num_gpus=1):
    mod = _load_example()
    return mod.main(["--output", str(tmp_path / "p.yaml"), "--run-local", "--data-dir", data_dir,
                     "--work-dir", str(tmp_path / "work"), "--steps", str(steps), "--hidden", hidden,
                     "--num-gpus", str(num_gpus)])


def _outputs(st, template):
    return [n for n in st["nodes"].values() if n["templateName"] == template][0]["outputs"]["parameters"]


def test_taxi_pipeline_runs_locally_on_synthetic_csv(tmp_path):
    data = tmp_path / "data"
    data.mkdir()
    _write_csv(data / "train.csv", synthetic_taxi_csv_rows(1200, seed=1))
    _write_csv(data / "eval.csv", synthetic_taxi_csv_rows(400, seed=2))
    (data / "column-names.json").write_text(json.dumps(TAXI_COLUMNS))
    st = _run(tmp_path, str(data), 40, "64")
    assert st["phase"] == "Succeeded", st["message"]
    auc = float(_outputs(st, "roc")[0]["value"])
    acc = float(_outputs(st, "confusion-matrix")[0]["value"])
    assert 0.5 < auc <= 1.0 and 0.5 < acc <= 1.0
    manifest = _outputs(st, "deployer")[0]["value"]
    docs = list(yaml.safe_load_all(open(manifest)))
    assert docs[0]["kind"] == "Deployment" and docs[1]["spec"]["type"] == "NodePort"


def test_taxi_pipeline_dnntrainer_data_parallel_two_ranks(tmp_path, monkeypatch):
    """--num-gpus 2: the dnntrainer step launches two ranks of itself (gloo on this CPU host; on GPUs: one
    per device, sparse backward-state all-gather) and the rest of the pipeline consumes rank 0's export."""
    monkeypatch.setenv("CUDA_VISIBLE_DEVICES", "")
    data = tmp_path / "data"
    data.mkdir()
    _write_csv(data / "train.csv", synthetic_taxi_csv_rows(1200, seed=1))
    _write_csv(data / "eval.csv", synthetic_taxi_csv_rows(400, seed=2))
    (data / "column-names.json").write_text(json.dumps(TAXI_COLUMNS))
    st = _run(tmp_path, str(data), 30, "64", num_gpus=2)
    assert st["phase"] == "Succeeded", st["message"]
    wf = yaml.safe_load(open(tmp_path / "p.yaml"))
    t = {x["name"]: x for x in wf["spec"]["templates"]}
    assert t["dnntrainer"]["container"]["resources"]["limits"]["amd.com/gpu"] == "2"
    logs = [p for p in (tmp_path / "work").rglob("rank1.log")]
    assert logs, "no rank logs"
    assert 0.5 < float(_outputs(st, "roc")[0]["value"]) <= 1.0


@pytest.mark.skipif(not os.path.exists(os.path.join(REF_TAXI, "train.csv")), reason="reference data not present")
def test_taxi_pipeline_on_reference_csv(tmp_path):
    """The reference's own train/eval CSVs (10k/5k Chicago-taxi rows; read as text only)."""
    st = _run(tmp_path, REF_TAXI, 300, "128")
    assert st["phase"] == "Succeeded", st["message"]
    assert float(_outputs(st, "roc")[0]["value"]) > 0.8


def test_target_lambda_whitelist():
    from mifx.kfp_components.taxi import _compile_target_lambda

    f = _compile_target_lambda("lambda x: (x['target'] > x['fare'] * 0.2)")
    assert f({"target": 3.0, "fare": 10.0}) is True
    assert _compile_target_lambda("lambda x: math.sqrt(abs(x)) if x else 0.0")(-4) == 2.0
    for bad in ("lambda x: ().__class__.__base__.__subclasses__()", "lambda x: open(x)", "__import__('os')",
                "lambda x: [y for y in x]", "lambda x: math.__dict__", "lambda x: (lambda: 1)()"):
        with pytest.raises((ValueError, SyntaxError)):
            _compile_target_lambda(bad)
