"""Data-parallel Trainer component (custom_config num_gpus): N ranks launched by the component, each training
its shard of every global batch, must equal one process on the global batch (CPU: gloo ranks)."""
import csv
import os
import sys

import numpy as np
import pytest
import torch
from safetensors.torch import load_file

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "examples", "taxi"))

from mifx.data.synthetic import TAXI_COLUMNS, synthetic_taxi_csv_rows  # noqa: E402
from mifx.orchestration import LocalDagRunner  # noqa: E402
from mifx.trainer.estimator import shard_records  # noqa: E402


def test_shard_records_interleaves_global_batches():
    r = torch.arange(2 * 3 * 5 + 4)
    shards = [shard_records(r, k, 3, 5) for k in range(3)]
    for i in range(2):  # step i of rank k == slice k of global batch i
        glob = r[i * 15:(i + 1) * 15]
        assert torch.equal(torch.cat([s[i * 5:(i + 1) * 5] for s in shards]), glob)
    assert sum(len(s) for s in shards) == 30  # remainder dropped


def _csv(d, n=2500):
    data = d / "data"
    data.mkdir()
    with open(data / "data.csv", "w", newline="") as f:
        w = csv.DictWriter(f, fieldnames=TAXI_COLUMNS)
        w.writeheader()
        for r in synthetic_taxi_csv_rows(n, seed=1):
            w.writerow({k: ("" if v is None else v) for k, v in r.items()})
    return data


def _run(d, data, name, num_gpus, batch, device, steps=25):
    import taxi_pipeline_local as tp

    p = tp.create_pipeline(name, str(d / name), str(data), str(d / f"serving_{name}"), train_steps=steps,
                           eval_steps=10, metadata_db_root=str(d / f"md_{name}"), batch_size=batch,
                           num_gpus=num_gpus)
    res = LocalDagRunner(device=device).run(p)
    assert res.succeeded
    tr = res.components["Trainer"].outputs["output"][0]
    ck = [f for f in os.listdir(os.path.join(tr.uri, "serving_model_dir")) if f.startswith("ckpt-")]
    assert ck == [f"ckpt-{steps}.safetensors"]
    return tr, load_file(os.path.join(tr.uri, "serving_model_dir", ck[0]))


def test_dp_trainer_component_equals_single_process_global_batch(tmp_path):
    data = _csv(tmp_path)
    tr1, one = _run(tmp_path, data, "single", 1, 40, "cpu")
    tr2, dp = _run(tmp_path, data, "dp2", 2, 20, "cpu")
    assert tr2.custom_properties["num_replicas"] == 2
    assert set(one) == set(dp)
    for k in one:  # same examples per step, gradients summed across ranks: fp32 summation order only
        np.testing.assert_allclose(dp[k].numpy(), one[k].numpy(), rtol=2e-4, atol=2e-5, err_msg=k)
    assert abs(tr2.custom_properties["eval_auc"] - tr1.custom_properties["eval_auc"]) < 1e-3


@pytest.mark.gpu
def test_dp_trainer_component_gpu_shared_rehearsal(tmp_path, monkeypatch):
    """2 ranks sharing cuda:0 (the multi-GPU flow on a 1-GPU box): the fused W&D step with the xGMI exchange in
    multi-step hipGraphs, launched by the component. The replicas must end bit-identical, and match one
    process on the global batch to fp32 summation order."""
    monkeypatch.setenv("MIFX_SHARED_GPU", "1")
    monkeypatch.setenv("MIFX_DIST_BACKEND", "gloo")
    import taxi_pipeline_local as tp

    data = _csv(tmp_path)
    one_tr, _ = _run(tmp_path, data, "single", 1, 40, "cuda", steps=300)
    p = tp.create_pipeline("dp2", str(tmp_path / "dp2"), str(data), str(tmp_path / "serving_dp2"), train_steps=300,
                           eval_steps=10, metadata_db_root=str(tmp_path / "md_dp2"), batch_size=20, num_gpus=2)
    trainer = next(c for c in p.components if c.id == "Trainer")
    trainer.exec_properties["custom_config"]["dump_replicas_dir"] = str(tmp_path / "replicas")
    res = LocalDagRunner(device="cuda").run(p)
    assert res.succeeded
    r0 = torch.load(tmp_path / "replicas" / "replica0.pt", weights_only=True)
    r1 = torch.load(tmp_path / "replicas" / "replica1.pt", weights_only=True)
    for k in r0:
        assert torch.equal(r0[k], r1[k]), k
    tr = res.components["Trainer"].outputs["output"][0]
    # (weights: bf16 MFMA + another fp32 association of the gradient sum; FTRL's threshold makes single weights
    # flip on last-bit differences, so the two runs are compared on their evaluation)
    # (400 evaluation examples: an AUC step is ~1/(pos x neg) per swapped pair; bf16 runs differ by a few pairs)
    assert abs(tr.custom_properties["eval_auc"] - one_tr.custom_properties["eval_auc"]) < 0.015
    log = open(os.path.join(tr.uri, "dp_run", "rank0.log")).read()
    assert "xGMI exchange unavailable" not in log
