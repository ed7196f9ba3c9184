"""Training-job specs (TFJob / PyTorchJob / MIFXJob) and the local multi-process launcher."""
import json
import sys

import pytest
import yaml

from mifx.launch import JobSpec, launch_local, to_indexed_job, validate

_WORKER = """
import json, os, sys
import torch.distributed as dist
dist.init_process_group("gloo")
t = __import__("torch").tensor([float(dist.get_rank() + 1)])
dist.all_reduce(t)
out = {"rank": dist.get_rank(), "world": dist.get_world_size(), "sum": float(t), "tf": os.environ.get("TF_CONFIG")}
open(os.path.join(sys.argv[1], f"r{dist.get_rank()}.json"), "w").write(json.dumps(out))
dist.destroy_process_group()
"""


def _job(kind, key, roles, worker, out):
    return {"apiVersion": "kubeflow.org/v1", "kind": kind, "metadata": {"name": "t"},
            "spec": {key: {role: {"replicas": n, "template": {"spec": {"containers": [
                {"name": "c", "image": "img", "command": ["python", str(worker), str(out)]}]}}} for role, n in roles}}}


def test_validation_rules():
    with pytest.raises(ValueError):
        JobSpec.from_dict({"kind": "TFJob", "spec": {"tfReplicaSpecs": {"Chief": {"replicas": 2, "template": {
            "spec": {"containers": [{"command": ["x"]}]}}}}}})
    with pytest.raises(ValueError):
        JobSpec.from_dict({"kind": "PyTorchJob", "spec": {"pytorchReplicaSpecs": {"Worker": {"replicas": 0}}}})


@pytest.mark.parametrize("kind,key,roles", [("PyTorchJob", "pytorchReplicaSpecs", [("Master", 1), ("Worker", 2)]),
                                             ("TFJob", "tfReplicaSpecs", [("Worker", 3)])])
def test_launch_local_ranks(tmp_path, kind, key, roles):
    worker = tmp_path / "w.py"
    worker.write_text(_WORKER)
    spec = JobSpec.from_dict(_job(kind, key, roles, worker, tmp_path))
    validate(spec)
    codes = launch_local(spec, num_gpus=0, timeout=120, log_dir=str(tmp_path / "logs"))
    assert all(c == 0 for c in codes.values()), codes
    outs = [json.loads((tmp_path / f"r{r}.json").read_text()) for r in range(3)]
    assert {o["rank"] for o in outs} == {0, 1, 2} and all(o["sum"] == 6.0 for o in outs)
    if kind == "TFJob":
        tf = json.loads(outs[0]["tf"])
        assert len(tf["cluster"]["worker"]) == 3 and tf["task"]["type"] == "worker"


def test_render_indexed_job(tmp_path):
    spec = JobSpec.from_yaml("deploy/k8s/wide-deep-bench-dp8-job.yaml")
    job = to_indexed_job(spec)
    c = job["spec"]["template"]["spec"]["containers"][0]
    assert "--nproc-per-node=8" in c["command"] and c["resources"]["limits"]["amd.com/gpu"] == "8"
    assert yaml.safe_load(yaml.safe_dump(job)) == job
    _ = sys


@pytest.mark.timeout(600)
def test_notebook10_distributed_training_job_runs_three_workers(tmp_path):
    import os

    from mifx.launch.job import JobSpec, launch_local

    root = os.path.join(os.path.dirname(__file__), "..")
    spec = JobSpec.from_yaml(os.path.join(root, "examples", "training-jobs", "distributed-training-job.yaml"))
    assert spec.world_size == 3
    spec.replicas[0].command = spec.replicas[0].command[:2] + ["--epochs", "1", "--steps_per_epoch", "2",
                                                               "--train_size", "3060", "--batch_size", "306",
                                                               "--weights", str(tmp_path / "w.safetensors")]
    spec.replicas[0].env["CUDA_VISIBLE_DEVICES"] = ""
    spec.replicas[0].env["OMP_NUM_THREADS"] = "2"
    codes = launch_local(spec, num_gpus=0, timeout=500, cwd=root, log_dir=str(tmp_path))
    assert set(codes.values()) == {0}, codes
    assert (tmp_path / "w.safetensors").exists()


def test_dp8_pipeline_job_runs_the_trainer_component():
    """The 8-GPU deployment runs the pipeline whose Trainer component trains data-parallel (not bench.py)."""
    import os

    job = yaml.safe_load(open("deploy/k8s/wide-deep-dp8-job.yaml"))
    c = job["spec"]["template"]["spec"]["containers"][0]
    assert c["resources"]["limits"]["amd.com/gpu"] == 8
    cmd = c["command"]
    assert cmd[1] == "examples/taxi/taxi_pipeline_local.py" and os.path.exists(cmd[1])
    assert cmd[cmd.index("--num-gpus") + 1] == "8" and "bench.py" not in cmd


def test_deploy_stack_manifests_parse_and_point_at_real_entry_points():
    """Every manifest of the stack parses; every container command that runs mifx names a module / script that
    exists in this tree (so `kubectl apply -k deploy/k8s` starts real services)."""
    import importlib.util
    import os

    root = os.path.join(os.path.dirname(__file__), "..")
    kust = yaml.safe_load(open(os.path.join(root, "deploy/k8s/kustomization.yaml")))
    assert len(kust["resources"]) >= 7
    seen = 0
    for res in kust["resources"]:
        for doc in yaml.safe_load_all(open(os.path.join(root, "deploy/k8s", res))):
            if not doc:
                continue
            spec = doc.get("spec", {})
            pod = spec.get("template", {}).get("spec", {})
            for c in pod.get("containers", []):
                cmd = c.get("command") or []
                if cmd[:2] == ["python3", "-m"] and cmd[2].startswith("mifx"):
                    assert importlib.util.find_spec(cmd[2]) is not None, cmd[2]
                    seen += 1
                elif cmd[:1] == ["python3"] and cmd[1].endswith(".py"):
                    assert os.path.exists(os.path.join(root, cmd[1])), cmd[1]
                    seen += 1
    assert seen >= 5
