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


# ---------------------------------------------------------------- restart policies and device visibility
_CKPT_WORKER = """
import os, sys, torch, torch.distributed as dist
out, fail_at = sys.argv[1], int(sys.argv[2])
dist.init_process_group("gloo")
rank, world = dist.get_rank(), dist.get_world_size()
w, start = torch.zeros(8, dtype=torch.float64), 0
ck = os.path.join(out, "ckpt.pt")
if os.path.exists(ck):  # resume from the latest checkpoint (what a restarted replica set does)
    st = torch.load(ck, weights_only=True)
    w, start = st["w"], int(st["step"])
for step in range(start, 10):
    g = torch.Generator().manual_seed(1000 * step + rank)
    x = torch.randn(16, 8, generator=g, dtype=torch.float64)
    grad = 2 * x.t() @ (x @ w - x.sum(1)) / 16
    dist.all_reduce(grad)
    w = w - 0.05 * grad / world
    if rank == 0:
        torch.save({"w": w, "step": step + 1}, ck + ".tmp")
        os.replace(ck + ".tmp", ck)
    dist.barrier()
    if step + 1 == fail_at and rank == 1 and os.environ["MIFX_RESTART_COUNT"] == "0":
        os._exit(3)  # injected rank failure, first attempt only
if rank == 0:
    torch.save({"w": w, "restart": os.environ["MIFX_RESTART_COUNT"]}, os.path.join(out, "final.pt"))
dist.destroy_process_group()
"""


def _ckpt_job(tmp_path, name, policy, fail_at, backoff=None):
    worker = tmp_path / "ck.py"
    worker.write_text(_CKPT_WORKER)
    out = tmp_path / name
    out.mkdir()
    d = {"kind": "PyTorchJob", "metadata": {"name": name},
         "spec": {"pytorchReplicaSpecs": {"Worker": {"replicas": 3, "restartPolicy": policy, "template": {"spec": {
             "containers": [{"name": "c", "command": ["python", str(worker), str(out), str(fail_at)]}]}}}}}}
    if backoff is not None:
        d["spec"]["runPolicy"] = {"backoffLimit": backoff}
    return JobSpec.from_dict(d), out


@pytest.mark.timeout(300)
def test_on_failure_restarts_from_checkpoint_bit_identical(tmp_path):
    import torch

    ref_spec, ref_out = _ckpt_job(tmp_path, "ref", "Never", -1)
    assert set(launch_local(ref_spec, num_gpus=0, timeout=120, log_dir=str(tmp_path / "l0")).values()) == {0}
    spec, out = _ckpt_job(tmp_path, "inj", "OnFailure", 4)
    stats = {}
    codes = launch_local(spec, num_gpus=0, timeout=200, log_dir=str(tmp_path / "l1"), backoff_s=0.05, stats=stats)
    assert set(codes.values()) == {0}, codes
    assert stats["restarts"] == 1 and stats["attempts"][0]["worker-1"] == 3
    a = torch.load(ref_out / "final.pt", weights_only=True)
    b = torch.load(out / "final.pt", weights_only=True)
    assert b["restart"] == "1" and torch.equal(a["w"], b["w"])  # resumed run == uninterrupted run, bit for bit


@pytest.mark.timeout(300)
def test_never_fails_fast_and_backoff_limit_is_honoured(tmp_path):
    spec, out = _ckpt_job(tmp_path, "never", "Never", 4)
    stats = {}
    codes = launch_local(spec, num_gpus=0, timeout=120, log_dir=str(tmp_path / "l"), stats=stats)
    assert codes["worker-1"] == 3 and stats["restarts"] == 0 and not (out / "final.pt").exists()
    # backoffLimit 0: OnFailure but no restart allowed
    spec, out = _ckpt_job(tmp_path, "bl0", "OnFailure", 4, backoff=0)
    assert spec.backoff_limit == 0
    codes = launch_local(spec, num_gpus=0, timeout=120, log_dir=str(tmp_path / "l2"), stats=stats)
    assert codes["worker-1"] == 3 and stats["restarts"] == 0


def test_exit_code_policy_restarts_only_retryable_codes():
    from mifx.launch.job import ReplicaSpec, _wants_restart

    r = ReplicaSpec("Worker", 2, ["x"], restart_policy="ExitCode")
    spec = JobSpec("PyTorchJob", "t", [r])
    roles = {"worker-0": r, "worker-1": r}
    assert _wants_restart(spec, {"worker-0": 0, "worker-1": 137}, roles)  # SIGKILL / OOM: retryable
    assert not _wants_restart(spec, {"worker-0": 0, "worker-1": 1}, roles)  # the program's own failure
    assert not _wants_restart(spec, {"worker-0": 0, "worker-1": 0}, roles)
    with pytest.raises(ValueError):
        validate(JobSpec("PyTorchJob", "t", [ReplicaSpec("Worker", 1, ["x"], restart_policy="Sometimes")]))


_ENV_WORKER = """
import json, os, sys
keys = ("RANK", "LOCAL_RANK", "LOCAL_WORLD_SIZE", "HIP_VISIBLE_DEVICES")
open(os.path.join(sys.argv[1], "env" + os.environ["RANK"] + ".json"), "w").write(
    json.dumps({k: os.environ.get(k) for k in keys}))
"""


@pytest.mark.parametrize("isolate", [False, True])
def test_data_parallel_ranks_see_every_gpu(tmp_path, monkeypatch, isolate):
    """A DP job's ranks must see all the node's GPUs (xGMI peer mapping, RCCL P2P) and pick theirs by LOCAL_RANK;
    one-device isolation is opt-in (independent trials)."""
    monkeypatch.delenv("HIP_VISIBLE_DEVICES", raising=False)
    worker = tmp_path / "env.py"
    worker.write_text(_ENV_WORKER)
    spec = JobSpec.from_dict(_job("PyTorchJob", "pytorchReplicaSpecs", [("Master", 1), ("Worker", 3)], worker,
                                  tmp_path))
    codes = launch_local(spec, num_gpus=8, timeout=60, log_dir=str(tmp_path / "logs"), isolate_gpus=isolate)
    assert set(codes.values()) == {0}
    envs = [json.loads((tmp_path / f"env{r}.json").read_text()) for r in range(4)]
    for r, e in enumerate(envs):
        if isolate:
            assert e["HIP_VISIBLE_DEVICES"] == str(r) and e["LOCAL_RANK"] == "0"
        else:
            assert e["HIP_VISIBLE_DEVICES"] is None and e["LOCAL_RANK"] == str(r) and e["LOCAL_WORLD_SIZE"] == "4"


# ---------------------------------------------------------------- job operator (CR -> replica set, status)
def test_operator_local_backend_runs_crs_and_reports_status(tmp_path):
    import time as _time

    from mifx.launch import operator as op

    worker = tmp_path / "w.py"
    worker.write_text(_WORKER)
    out = tmp_path / "out"
    out.mkdir()
    crs = tmp_path / "crs"
    crs.mkdir()
    ok = _job("PyTorchJob", "pytorchReplicaSpecs", [("Master", 1), ("Worker", 2)], worker, out)
    ok["metadata"]["name"] = "good"
    bad = {"kind": "MIFXJob", "metadata": {"name": "bad"}, "spec": {"replicaSpecs": {"Worker": {
        "replicas": 2, "restartPolicy": "Never",
        "template": {"spec": {"containers": [{"command": ["python", "-c", "import sys; sys.exit(4)"]}]}}}}}}
    invalid = {"kind": "TFJob", "metadata": {"name": "invalid"}, "spec": {"tfReplicaSpecs": {"Chief": {
        "replicas": 2, "template": {"spec": {"containers": [{"command": ["x"]}]}}}}}}
    for cr in (ok, bad, invalid):
        (crs / f"{cr['metadata']['name']}.yaml").write_text(yaml.safe_dump(cr))
    be = op.LocalBackend(str(crs), num_gpus=0)
    deadline = _time.time() + 120
    while op.reconcile_all(be) and _time.time() < deadline:
        _time.sleep(0.2)
    st = {n: s for n, _, s in be.list()}
    assert st["good"]["phase"] == "Succeeded" and [c["type"] for c in st["good"]["conditions"]] == \
        ["Created", "Running", "Succeeded"]
    assert st["bad"]["phase"] == "Failed" and set(st["bad"]["exitCodes"].values()) <= {4, -9}
    assert st["invalid"]["phase"] == "Failed" and st["invalid"]["conditions"][-1]["reason"] == "InvalidSpec"
    assert {json.loads((out / f"r{r}.json").read_text())["sum"] for r in range(3)} == {6.0}


def test_operator_kube_backend_creates_job_and_mirrors_status():
    from mifx.launch import operator as op

    class FakeApi:
        def __init__(self):
            self.objs, self.status = {}, {}

        def get(self, path):
            if path.endswith("/mifxjobs"):
                return {"items": [self.cr]}
            if path.endswith(("/tfjobs", "/pytorchjobs")):
                return None
            return self.objs.get(path)

        def post(self, path, body):
            self.objs[f"{path}/{body['metadata']['name']}"] = body
            return body

        def patch_status(self, path, status):
            self.status[path] = status
            self.cr["status"] = status

    api = FakeApi()
    api.cr = {"kind": "MIFXJob", "metadata": {"name": "dp8", "uid": "u1"}, "spec": {
        "runPolicy": {"backoffLimit": 2},
        "replicaSpecs": {"Worker": {"replicas": 8, "restartPolicy": "OnFailure", "template": {"spec": {"containers": [
            {"image": "img", "command": ["python3", "bench.py", "--gpus", "8"],
             "resources": {"limits": {"amd.com/gpu": 1}}}]}}}}}}
    be = op.KubeBackend(api, "kubeflow")
    assert op.reconcile_all(be) == 1
    job = api.objs["/apis/batch/v1/namespaces/kubeflow/jobs/dp8"]
    c = job["spec"]["template"]["spec"]["containers"][0]
    assert "--nproc-per-node=8" in c["command"] and c["resources"]["limits"]["amd.com/gpu"] == "8"
    assert job["spec"]["backoffLimit"] == 2 and job["metadata"]["ownerReferences"][0]["uid"] == "u1"
    assert api.cr["status"]["phase"] == "Created"
    op.reconcile_all(be)  # no Job status yet: nothing changes, no second Job
    assert len(api.objs) == 1
    job["status"] = {"active": 1}
    op.reconcile_all(be)
    assert api.cr["status"]["phase"] == "Running"
    job["status"] = {"failed": 1, "active": 1}
    op.reconcile_all(be)
    assert api.cr["status"]["phase"] == "Restarting" and api.cr["status"]["restarts"] == 1
    job["status"] = {"succeeded": 1, "failed": 1}
    assert op.reconcile_all(be) == 1  # (the pass that observes success)
    assert api.cr["status"]["phase"] == "Succeeded"
    assert op.reconcile_all(be) == 0


def test_central_dashboard_reports_live_services(tmp_path):
    """The dashboard probes each service: one that answers is 'up', one that does not is 'down'."""
    import threading

    import uvicorn
    from fastapi.testclient import TestClient

    from mifx import dashboard
    from mifx.board.server import create_app as board_app

    import socket as _s
    with _s.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    srv = uvicorn.Server(uvicorn.Config(board_app(str(tmp_path)), host="127.0.0.1", port=port, log_level="error"))
    t = threading.Thread(target=srv.run, daemon=True)
    t.start()
    import time as _time
    for _ in range(100):
        if srv.started:
            break
        _time.sleep(0.05)
    try:
        services = [("board", "scalars", f"http://127.0.0.1:{port}/healthz", "/tensorboard/"),
                    ("gone", "nothing listens", "http://127.0.0.1:9/healthz", "/gone/"),
                    ("tracking", "files", None, "/tracking/")]
        c = TestClient(dashboard.create_app(services))
        st = {s["name"]: s["state"] for s in c.get("/api/services").json()["services"]}
        assert st == {"board": "up", "gone": "down", "tracking": "static"}
        assert "board" in c.get("/").text
    finally:
        srv.should_exit = True
        t.join(5)


def test_reverse_proxy_and_bootstrap_cover_every_service():
    """deploy/nginx.conf routes every local service of the dashboard's list and the bootstrap script starts them
    (and parses as bash)."""
    import os
    import re
    import subprocess

    from mifx import dashboard

    root = os.path.join(os.path.dirname(__file__), "..")
    conf = open(os.path.join(root, "deploy/nginx.conf")).read()
    for _, _, _, link in dashboard.SERVICES:
        assert re.search(r"location\s+" + re.escape(link) + r"\s", conf), link
    boot = os.path.join(root, "deploy/scripts/bootstrap-node.sh")
    subprocess.run(["bash", "-n", boot], check=True)
    text = open(boot).read()
    for mod in ("mifx.dashboard", "mifx.kfp.server", "mifx.metadata.server", "mifx.board", "mifx.notebook_server",
                "mifx.launch.operator", "mifx.serving.resp_server", "mifx.serving.server"):
        assert mod in text, mod
    assert "kubectl apply -k" in text and "mifxjob-crd.yaml" in text


def test_operator_local_studyjob_and_notebook(tmp_path):
    """Katib StudyJob CR -> a hyper-parameter study (trials parse `name=value` metrics from their logs), status
    Succeeded with the best trial; Notebook CR -> a supervised notebook server that answers on its port and is
    restarted if it exits."""
    import socket
    import sys
    import time as _time

    import requests

    from mifx.launch import operator as op

    crs = tmp_path / "crs"
    crs.mkdir()
    trial = "import sys; lr = float(sys.argv[1].split('=')[1]); print(f'accuracy={1 - abs(lr - 0.02):.6f}')"
    study = {"apiVersion": "kubeflow.org/v1alpha1", "kind": "StudyJob", "metadata": {"name": "random-search"},
             "spec": {"studyName": "random-search", "optimizationtype": "maximize", "objectivevaluename": "accuracy",
                      "optimizationgoal": 0.9999, "requestcount": 2, "metricsnames": ["accuracy"],
                      "parameterconfigs": [{"name": "--lr", "parametertype": "double",
                                            "feasible": {"min": "0.01", "max": "0.03"}}],
                      "suggestionSpec": {"suggestionAlgorithm": "random", "requestNumber": 3},
                      "workerSpec": {"command": [sys.executable, "-c", trial]}}}
    with socket.socket() as s_:
        s_.bind(("127.0.0.1", 0))
        port = s_.getsockname()[1]
    nb = {"apiVersion": "kubeflow.org/v1alpha1", "kind": "Notebook", "metadata": {"name": "nb"},
          "spec": {"template": {"spec": {"containers": [{"ports": [{"containerPort": port}]}]}}}}
    for cr in (study, nb):
        (crs / f"{cr['metadata']['name']}.yaml").write_text(yaml.safe_dump(cr))
    be = op.LocalBackend(str(crs), num_gpus=0)
    try:
        deadline = _time.time() + 120
        while op.reconcile_all(be) and _time.time() < deadline:
            _time.sleep(0.2)
        st = {n: s for n, _, s in be.list()}
        s = st["random-search"]
        assert s["phase"] == "Succeeded" and s["trials"] == 6, s
        assert s["bestTrial"]["metrics"]["accuracy"] > 0.99 and "--lr" in s["bestTrial"]["parameters"]
        assert st["nb"]["phase"] == "Running" and st["nb"]["url"].endswith(f":{port}/")
        ok = False
        for _ in range(100):
            try:
                ok = requests.get(f"http://127.0.0.1:{port}/api/notebooks", timeout=2).status_code == 200
                break
            except requests.RequestException:
                _time.sleep(0.3)
        assert ok
        be._procs["nb"].terminate()  # the server exits: the next pass restarts it
        be._procs["nb"].wait(timeout=10)
        op.reconcile_all(be)
        st = {n: s for n, _, s in be.list()}
        assert st["nb"]["restarts"] == 1 and st["nb"]["phase"] == "Running"
        assert be._procs["nb"].poll() is None
    finally:
        be.stop()


def test_operator_kube_backend_studyjob_and_notebook():
    from mifx.launch import operator as op

    class FakeApi:
        def __init__(self, crs):
            self.objs, self.crs = {}, crs

        def get(self, path):
            for plural, kind in (("/studyjobs", "StudyJob"), ("/notebooks", "Notebook")):
                if path.endswith(plural):
                    return {"items": [c for c in self.crs if c["kind"] == kind]}
            if path.endswith(("/mifxjobs", "/tfjobs", "/pytorchjobs")):
                return None
            return self.objs.get(path)

        def post(self, path, body):
            self.objs[f"{path}/{body['metadata']['name']}"] = body
            return body

        def patch_status(self, path, status):
            for c in self.crs:
                if path.endswith(f"/{c['metadata']['name']}"):
                    c["status"] = status

    study = {"kind": "StudyJob", "metadata": {"name": "s1", "uid": "u2"},
             "spec": {"studyName": "s1", "objectivevaluename": "accuracy", "requestcount": 1,
                      "parameterconfigs": [{"name": "--lr", "parametertype": "double",
                                            "feasible": {"min": "0.01", "max": "0.03"}}],
                      "workerSpec": {"command": ["python3", "train.py"]}}}
    nb = {"kind": "Notebook", "metadata": {"name": "nb1", "uid": "u3"}, "spec": {}}
    api = FakeApi([study, nb])
    be = op.KubeBackend(api, "kubeflow", image="img")
    op.reconcile_all(be)
    job = api.objs["/apis/batch/v1/namespaces/kubeflow/jobs/s1"]
    cmd = job["spec"]["template"]["spec"]["containers"][0]["command"]
    assert cmd[:4] == ["python3", "-m", "mifx.hpo.study", "--spec-json"]
    assert json.loads(cmd[4])["spec"]["studyName"] == "s1" and study["status"]["phase"] == "Created"
    dep = api.objs["/apis/apps/v1/namespaces/kubeflow/deployments/nb1"]
    assert dep["spec"]["template"]["spec"]["containers"][0]["ports"][0]["containerPort"] == 8888
    assert "/api/v1/namespaces/kubeflow/services/nb1" in api.objs and nb["status"]["phase"] == "Created"
    dep["status"] = {"readyReplicas": 1}
    job["status"] = {"succeeded": 1}
    op.reconcile_all(be)
    assert nb["status"]["phase"] == "Running" and study["status"]["phase"] == "Succeeded"
