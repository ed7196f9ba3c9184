"""Cluster execution of compiled pipelines (mifx.kfp.local.kube.KubeStepRunner: the Argo controller's role, one Pod
per step) against an in-memory Kubernetes API whose fake kubelet runs each Pod's `main` container as a local process:
volume mounts become directories (one per PVC claim, shared by every pod that mounts it; per-pod otherwise), absolute
output paths are remapped into the pod's own root, and the container's termination message is the file the step's
wrapper wrote, cut to the kubelet's 4 KB. So the tests check what a cluster would see -- the Pod specs (image, GPU
limit, PVC mounts, sidecars), the DAG order of pod creation, resource templates applied with their conditions, output
parameters handed back through the termination message -- AND that the compiled pipelines run to the same results as
on the host-local executor (taxi pipeline, condition, exit handler, recursion, VolumeOp DAG)."""
import copy
import importlib.util
import json
import os
import re
import subprocess
import sys
import threading

import pytest
import yaml

ROOT = os.path.dirname(os.path.dirname(__file__))
sys.path.insert(0, os.path.join(ROOT, "tests"))


class FakeKube:
    """Objects by REST path; Pods 'run' at creation (on the creating thread) through `kubelet`."""

    def __init__(self, root: str):
        self.root = root
        self.objs, self.logs, self.order = {}, {}, []
        self.lock = threading.Lock()
        self.n = 0

    # ---- REST surface used by KubeStepRunner
    def get(self, path):
        with self.lock:
            o = self.objs.get(path)
            return copy.deepcopy(o) if o is not None else None

    def get_text(self, path):
        return self.logs.get(path.split("/log")[0], "")

    def post(self, coll, body):
        body = copy.deepcopy(body)
        meta = body.setdefault("metadata", {})
        with self.lock:
            if not meta.get("name"):
                self.n += 1
                meta["name"] = meta.get("generateName", "obj-") + f"{self.n:05d}"
            path = f"{coll}/{meta['name']}"
            if path in self.objs:
                raise RuntimeError(f"409 Conflict: {path} exists")
            self.objs[path] = body
            self.order.append(path)
        if body["kind"] == "PersistentVolumeClaim":
            body["status"] = {"phase": "Bound", "capacity": {"storage": body["spec"]["resources"]["requests"]["storage"]}}
        elif body["kind"] == "Pod":
            self._kubelet(path, body)
        return copy.deepcopy(body)

    def patch(self, path, body, content_type):
        with self.lock:
            cur = self.objs[path]
            cur.update({k: v for k, v in body.items() if k != "metadata"})
            return copy.deepcopy(cur)

    def delete(self, path):
        with self.lock:
            self.objs.pop(path, None)

    # ---- kubelet
    def _kubelet(self, path, pod):
        name = pod["metadata"]["name"]
        proot = os.path.join(self.root, "pods", name)
        os.makedirs(proot, exist_ok=True)
        vols = {v["name"]: v for v in pod["spec"].get("volumes", [])}
        main = pod["spec"]["containers"][0]
        assert main["name"] == "main" and main["command"][:2] == ["sh", "-c"]
        remap = {}
        for m in main.get("volumeMounts", []):
            v = vols[m["name"]]  # a mount without its volume would not schedule
            if "persistentVolumeClaim" in v:
                claim = v["persistentVolumeClaim"]["claimName"]
                with self.lock:  # a PVC must exist (VolumeOp created it) unless provisioned outside the run
                    assert any(p.endswith(f"/persistentvolumeclaims/{claim}") for p in self.objs) or \
                        claim in self.preexisting, claim
                host = os.path.join(self.root, "pvcs", claim)
            else:
                host = os.path.join(proot, "vol-" + m["name"])
            os.makedirs(host, exist_ok=True)
            remap[m["mountPath"].rstrip("/")] = host
        env = {e["name"]: e["value"] for e in main.get("env", []) if "value" in e}
        for kv in env.get("MIFX_OUTPUTS", "").split():
            p = kv.split("=", 1)[1]
            if not any(p == mp or p.startswith(mp + "/") for mp in remap):
                remap[p] = os.path.join(proot, "fs", p.lstrip("/"))
        pats = sorted(remap, key=len, reverse=True)

        def fix(s):
            for mp in pats:
                s = re.sub(r"(?<![\w/.])" + re.escape(mp) + r"(?=/|$|\s|['\"])", remap[mp], s)
            return s

        for dst in remap.values():
            os.makedirs(os.path.dirname(dst), exist_ok=True)
        argv = [fix(x) for x in main["command"]]
        env = dict(os.environ, **{k: fix(v) for k, v in env.items()})
        env["PYTHONPATH"] = ROOT
        env["MIFX_TERMINATION_LOG"] = os.path.join(proot, "termination-log")
        r = subprocess.run(argv, cwd=proot, env=env, capture_output=True, text=True, timeout=600)
        try:
            with open(env["MIFX_TERMINATION_LOG"]) as f:
                msg = f.read()[:4096]
        except FileNotFoundError:
            msg = ""
        self.logs[path] = r.stdout + r.stderr
        with self.lock:
            self.objs[path]["status"] = {
                "phase": "Succeeded" if r.returncode == 0 else "Failed",
                "containerStatuses": [{"name": "main", "state": {"terminated": {
                    "exitCode": r.returncode, "message": msg, "reason": "Completed" if r.returncode == 0 else "Error"}}}]}

    preexisting: set = set()

    def pods(self):
        return [self.objs[p] for p in self.order if "/pods/" in p and p in self.objs]


def _runner(fake):
    from mifx.kfp.local.kube import KubeStepRunner

    return KubeStepRunner(fake, "kubeflow", poll_s=0.01)


def _load(path, name):
    spec = importlib.util.spec_from_file_location(name, os.path.join(ROOT, path))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def _nodes(st, template):
    return [n for n in st["nodes"].values() if n["templateName"] == template]


def test_wrapper_hands_outputs_through_the_termination_message(tmp_path):
    """The sh wrapper a step's main container runs: the step's own exit code, and one name<TAB>base64 line per
    output file that exists (decoded by the runner; a missing file is an error there)."""
    from mifx.kfp.local.kube import KubeStepRunner, wrapper_command

    out = tmp_path / "o.txt"
    term = tmp_path / "term"
    env = dict(os.environ, MIFX_OUTPUTS=f"a={out} b={tmp_path}/missing", MIFX_TERMINATION_LOG=str(term))
    r = subprocess.run(wrapper_command(["sh", "-c", f"printf 'tails\\n' > {out}; exit 3"]), env=env)
    assert r.returncode == 3
    lines = term.read_text().splitlines()
    assert len(lines) == 1 and lines[0].startswith("a\t")
    assert KubeStepRunner._outputs("s", term.read_text(), {"a": str(out)}) == {"a": "tails"}
    from mifx.kfp.local import WorkflowError

    with pytest.raises(WorkflowError, match="not written"):
        KubeStepRunner._outputs("s", term.read_text(), {"a": str(out), "b": "/x"})
    with pytest.raises(WorkflowError, match="termination message"):
        KubeStepRunner._outputs("s", "a\tAAAA@@", {"a": str(out)})


def test_resource_conditions_paths_and_jsonpath():
    from mifx.kfp.local.kube import condition_holds, json_path, resource_path

    o = {"status": {"phase": "Bound", "readyToUse": True, "succeeded": 2, "capacity": {"storage": "10Gi"}},
         "metadata": {"name": "p"}}
    assert condition_holds(o, "status.phase == Bound") and condition_holds(o, "status.readyToUse == true")
    assert condition_holds(o, "status.succeeded > 1, status.phase in (Bound, Lost)")
    assert not condition_holds(o, "status.phase notin (Bound)") and not condition_holds(o, "status.failed > 0")
    assert json_path(o, "{.status.capacity.storage}") == "10Gi" and json.loads(json_path(o, "{}")) == o
    assert resource_path({"apiVersion": "v1", "kind": "PersistentVolumeClaim"}, "ns") == \
        "/api/v1/namespaces/ns/persistentvolumeclaims"
    assert resource_path({"apiVersion": "snapshot.storage.k8s.io/v1alpha1", "kind": "VolumeSnapshot"}, "ns", "s") \
        == "/apis/snapshot.storage.k8s.io/v1alpha1/namespaces/ns/volumesnapshots/s"
    assert resource_path({"apiVersion": "batch/v1", "kind": "Job"}, "ns") == "/apis/batch/v1/namespaces/ns/jobs"


def test_volumeop_dag_creates_the_pvc_and_shares_it_between_pods(tmp_path):
    from kfp_testdata.pipelines import PIPELINES

    from mifx.kfp import compiler
    from mifx.kfp.local import LocalWorkflowExecutor

    wf = compiler.Compiler().compile_to_workflow(PIPELINES["volumeop_dag"])
    fake = _FK(str(tmp_path / "k8s"))
    st = LocalWorkflowExecutor(wf, str(tmp_path / "run"), steps=_runner(fake), timeout=300).run()
    assert st["phase"] == "Succeeded", st["message"]
    pvc = [p for p in fake.order if "/persistentvolumeclaims/" in p]
    assert len(pvc) == 1 and pvc[0].endswith("-my-pvc") and fake.order.index(pvc[0]) == 0  # created first
    pods = fake.pods()
    assert [p["metadata"]["labels"]["mifx.amd.com/step"] for p in pods][-1] == "step3"  # after step1 and step2
    claim = pvc[0].rsplit("/", 1)[1]
    for p in pods:
        assert p["spec"]["containers"][0]["image"] == "library/bash:4.4.23"
        assert p["spec"]["volumes"] == [{"name": "create-pvc", "persistentVolumeClaim": {"claimName": claim}}]
        assert p["spec"]["restartPolicy"] == "Never" and p["spec"]["serviceAccountName"] == "pipeline-runner"
    step3 = [k for k in fake.order if "/pods/" in k][-1]
    assert fake.logs[step3].split() == ["1", "2"]  # step3 reads what step1 and step2 wrote on the shared PVC
    size = _nodes(st, "create-pvc")[0]["outputs"]["parameters"]
    assert {"name": "create-pvc-size", "value": "10Gi"} in size


class _FK(FakeKube):
    preexisting = {"users-pvc"}


@pytest.mark.parametrize("name", ["condition", "exit_handler", "recursion"])
def test_basic_samples_run_as_pods(tmp_path, name):
    """The KFP basic samples with `when` conditions, an exit handler and recursion through a graph component, each
    container step a Pod; output parameters (the coin flips) come back through the termination message."""
    bs = _load("examples/kfp/basic_samples.py", "basic_samples_kube")
    from mifx.kfp.local import LocalWorkflowExecutor

    wf = bs.compiler.Compiler().compile_to_workflow(bs.SAMPLES[name])
    fake = _FK(str(tmp_path / "k8s"))
    st = LocalWorkflowExecutor(wf, str(tmp_path / "run"), steps=_runner(fake), timeout=300).run()
    assert st["phase"] == "Succeeded", st["message"]
    pods = fake.pods()
    assert pods and all(p["spec"]["containers"][0]["name"] == "main" for p in pods)
    if name == "condition":  # the flip's output decided which branch ran: the skipped ones made no pod
        flip = _nodes(st, "flip-coin")[0]["outputs"]["parameters"][0]["value"]
        assert flip in ("heads", "tails")
        ran = {p["metadata"]["labels"]["mifx.amd.com/step"] for p in pods}
        assert ran >= {"flip-coin"} and len(pods) < len(wf["spec"]["templates"])
    if name == "exit_handler":  # the exit step's pod is the last one created
        assert pods[-1]["metadata"]["annotations"]["workflows.argoproj.io/node-name"].endswith(".onExit")
    if name == "recursion":
        flips = [n for n in st["nodes"].values() if n["templateName"].startswith("flip") and n["outputs"]["parameters"]]
        assert flips[-1]["outputs"]["parameters"][0]["value"] == "tails"  # the loop ran until tails


def test_taxi_pipeline_runs_as_pods_with_gpu_limit_and_users_pvc(tmp_path):
    """The compiled KFP taxi pipeline (8 steps) on the fake cluster: every step a Pod mounting the users-pvc claim,
    the trainer's Pod asking for amd.com/gpu, DAG order respected, the same results as the host-local run."""
    from mifx.data.synthetic import TAXI_COLUMNS, synthetic_taxi_csv_rows
    from mifx.kfp.local import LocalWorkflowExecutor

    mod = _load("examples/kfp/taxi/taxi_pipeline.py", "kfp_taxi_kube")
    out = str(tmp_path / "taxi.yaml")
    mod.main(["--output", out])
    wf = yaml.safe_load(open(out))
    fake = _FK(str(tmp_path / "k8s"))
    data = tmp_path / "k8s" / "pvcs" / "users-pvc" / "taxi"
    data.mkdir(parents=True)
    import csv

    for fn, n, seed in (("train.csv", 1200, 1), ("eval.csv", 400, 2)):
        with open(data / fn, "w", newline="") as f:
            w = csv.writer(f)
            for r in synthetic_taxi_csv_rows(n, seed=seed):
                w.writerow(["" if r[c] is None else r[c] for c in TAXI_COLUMNS])
    (data / "column-names.json").write_text(json.dumps(TAXI_COLUMNS))
    (data / "preprocessing.py").write_text(open(os.path.join(ROOT, "examples/kfp/taxi/preprocessing.py")).read())
    st = LocalWorkflowExecutor(wf, str(tmp_path / "run"), {"steps": 40, "hidden_layer_size": "64"},
                               steps=_runner(fake), timeout=900).run()
    assert st["phase"] == "Succeeded", st["message"]
    pods = {p["metadata"]["labels"]["mifx.amd.com/step"]: p for p in fake.pods()}
    assert set(pods) == {"tfdv", "tft", "dnntrainer", "tfma", "predict", "confusion-matrix", "roc", "deployer"}
    for step, p in pods.items():
        c = p["spec"]["containers"][0]
        assert {"mountPath": "/mnt", "name": "local-storage"} in c["volumeMounts"], step
        assert {"name": "local-storage", "persistentVolumeClaim": {"claimName": "users-pvc"}} in p["spec"]["volumes"]
        assert c["image"] == wf["spec"]["templates"][[t["name"] for t in wf["spec"]["templates"]].index(step)][
            "container"]["image"]
    assert pods["dnntrainer"]["spec"]["containers"][0]["resources"]["limits"]["amd.com/gpu"] == "1"
    order = [p["metadata"]["labels"]["mifx.amd.com/step"] for p in fake.pods()]
    for a, b in (("tfdv", "tft"), ("tft", "dnntrainer"), ("dnntrainer", "tfma"), ("dnntrainer", "predict"),
                 ("predict", "roc"), ("predict", "confusion-matrix"), ("dnntrainer", "deployer")):
        assert order.index(a) < order.index(b), order
    auc = float(_nodes(st, "roc")[0]["outputs"]["parameters"][0]["value"])
    assert 0.5 < auc <= 1.0


def test_pipelines_api_server_runs_steps_as_pods(tmp_path):
    """The API server with the Kubernetes executor (what deploy/k8s/pipelines-api.yaml runs): a run created over REST
    executes every step as a Pod and reports the Argo status."""
    import time

    from fastapi.testclient import TestClient

    from mifx.kfp.local.kube import KubeStepRunner
    from mifx.kfp.server import create_app

    bs = _load("examples/kfp/basic_samples.py", "basic_samples_api")
    wf = bs.compiler.Compiler().compile_to_workflow(bs.SAMPLES["sequential"])
    fake = _FK(str(tmp_path / "k8s"))
    app = create_app(str(tmp_path / "api"), steps_factory=lambda: KubeStepRunner(fake, "kubeflow", poll_s=0.01))
    c = TestClient(app)
    assert c.get("/apis/v1beta1/healthz").json()["backend"] == "kubernetes"
    rid = c.post("/apis/v1beta1/runs", json={"name": "r", "pipeline_spec": {
        "workflow_manifest": json.dumps(wf), "parameters": []}}).json()["run"]["id"]
    for _ in range(600):
        run = c.get(f"/apis/v1beta1/runs/{rid}").json()
        if run["run"]["status"] not in ("Running", None):
            break
        time.sleep(0.05)
    assert run["run"]["status"] == "Succeeded", run
    assert [p["metadata"]["labels"]["mifx.amd.com/step"] for p in fake.pods()] == ["download", "echo"]
