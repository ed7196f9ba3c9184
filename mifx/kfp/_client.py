"""Pipelines API client: experiments, runs, pipeline packages.

Reference: `sdk/python/kfp/_client.py:32-316` (swagger `kfp_server_api` over the ml-pipeline REST API
v1beta1, IAP token auth, in-cluster DNS / kube-proxy host discovery, notebook links).
Here there are two backends behind the same methods:

* REST (`host='http(s)://…'` or `'host:port/pipeline'`): plain `requests` calls against
  `/apis/v1beta1/{experiments,runs,pipelines}` with optional bearer token (`client_id` -> IAP token
  via `_auth.get_auth_token`). No generated client library is needed.
* local (`host='local'` or `'local:///some/dir'`): experiments and runs are kept as JSON under a
  directory and `run_pipeline` executes the workflow on this host with
  `mifx.kfp.local.LocalWorkflowExecutor` (in a background thread; `wait_for_run_completion` joins)."""
from __future__ import annotations

import datetime as _dt
import json
import logging
import os
import tarfile
import threading
import time
import uuid
import zipfile

import yaml

from .compiler._k8s_helper import K8sHelper


class ApiObject(dict):
    """JSON response with attribute access (`run.id`, `resp.experiments[0].name`)."""

    def __getattr__(self, item):
        if item.startswith("__"):
            raise AttributeError(item)
        v = self.get(item)
        return _wrap(v)


def _wrap(v):
    if isinstance(v, dict) and not isinstance(v, ApiObject):
        return ApiObject(v)
    if isinstance(v, list):
        return [_wrap(x) for x in v]
    return v


def _now() -> str:
    return _dt.datetime.now(_dt.timezone.utc).isoformat()


class _RestBackend:
    def __init__(self, host: str, token: str | None):
        import requests

        self._s = requests.Session()
        if token:
            self._s.headers["Authorization"] = "Bearer " + token
        if not host.startswith(("http://", "https://")):
            host = "http://" + host
        self.base = host.rstrip("/") + "/apis/v1beta1"

    def _call(self, method, path, **kw):
        r = self._s.request(method, self.base + path, timeout=60, **kw)
        if r.status_code >= 400:
            raise RuntimeError(f"{method} {path}: HTTP {r.status_code}: {r.text[:500]}")
        return ApiObject(r.json() if r.content else {})

    def create_experiment(self, name, description=""):
        return self._call("POST", "/experiments", json={"name": name, "description": description})

    def get_experiment(self, eid):
        return self._call("GET", f"/experiments/{eid}")

    def list_experiments(self, page_token, page_size, sort_by):
        return self._call("GET", "/experiments", params={"page_token": page_token, "page_size": page_size,
                                                         "sort_by": sort_by})

    def create_run(self, body):
        return self._call("POST", "/runs", json=body)

    def list_runs(self, page_token, page_size, sort_by, experiment_id):
        params = {"page_token": page_token, "page_size": page_size, "sort_by": sort_by}
        if experiment_id is not None:
            params.update({"resource_reference_key.type": "EXPERIMENT", "resource_reference_key.id": experiment_id})
        return self._call("GET", "/runs", params=params)

    def get_run(self, run_id):
        return self._call("GET", f"/runs/{run_id}")

    def upload_pipeline(self, path, name):
        with open(path, "rb") as f:
            return self._call("POST", "/pipelines/upload", params={"name": name}, files={"uploadfile": f})

    def list_pipelines(self, page_token, page_size, sort_by):
        return self._call("GET", "/pipelines", params={"page_token": page_token, "page_size": page_size,
                                                       "sort_by": sort_by})


class _LocalBackend:
    """Experiments/runs/pipelines as JSON files; runs execute through the local workflow executor."""

    def __init__(self, root: str, max_parallel: int = 4, steps_factory=None):
        """steps_factory: () -> a step runner for each run (mifx.kfp.local.kube.KubeStepRunner: every step a Pod on
        the cluster); None runs the steps on this host."""
        self.root = os.path.abspath(root)
        for d in ("experiments", "runs", "pipelines"):
            os.makedirs(os.path.join(self.root, d), exist_ok=True)
        self.max_parallel = max_parallel
        self.steps_factory = steps_factory
        self.executor = "kubernetes" if steps_factory is not None else "local"
        self._threads: dict[str, threading.Thread] = {}
        self._lock = threading.Lock()

    def _path(self, kind, oid):
        return os.path.join(self.root, kind, oid + ".json")

    def _write(self, kind, obj):
        tmp = self._path(kind, obj["id"]) + ".tmp"
        with open(tmp, "w") as f:
            json.dump(obj, f, indent=1, default=str)
        os.replace(tmp, self._path(kind, obj["id"]))

    def _read(self, kind, oid):
        p = self._path(kind, oid)
        if not os.path.exists(p):
            raise ValueError(f"{kind[:-1]} {oid} not found")
        with open(p) as f:
            return json.load(f)

    def _list(self, kind, page_token, page_size, sort_by, pred=lambda o: True):
        objs = []
        for fn in os.listdir(os.path.join(self.root, kind)):
            if fn.endswith(".json"):
                with open(os.path.join(self.root, kind, fn)) as f:
                    o = json.load(f)
                if pred(o):
                    objs.append(o)
        field, desc = "created_at", False
        if sort_by:
            parts = sort_by.split()
            field, desc = parts[0], len(parts) > 1 and parts[1] == "des"
        objs.sort(key=lambda o: str(o.get(field, "")), reverse=desc)
        start = int(page_token or 0)
        page = objs[start:start + page_size]
        nxt = str(start + page_size) if start + page_size < len(objs) else None
        return ApiObject({kind: page, "total_size": len(objs), "next_page_token": nxt})

    def create_experiment(self, name, description=""):
        e = {"id": str(uuid.uuid4()), "name": name, "description": description, "created_at": _now()}
        self._write("experiments", e)
        return ApiObject(e)

    def get_experiment(self, eid):
        return ApiObject(self._read("experiments", eid))

    def list_experiments(self, page_token, page_size, sort_by):
        return self._list("experiments", page_token, page_size, sort_by)

    def create_run(self, body):
        from .local import LocalWorkflowExecutor

        spec = body["pipeline_spec"]
        if spec.get("workflow_manifest"):
            wf = json.loads(spec["workflow_manifest"])
        elif spec.get("pipeline_id"):
            wf = self._read("pipelines", spec["pipeline_id"])["workflow"]
        else:
            raise ValueError("either a pipeline package or a pipeline_id is required")
        params = {p["name"]: p["value"] for p in spec.get("parameters") or []}
        rid = str(uuid.uuid4())
        exp = next((r["key"]["id"] for r in body.get("resource_references", [])
                    if r["key"]["type"] == "EXPERIMENT"), None)
        run = {"id": rid, "name": body["name"], "status": "Running", "created_at": _now(), "experiment_id": exp,
               "pipeline_spec": {"parameters": spec.get("parameters") or [], "pipeline_id": spec.get("pipeline_id")},
               "resource_references": body.get("resource_references", [])}
        rec = {**run, "workflow": wf, "workflow_status": None}
        self._write("runs", rec)
        run_dir = os.path.join(self.root, "run_data", rid)

        def body_fn():
            try:
                steps = self.steps_factory() if self.steps_factory is not None else None
                st = LocalWorkflowExecutor(wf, run_dir, params, max_parallel=self.max_parallel, steps=steps).run()
                phase = st["phase"]
            except Exception as e:  # noqa: BLE001 - recorded as the run's failure
                st, phase = {"phase": "Error", "message": str(e)}, "Error"
            with self._lock:
                r = self._read("runs", rid)
                r.update(status=phase, finished_at=_now(), workflow_status=st)
                self._write("runs", r)

        t = threading.Thread(target=body_fn, daemon=True)
        self._threads[rid] = t
        t.start()
        return ApiObject({"run": run})

    def list_runs(self, page_token, page_size, sort_by, experiment_id):
        pred = (lambda o: o.get("experiment_id") == experiment_id) if experiment_id else (lambda o: True)
        resp = self._list("runs", page_token, page_size, sort_by, pred)
        for r in resp["runs"]:
            r.pop("workflow", None)
            r.pop("workflow_status", None)
        return resp

    def get_run(self, run_id):
        with self._lock:
            r = self._read("runs", run_id)
        wf = dict(r.pop("workflow"))
        wf["status"] = r.pop("workflow_status")
        return ApiObject({"run": r, "pipeline_runtime": {"workflow_manifest": json.dumps(wf, default=str)}})

    def join(self, run_id, timeout=None):
        t = self._threads.get(run_id)
        if t is not None:
            t.join(timeout)

    def upload_pipeline(self, path, name):
        wf = Client._extract_pipeline_yaml(path)
        p = {"id": str(uuid.uuid4()), "name": name or os.path.basename(path), "created_at": _now(), "workflow": wf,
             "parameters": wf.get("spec", {}).get("arguments", {}).get("parameters", [])}
        self._write("pipelines", p)
        return ApiObject({k: v for k, v in p.items() if k != "workflow"})

    def list_pipelines(self, page_token, page_size, sort_by):
        resp = self._list("pipelines", page_token, page_size, sort_by)
        for p in resp["pipelines"]:
            p.pop("workflow", None)
        return resp


class Client:
    """API client for Pipelines (REST or host-local backend)."""

    IN_CLUSTER_DNS_NAME = "ml-pipeline.{}.svc.cluster.local:8888"
    KUBE_PROXY_PATH = "api/v1/namespaces/{}/services/ml-pipeline:http/proxy/"

    def __init__(self, host: str | None = None, client_id: str | None = None, namespace: str = "kubeflow",
                 max_parallel: int = 4, poll_interval: float = 5.0):
        self._host = host
        self.poll_interval = poll_interval
        if host is not None and (host == "local" or host.startswith("local://")):
            root = host[len("local://"):] if host.startswith("local://") else \
                os.path.join(os.path.expanduser("~"), ".mifx", "pipelines")
            self._backend = _LocalBackend(root, max_parallel)
            return
        token = None
        if host and client_id:
            from ._auth import get_auth_token

            token = get_auth_token(client_id)
        if not host:
            host = self._discover_host(namespace)
        self._backend = _RestBackend(host, token)

    @staticmethod
    def _discover_host(namespace: str) -> str:
        if os.environ.get("KUBERNETES_SERVICE_HOST"):  # running in a pod of the cluster
            return Client.IN_CLUSTER_DNS_NAME.format(namespace)
        try:
            server = K8sHelper()._run("config", "view", "--minify", "-o", "jsonpath={.clusters[0].cluster.server}")
        except Exception:  # noqa: BLE001 - no kubectl / kubeconfig
            server = ""
        if not server:
            raise RuntimeError("No pipelines host given and no cluster found; pass host=... (or host='local')")
        return os.path.join(server, Client.KUBE_PROXY_PATH.format(namespace))

    @property
    def is_local(self) -> bool:
        return isinstance(self._backend, _LocalBackend)

    def _is_ipython(self) -> bool:
        try:
            import IPython

            return IPython.get_ipython() is not None
        except ImportError:
            return False

    def _get_url_prefix(self) -> str:
        if self._host:
            return self._host if self._host.startswith(("http://", "https://")) else "http://" + self._host
        return "/pipeline"

    def _display_link(self, what: str, path: str) -> None:
        if self._is_ipython() and not self.is_local:
            import IPython

            IPython.display.display(IPython.display.HTML(
                f'{what} link <a href="{self._get_url_prefix()}/#/{path}" target="_blank" >here</a>'))

    # ---- experiments --------------------------------------------------------------------------
    def create_experiment(self, name: str, description: str = ""):
        try:
            exp = self.get_experiment(experiment_name=name)
        except ValueError:
            exp = None
        if exp is None:
            logging.info("Creating experiment %s.", name)
            exp = self._backend.create_experiment(name, description)
        self._display_link("Experiment", f"experiments/details/{exp.id}")
        return exp

    def list_experiments(self, page_token: str = "", page_size: int = 10, sort_by: str = ""):
        return self._backend.list_experiments(page_token, page_size, sort_by)

    def get_experiment(self, experiment_id: str | None = None, experiment_name: str | None = None):
        if experiment_id is None and experiment_name is None:
            raise ValueError("Either experiment_id or experiment_name is required")
        if experiment_id is not None:
            return self._backend.get_experiment(experiment_id)
        token = ""
        while token is not None:
            resp = self.list_experiments(page_size=100, page_token=token)
            token = resp.next_page_token
            for e in resp.experiments or []:
                if e.name == experiment_name:
                    return self._backend.get_experiment(e.id)
        raise ValueError("No experiment is found with name {}.".format(experiment_name))

    # ---- pipelines ----------------------------------------------------------------------------
    @staticmethod
    def _extract_pipeline_yaml(package_file: str) -> dict:
        def choose(names):
            ys = [n for n in names if n.endswith(".yaml")]
            if not ys:
                raise ValueError("Invalid package. Missing pipeline yaml file in the package.")
            if "pipeline.yaml" in ys:
                return "pipeline.yaml"
            if len(ys) == 1:
                return ys[0]
            raise ValueError("Invalid package. There is no pipeline.yaml file and there are multiple yaml files.")

        if package_file.endswith((".tar.gz", ".tgz")):
            with tarfile.open(package_file, "r:gz") as tar:
                member = choose([m.name for m in tar if m.isfile()])
                with tar.extractfile(tar.getmember(member)) as f:
                    return yaml.safe_load(f)
        if package_file.endswith(".zip"):
            with zipfile.ZipFile(package_file) as z:
                with z.open(choose(z.namelist())) as f:
                    return yaml.safe_load(f)
        if package_file.endswith((".yaml", ".yml")):
            with open(package_file) as f:
                return yaml.safe_load(f)
        raise ValueError("The package_file " + package_file + " should ends with one of the following formats: "
                         "[.tar.gz, .tgz, .zip, .yaml, .yml]")

    def upload_pipeline(self, pipeline_package_path: str, pipeline_name: str | None = None):
        return self._backend.upload_pipeline(pipeline_package_path, pipeline_name)

    def list_pipelines(self, page_token: str = "", page_size: int = 10, sort_by: str = ""):
        return self._backend.list_pipelines(page_token, page_size, sort_by)

    # ---- runs ---------------------------------------------------------------------------------
    def run_pipeline(self, experiment_id: str, job_name: str, pipeline_package_path: str | None = None,
                     params: dict | None = None, pipeline_id: str | None = None):
        manifest = json.dumps(self._extract_pipeline_yaml(pipeline_package_path)) if pipeline_package_path else None
        body = {"name": job_name,
                "pipeline_spec": {"pipeline_id": pipeline_id, "workflow_manifest": manifest,
                                  "parameters": [{"name": K8sHelper.sanitize_k8s_name(k), "value": str(v)}
                                                 for k, v in (params or {}).items()]},
                "resource_references": [{"key": {"id": experiment_id, "type": "EXPERIMENT"},
                                         "relationship": "OWNER"}]}
        run = self._backend.create_run(body).run
        self._display_link("Run", f"runs/details/{run.id}")
        return run

    def create_run_from_pipeline_func(self, pipeline_func, arguments: dict, run_name: str | None = None,
                                      experiment_name: str | None = None):
        """Compile `pipeline_func` to a temporary package and run it."""
        import tempfile

        from .compiler import Compiler

        with tempfile.TemporaryDirectory() as d:
            pkg = os.path.join(d, "pipeline.yaml")
            Compiler().compile(pipeline_func, pkg)
            exp = self.create_experiment(experiment_name or "Default")
            name = run_name or (pipeline_func.__name__ + " " + time.strftime("%Y-%m-%d %H-%M-%S"))
            return self.run_pipeline(exp.id, name, pkg, arguments)

    def list_runs(self, page_token: str = "", page_size: int = 10, sort_by: str = "",
                  experiment_id: str | None = None):
        return self._backend.list_runs(page_token, page_size, sort_by, experiment_id)

    def get_run(self, run_id: str):
        return self._backend.get_run(run_id)

    def wait_for_run_completion(self, run_id: str, timeout: float):
        start = time.time()
        while True:
            if self.is_local:
                self._backend.join(run_id, timeout=min(5.0, max(0.0, timeout - (time.time() - start))))
            resp = self.get_run(run_id)
            status = resp.run.status
            if status is not None and status.lower() in ("succeeded", "failed", "skipped", "error"):
                return resp
            if time.time() - start > timeout:
                raise TimeoutError("Run timeout")
            logging.info("Waiting for the job to complete...")
            if not self.is_local:
                time.sleep(self.poll_interval)

    def _get_workflow_json(self, run_id: str) -> dict:
        return json.loads(self.get_run(run_id).pipeline_runtime.workflow_manifest)
