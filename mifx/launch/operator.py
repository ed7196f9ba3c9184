"""Training-job operator: reconciles MIFXJob / TFJob / PyTorchJob custom resources into running replica sets.

Reference: the Kubeflow tf-job-operator / pytorch-operator the workshop installs (`install-kubeflow/app.yaml:15-27`,
CRD `infrastructure/crd/tfjob-crd-v1.yaml`), which watch job CRs, create the replica pods, restart them per
`restartPolicy` and report `status.conditions` (Created / Running / Restarting / Succeeded / Failed). Two backends:

  * `KubeBackend` -- the Kubernetes REST API through the pod's service account (no client library needed): each new
    CR becomes the single-node batch/v1 Job of `mifx.launch.job.to_indexed_job` (one pod, all GPUs of the node, one
    rank per GPU under torch.distributed.run; restartPolicy OnFailure / Always / ExitCode -> the Job's backoffLimit,
    Never -> 0), owned by the CR, and the Job's status is mirrored into the CR's status subresource.
    Deployed by `deploy/k8s/mifxjob-operator.yaml` (ServiceAccount + RBAC + Deployment).
  * `LocalBackend` -- CRs as YAML files in a directory (the single-node stand-in for the API server): each is run by
    `launch_local` (restart semantics included) on a worker thread and its status written next to it as JSON.

It also reconciles the two other controllers of the reference's Kubeflow app (`install-kubeflow/app.yaml:15-27`):
  * Katib `StudyJob` (`notebooks/hyperparameter-tuning/random-search-job.yaml`) -> a hyper-parameter study
    (mifx.hpo.study.StudyRunner: rounds of parallel trials, one GPU each); local: a worker thread, Kubernetes: a
    batch/v1 Job running the study on one node; status Succeeded / Failed with the best trial;
  * `Notebook` (the notebook-controller's CR) -> the notebook server (mifx.notebook_server); local: a supervised
    process (restarted if it exits), Kubernetes: a Deployment + Service; status Running with its URL.

`python -m mifx.launch.operator --local DIR` / `--kube [--namespace NS]` runs the control loop."""
from __future__ import annotations

import json
import os
import threading
import time

import yaml

from .job import JobSpec, launch_local, to_indexed_job

KINDS = {"MIFXJob": ("mifx.amd.com", "v1", "mifxjobs"), "TFJob": ("kubeflow.org", "v1", "tfjobs"),
         "PyTorchJob": ("kubeflow.org", "v1", "pytorchjobs"), "StudyJob": ("kubeflow.org", "v1alpha1", "studyjobs"),
         "Notebook": ("kubeflow.org", "v1alpha1", "notebooks")}
TERMINAL = ("Succeeded", "Failed")
JOB_KINDS = ("MIFXJob", "TFJob", "PyTorchJob")


def notebook_port(cr: dict) -> int:
    """The container port of a Notebook CR (spec.template.spec.containers[0].ports[0].containerPort, default 8888)."""
    try:
        return int(cr["spec"]["template"]["spec"]["containers"][0]["ports"][0]["containerPort"])
    except (KeyError, IndexError, TypeError, ValueError):
        return int((cr.get("spec") or {}).get("port", 8888))


def study_summary(res: dict) -> dict:
    best = res.get("best")
    return {"trials": len(res.get("trials", [])), "goalReached": bool(res.get("goal_reached")),
            "bestTrial": None if best is None else {"name": best["trial"], "parameters": best["params"],
                                                     "metrics": best["metrics"]}}


def _now() -> str:
    return time.strftime("%Y-%m-%dT%H:%M:%SZ", time.gmtime())


def _condition(status: dict, ctype: str, reason: str, message: str = "") -> dict:
    """Append a condition (TFJob status convention: the last condition is the current phase)."""
    conds = status.setdefault("conditions", [])
    if not conds or conds[-1]["type"] != ctype:
        conds.append({"type": ctype, "status": "True", "reason": reason, "message": message,
                      "lastTransitionTime": _now()})
    status["phase"] = ctype
    return status


def phase(status: dict | None) -> str | None:
    return (status or {}).get("phase")


# ---------------------------------------------------------------- local backend
class LocalBackend:
    """CRs are `<dir>/<name>.yaml`; status goes to `<dir>/<name>.status.json`; logs under `<dir>/logs/<name>/`."""

    def __init__(self, root: str, num_gpus: int | None = None, cwd: str | None = None):
        self.root, self.num_gpus, self.cwd = root, num_gpus, cwd
        self._threads: dict[str, threading.Thread] = {}
        self._procs: dict[str, object] = {}  # Notebook name -> its server process

    def _status_path(self, name: str) -> str:
        return os.path.join(self.root, f"{name}.status.json")

    def list(self) -> list[tuple[str, dict, dict | None]]:
        out = []
        for fn in sorted(os.listdir(self.root)):
            if not fn.endswith((".yaml", ".yml")):
                continue
            with open(os.path.join(self.root, fn)) as f:
                cr = yaml.safe_load(f)
            if not isinstance(cr, dict) or cr.get("kind") not in KINDS:
                continue
            name = cr.get("metadata", {}).get("name") or os.path.splitext(fn)[0]
            st = None
            if os.path.exists(self._status_path(name)):
                with open(self._status_path(name)) as f:
                    st = json.load(f)
            out.append((name, cr, st))
        return out

    def set_status(self, name: str, status: dict) -> None:
        tmp = self._status_path(name) + ".tmp"
        with open(tmp, "w") as f:
            json.dump(status, f, indent=1)
        os.replace(tmp, self._status_path(name))

    def reconcile(self, name: str, cr: dict, status: dict | None) -> None:
        kind = cr.get("kind")
        if kind == "Notebook":
            return self._reconcile_notebook(name, cr, status)
        if phase(status) in TERMINAL or name in self._threads:
            return
        if kind == "StudyJob":
            return self._reconcile_study(name, cr)
        try:
            spec = JobSpec.from_dict(cr)
        except ValueError as e:
            self.set_status(name, _condition({}, "Failed", "InvalidSpec", str(e)))
            return
        st = _condition(_condition({"startTime": _now()}, "Created", "JobCreated"), "Running", "JobRunning")
        self.set_status(name, st)

        def run():
            stats: dict = {}
            codes = launch_local(spec, num_gpus=self.num_gpus, cwd=self.cwd,
                                 log_dir=os.path.join(self.root, "logs", name), stats=stats)
            st2 = dict(st, restarts=stats.get("restarts", 0), exitCodes=codes, completionTime=_now())
            if stats.get("restarts"):
                _condition(st2, "Restarting", "JobRestarting", f"{stats['restarts']} restart(s) of the replica set")
            ok = all(c == 0 for c in codes.values())
            _condition(st2, "Succeeded" if ok else "Failed", "JobSucceeded" if ok else "JobFailed",
                       "" if ok else f"replica exit codes {codes}")
            self.set_status(name, st2)

        t = threading.Thread(target=run, daemon=True)
        self._threads[name] = t
        t.start()

    def _reconcile_study(self, name: str, cr: dict) -> None:
        from ..hpo.study import StudyRunner, StudySpec

        try:
            spec = StudySpec.from_dict(cr)
        except (KeyError, ValueError, TypeError) as e:
            self.set_status(name, _condition({}, "Failed", "InvalidSpec", str(e)))
            return
        st = _condition(_condition({"startTime": _now()}, "Created", "StudyJobCreated"), "Running", "StudyJobRunning")
        self.set_status(name, st)

        def run():
            try:
                res = StudyRunner(spec, workdir=os.path.join(self.root, "studies", name), num_gpus=self.num_gpus).run()
                st2 = dict(st, completionTime=_now(), **study_summary(res))
                ok = res.get("best") is not None
                _condition(st2, "Succeeded" if ok else "Failed", "StudyJobCompleted" if ok else "NoTrialSucceeded")
            except Exception as e:  # noqa: BLE001 -- reported in the CR status
                st2 = _condition(dict(st, completionTime=_now()), "Failed", "StudyJobFailed", str(e))
            self.set_status(name, st2)

        t = threading.Thread(target=run, daemon=True)
        self._threads[name] = t
        t.start()

    def _reconcile_notebook(self, name: str, cr: dict, status: dict | None) -> None:
        import subprocess
        import sys

        p = self._procs.get(name)
        if p is not None and p.poll() is None:
            return
        port = notebook_port(cr)
        st = dict(status or {})
        if p is not None:  # the server exited: restart it (the controller keeps a Notebook running)
            st["restarts"] = int(st.get("restarts", 0)) + 1
            _condition(st, "Restarting", "NotebookRestarting", f"server exited with {p.returncode}")
        os.makedirs(os.path.join(self.root, "logs"), exist_ok=True)
        cmd = [sys.executable, "-m", "mifx.notebook_server", "--port", str(port)]
        root = (cr.get("spec") or {}).get("notebooksDir")
        if root:
            cmd += ["--root", root]
        with open(os.path.join(self.root, "logs", f"{name}.notebook.log"), "ab") as log:
            self._procs[name] = subprocess.Popen(cmd, stdout=log, stderr=subprocess.STDOUT, cwd=self.cwd)
        st.setdefault("startTime", _now())
        st["url"] = f"http://127.0.0.1:{port}/"
        self.set_status(name, _condition(st, "Running", "NotebookRunning", st["url"]))

    def stop(self) -> None:
        """Stop the supervised notebook servers (the jobs / studies are threads that finish on their own)."""
        for p in self._procs.values():
            if p.poll() is None:
                p.terminate()
                try:
                    p.wait(timeout=10)
                except Exception:  # noqa: BLE001
                    p.kill()
        self._procs.clear()

    def idle(self) -> bool:
        return all(not t.is_alive() for t in self._threads.values())


# ---------------------------------------------------------------- Kubernetes backend
class KubeApi:
    """Minimal Kubernetes REST client: in-cluster service-account token + CA (or an explicit base URL / token)."""

    SA = "/var/run/secrets/kubernetes.io/serviceaccount"

    def __init__(self, base: str | None = None, token: str | None = None, verify=None):
        import requests

        self.s = requests.Session()
        if base is None:
            base = f"https://{os.environ['KUBERNETES_SERVICE_HOST']}:{os.environ.get('KUBERNETES_SERVICE_PORT', '443')}"
        if token is None and os.path.exists(f"{self.SA}/token"):
            with open(f"{self.SA}/token") as f:
                token = f.read().strip()
        if token:
            self.s.headers["Authorization"] = f"Bearer {token}"
        self.s.verify = verify if verify is not None else (f"{self.SA}/ca.crt" if os.path.exists(f"{self.SA}/ca.crt")
                                                          else True)
        self.base = base.rstrip("/")

    def get(self, path: str):
        r = self.s.get(self.base + path, timeout=30)
        if r.status_code == 404:
            return None
        r.raise_for_status()
        return r.json()

    def post(self, path: str, body: dict):
        r = self.s.post(self.base + path, json=body, timeout=30)
        r.raise_for_status()
        return r.json()

    def patch(self, path: str, body: dict, content_type: str = "application/merge-patch+json"):
        r = self.s.patch(self.base + path, data=json.dumps(body), timeout=30, headers={"Content-Type": content_type})
        r.raise_for_status()
        return r.json()

    def delete(self, path: str):
        r = self.s.delete(self.base + path, timeout=30)
        if r.status_code not in (200, 202, 404):
            r.raise_for_status()

    def get_text(self, path: str) -> str:
        r = self.s.get(self.base + path, timeout=60)
        r.raise_for_status()
        return r.text

    def patch_status(self, path: str, status: dict):
        r = self.s.patch(self.base + path + "/status", data=json.dumps({"status": status}), timeout=30,
                         headers={"Content-Type": "application/merge-patch+json"})
        r.raise_for_status()
        return r.json()


class KubeBackend:
    def __init__(self, api, namespace: str = "kubeflow", image: str | None = None):
        self.api, self.ns, self.image = api, namespace, image

    def _cr_path(self, kind: str, name: str | None = None) -> str:
        g, v, plural = KINDS[kind]
        p = f"/apis/{g}/{v}/namespaces/{self.ns}/{plural}"
        return p + (f"/{name}" if name else "")

    def list(self) -> list[tuple[str, dict, dict | None]]:
        out = []
        for kind in KINDS:
            try:
                lst = self.api.get(self._cr_path(kind))
            except Exception:  # noqa: BLE001 -- a CRD that is not installed
                lst = None
            for cr in (lst or {}).get("items", []):
                cr.setdefault("kind", kind)
                out.append((cr["metadata"]["name"], cr, cr.get("status")))
        return out

    def set_status(self, name: str, status: dict, kind: str = "MIFXJob") -> None:
        self.api.patch_status(self._cr_path(kind, name), status)

    def _owner(self, kind: str, name: str, cr: dict) -> list:
        return [{"apiVersion": f"{KINDS[kind][0]}/{KINDS[kind][1]}", "kind": kind, "name": name,
                 "uid": cr["metadata"].get("uid", ""), "controller": True, "blockOwnerDeletion": True}]

    def _study_job(self, name: str, cr: dict) -> dict:
        """A one-node batch/v1 Job running the study (trials in parallel over the node's GPUs)."""
        spec_json = json.dumps({"spec": cr.get("spec", {}), "metadata": {"name": name}})
        return {"apiVersion": "batch/v1", "kind": "Job",
                "metadata": {"name": name, "namespace": self.ns, "labels": {"mifx.amd.com/study": name},
                             "ownerReferences": self._owner("StudyJob", name, cr)},
                "spec": {"backoffLimit": 0, "template": {"metadata": {"labels": {"mifx.amd.com/study": name}}, "spec": {
                    "restartPolicy": "Never",
                    "containers": [{"name": "study", "image": self.image or "mifx:latest",
                                    "command": ["python3", "-m", "mifx.hpo.study", "--spec-json", spec_json],
                                    "resources": {"limits": {"amd.com/gpu": "8"}}}]}}}}

    def _reconcile_notebook(self, name: str, cr: dict, status: dict | None) -> None:
        port = notebook_port(cr)
        dpath = f"/apis/apps/v1/namespaces/{self.ns}/deployments"
        dep = self.api.get(f"{dpath}/{name}")
        st = dict(status or {})
        if dep is None:
            labels = {"mifx.amd.com/notebook": name}
            self.api.post(dpath, {
                "apiVersion": "apps/v1", "kind": "Deployment",
                "metadata": {"name": name, "namespace": self.ns, "labels": labels,
                             "ownerReferences": self._owner("Notebook", name, cr)},
                "spec": {"replicas": 1, "selector": {"matchLabels": labels}, "template": {
                    "metadata": {"labels": labels}, "spec": {"containers": [{
                        "name": "notebook", "image": self.image or "mifx:latest",
                        "command": ["python3", "-m", "mifx.notebook_server", "--host", "0.0.0.0", "--port", str(port)],
                        "ports": [{"containerPort": port}],
                        "resources": {"limits": {"amd.com/gpu": "1"}}}]}}}})
            self.api.post(f"/api/v1/namespaces/{self.ns}/services", {
                "apiVersion": "v1", "kind": "Service",
                "metadata": {"name": name, "namespace": self.ns, "ownerReferences": self._owner("Notebook", name, cr)},
                "spec": {"selector": labels, "ports": [{"port": 80, "targetPort": port}]}})
            st.setdefault("startTime", _now())
            self.set_status(name, _condition(st, "Created", "NotebookCreated", f"Deployment {name}"), "Notebook")
            return
        ready = int((dep.get("status") or {}).get("readyReplicas", 0))
        if ready >= 1 and phase(st) != "Running":
            st["url"] = f"http://{name}.{self.ns}.svc/"
            self.set_status(name, _condition(st, "Running", "NotebookRunning", st["url"]), "Notebook")

    def reconcile(self, name: str, cr: dict, status: dict | None) -> None:
        kind = cr.get("kind", "MIFXJob")
        if kind == "Notebook":
            return self._reconcile_notebook(name, cr, status)
        if phase(status) in TERMINAL:
            return
        spec = None
        if kind != "StudyJob":
            try:
                spec = JobSpec.from_dict(cr)
            except ValueError as e:
                self.set_status(name, _condition({}, "Failed", "InvalidSpec", str(e)), kind)
                return
        jpath = f"/apis/batch/v1/namespaces/{self.ns}/jobs"
        job = self.api.get(f"{jpath}/{name}")
        st = dict(status or {})
        if job is None and kind == "StudyJob":
            self.api.post(jpath, self._study_job(name, cr))
            st.setdefault("startTime", _now())
            self.set_status(name, _condition(st, "Created", "StudyJobCreated", f"batch/v1 Job {name}"), kind)
            return
        if job is None:
            body = to_indexed_job(spec, self.ns, self.image)
            body["metadata"]["name"] = name
            body["metadata"]["ownerReferences"] = self._owner(kind, name, cr)
            policies = {r.restart_policy for r in spec.replicas}
            restart = bool(policies & {"OnFailure", "Always", "ExitCode"})
            body["spec"]["backoffLimit"] = (spec.backoff_limit if spec.backoff_limit is not None else 3) \
                if restart else 0
            self.api.post(jpath, body)
            st.setdefault("startTime", _now())
            self.set_status(name, _condition(st, "Created", "JobCreated", f"batch/v1 Job {name}"), kind)
            return
        js = job.get("status") or {}
        if js.get("succeeded"):
            _condition(st, "Succeeded", "JobSucceeded")
            st["completionTime"] = _now()
        elif any(c.get("type") == "Failed" and c.get("status") == "True" for c in js.get("conditions") or []):
            _condition(st, "Failed", "JobFailed", f"{js.get('failed', 0)} failed pod(s)")
            st["completionTime"] = _now()
        elif js.get("failed"):
            _condition(st, "Restarting", "JobRestarting", f"{js['failed']} failed attempt(s), retrying")
            st["restarts"] = int(js["failed"])
        elif js.get("active"):
            _condition(st, "Running", "JobRunning")
        else:
            return
        self.set_status(name, st, kind)


# ---------------------------------------------------------------- control loop
def reconcile_all(backend) -> int:
    """One pass over every CR; returns how many are not yet terminal."""
    pending = 0
    for name, cr, st in backend.list():
        try:
            backend.reconcile(name, cr, st)
        except Exception as e:  # noqa: BLE001 -- one bad CR never stops the loop
            print(f"[mifx-operator] {name}: {e}", flush=True)
        if phase(st) not in TERMINAL and cr.get("kind") != "Notebook":  # (a Notebook is a service: never "done")
            pending += 1
    return pending


def run(backend, interval_s: float = 2.0, stop: threading.Event | None = None) -> None:
    stop = stop or threading.Event()
    while not stop.is_set():
        reconcile_all(backend)
        stop.wait(interval_s)


def main(argv=None) -> int:
    import argparse

    ap = argparse.ArgumentParser(prog="python -m mifx.launch.operator", description=__doc__.split("\n")[0])
    g = ap.add_mutually_exclusive_group(required=True)
    g.add_argument("--local", metavar="DIR", help="watch CR YAML files in DIR and run them as local processes")
    g.add_argument("--kube", action="store_true", help="reconcile CRs through the Kubernetes API (in-cluster)")
    ap.add_argument("--namespace", default=os.environ.get("POD_NAMESPACE", "kubeflow"))
    ap.add_argument("--image", default=None, help="container image for the rendered Jobs")
    ap.add_argument("--interval", type=float, default=2.0)
    a = ap.parse_args(argv)
    backend = LocalBackend(a.local) if a.local else KubeBackend(KubeApi(), a.namespace, a.image)
    run(backend, a.interval)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
