"""File-store experiment tracking.

Layout: <root>/<experiment_id>/meta.json, <root>/<experiment_id>/<run_id>/{meta.json, params/<k>,
metrics/<k> (lines "timestamp value step"), tags/<k>, artifacts/...}."""
from __future__ import annotations

import json
import os
import shutil
import time
import uuid

_state = {"uri": None, "experiment": None, "runs": []}


def _root() -> str:
    uri = _state["uri"] or os.environ.get("MIFX_TRACKING_URI") or os.path.abspath("mlruns")
    return uri[len("file://"):] if uri.startswith("file://") else uri


def set_tracking_uri(uri: str) -> None:
    _state["uri"] = uri


def get_tracking_uri() -> str:
    return "file://" + _root()


class FileStore:
    def __init__(self, root: str | None = None):
        self.root = root or _root()
        os.makedirs(self.root, exist_ok=True)

    def _exp_dirs(self):
        for d in sorted(os.listdir(self.root)):
            p = os.path.join(self.root, d, "meta.json")
            if os.path.exists(p):
                with open(p) as f:
                    yield json.load(f)

    def get_experiment_by_name(self, name: str):
        return next((e for e in self._exp_dirs() if e["name"] == name), None)

    def create_experiment(self, name: str) -> str:
        if self.get_experiment_by_name(name):
            raise ValueError(f"experiment {name!r} already exists")
        eid = str(sum(1 for _ in self._exp_dirs()))
        os.makedirs(os.path.join(self.root, eid), exist_ok=True)
        with open(os.path.join(self.root, eid, "meta.json"), "w") as f:
            json.dump({"experiment_id": eid, "name": name, "artifact_location": os.path.join(self.root, eid),
                       "lifecycle_stage": "active", "creation_time": int(time.time() * 1000)}, f)
        return eid

    def run_dir(self, exp_id: str, run_id: str) -> str:
        return os.path.join(self.root, exp_id, run_id)

    def create_run(self, exp_id: str, run_name: str | None = None) -> dict:
        rid = uuid.uuid4().hex
        d = self.run_dir(exp_id, rid)
        for sub in ("params", "metrics", "tags", "artifacts"):
            os.makedirs(os.path.join(d, sub), exist_ok=True)
        meta = {"run_id": rid, "experiment_id": exp_id, "run_name": run_name or rid[:8], "status": "RUNNING",
                "start_time": int(time.time() * 1000), "end_time": None, "artifact_uri": os.path.join(d, "artifacts")}
        self._write_meta(d, meta)
        return meta

    @staticmethod
    def _write_meta(d, meta):
        with open(os.path.join(d, "meta.json"), "w") as f:
            json.dump(meta, f, indent=1)

    def get_run(self, run_id: str) -> dict:
        for e in self._exp_dirs():
            d = self.run_dir(e["experiment_id"], run_id)
            if os.path.isdir(d):
                with open(os.path.join(d, "meta.json")) as f:
                    meta = json.load(f)
                return {"info": meta, "data": self._data(d)}
        raise KeyError(f"run {run_id} not found")

    @staticmethod
    def _data(d: str) -> dict:
        def read_dir(sub):
            out = {}
            p = os.path.join(d, sub)
            for k in sorted(os.listdir(p)) if os.path.isdir(p) else []:
                with open(os.path.join(p, k)) as f:
                    out[k] = f.read()
            return out

        metrics, history = {}, {}
        for k, txt in read_dir("metrics").items():
            rows = [ln.split() for ln in txt.splitlines() if ln.strip()]
            history[k] = [{"timestamp": int(r[0]), "value": float(r[1]), "step": int(r[2])} for r in rows]
            metrics[k] = history[k][-1]["value"]
        return {"params": read_dir("params"), "metrics": metrics, "metric_history": history, "tags": read_dir("tags")}

    def finish(self, exp_id: str, run_id: str, status: str = "FINISHED") -> None:
        d = self.run_dir(exp_id, run_id)
        with open(os.path.join(d, "meta.json")) as f:
            meta = json.load(f)
        meta.update(status=status, end_time=int(time.time() * 1000))
        self._write_meta(d, meta)

    def search_runs(self, experiment_ids: list[str], filter_fn=None, order_by: str | None = None) -> list[dict]:
        runs = []
        for eid in experiment_ids:
            base = os.path.join(self.root, eid)
            for rid in sorted(os.listdir(base)) if os.path.isdir(base) else []:
                if os.path.isdir(os.path.join(base, rid)):
                    r = self.get_run(rid)
                    if filter_fn is None or filter_fn(r):
                        runs.append(r)
        if order_by:
            key, _, direction = order_by.partition(" ")
            kind, _, name = key.partition(".")
            runs.sort(key=lambda r: r["data"][{"metrics": "metrics", "params": "params"}[kind]].get(name, float("nan")),
                      reverse=direction.upper() == "DESC")
        return runs


class ActiveRun:
    def __init__(self, store: FileStore, meta: dict):
        self.store, self.info = store, meta
        self.dir = store.run_dir(meta["experiment_id"], meta["run_id"])

    def __enter__(self):
        return self

    def __exit__(self, exc_type, exc, tb):
        end_run("FAILED" if exc_type else "FINISHED")
        return False


def create_experiment(name: str) -> str:
    return FileStore().create_experiment(name)


def get_experiment_by_name(name: str):
    return FileStore().get_experiment_by_name(name)


def set_experiment(name: str) -> str:
    st = FileStore()
    e = st.get_experiment_by_name(name)
    eid = e["experiment_id"] if e else st.create_experiment(name)
    _state["experiment"] = eid
    return eid


def start_run(run_name: str | None = None, experiment_id: str | None = None, nested: bool = False) -> ActiveRun:
    if _state["runs"] and not nested:
        raise RuntimeError("a run is already active; use nested=True or end_run()")
    st = FileStore()
    eid = experiment_id or _state["experiment"] or set_experiment("Default")
    run = ActiveRun(st, st.create_run(eid, run_name))
    _state["runs"].append(run)
    return run


def active_run() -> ActiveRun | None:
    return _state["runs"][-1] if _state["runs"] else None


def _run() -> ActiveRun:
    return active_run() or start_run()


def end_run(status: str = "FINISHED") -> None:
    if _state["runs"]:
        r = _state["runs"].pop()
        r.store.finish(r.info["experiment_id"], r.info["run_id"], status)


def _write(sub: str, key: str, text: str, append: bool = False) -> None:
    r = _run()
    if "/" in key or key.startswith("."):
        raise ValueError(f"invalid key {key!r}")
    with open(os.path.join(r.dir, sub, key), "a" if append else "w") as f:
        f.write(text)


def log_param(key: str, value) -> None:
    p = os.path.join(_run().dir, "params", key)
    if os.path.exists(p) and open(p).read() != str(value):
        raise ValueError(f"param {key!r} already logged with a different value")
    _write("params", key, str(value))


def log_params(params: dict) -> None:
    for k, v in params.items():
        log_param(k, v)


def log_metric(key: str, value: float, step: int = 0) -> None:
    _write("metrics", key, f"{int(time.time() * 1000)} {float(value)!r} {int(step)}\n", append=True)


def log_metrics(metrics: dict, step: int = 0) -> None:
    for k, v in metrics.items():
        log_metric(k, v, step)


def set_tag(key: str, value) -> None:
    _write("tags", key, str(value))


def log_artifact(local_path: str, artifact_path: str | None = None) -> str:
    dst = os.path.join(_run().dir, "artifacts", artifact_path or "")
    os.makedirs(dst, exist_ok=True)
    target = os.path.join(dst, os.path.basename(local_path))
    (shutil.copytree if os.path.isdir(local_path) else shutil.copyfile)(local_path, target)
    return target


def log_model(model, artifact_path: str = "model", module_class: str | None = None, config: dict | None = None) -> str:
    """torch modules -> mifx saved-model (safetensors); other estimators (e.g. sklearn) -> joblib."""
    dst = os.path.join(_run().dir, "artifacts", artifact_path)
    os.makedirs(dst, exist_ok=True)
    try:
        import torch

        is_torch = isinstance(model, torch.nn.Module)
    except ImportError:
        is_torch = False
    if is_torch:
        from ..serving.saved_model import save_module

        cls = module_class or f"{type(model).__module__}:{type(model).__name__}"
        save_module(dst, model, cls, config or {})
        flavor = "mifx.torch"
    else:
        import joblib

        joblib.dump(model, os.path.join(dst, "model.joblib"))
        flavor = "sklearn"
    with open(os.path.join(dst, "MLmodel.json"), "w") as f:
        json.dump({"flavor": flavor, "run_id": _run().info["run_id"], "class": type(model).__name__}, f)
    return dst


def get_run(run_id: str) -> dict:
    return FileStore().get_run(run_id)


def search_runs(experiment_ids: list[str] | None = None, order_by: str | None = None) -> list[dict]:
    st = FileStore()
    ids = experiment_ids or [e["experiment_id"] for e in st._exp_dirs()]
    return st.search_runs(ids, order_by=order_by)

