"""Model server with the TF-Serving REST API, version management and GPU dynamic batching.

Reference: the TF-Serving deployment (`tensorflow_model_server --port=9000 --rest_api_port=8500
--model_name --model_base_path`; the gRPC API on --port is mifx.serving.grpc_service, ksonnet `tf-serving` prototypes, optional Prometheus monitoring
config) and the notebook's REST usage (`serving/Predict_Fashion_MNIST.ipynb`: POST
`/v1/models/<name>:predict` and `/v1/models/<name>/versions/<v>:predict` with `{"instances": ...}`).

Endpoints (TF-Serving REST v1 semantics):
  GET  /v1/models/{name}[/versions/{v}]            model version status
  GET  /v1/models/{name}[/versions/{v}]/metadata   signature metadata
  POST /v1/models/{name}[/versions/{v}]:predict    {"instances": [...]} | {"inputs": ...}
  POST /v1/models/{name}[/versions/{v}]:classify   {"examples": [{feature: value}, ...]}
  GET  /monitoring/prometheus/metrics              request counters / latency histograms
Versions are integer sub-directories of the base path (highest = latest); a watcher thread
loads new versions and unloads ones outside the policy. On a GPU, concurrent predict calls for
the same version are merged by a `DynamicBatcher` (max batch / timeout) into one device launch."""

import argparse
import os
import threading
import time
from concurrent.futures import Future

import numpy as np

from .saved_model import LoadedModel


class DynamicBatcher:
    """Merge concurrent requests into one forward (TF-Serving's `--enable_batching` equivalent)."""

    def __init__(self, run_fn, max_batch_size: int = 4096, batch_timeout_s: float = 0.002):
        self.run_fn = run_fn
        self.max_batch = max_batch_size
        self.timeout = batch_timeout_s
        self._q: list = []
        self._cv = threading.Condition()
        self._stop = False
        self.batches_run = 0
        self._t = threading.Thread(target=self._loop, daemon=True)
        self._t.start()

    def submit(self, items: list) -> Future:
        f: Future = Future()
        with self._cv:
            self._q.append((items, f))
            self._cv.notify()
        return f

    def _loop(self):
        while True:
            with self._cv:
                while not self._q and not self._stop:
                    self._cv.wait()
                if self._stop:
                    return
                deadline = time.monotonic() + self.timeout
                while sum(len(i) for i, _ in self._q) < self.max_batch:
                    left = deadline - time.monotonic()
                    if left <= 0:
                        break
                    self._cv.wait(left)
                batch, total = [], 0
                while self._q and (not batch or total + len(self._q[0][0]) <= self.max_batch):
                    items, f = self._q.pop(0)
                    batch.append((items, f))
                    total += len(items)
            try:
                merged = [x for items, _ in batch for x in items]
                out = self.run_fn(merged)
                self.batches_run += 1
                off = 0
                for items, f in batch:
                    f.set_result({k: v[off:off + len(items)] for k, v in out.items()})
                    off += len(items)
            except Exception as e:  # noqa: BLE001 - delivered to each waiting request
                for _, f in batch:
                    f.set_exception(e)

    def close(self):
        with self._cv:
            self._stop = True
            self._cv.notify_all()


class ServableVersion:
    def __init__(self, name: str, version: int, path: str, device=None, batching: bool = True,
                 max_batch_size: int = 4096, batch_timeout_s: float = 0.002):
        self.name, self.version, self.path = name, version, path
        self.model = LoadedModel(path, device)
        self.state = "AVAILABLE"
        self.batcher = DynamicBatcher(self.model.predict, max_batch_size, batch_timeout_s) \
            if batching and self.model.device.type == "cuda" else None

    def predict(self, instances) -> dict:
        if self.batcher is not None and isinstance(instances, list):
            return self.batcher.submit(instances).result()
        return self.model.predict(instances)

    def unload(self):
        if self.batcher:
            self.batcher.close()
        self.state = "END"


class ModelManager:
    """Loads integer-versioned exports under `base_path` per a version policy and keeps them fresh."""

    def __init__(self, name: str, base_path: str, policy: str = "latest", versions: list | None = None,
                 device=None, poll_s: float = 2.0, batching: bool = True):
        self.name, self.base_path, self.policy, self.pinned = name, base_path, policy, versions or []
        self.device, self.batching = device, batching
        self.servables: dict[int, ServableVersion] = {}
        self._lock = threading.Lock()
        self.refresh()
        self._stop = threading.Event()
        if poll_s > 0:
            threading.Thread(target=self._watch, args=(poll_s,), daemon=True).start()

    def _on_disk(self) -> list[int]:
        if not os.path.isdir(self.base_path):
            return []
        return sorted(int(d) for d in os.listdir(self.base_path)
                      if d.isdigit() and os.path.exists(os.path.join(self.base_path, d, "saved_model.json")))

    def _wanted(self, disk: list[int]) -> list[int]:
        if not disk:
            return []
        if self.policy == "all":
            return disk
        if self.policy == "specific":
            return [v for v in disk if v in self.pinned]
        return [disk[-1]]

    def refresh(self) -> None:
        want = set(self._wanted(self._on_disk()))
        with self._lock:
            for v in sorted(want - set(self.servables)):
                self.servables[v] = ServableVersion(self.name, v, os.path.join(self.base_path, str(v)), self.device,
                                                    self.batching)
            for v in sorted(set(self.servables) - want):
                self.servables.pop(v).unload()

    def _watch(self, poll_s):
        while not self._stop.wait(poll_s):
            try:
                self.refresh()
            except Exception:  # noqa: BLE001 - keep serving the loaded versions
                pass

    def get(self, version: int | None = None) -> ServableVersion:
        with self._lock:
            if not self.servables:
                raise KeyError(f"Servable not found for request: Latest({self.name})")
            if version is None:
                return self.servables[max(self.servables)]
            if version not in self.servables:
                raise KeyError(f"Servable not found for request: Specific({self.name}, {version})")
            return self.servables[version]

    def status(self, version: int | None = None) -> dict:
        with self._lock:
            vs = [version] if version is not None else sorted(self.servables, reverse=True)
            return {"model_version_status": [{"version": str(v), "state": self.servables[v].state if v in
                                              self.servables else "UNKNOWN",
                                              "status": {"error_code": "OK", "error_message": ""}} for v in vs]}

    def close(self):
        self._stop.set()
        with self._lock:
            for s in self.servables.values():
                s.unload()
            self.servables.clear()


def _jsonable(out: dict, columnar: bool):
    conv = {k: np.asarray(v).tolist() for k, v in out.items()}
    if columnar:
        return {"outputs": conv if len(conv) > 1 else next(iter(conv.values()))}
    keys = list(conv)
    if len(keys) == 1:
        return {"predictions": conv[keys[0]]}
    n = len(conv[keys[0]])
    return {"predictions": [{k: conv[k][i] for k in keys} for i in range(n)]}


def create_app(models: dict[str, ModelManager]):
    """FastAPI app exposing the TF-Serving REST API for `models` (name -> manager)."""
    from fastapi import FastAPI, HTTPException, Request
    from fastapi.responses import JSONResponse, PlainTextResponse
    from prometheus_client import CONTENT_TYPE_LATEST, CollectorRegistry, Counter, Histogram, generate_latest

    reg = CollectorRegistry()
    req_count = Counter("mifx_serving_requests", "requests", ["model", "method", "status"], registry=reg)
    latency = Histogram("mifx_serving_request_latency_seconds", "latency", ["model", "method"], registry=reg)
    app = FastAPI(title="mifx model server")

    def _mgr(name):
        if name not in models:
            raise HTTPException(404, detail=f"Servable not found for request: Latest({name})")
        return models[name]

    def _parse(name_action: str):
        name, _, action = name_action.partition(":")
        return name, action

    @app.get("/v1/models/{name}")
    def status(name: str):
        return _mgr(name).status()

    @app.get("/v1/models/{name}/versions/{version}")
    def status_v(name: str, version: int):
        return _mgr(name).status(version)

    @app.get("/v1/models/{name}/metadata")
    def metadata(name: str):
        s = _mgr(name).get()
        return {"model_spec": {"name": name, "version": str(s.version)},
                "metadata": {"signature_def": s.model.signatures}}

    @app.get("/v1/models/{name}/versions/{version}/metadata")
    def metadata_v(name: str, version: int):
        s = _mgr(name).get(version)
        return {"model_spec": {"name": name, "version": str(version)},
                "metadata": {"signature_def": s.model.signatures}}

    async def _run(name: str, version, action: str, request: Request):
        t0 = time.perf_counter()
        try:
            mgr = _mgr(name)
            try:
                s = mgr.get(version)
            except KeyError as e:
                raise HTTPException(404, detail=str(e)) from e
            body = await request.json()
            if action == "predict":
                if "instances" in body:
                    out, columnar = s.predict(body["instances"]), False
                elif "inputs" in body:
                    out, columnar = s.predict(body["inputs"]), True
                else:
                    raise HTTPException(400, detail="JSON body must contain 'instances' or 'inputs'")
                resp = _jsonable(out, columnar)
            elif action in ("classify", "regress"):
                out = s.predict(body.get("examples", []))
                if action == "classify":
                    probs = np.asarray(out.get("probabilities", out.get("scores")))
                    resp = {"results": [[[str(c), float(p)] for c, p in enumerate(row)] for row in probs]}
                else:
                    key = "logistic" if "logistic" in out else next(iter(out))
                    resp = {"results": np.asarray(out[key]).reshape(-1).tolist()}
            else:
                raise HTTPException(400, detail=f"unsupported method {action}")
            req_count.labels(name, action, "ok").inc()
            return JSONResponse(resp)
        except HTTPException:
            req_count.labels(name, action, "error").inc()
            raise
        except Exception as e:  # noqa: BLE001 - TF-Serving returns {"error": ...}
            req_count.labels(name, action, "error").inc()
            return JSONResponse({"error": str(e)}, status_code=400)
        finally:
            latency.labels(name, action).observe(time.perf_counter() - t0)

    @app.post("/v1/models/{name_action}")
    async def call(name_action: str, request: Request):
        name, action = _parse(name_action)
        return await _run(name, None, action, request)

    @app.post("/v1/models/{name}/versions/{version_action}")
    async def call_v(name: str, version_action: str, request: Request):
        v, action = _parse(version_action)
        return await _run(name, int(v), action, request)

    @app.get("/monitoring/prometheus/metrics")
    def metrics():
        return PlainTextResponse(generate_latest(reg), media_type=CONTENT_TYPE_LATEST)

    return app


def main(argv=None):
    ap = argparse.ArgumentParser(prog="mifx-model-server")
    ap.add_argument("--rest_api_port", type=int, default=8500)
    ap.add_argument("--port", type=int, default=9000,
                    help="gRPC PredictionService / ModelService port (tensorflow_model_server --port); -1 disables")
    ap.add_argument("--model_name", required=True)
    ap.add_argument("--model_base_path", required=True)
    ap.add_argument("--version_policy", default="latest", choices=["latest", "all", "specific"])
    ap.add_argument("--versions", type=int, nargs="*", default=[])
    ap.add_argument("--enable_batching", type=int, default=1)
    ap.add_argument("--file_system_poll_wait_seconds", type=float, default=2.0)
    ap.add_argument("--device", default=None)
    a = ap.parse_args(argv)
    import uvicorn

    mgr = ModelManager(a.model_name, a.model_base_path, a.version_policy, a.versions, a.device,
                       a.file_system_poll_wait_seconds, bool(a.enable_batching))
    models = {a.model_name: mgr}
    grpc_server = None
    if a.port >= 0:  # the gRPC API beside REST, sharing the loaded versions and the dynamic batcher
        from .grpc_service import serve

        grpc_server, _ = serve(models, a.port)
    try:
        uvicorn.run(create_app(models), host="0.0.0.0", port=a.rest_api_port, log_level="warning")
    finally:
        if grpc_server is not None:
            grpc_server.stop(grace=1.0)


if __name__ == "__main__":
    main()
