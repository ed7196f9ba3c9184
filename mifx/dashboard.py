"""Central dashboard: one page linking every service of the single-node stack, with live health.

Reference: the Kubeflow central dashboard the workshop deploys (`install-kubeflow/app.yaml:15-27` component
`centraldashboard`) and the PipelineAI reverse proxy's dashboards (`infrastructure/config/nginx/pipelineai-nginx.conf`).
Each service is probed with a short HTTP GET from the server side; `/api/services` returns the same as JSON.

  python -m mifx.dashboard --port 8082   (behind deploy/nginx.conf at /)"""
from __future__ import annotations

import html
import os
import time

# (name, what, upstream URL probed by the dashboard, path under the reverse proxy)
SERVICES = [
    ("pipelines", "KFP pipelines API + run list (mifx.kfp.server)", "http://127.0.0.1:8888/apis/v1beta1/healthz",
     "/pipeline/"),
    ("metadata", "ML-Metadata lineage + run dashboard (mifx.metadata.server)", "http://127.0.0.1:8080/healthz",
     "/metadata/"),
    ("serving", "TF-Serving REST model server (mifx.serving.server; gRPC on :9000)",
     "http://127.0.0.1:8500/monitoring/prometheus/metrics", "/predict/"),
    ("board", "TensorBoard-compatible scalar dashboard (mifx.board)", "http://127.0.0.1:6006/healthz", "/tensorboard/"),
    ("notebooks", "notebook runner (mifx.notebook_server)", "http://127.0.0.1:8889/healthz", "/notebooks/"),
    ("operator", "training-job operator (mifx.launch.operator): MIFXJob / TFJob / PyTorchJob status", None, "/jobs/"),
    ("tracking", "MLflow-compatible experiment store (file browser)", None, "/tracking/"),
    ("prometheus", "Prometheus scrape of the model server", "http://127.0.0.1:8500/monitoring/prometheus/metrics",
     "/metrics"),
]


def probe(url: str | None, timeout: float = 0.5) -> dict:
    if url is None:
        return {"state": "static"}
    import requests

    t0 = time.perf_counter()
    try:
        r = requests.get(url, timeout=timeout)
        return {"state": "up" if r.status_code < 500 else "error", "code": r.status_code,
                "ms": round(1e3 * (time.perf_counter() - t0), 1)}
    except Exception as e:  # noqa: BLE001
        return {"state": "down", "error": type(e).__name__}


def create_app(services=None):
    from fastapi import FastAPI
    from fastapi.responses import HTMLResponse

    services = services if services is not None else SERVICES
    app = FastAPI(title="mifx central dashboard")

    def status():
        return [{"name": n, "what": w, "link": link, **probe(u)} for n, w, u, link in services]

    @app.get("/api/services")
    def api_services():
        return {"services": status(), "gpus": _gpus()}

    @app.get("/healthz")
    def healthz():
        return {"ok": True}

    @app.get("/", response_class=HTMLResponse)
    def index():
        rows = "".join(
            f"<tr><td><a href='{html.escape(s['link'])}'>{html.escape(s['name'])}</a></td>"
            f"<td>{html.escape(s['what'])}</td><td class='{s['state']}'>{s['state']}</td></tr>" for s in status())
        g = _gpus()
        return ("<html><head><title>mifx</title><style>td{padding:4px 12px}.up{color:green}.down{color:red}"
                "</style></head><body><h2>mifx single-node stack</h2>"
                f"<p>{g['count']} GPU(s) {html.escape(', '.join(g['names']))}</p>"
                f"<table><tr><th>service</th><th>what</th><th>state</th></tr>{rows}</table></body></html>")

    return app


def _gpus() -> dict:
    try:
        import torch

        n = torch.cuda.device_count()
        names = sorted({torch.cuda.get_device_properties(i).name for i in range(n)}) if n else []
    except Exception:  # noqa: BLE001
        n, names = 0, []
    return {"count": n, "names": names}


def main(argv=None) -> int:
    import argparse

    import uvicorn

    ap = argparse.ArgumentParser(prog="python -m mifx.dashboard")
    ap.add_argument("--host", default=os.environ.get("MIFX_BIND", "127.0.0.1"))
    ap.add_argument("--port", type=int, default=8082)
    a = ap.parse_args(argv)
    uvicorn.run(create_app(), host=a.host, port=a.port, log_level="warning")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
