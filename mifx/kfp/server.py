"""Pipelines API server: the `ml-pipeline` REST API v1beta1 subset the SDK client uses, backed by the workflow
executor -- steps on this host, or (`--executor kubernetes`) one Pod per step on the cluster.

Reference: the KFP API server the workshop deploys (`install-kubeflow/ks_app/vendor/kubeflow/pipeline`
prototypes, api-server on 8888) and the client calls in `sdk/python/kfp/_client.py:124-316`
(experiments create/get/list, runs create/get/list with resource references, pipeline upload).
Run: `python -m mifx.kfp.server --port 8888 --root /var/lib/mifx/pipelines`, then
`Client(host="http://<host>:8888")`; the same port serves the pipelines UI (mifx.kfp.ui) at `/`."""
import argparse
import email.parser
import email.policy
import os
import tempfile

from ._client import _LocalBackend


def parse_multipart(body: bytes, content_type: str) -> dict:
    """multipart/form-data -> {field: (filename, bytes)} with the stdlib MIME parser."""
    msg = email.parser.BytesParser(policy=email.policy.HTTP).parsebytes(
        b"Content-Type: " + content_type.encode() + b"\r\n\r\n" + body)
    out = {}
    for part in msg.iter_parts():
        name = part.get_param("name", header="content-disposition")
        out[name] = (part.get_filename(), part.get_payload(decode=True) or b"")
    return out


def create_app(root: str, max_parallel: int = 4, steps_factory=None):
    """steps_factory: per-run step runner (None: steps on this host; see `main --executor kubernetes`)."""
    from fastapi import FastAPI, HTTPException, Request

    backend = _LocalBackend(root, max_parallel, steps_factory)
    app = FastAPI(title="mifx pipelines API")

    def _page(req: Request):
        q = req.query_params
        return q.get("page_token", ""), int(q.get("page_size", 10) or 10), q.get("sort_by", "")

    @app.post("/apis/v1beta1/experiments")
    async def create_experiment(req: Request):
        body = await req.json()
        return backend.create_experiment(body["name"], body.get("description", ""))

    @app.get("/apis/v1beta1/experiments/{eid}")
    def get_experiment(eid: str):
        try:
            return backend.get_experiment(eid)
        except ValueError as e:
            raise HTTPException(404, str(e)) from e

    @app.get("/apis/v1beta1/experiments")
    def list_experiments(req: Request):
        return backend.list_experiments(*_page(req))

    @app.post("/apis/v1beta1/runs")
    async def create_run(req: Request):
        return backend.create_run(await req.json())

    @app.get("/apis/v1beta1/runs/{run_id}")
    def get_run(run_id: str):
        try:
            return backend.get_run(run_id)
        except ValueError as e:
            raise HTTPException(404, str(e)) from e

    @app.get("/apis/v1beta1/runs")
    def list_runs(req: Request):
        exp = req.query_params.get("resource_reference_key.id")
        return backend.list_runs(*_page(req), exp)

    @app.post("/apis/v1beta1/pipelines/upload")
    async def upload(req: Request):
        parts = parse_multipart(await req.body(), req.headers.get("content-type", ""))
        if "uploadfile" not in parts:
            raise HTTPException(400, "multipart field 'uploadfile' is required")
        filename, data = parts["uploadfile"]
        name = req.query_params.get("name") or filename
        suffix = ".tar.gz" if (filename or "").endswith(".tar.gz") else (os.path.splitext(filename or "")[1] or ".yaml")
        with tempfile.NamedTemporaryFile(suffix=suffix, delete=False) as f:
            f.write(data)
        try:
            return backend.upload_pipeline(f.name, name)
        finally:
            os.unlink(f.name)

    @app.get("/apis/v1beta1/pipelines")
    def list_pipelines(req: Request):
        return backend.list_pipelines(*_page(req))

    @app.get("/apis/v1beta1/healthz")
    def healthz():
        return {"status": "ok", "backend": backend.executor, "root": backend.root}

    # ---- pipelines UI (mifx.kfp.ui): read-only HTML views
    from fastapi.responses import HTMLResponse

    from . import ui

    @app.get("/", response_class=HTMLResponse)
    def ui_index():
        return ui.index(backend)

    @app.get("/ui/runs/{run_id}", response_class=HTMLResponse)
    def ui_run(run_id: str):
        try:
            return ui.run_page(backend, run_id)
        except ValueError as e:
            raise HTTPException(404, str(e)) from e

    @app.get("/ui/pipelines/{pid}", response_class=HTMLResponse)
    def ui_pipeline(pid: str):
        try:
            return ui.pipeline_page(backend, pid)
        except ValueError as e:
            raise HTTPException(404, str(e)) from e

    app.state.backend = backend
    return app


def main(argv=None):
    ap = argparse.ArgumentParser(prog="mifx-pipelines-api")
    ap.add_argument("--port", type=int, default=8888)
    ap.add_argument("--root", default=os.path.join(os.path.expanduser("~"), ".mifx", "pipelines"))
    ap.add_argument("--max-parallel", type=int, default=4)
    ap.add_argument("--executor", choices=("local", "kubernetes"), default=os.environ.get("MIFX_KFP_EXECUTOR", "local"),
                    help="where pipeline steps run: this host, or one Pod per step through the Kubernetes API "
                         "(in-cluster service account; the Argo controller's role)")
    ap.add_argument("--namespace", default=os.environ.get("POD_NAMESPACE", "kubeflow"))
    a = ap.parse_args(argv)
    import uvicorn

    factory = None
    if a.executor == "kubernetes":
        from ..launch.operator import KubeApi
        from .local.kube import KubeStepRunner

        api = KubeApi()
        factory = lambda: KubeStepRunner(api, a.namespace)  # noqa: E731
    uvicorn.run(create_app(a.root, a.max_parallel, factory), host="0.0.0.0", port=a.port, log_level="warning")


if __name__ == "__main__":
    main()
