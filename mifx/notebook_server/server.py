"""Notebook server: browse and run the workshop notebooks over HTTP (the Jupyter role of the reference deployment).

The reference's Kubeflow app runs per-user Jupyter servers (jupyter-web-app + notebook-controller,
`install-kubeflow/app.yaml:15-46`, `install-kubeflow/ks_app/components/params.libsonnet:75-82`) in which the
workshop's 21 notebooks run. Jupyter is not part of this stack; the notebooks are plain Python modules
(`examples/notebooks/nXX_*.py`, one function per notebook cell group, tests in tests/test_notebook_examples.py).
This service lists them with their docstrings, shows their source, and runs one of THEM on request in its own
process (the server's GPU / device environment, a per-run timeout), keeping each run's status and output:

    GET  /api/notebooks                  [{name, title}]
    GET  /api/notebooks/{name}           {name, title, source}
    POST /api/notebooks/{name}/run       {run_id}
    GET  /api/runs, /api/runs/{run_id}   {run_id, notebook, status, returncode, output, seconds}
    GET  /                               HTML index with run buttons and recent runs

Only the notebooks found in --root can be run (a name is looked up in that listing, never joined into a path from
the request), with no request-supplied arguments, and the server binds to 127.0.0.1 unless told otherwise: like a
Jupyter server it executes code, so it is a single-user tool (reach it through a port-forward, not a Service).

    python -m mifx.notebook_server --root examples/notebooks --port 8888
"""
from __future__ import annotations

import argparse
import ast
import html
import os
import subprocess
import sys
import threading
import time
import uuid


def list_notebooks(root: str) -> list[dict]:
    out = []
    for f in sorted(os.listdir(root)):
        if f.endswith(".py") and not f.startswith("_"):
            out.append({"name": f[:-3], "title": _title(os.path.join(root, f))})
    return out


def _title(path: str) -> str:
    try:
        doc = ast.get_docstring(ast.parse(open(path).read())) or ""
    except SyntaxError:
        doc = ""
    return doc.strip().splitlines()[0] if doc.strip() else os.path.basename(path)


class Runner:
    """Runs the listed notebooks as child processes (`python <notebook>.py`), one thread per run."""

    def __init__(self, root: str, timeout_s: float = 1800.0, max_output: int = 1 << 20):
        self.root, self.timeout_s, self.max_output = os.path.abspath(root), timeout_s, max_output
        self.runs: dict[str, dict] = {}
        self._lock = threading.Lock()

    def start(self, name: str) -> str:
        known = {n["name"] for n in list_notebooks(self.root)}
        if name not in known:  # only the listed notebooks; the request never names a path
            raise FileNotFoundError(name)
        path = os.path.join(self.root, name + ".py")
        rid = uuid.uuid4().hex[:12]
        with self._lock:
            self.runs[rid] = {"run_id": rid, "notebook": name, "status": "running", "returncode": None, "output": "",
                              "seconds": None, "started": time.time()}
        threading.Thread(target=self._run, args=(rid, path), daemon=True).start()
        return rid

    def _run(self, rid: str, path: str) -> None:
        t0 = time.time()
        repo = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
        env = dict(os.environ, PYTHONPATH=os.pathsep.join([repo, os.environ.get("PYTHONPATH", "")]).rstrip(os.pathsep))
        try:
            p = subprocess.run([sys.executable, path], capture_output=True, text=True, timeout=self.timeout_s,
                               cwd=self.root, env=env)
            status, rc, out = ("succeeded" if p.returncode == 0 else "failed"), p.returncode, p.stdout + p.stderr
        except subprocess.TimeoutExpired as e:
            status, rc = "timeout", None
            out = (e.stdout or "") if isinstance(e.stdout, str) else ""
        with self._lock:
            self.runs[rid].update(status=status, returncode=rc, output=out[-self.max_output:],
                                  seconds=time.time() - t0)

    def get(self, rid: str) -> dict | None:
        with self._lock:
            r = self.runs.get(rid)
            return dict(r) if r else None

    def wait(self, rid: str, timeout: float = 60.0) -> dict:
        t0 = time.time()
        while time.time() - t0 < timeout:
            r = self.get(rid)
            if r and r["status"] != "running":
                return r
            time.sleep(0.05)
        return self.get(rid)


def create_app(root: str, timeout_s: float = 1800.0):
    from fastapi import FastAPI, HTTPException
    from fastapi.responses import HTMLResponse

    app = FastAPI(title="mifx notebook server")
    runner = Runner(root, timeout_s)
    app.state.runner = runner

    @app.get("/healthz")
    def healthz():
        return {"status": "ok"}

    @app.get("/api/notebooks")
    def notebooks():
        return list_notebooks(root)

    @app.get("/api/notebooks/{name}")
    def notebook(name: str):
        if name not in {n["name"] for n in list_notebooks(root)}:
            raise HTTPException(404, f"no notebook {name!r}")
        path = os.path.join(root, name + ".py")
        return {"name": name, "title": _title(path), "source": open(path).read()}

    @app.post("/api/notebooks/{name}/run")
    def run(name: str):
        try:
            return {"run_id": runner.start(name)}
        except FileNotFoundError:
            raise HTTPException(404, f"no notebook {name!r}")

    @app.get("/api/runs")
    def runs():
        return [runner.get(r) for r in list(runner.runs)]

    @app.get("/api/runs/{rid}")
    def run_status(rid: str):
        r = runner.get(rid)
        if r is None:
            raise HTTPException(404, f"no run {rid!r}")
        return r

    @app.get("/", response_class=HTMLResponse)
    def index():
        rows = "".join(f"<tr><td>{html.escape(n['name'])}</td><td>{html.escape(n['title'])}</td>"
                       f"<td><form method='post' action='/api/notebooks/{html.escape(n['name'])}/run'>"
                       f"<button>run</button></form></td></tr>" for n in list_notebooks(root))
        recent = "".join(f"<li>{html.escape(r['notebook'])}: {r['status']} "
                         f"(<a href='/api/runs/{r['run_id']}'>{r['run_id']}</a>)</li>"
                         for r in sorted((runner.get(x) for x in list(runner.runs)), key=lambda r: -r["started"])[:20])
        return (f"<html><head><title>mifx notebooks</title></head><body><h1>Notebooks</h1><table>{rows}</table>"
                f"<h2>Recent runs</h2><ul>{recent}</ul></body></html>")

    return app


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--root", default=os.path.join(os.path.dirname(__file__), "..", "..", "examples", "notebooks"))
    ap.add_argument("--host", default="127.0.0.1", help="bind address (the server runs code: keep it local)")
    ap.add_argument("--port", type=int, default=8888)
    ap.add_argument("--timeout", type=float, default=1800.0, help="seconds per notebook run")
    a = ap.parse_args(argv)
    import uvicorn

    uvicorn.run(create_app(os.path.abspath(a.root), a.timeout), host=a.host, port=a.port, log_level="warning")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
