"""Scalar dashboard over TF event files: the TensorBoard component of the reference's Kubeflow deployment.

The reference deploys TensorBoard next to the notebook servers (`install-kubeflow/ks_app/components/
params.libsonnet:75-82`, the `tensorboard` package of `install-kubeflow/app.yaml:15-46`) and its training code
writes `tf.summary.scalar` events into a log dir (`kubeflow-pipelines/fairing/fairing_tf.py:54-74`,
`research/pate_2017/deep_cnn.py:402,415-417`). mifx writes the same `events.out.tfevents.*` files without
TensorFlow (mifx.utils.summary.SummaryWriter); this service reads them and serves

* TensorBoard's scalar-plugin JSON routes -- `/data/runs`, `/data/plugin/scalars/tags`,
  `/data/plugin/scalars/scalars?run=&tag=` (rows `[wall_time, step, value]`), so scripts written against a
  TensorBoard endpoint keep working;
* `/` an HTML page with one SVG line chart per (tag, run), re-read on every request (live training runs).

A run is every directory under --logdir that holds event files (its path relative to the log dir).

    python -m mifx.board --logdir /mnt/logs --port 6006
"""
from __future__ import annotations

import argparse
import html
import os

from ..utils.summary import read_scalars


def find_runs(logdir: str) -> dict[str, list[str]]:
    """run name -> event files (sorted), for every directory under logdir holding `events.out.tfevents.*`."""
    runs: dict[str, list[str]] = {}
    for root, _, files in os.walk(logdir):
        ev = sorted(f for f in files if f.startswith("events.out.tfevents."))
        if ev:
            name = os.path.relpath(root, logdir)
            runs["." if name == "." else name] = [os.path.join(root, f) for f in ev]
    return dict(sorted(runs.items()))


def run_scalars(files: list[str]) -> dict[str, list[tuple[float, int, float]]]:
    """tag -> [(wall_time, step, value)] over a run's event files, in file then record order."""
    out: dict[str, list[tuple[float, int, float]]] = {}
    for f in files:
        for tag, rows in read_scalars(f, with_wall_time=True).items():
            out.setdefault(tag, []).extend(rows)
    return out


def _svg(series: dict[str, list[tuple[float, int, float]]], w: int = 420, h: int = 180) -> str:
    pts = [(s, v) for rows in series.values() for _, s, v in rows]
    if not pts:
        return "<svg/>"
    x0, x1 = min(p[0] for p in pts), max(p[0] for p in pts)
    y0, y1 = min(p[1] for p in pts), max(p[1] for p in pts)
    xs = (w - 50) / max(x1 - x0, 1)
    ys = (h - 30) / max(y1 - y0, 1e-12)
    colors = ["#1f77b4", "#d62728", "#2ca02c", "#9467bd", "#ff7f0e", "#8c564b"]
    lines = []
    for i, (run, rows) in enumerate(series.items()):
        path = " ".join(f"{40 + (s - x0) * xs:.1f},{h - 20 - (v - y0) * ys:.1f}" for _, s, v in rows)
        lines.append(f'<polyline fill="none" stroke="{colors[i % len(colors)]}" stroke-width="1.5" points="{path}">'
                     f"<title>{html.escape(run)}</title></polyline>")
    axes = (f'<text x="2" y="12" font-size="10">{y1:.4g}</text><text x="2" y="{h - 20}" font-size="10">{y0:.4g}'
            f'</text><text x="40" y="{h - 4}" font-size="10">step {x0}</text>'
            f'<text x="{w - 60}" y="{h - 4}" font-size="10">{x1}</text>')
    return f'<svg width="{w}" height="{h}" style="border:1px solid #ccc">{axes}{"".join(lines)}</svg>'


def create_app(logdir: str):
    from fastapi import FastAPI, HTTPException
    from fastapi.responses import HTMLResponse

    app = FastAPI(title="mifx board (TensorBoard scalars)")

    @app.get("/healthz")
    def healthz():
        return {"status": "ok"}

    @app.get("/data/runs")
    def runs():
        return list(find_runs(logdir))

    @app.get("/data/plugin/scalars/tags")
    def tags():
        return {run: {tag: {"displayName": tag, "description": ""} for tag in run_scalars(files)}
                for run, files in find_runs(logdir).items()}

    @app.get("/data/plugin/scalars/scalars")
    def scalars(run: str, tag: str):
        files = find_runs(logdir).get(run)
        if files is None:
            raise HTTPException(404, f"no run {run!r}")
        rows = run_scalars(files).get(tag)
        if rows is None:
            raise HTTPException(404, f"no tag {tag!r} in run {run!r}")
        return [[wt, st, v] for wt, st, v in rows]

    @app.get("/", response_class=HTMLResponse)
    def index():
        data = {run: run_scalars(files) for run, files in find_runs(logdir).items()}
        by_tag: dict[str, dict[str, list]] = {}
        for run, tags_ in data.items():
            for tag, rows in tags_.items():
                by_tag.setdefault(tag, {})[run] = rows
        body = [f"<h1>Scalars</h1><p>log dir <code>{html.escape(logdir)}</code>: {len(data)} run(s)</p>"]
        for tag, series in sorted(by_tag.items()):
            legend = ", ".join(html.escape(r) for r in series)
            body.append(f"<h3>{html.escape(tag)}</h3><p style='font-size:small'>{legend}</p>{_svg(series)}")
        return "<html><head><title>mifx board</title></head><body>" + "".join(body) + "</body></html>"

    return app


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(description=__doc__.split("\n\n")[0])
    ap.add_argument("--logdir", required=True)
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=6006)
    a = ap.parse_args(argv)
    import uvicorn

    uvicorn.run(create_app(a.logdir), host=a.host, port=a.port, log_level="warning")
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
