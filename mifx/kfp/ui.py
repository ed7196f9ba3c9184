"""Pipelines UI: HTML views of the pipelines API server's experiments, runs and pipelines (the role of the KFP
frontend the reference deploys next to the api-server, `install-kubeflow/app.yaml:15-27` ml-pipeline-ui).

Served by mifx.kfp.server at `/` (experiments, runs with status, uploaded pipelines), `/ui/runs/{id}` (the run's
graph: every node of the executed workflow as an SVG box coloured by phase, laid out by depth along its `children`
edges, and a table with times, attempts, outputs and messages) and `/ui/pipelines/{id}` (the pipeline's DAG from its
workflow spec). Read-only: runs are created through the API / SDK client. All text from the stores is HTML-escaped."""
from __future__ import annotations

import html
import json
import time

_PHASE_COLOURS = {"Succeeded": "#2e7d32", "Failed": "#c62828", "Error": "#c62828", "Running": "#1565c0",
                  "Pending": "#9e9e9e", "Skipped": "#bdbdbd", "Omitted": "#bdbdbd"}
_CSS = ("body{font-family:sans-serif;margin:24px}table{border-collapse:collapse}td,th{border:1px solid #ccc;"
        "padding:4px 8px;font-size:13px}th{background:#f4f4f4}.ph{color:#fff;padding:1px 6px;border-radius:3px}")


def _e(x) -> str:
    return html.escape(str(x if x is not None else ""))


def _page(title: str, body: str) -> str:
    return (f"<!doctype html><html><head><meta charset='utf-8'><title>{_e(title)}</title><style>{_CSS}</style>"
            f"</head><body><p><a href='/'>pipelines</a></p><h2>{_e(title)}</h2>{body}</body></html>")


def _phase(p) -> str:
    return f"<span class='ph' style='background:{_PHASE_COLOURS.get(str(p), '#616161')}'>{_e(p)}</span>"


def _ts(t) -> str:
    try:
        t = float(t)
    except (TypeError, ValueError):
        return _e(t)
    return time.strftime("%Y-%m-%d %H:%M:%S", time.localtime(t)) if t > 0 else ""


def index(backend) -> str:
    exps = backend.list_experiments("", 1000, "created_at des")["experiments"]
    runs = backend.list_runs("", 1000, "created_at des", None)["runs"]
    pipes = backend.list_pipelines("", 1000, "created_at des")["pipelines"]
    ename = {e["id"]: e["name"] for e in exps}
    rows = "".join(f"<tr><td><a href='/ui/runs/{_e(r['id'])}'>{_e(r['name'])}</a></td><td>{_phase(r.get('status'))}"
                   f"</td><td>{_e(ename.get(r.get('experiment_id'), ''))}</td><td>{_e(r.get('created_at'))}</td>"
                   f"<td>{_e(r.get('finished_at', ''))}</td></tr>" for r in runs)
    erows = "".join(f"<tr><td>{_e(e['name'])}</td><td>{_e(e.get('description', ''))}</td>"
                    f"<td>{_e(e.get('created_at'))}</td></tr>" for e in exps)
    prows = "".join(f"<tr><td><a href='/ui/pipelines/{_e(p['id'])}'>{_e(p['name'])}</a></td>"
                    f"<td>{_e(', '.join(x.get('name', '') for x in p.get('parameters') or []))}</td>"
                    f"<td>{_e(p.get('created_at'))}</td></tr>" for p in pipes)
    body = (f"<h3>Runs ({len(runs)})</h3><table><tr><th>run</th><th>status</th><th>experiment</th><th>created</th>"
            f"<th>finished</th></tr>{rows}</table><h3>Experiments ({len(exps)})</h3><table><tr><th>name</th>"
            f"<th>description</th><th>created</th></tr>{erows}</table><h3>Pipelines ({len(pipes)})</h3><table><tr>"
            f"<th>name</th><th>parameters</th><th>uploaded</th></tr>{prows}</table>")
    return _page("Pipelines", body)


def layout(nodes: dict[str, list[str]]) -> dict[str, tuple[int, int]]:
    """Longest-path depth of every node of a DAG given as {node: [children]} -> {node: (depth, index in layer)}."""
    parents: dict[str, list[str]] = {n: [] for n in nodes}
    for n, ch in nodes.items():
        for c in ch:
            parents.setdefault(c, []).append(n)
    depth: dict[str, int] = {}

    def d(n, seen=()):
        if n in depth:
            return depth[n]
        if n in seen:  # (a cycle cannot come from a valid workflow; do not recurse forever)
            return 0
        depth[n] = v = 1 + max((d(p, seen + (n,)) for p in parents.get(n, [])), default=-1)
        return v

    for n in parents:
        d(n)
    layers: dict[int, list[str]] = {}
    for n in sorted(depth, key=lambda k: (depth[k], k)):
        layers.setdefault(depth[n], []).append(n)
    return {n: (dep, i) for dep, ns in layers.items() for i, n in enumerate(ns)}


def _svg(nodes: dict[str, list[str]], label, colour) -> str:
    pos = layout(nodes)
    if not pos:
        return ""
    W, H, GX, GY = 170, 34, 40, 30
    cols = max(i for _, i in pos.values()) + 1
    rows = max(d for d, _ in pos.values()) + 1
    xy = {n: (10 + i * (W + GX), 10 + dep * (H + GY)) for n, (dep, i) in pos.items()}
    edges = "".join(f"<line x1='{xy[a][0] + W / 2}' y1='{xy[a][1] + H}' x2='{xy[b][0] + W / 2}' y2='{xy[b][1]}' "
                    f"stroke='#888' marker-end='url(#ar)'/>" for a, ch in nodes.items() for b in ch if b in xy)
    boxes = "".join(f"<g><rect x='{x}' y='{y}' width='{W}' height='{H}' rx='5' fill='{colour(n)}'/>"
                    f"<text x='{x + W / 2}' y='{y + H / 2 + 4}' text-anchor='middle' fill='#fff' font-size='12'>"
                    f"{_e(str(label(n))[:26])}</text></g>" for n, (x, y) in xy.items())
    return (f"<svg width='{20 + cols * (W + GX)}' height='{20 + rows * (H + GY)}' xmlns='http://www.w3.org/2000/svg'>"
            "<defs><marker id='ar' markerWidth='8' markerHeight='8' refX='6' refY='3' orient='auto'>"
            f"<path d='M0,0 L6,3 L0,6 z' fill='#888'/></marker></defs>{edges}{boxes}</svg>")


def run_page(backend, run_id: str) -> str:
    res = backend.get_run(run_id)
    run = res["run"]
    wf = json.loads(res["pipeline_runtime"]["workflow_manifest"])
    st = wf.get("status") or {}
    nodes = st.get("nodes") or {}
    graph = {k: [c for c in v.get("children", []) if c in nodes] for k, v in nodes.items()}
    svg = _svg(graph, lambda k: nodes[k].get("name", k),
               lambda k: _PHASE_COLOURS.get(nodes[k].get("phase"), "#616161"))

    def outs(v) -> str:
        return ", ".join(f"{p['name']}={p['value']}" for p in (v.get("outputs") or {}).get("parameters", []))

    rows = "".join(
        f"<tr><td>{_e(v.get('name', k))}</td><td>{_e(v.get('templateName'))}</td><td>{_phase(v.get('phase'))}</td>"
        f"<td>{_ts(v.get('startedAt'))}</td><td>{_ts(v.get('finishedAt'))}</td><td>{_e(v.get('attempts', ''))}</td>"
        f"<td>{_e(outs(v))}</td><td>{_e(v.get('message', ''))}</td></tr>"
        for k, v in sorted(nodes.items(), key=lambda kv: kv[1].get("startedAt") or 0))
    params = ", ".join(f"{p['name']}={p['value']}" for p in (run.get("pipeline_spec") or {}).get("parameters", []))
    body = (f"<p>status {_phase(run.get('status'))} &middot; created {_e(run.get('created_at'))} &middot; finished "
            f"{_e(run.get('finished_at', ''))} &middot; parameters {_e(params)}</p>{svg}"
            f"<table><tr><th>node</th><th>template</th><th>phase</th><th>started</th><th>finished</th><th>attempts</th>"
            f"<th>outputs</th><th>message</th></tr>{rows}</table>"
            f"{('<p>' + _e(st.get('message')) + '</p>') if st.get('message') else ''}")
    return _page(f"Run {run.get('name')}", body)


def pipeline_page(backend, pipeline_id: str) -> str:
    p = backend._read("pipelines", pipeline_id)
    wf = p.get("workflow") or {}
    spec = wf.get("spec", {})
    graph: dict[str, list[str]] = {}
    for t in spec.get("templates", []):
        for task in (t.get("dag") or {}).get("tasks", []):
            graph.setdefault(task["name"], [])
            for dep in task.get("dependencies", []) or []:
                graph.setdefault(dep, []).append(task["name"])
    svg = _svg(graph, lambda k: k, lambda k: "#455a64")
    tmpl = "".join(f"<tr><td>{_e(t.get('name'))}</td><td>{_e((t.get('container') or {}).get('image', ''))}</td></tr>"
                   for t in spec.get("templates", []))
    return _page(f"Pipeline {p.get('name')}", f"{svg}<table><tr><th>template</th><th>image</th></tr>{tmpl}</table>")
