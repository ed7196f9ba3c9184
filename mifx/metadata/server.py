"""Metadata service: the MLMD store over HTTP (+ a lineage / run dashboard page).

The reference deploys ML Metadata behind Kubeflow (the notebooks open the TFX sqlite store directly:
`notebooks/tfx_utils.py:53-65`, `notebooks/utils.py:214-503`) and the Kubeflow UI shows runs and artifacts
(`install-kubeflow/app.yaml:15-46`: centraldashboard, pipeline UI). This service exposes the read API those
notebooks use -- types, artifacts, executions, events, contexts, and the recursive source / destination artifact
search of `ReadonlyMetadataStore` -- as JSON, and renders one HTML page listing the pipeline runs (contexts)
with their executions and artifacts. It reads the same sqlite store the runners write
(`<root>/metadata/<pipeline>/metadata.db`).

    python -m mifx.metadata.server --db /mnt/pipelines/metadata/taxi/metadata.db --port 8080
"""
from __future__ import annotations

import argparse
import html

from .lineage import ReadonlyMetadataStore, _value_str
from .store import MetadataStore


def _props(obj) -> dict:
    out = {k: _value_str(v) for k, v in obj.properties.items()}
    out.update({k: _value_str(v) for k, v in obj.custom_properties.items()})
    return out


def _artifact(a, types: dict) -> dict:
    return {"id": a.id, "type": types.get(a.type_id), "uri": a.uri, "properties": _props(a)}


def _execution(e, types: dict) -> dict:
    return {"id": e.id, "type": types.get(e.type_id), "properties": _props(e)}


def create_app(db_path: str):
    from fastapi import FastAPI, HTTPException
    from fastapi.responses import HTMLResponse

    app = FastAPI(title="mifx metadata service")

    db = MetadataStore(db_path)  # sqlite (WAL): sees what the runners commit; one connection for the service

    def store() -> MetadataStore:
        return db

    def atypes(s):
        return {t.id: t.name for t in s.get_artifact_types()}

    def etypes(s):
        return {t.id: t.name for t in s.get_execution_types()}

    @app.get("/healthz")
    def healthz():
        return {"status": "ok"}

    @app.get("/api/v1/artifact_types")
    def artifact_types():
        s = store()
        return [{"id": t.id, "name": t.name} for t in s.get_artifact_types()]

    @app.get("/api/v1/execution_types")
    def execution_types():
        s = store()
        return [{"id": t.id, "name": t.name} for t in s.get_execution_types()]

    @app.get("/api/v1/artifacts")
    def artifacts(type: str | None = None):  # noqa: A002 (query parameter name)
        s = store()
        arts = s.get_artifacts_by_type(type) if type else s.get_artifacts()
        t = atypes(s)
        return [_artifact(a, t) for a in arts]

    @app.get("/api/v1/artifacts/{aid}")
    def artifact(aid: int):
        s = store()
        got = s.get_artifacts_by_id([aid])
        if not got:
            raise HTTPException(404, f"artifact {aid} not found")
        return _artifact(got[0], atypes(s))

    @app.get("/api/v1/executions")
    def executions(type: str | None = None):  # noqa: A002
        s = store()
        ex = s.get_executions_by_type(type) if type else s.get_executions()
        t = etypes(s)
        return [_execution(e, t) for e in ex]

    @app.get("/api/v1/executions/{eid}")
    def execution(eid: int):
        s = store()
        got = s.get_executions_by_id([eid])
        if not got:
            raise HTTPException(404, f"execution {eid} not found")
        return _execution(got[0], etypes(s))

    @app.get("/api/v1/events")
    def events(artifact_id: int | None = None, execution_id: int | None = None):
        s = store()
        if artifact_id is None and execution_id is None:
            raise HTTPException(400, "artifact_id or execution_id required")
        ev = s.get_events_by_artifact_ids([artifact_id]) if artifact_id is not None else \
            s.get_events_by_execution_ids([execution_id])
        return [{"artifact_id": e.artifact_id, "execution_id": e.execution_id, "type": int(e.type),
                 "path": [p.key for p in e.path] if e.path else []} for e in ev]

    @app.get("/api/v1/contexts")
    def contexts():
        s = store()
        return [{"id": c.id, "name": c.name, "properties": _props(c)} for c in s.get_contexts()]

    @app.get("/api/v1/lineage/{aid}")
    def lineage(aid: int, direction: str = "upstream", type: str | None = None):  # noqa: A002
        """The nearest upstream (source) or downstream (destination) artifact of a type -- the notebooks'
        get_source_artifact_of_type / get_dest_artifact_of_type -- or, without a type, the lineage graph."""
        s = store()
        ro = ReadonlyMetadataStore(s)
        if type:
            fn = ro.get_source_artifact_of_type if direction == "upstream" else ro.get_dest_artifact_of_type
            a = fn(aid, type)
            return _artifact(a, atypes(s)) if a is not None else None
        g = ro.get_artifact_lineage(aid)
        return {"nodes": [{"id": n, **{k: str(v) for k, v in d.items()}} for n, d in g.nodes(data=True)],
                "edges": [[u, v] for u, v in g.edges()]}

    @app.get("/", response_class=HTMLResponse)
    def dashboard():
        s = store()
        t_a, t_e = atypes(s), etypes(s)
        rows = []
        for c in s.get_contexts():
            ex = s.get_executions_by_context(c.id)
            arts = s.get_artifacts_by_context(c.id)
            rows.append(f"<h2>{html.escape(c.name)}</h2><table border=1><tr><th>execution</th><th>type</th>"
                        f"<th>state</th></tr>" + "".join(
                            f"<tr><td>{e.id}</td><td>{html.escape(str(t_e.get(e.type_id)))}</td>"
                            f"<td>{html.escape(_props(e).get('state', ''))}</td></tr>" for e in ex) + "</table>"
                        "<table border=1><tr><th>artifact</th><th>type</th><th>uri</th></tr>" + "".join(
                            f"<tr><td>{a.id}</td><td>{html.escape(str(t_a.get(a.type_id)))}</td>"
                            f"<td>{html.escape(a.uri)}</td></tr>" for a in arts) + "</table>")
        return "<html><head><title>mifx metadata</title></head><body><h1>Pipeline runs</h1>" + "".join(rows) + \
            "</body></html>"

    return app


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="python -m mifx.metadata.server")
    ap.add_argument("--db", required=True, help="sqlite MLMD file (<root>/metadata/<pipeline>/metadata.db)")
    ap.add_argument("--host", default="0.0.0.0")
    ap.add_argument("--port", type=int, default=8080)
    a = ap.parse_args(argv)
    import uvicorn

    uvicorn.run(create_app(a.db), host=a.host, port=a.port)
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
