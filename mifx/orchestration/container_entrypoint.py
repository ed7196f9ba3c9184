"""Run ONE component of a TFX-style pipeline in its own process / container.

Used by `KubeflowDagRunner` (each Argo step) and `AirflowDagRunner` (each Airflow task): the
pipeline is rebuilt from an importable factory (`module:function` + JSON kwargs), upstream
outputs of this run are resolved from the shared MLMD store (OUTPUT events of the producers'
executions in the run context), and the component is launched exactly as LocalDagRunner would
(driver -> executor -> publisher, cache fingerprinting, lineage).

    python3 -m mifx.orchestration.container_entrypoint --pipeline-factory examples.taxi.p:create \\
        --factory-args '{"root": "/mnt"}' --component-id StatisticsGen --run-id <uid>"""
from __future__ import annotations

import argparse
import importlib
import json
import logging
import sys

from ..metadata.proto import Event
from ..metadata.store import MetadataStore
from .artifact import Artifact
from .runner import Launcher


def load_factory(spec: str):
    mod, _, fn = spec.partition(":")
    return getattr(importlib.import_module(mod), fn)


def _upstream_closure(comp) -> list:
    seen, stack = [], list(comp.upstream_nodes)
    while stack:
        c = stack.pop()
        if c not in seen:
            seen.append(c)
            stack.extend(c.upstream_nodes)
    return seen


def resolve_outputs_from_mlmd(store: MetadataStore, pipeline_name: str, run_id: str, comp) -> bool:
    """Fill `comp.outputs` with the artifacts its execution in this run published. False if none."""
    ctx_name = f"{pipeline_name}.{run_id}"
    ctx = next((c for c in store.get_contexts() if c.name == ctx_name), None)
    if ctx is None:
        return False
    execs = [e for e in store.get_executions_by_context(ctx.id)
             if e.properties.get("component_id") is not None
             and e.properties["component_id"].string_value == comp.id
             and e.properties["state"].string_value in ("complete", "cached")]
    if not execs:
        return False
    ex = execs[-1]
    evs = [e for e in store.get_events_by_execution_ids([ex.id]) if e.type == Event.Type.OUTPUT]
    arts = {a.id: a for a in store.get_artifacts_by_id([e.artifact_id for e in evs])}
    types = {t.id: t.name for t in store.get_artifact_types()}
    outs: dict = {}
    for e in evs:
        key = e.path[0].key if e.path else "output"
        a = arts[e.artifact_id]
        outs.setdefault(key, []).append(Artifact.from_mlmd(a, types[a.type_id]))
    for k, v in outs.items():
        if k in comp.outputs:
            comp.outputs[k].set(v)
    return True


def run_component(pipeline, component_id: str, run_id: str, device: str | None = None):
    comp = next((c for c in pipeline.components if c.id == component_id), None)
    if comp is None:
        raise KeyError(f"component {component_id!r} not in pipeline {pipeline.pipeline_name}")
    store = MetadataStore(pipeline.metadata_connection_config)
    try:
        for up in _upstream_closure(comp):
            if not resolve_outputs_from_mlmd(store, pipeline.pipeline_name, run_id, up):
                raise RuntimeError(f"{component_id}: upstream {up.id} has no outputs in run {run_id}")
        return Launcher(pipeline, store, run_id, device).launch(comp, pipeline.enable_cache)
    finally:
        store.close()


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="python3 -m mifx.orchestration.container_entrypoint")
    ap.add_argument("--pipeline-factory", required=True)
    ap.add_argument("--factory-args", default="{}")
    ap.add_argument("--component-id", required=True)
    ap.add_argument("--run-id", required=True)
    ap.add_argument("--device", default=None)
    a = ap.parse_args(argv)
    logging.basicConfig(level=logging.INFO)
    pipeline = load_factory(a.pipeline_factory)(**json.loads(a.factory_args))
    r = run_component(pipeline, a.component_id, a.run_id, a.device)
    print(json.dumps({"component": r.component_id, "state": r.state, "execution_id": r.execution_id,
                      "seconds": round(r.seconds, 3)}))
    if r.state == "failed":
        print(r.error, file=sys.stderr)
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
