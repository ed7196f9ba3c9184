"""Component launcher (driver -> executor -> publisher) with MLMD lineage and caching, and the
in-process ``LocalDagRunner``.

Reference behaviour: each component's driver resolves input artifacts from MLMD
and, with ``enable_cache=True``, skips execution when an identical execution (same inputs, exec
properties and module code) already completed; the executor runs; the publisher records output
artifacts and INPUT/OUTPUT events. Execution type names follow `notebooks/tfx_utils.py:39-47`.
Independent components may run concurrently (Argo-style task parallelism).
"""
from __future__ import annotations

import concurrent.futures as cf
import hashlib
import json
import logging
import os
import shutil
import tempfile
import time
import traceback
import uuid
from dataclasses import dataclass, field

from ..metadata.proto import (ContextType, Context, Event, EventPathStep, Execution, ExecutionState,
                              ExecutionType, STRING, INT)
from ..metadata.store import MetadataStore
from .artifact import EXTERNAL, Artifact
from .component import BaseComponent, ExecutorContext
from .pipeline import Pipeline

log = logging.getLogger("mifx.orchestration")

FRAMEWORK_VERSION = "mifx-0.1"


def _file_digest(path: str) -> str:
    h = hashlib.sha256()
    if os.path.isdir(path):
        for root, _, files in sorted(os.walk(path)):
            for f in sorted(files):
                p = os.path.join(root, f)
                h.update(os.path.relpath(p, path).encode())
                with open(p, "rb") as fh:
                    h.update(fh.read())
    elif os.path.exists(path):
        with open(path, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()


@dataclass
class ComponentRun:
    component_id: str
    execution_id: int
    state: str
    outputs: dict = field(default_factory=dict)
    seconds: float = 0.0
    error: str | None = None


@dataclass
class RunResult:
    pipeline_name: str
    run_id: str
    components: dict = field(default_factory=dict)  # id -> ComponentRun

    @property
    def succeeded(self) -> bool:
        return all(r.state in ("complete", "cached") for r in self.components.values())


class Launcher:
    def __init__(self, pipeline: Pipeline, store: MetadataStore, run_id: str, device: str | None = None):
        self.pipeline = pipeline
        self.store = store
        self.run_id = run_id
        self.device = device
        ctype = ContextType(name="pipeline", properties={"pipeline_name": STRING})
        rtype = ContextType(name="run", properties={"pipeline_name": STRING, "run_id": STRING})
        self.store.put_context_type(ctype)
        self.store.put_context_type(rtype)
        self.contexts = [Context(type_id=ctype.id, name=pipeline.pipeline_name),
                         Context(type_id=rtype.id, name=f"{pipeline.pipeline_name}.{run_id}")]
        self.contexts[0].properties["pipeline_name"] = pipeline.pipeline_name
        self.contexts[1].properties["pipeline_name"] = pipeline.pipeline_name
        self.contexts[1].properties["run_id"] = run_id
        self.store.put_contexts(self.contexts)

    # ---------------------------------------------------------------------- driver
    def _register(self, art: Artifact) -> Artifact:
        art.type_id = self.store.put_artifact_type(art.mlmd_type())
        return art

    def _resolve_inputs(self, comp: BaseComponent) -> dict[str, list[Artifact]]:
        out = {}
        for key, ch in comp.inputs.items():
            arts = ch.get()
            if not arts:
                raise RuntimeError(f"{comp.id}: input {key!r} has no artifacts (did its producer run?)")
            resolved = []
            for a in arts:
                if a.id is None:  # external input: register once per uri
                    self._register(a)
                    existing = [x for x in self.store.get_artifacts_by_uri(a.uri) if x.type_id == a.type_id]
                    if existing:
                        a.id = existing[0].id
                    else:
                        [a.id] = self.store.put_artifacts([a.to_mlmd()])
                resolved.append(a)
            out[key] = resolved
        return out

    def _fingerprint(self, comp: BaseComponent, inputs: dict[str, list[Artifact]]) -> str:
        props = comp.serializable_exec_properties()
        code = {}
        for k, v in comp.exec_properties.items():
            if isinstance(v, str) and k.endswith(("module_file", "_file")) and os.path.exists(v):
                code[k] = _file_digest(v)
        ins = {k: [(a.type_name, a.uri, a.split, _file_digest(a.uri) if a.type_name == EXTERNAL else a.id)
                   for a in v] for k, v in sorted(inputs.items())}
        blob = json.dumps({"component": comp.id, "executor": f"{comp.executor_class.__module__}."
                           f"{comp.executor_class.__qualname__}", "props": props, "code": code, "inputs": ins,
                           "version": FRAMEWORK_VERSION}, sort_keys=True, default=str)
        return hashlib.sha256(blob.encode()).hexdigest()

    def _cached_outputs(self, comp: BaseComponent, fp: str) -> dict[str, list[Artifact]] | None:
        for ex in reversed(self.store.get_executions_by_type(comp.EXECUTION_TYPE)):
            if ex.last_known_state != ExecutionState.COMPLETE:
                continue
            if ex.custom_properties["fingerprint"].string_value != fp:
                continue
            outs: dict[str, list[Artifact]] = {}
            evs = [e for e in self.store.get_events_by_execution_ids([ex.id]) if e.type == Event.Type.OUTPUT]
            arts = {a.id: a for a in self.store.get_artifacts_by_id([e.artifact_id for e in evs])}
            types = {t.id: t.name for t in self.store.get_artifact_types()}
            ok = True
            for e in evs:
                key = e.path[0].key if e.path else "output"
                a = arts[e.artifact_id]
                if not os.path.exists(a.uri):
                    ok = False
                outs.setdefault(key, []).append(Artifact.from_mlmd(a, types[a.type_id]))
            if ok and set(outs) == set(comp.outputs):
                return outs
        return None

    # ---------------------------------------------------------------------- launch
    def launch(self, comp: BaseComponent, enable_cache: bool) -> ComponentRun:
        t0 = time.time()
        etype = ExecutionType(name=comp.EXECUTION_TYPE, properties={
            "component_id": STRING, "pipeline_name": STRING, "run_id": STRING, "state": STRING,
            "pipeline_root": STRING, "checksum_md5": STRING, "num_retries": INT})
        self.store.put_execution_type(etype)
        inputs = self._resolve_inputs(comp)
        fp = self._fingerprint(comp, inputs)
        ex = Execution(type_id=etype.id, name=f"{comp.id}.{self.run_id}", last_known_state=ExecutionState.RUNNING)
        ex.properties["component_id"] = comp.id
        ex.properties["pipeline_name"] = self.pipeline.pipeline_name
        ex.properties["run_id"] = self.run_id
        ex.properties["pipeline_root"] = self.pipeline.pipeline_root
        ex.properties["state"] = "running"
        ex.custom_properties["fingerprint"] = fp
        for k, v in comp.serializable_exec_properties().items():
            ex.custom_properties[k] = v if isinstance(v, (int, float, str)) and not isinstance(v, bool) \
                else json.dumps(v, default=str)
        cached = self._cached_outputs(comp, fp) if enable_cache else None
        if cached is not None:
            ex.last_known_state = ExecutionState.CACHED
            ex.properties["state"] = "cached"
            self._publish(comp, ex, inputs, cached)
            for k, arts in cached.items():
                comp.outputs[k].set(arts)
            log.info("%s: cache hit (execution %s)", comp.id, ex.id)
            return ComponentRun(comp.id, ex.id, "cached", cached, time.time() - t0)
        [eid] = self.store.put_executions([ex])
        outputs: dict[str, list[Artifact]] = {}
        for key, ch in comp.outputs.items():
            arts = []
            for split in comp.output_splits(key, inputs):
                uri = os.path.join(self.pipeline.pipeline_root, comp.id, key, str(eid), split)
                if os.path.exists(uri):
                    shutil.rmtree(uri)
                os.makedirs(uri, exist_ok=True)
                a = self._register(Artifact(ch.type_name, split=split, uri=uri))
                a.producer_component = comp.id
                a.name = f"{comp.id}.{key}"
                arts.append(a)
            outputs[key] = arts
        tmp = tempfile.mkdtemp(prefix=f"mifx-{comp.id}-")
        try:
            extra = dict(self.pipeline.additional_pipeline_args)
            extra["__metadata_store__"] = self.store
            extra["__pipeline__"] = self.pipeline
            executor = comp.executor_class(ExecutorContext(tmp_dir=tmp, device=self.device, extra=extra))
            executor.Do(inputs, outputs, dict(comp.exec_properties))
        except Exception as e:  # record the failure in MLMD, then propagate
            ex.last_known_state = ExecutionState.FAILED
            ex.properties["state"] = "failed"
            ex.custom_properties["error"] = f"{type(e).__name__}: {e}"
            self.store.put_executions([ex])
            self.store.put_attributions_and_associations([], [(c.id, ex.id) for c in self.contexts])
            return ComponentRun(comp.id, ex.id, "failed", {}, time.time() - t0, traceback.format_exc())
        finally:
            shutil.rmtree(tmp, ignore_errors=True)
        ex.last_known_state = ExecutionState.COMPLETE
        ex.properties["state"] = "complete"
        self._publish(comp, ex, inputs, outputs)
        for k, arts in outputs.items():
            comp.outputs[k].set(arts)
        return ComponentRun(comp.id, ex.id, "complete", outputs, time.time() - t0)

    def _publish(self, comp, ex: Execution, inputs, outputs) -> None:
        pairs = []
        for key, arts in inputs.items():
            for i, a in enumerate(arts):
                m = a.to_mlmd()
                pairs.append((m, Event(type=Event.Type.INPUT, path=[EventPathStep(key=key), EventPathStep(index=i)])))
        out_objs = []
        for key, arts in outputs.items():
            for i, a in enumerate(arts):
                m = a.to_mlmd()
                out_objs.append((a, m))
                pairs.append((m, Event(type=Event.Type.OUTPUT, path=[EventPathStep(key=key), EventPathStep(index=i)])))
        self.store.put_execution(ex, pairs, self.contexts)
        for a, m in out_objs:
            a.id = m.id


class LocalDagRunner:
    """Runs a pipeline in-process, topologically, optionally with concurrent independent tasks."""

    def __init__(self, max_parallel: int = 1, device: str | None = None, fail_fast: bool = True):
        self.max_parallel = max(1, max_parallel)
        self.device = device
        self.fail_fast = fail_fast

    def _configure_logging(self, pipeline: Pipeline):
        la = pipeline.additional_pipeline_args.get("logger_args")
        if la and la.get("log_root"):
            os.makedirs(la["log_root"], exist_ok=True)
            h = logging.FileHandler(os.path.join(la["log_root"], f"{pipeline.pipeline_name}.log"))
            h.setFormatter(logging.Formatter("%(asctime)s %(levelname)s %(name)s: %(message)s"))
            lg = logging.getLogger("mifx")
            lg.addHandler(h)
            lg.setLevel(getattr(logging, str(la.get("log_level", "INFO")).upper(), logging.INFO))

    def run(self, pipeline: Pipeline, run_id: str | None = None) -> RunResult:
        self._configure_logging(pipeline)
        store = MetadataStore(pipeline.metadata_connection_config)
        run_id = run_id or time.strftime("%Y%m%d-%H%M%S") + "-" + uuid.uuid4().hex[:6]
        launcher = Launcher(pipeline, store, run_id, self.device)
        result = RunResult(pipeline.pipeline_name, run_id)
        done: set = set()
        failed: set = set()
        pending = list(pipeline.components)
        with cf.ThreadPoolExecutor(self.max_parallel) as pool:
            running: dict = {}
            while pending or running:
                for c in list(pending):
                    if len(running) >= self.max_parallel:
                        break
                    if any(u in failed for u in c.upstream_nodes):
                        pending.remove(c)
                        failed.add(c)
                        result.components[c.id] = ComponentRun(c.id, -1, "skipped")
                        continue
                    if all(u in done for u in c.upstream_nodes):
                        pending.remove(c)
                        running[pool.submit(launcher.launch, c, pipeline.enable_cache)] = c
                if not running:
                    break
                fin, _ = cf.wait(list(running), return_when=cf.FIRST_COMPLETED)
                for f in fin:
                    c = running.pop(f)
                    r = f.result()
                    result.components[c.id] = r
                    if r.state == "failed":
                        failed.add(c)
                        log.error("%s failed:\n%s", c.id, r.error)
                        if self.fail_fast:
                            pending.clear()
                    else:
                        done.add(c)
        store.close()
        if not result.succeeded and self.fail_fast:
            errs = {k: v.error for k, v in result.components.items() if v.state == "failed"}
            raise RuntimeError(f"pipeline {pipeline.pipeline_name} failed: {errs}")
        return result
