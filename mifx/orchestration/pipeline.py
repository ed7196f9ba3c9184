"""Logical pipeline: a DAG of components wired by channels.

Reference: ``tfx.orchestration.pipeline.Pipeline(pipeline_name, pipeline_root, components,
enable_cache, metadata_db_root, additional_pipeline_args={'logger_args': ...})``
(`airflow-dags/taxi_pipeline.py:122-132`). Topological order uses Kahn's algorithm with the same
cycle detection semantics as the KFP GraphSpec toposort (`sdk/python/kfp/components/_structures.py:499-533`).
"""
from __future__ import annotations

import os
from typing import Sequence

from ..metadata.proto import ConnectionConfig
from .component import BaseComponent


class CycleError(ValueError):
    pass


def topological_sort(components: Sequence[BaseComponent]) -> list[BaseComponent]:
    comps = list(components)
    indeg = {c: 0 for c in comps}
    for c in comps:
        for u in c.upstream_nodes:
            if u in indeg:
                indeg[c] += 1
    ready = [c for c in comps if indeg[c] == 0]
    order = []
    while ready:
        c = ready.pop(0)
        order.append(c)
        for d in sorted(c.downstream_nodes, key=lambda x: comps.index(x) if x in comps else 0):
            if d in indeg:
                indeg[d] -= 1
                if indeg[d] == 0:
                    ready.append(d)
    if len(order) != len(comps):
        stuck = [c.id for c in comps if c not in order]
        raise CycleError(f"pipeline has a cycle involving {stuck}")
    return order


def sqlite_metadata_connection_config(path: str) -> ConnectionConfig:
    cfg = ConnectionConfig()
    cfg.sqlite.filename_uri = path
    return cfg


class Pipeline:
    def __init__(self, pipeline_name: str, pipeline_root: str, components: Sequence[BaseComponent],
                 enable_cache: bool = False, metadata_db_root: str | None = None,
                 metadata_connection_config: ConnectionConfig | None = None,
                 additional_pipeline_args: dict | None = None, beam_pipeline_args: list | None = None):
        self.pipeline_name = pipeline_name
        self.pipeline_root = pipeline_root
        self.enable_cache = enable_cache
        self.additional_pipeline_args = additional_pipeline_args or {}
        self.beam_pipeline_args = beam_pipeline_args or []
        if metadata_connection_config is None:
            root = metadata_db_root or os.path.join(pipeline_root, "metadata")
            metadata_connection_config = sqlite_metadata_connection_config(
                os.path.join(root, pipeline_name, "metadata.db"))
        self.metadata_connection_config = metadata_connection_config
        ids = [c.id for c in components]
        dup = {i for i in ids if ids.count(i) > 1}
        if dup:
            raise ValueError(f"duplicate component ids {sorted(dup)}; pass name= to disambiguate")
        # wire implicit dependencies from channels
        producers = {}
        for c in components:
            for ch in c.outputs.values():
                producers[id(ch)] = c
        for c in components:
            for ch in c.inputs.values():
                p = producers.get(id(ch))
                if p is not None and p is not c:
                    c.add_upstream_node(p)
        self.components = topological_sort(components)

    def __repr__(self):
        return f"Pipeline({self.pipeline_name}, {[c.id for c in self.components]})"
