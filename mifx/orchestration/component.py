"""Component model: spec (parameters / input channels / output channels), executor, and the
driver -> executor -> publisher contract of a TFX 0.13-style component.

Reference: components used in `airflow-dags/taxi_pipeline.py:73-120` and their channel names
(SURVEY §2.3 T1-T9). Executors implement ``Do(input_dict, output_dict, exec_properties)``.
"""
from __future__ import annotations

import json
import logging
from typing import Any

from .artifact import Artifact, Channel, ChannelMap


class ExecutionParameter:
    def __init__(self, type=None, optional: bool = False, default: Any = None):  # noqa: A002
        self.type = type
        self.optional = optional
        self.default = default


class ChannelParameter:
    def __init__(self, type_name: str, optional: bool = False):
        self.type_name = type_name
        self.optional = optional


class ComponentSpec:
    PARAMETERS: dict[str, ExecutionParameter] = {}
    INPUTS: dict[str, ChannelParameter] = {}
    OUTPUTS: dict[str, ChannelParameter] = {}

    def __init__(self, **kwargs):
        self.exec_properties: dict[str, Any] = {}
        self.inputs = ChannelMap()
        self.outputs = ChannelMap()
        for k, p in self.PARAMETERS.items():
            if k in kwargs and kwargs[k] is not None:
                self.exec_properties[k] = kwargs[k]
            elif not p.optional:
                raise ValueError(f"{type(self).__name__}: missing required parameter {k!r}")
            else:
                self.exec_properties[k] = p.default
        for k, p in self.INPUTS.items():
            ch = kwargs.get(k)
            if ch is None:
                if not p.optional:
                    raise ValueError(f"{type(self).__name__}: missing required input {k!r}")
                continue
            if not isinstance(ch, Channel):
                raise TypeError(f"{type(self).__name__}.{k}: expected Channel, got {type(ch).__name__}")
            if ch.type_name != p.type_name:
                raise TypeError(f"{type(self).__name__}.{k}: expected {p.type_name}, got {ch.type_name}")
            self.inputs[k] = ch
        for k, p in self.OUTPUTS.items():
            ch = kwargs.get(k)
            self.outputs[k] = ch if isinstance(ch, Channel) else Channel(p.type_name)
        unknown = set(kwargs) - set(self.PARAMETERS) - set(self.INPUTS) - set(self.OUTPUTS)
        if unknown:
            raise ValueError(f"{type(self).__name__}: unknown arguments {sorted(unknown)}")


class ExecutorContext:
    def __init__(self, tmp_dir: str = "", device: str | None = None, extra: dict | None = None,
                 logger: logging.Logger | None = None):
        self.tmp_dir = tmp_dir
        self.device = device
        self.extra = extra or {}
        self.logger = logger or logging.getLogger("mifx.executor")


class BaseExecutor:
    def __init__(self, context: ExecutorContext | None = None):
        self.context = context or ExecutorContext()

    def Do(self, input_dict: dict[str, list[Artifact]], output_dict: dict[str, list[Artifact]],  # noqa: N802
           exec_properties: dict[str, Any]) -> None:
        raise NotImplementedError


class BaseComponent:
    SPEC_CLASS = ComponentSpec
    EXECUTOR_CLASS = BaseExecutor
    EXECUTION_TYPE = "component"
    # output key -> list of split names (one artifact per split); missing key -> single artifact
    OUTPUT_SPLITS: dict[str, list[str]] = {}

    def __init__(self, spec: ComponentSpec, name: str | None = None, executor_class=None):
        self.spec = spec
        self.component_name = type(self).__name__
        self.name = name
        self.executor_class = executor_class or self.EXECUTOR_CLASS
        self.upstream_nodes: set[BaseComponent] = set()
        self.downstream_nodes: set[BaseComponent] = set()
        for k, ch in self.outputs.items():
            ch.producer = (self, k)

    @property
    def id(self) -> str:
        return f"{self.component_name}.{self.name}" if self.name else self.component_name

    @property
    def inputs(self) -> ChannelMap:
        return self.spec.inputs

    @property
    def outputs(self) -> ChannelMap:
        return self.spec.outputs

    @property
    def exec_properties(self) -> dict:
        return self.spec.exec_properties

    def output_splits(self, key: str, input_dict: dict[str, list[Artifact]]) -> list[str]:
        return self.OUTPUT_SPLITS.get(key, [""])

    def add_upstream_node(self, other: "BaseComponent") -> None:
        self.upstream_nodes.add(other)
        other.downstream_nodes.add(self)

    def serializable_exec_properties(self) -> dict:
        out = {}
        for k, v in self.exec_properties.items():
            out[k] = to_jsonable(v)
        return out

    def __repr__(self):
        return f"<{self.id}>"


def to_jsonable(v):
    if hasattr(v, "to_dict"):
        return v.to_dict()
    if isinstance(v, (list, tuple)):
        return [to_jsonable(x) for x in v]
    if isinstance(v, dict):
        return {k: to_jsonable(x) for k, x in v.items()}
    try:
        json.dumps(v)
        return v
    except TypeError:
        return repr(v)
