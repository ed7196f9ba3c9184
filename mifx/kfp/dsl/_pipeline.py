"""@pipeline decorator, PipelineConf and the Pipeline context that registers ops and groups.

Reference: `sdk/python/kfp/dsl/_pipeline.py:25-240` (decorator hook used by dsl-compile's
PipelineCollectorContext; unique op names by appending " 2", " 3", ...; nested pipelines
rejected)."""
from __future__ import annotations

from . import _container_op, _ops_group
from ._metadata import PipelineMeta, _extract_pipeline_metadata


def _pipeline_decorator_handler(func):  # swapped by compiler.main.PipelineCollectorContext
    return func


def pipeline(name: str | None = None, description: str | None = None):
    def _pipeline(func):
        if name:
            func._pipeline_name = name
        if description:
            func._pipeline_description = description
        from .. import _config

        if _config.type_check_enabled():
            func._pipeline_meta = _extract_pipeline_metadata(func, validate=False)
        from . import _pipeline as me

        return me._pipeline_decorator_handler(func) or func

    return _pipeline


class PipelineConf:
    def __init__(self):
        self.image_pull_secrets = []
        self.timeout = 0
        self.artifact_location = None
        self.op_transformers = []

    def set_image_pull_secrets(self, image_pull_secrets):
        self.image_pull_secrets = image_pull_secrets
        return self

    def set_timeout(self, seconds: int):
        self.timeout = seconds
        return self

    def set_artifact_location(self, artifact_location):
        self.artifact_location = artifact_location
        return self

    def add_op_transformer(self, transformer):
        self.op_transformers.append(transformer)
        return self


def get_pipeline_conf() -> PipelineConf:
    p = Pipeline.get_default_pipeline()
    if p is None:
        raise ValueError("get_pipeline_conf() must be called inside a pipeline function being compiled")
    return p.conf


def _make_name_unique_by_adding_index(name: str, collection, delimiter: str) -> str:
    unique = name
    i = 2
    while unique in collection:
        unique = f"{name}{delimiter}{i}"
        i += 1
    return unique


class Pipeline:
    _default_pipeline = None

    @staticmethod
    def get_default_pipeline():
        return Pipeline._default_pipeline

    @staticmethod
    def add_pipeline(name, description, func):
        return pipeline(name=name, description=description)(func)

    def __init__(self, name: str):
        self.name = name
        self.ops = {}
        self.groups = [_ops_group.OpsGroup("pipeline", name=name)]
        self.group_id = 0
        self.conf = PipelineConf()
        self._metadata = None

    def __enter__(self):
        if Pipeline._default_pipeline:
            raise Exception("Nested pipelines are not allowed.")
        Pipeline._default_pipeline = self
        self._old_handler = _container_op._register_op_handler
        _container_op._register_op_handler = lambda op: self.add_op(op, op.is_exit_handler)
        return self

    def __exit__(self, *args):
        Pipeline._default_pipeline = None
        _container_op._register_op_handler = self._old_handler

    def add_op(self, op, define_only: bool) -> str:
        op_name = _make_name_unique_by_adding_index(op.human_name, list(self.ops.keys()), " ")
        self.ops[op_name] = op
        if not define_only:
            self.groups[-1].ops.append(op)
        return op_name

    def push_ops_group(self, group):
        self.groups[-1].groups.append(group)
        self.groups.append(group)

    def pop_ops_group(self):
        del self.groups[-1]

    def get_next_group_id(self) -> int:
        self.group_id += 1
        return self.group_id

    def _set_metadata(self, metadata):
        if not isinstance(metadata, PipelineMeta):
            raise ValueError("_set_metadata is expecting PipelineMeta.")
        self._metadata = metadata
