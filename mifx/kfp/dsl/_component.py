"""Component decorators: python_component (metadata), component (argument type checks),
graph_component (recursive sub-graphs).

Reference: `sdk/python/kfp/dsl/_component.py:21-125`."""
from __future__ import annotations

import functools

from ._metadata import TypeMeta, _extract_component_metadata
from ._ops_group import Graph
from ._pipeline_param import PipelineParam
from .types import InconsistentTypeException, check_types


def python_component(name, description=None, base_image=None, target_component_file: str | None = None):
    def _python_component(func):
        func._component_human_name = name
        if description:
            func._component_description = description
        if base_image:
            func._component_base_image = base_image
        if target_component_file:
            func._component_target_component_file = target_component_file
        return func

    return _python_component


def component(func):
    """Type-checks PipelineParam arguments against the annotations when kfp.TYPE_CHECK is on and
    attaches component metadata to the produced ContainerOp."""

    @functools.wraps(func)
    def _component(*args, **kwargs):
        from .. import _config

        if not _config.type_check_enabled():
            op = func(*args, **kwargs)
            op._set_metadata(_extract_component_metadata(func))
            return op
        meta = _extract_component_metadata(func)
        params = {p.name: p for p in meta.inputs}
        bound = dict(zip([p.name for p in meta.inputs], args))
        bound.update(kwargs)
        for k, v in bound.items():
            if isinstance(v, PipelineParam) and k in params:
                expected = params[k].param_type.to_dict_or_str()
                got = v.param_type.to_dict_or_str() if v.param_type else ""
                if expected and got and not check_types(got, expected):
                    raise InconsistentTypeException(
                        f"Component {meta.name} is expecting {k} to be type({expected}), but the passed argument is "
                        f"type({got})")
        op = func(*args, **kwargs)
        op._set_metadata(meta)
        return op

    return _component


def graph_component(func):
    @functools.wraps(func)
    def _graph_component(*args, **kwargs):
        g = Graph(func.__name__)
        g.inputs = list(args) + list(kwargs.values())
        for i in g.inputs:
            if not isinstance(i, PipelineParam):
                raise ValueError(f"arguments to {func.__name__} should be PipelineParams.")
        with g:
            if not g.recursive_ref:
                func(*args, **kwargs)
        return g

    return _graph_component


_ = TypeMeta
