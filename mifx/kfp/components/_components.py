"""Component loading (file / URL / text / zip) and task-factory creation.

Reference: `sdk/python/kfp/components/_components.py:35-256` — the factory gets a generated
signature (required inputs first, defaults kept), PipelineParam arguments are type-checked against
input types when `kfp.TYPE_CHECK` is on, default I/O file paths are `/inputs/<name>/data` and
`/outputs/<name>/data` (the outputs dir is swappable for local execution tests)."""
from __future__ import annotations

import hashlib
import inspect
import os
import zipfile

from .. import _config
from ..dsl._pipeline_param import PipelineParam
from ..dsl.types import InconsistentTypeException, check_types
from . import _dynamic
from ._naming import _sanitize_file_name, _sanitize_python_function_name, generate_unique_name_conversion_table
from ._structures import ComponentReference, ComponentSpec, GraphInputArgument, TaskOutputArgument, TaskSpec
from ._yaml_utils import load_yaml

_default_component_name = "Component"
_inputs_dir = "/inputs"
_outputs_dir = "/outputs"
_single_io_file_name = "data"


def _generate_input_file_name(port_name: str) -> str:
    return _inputs_dir + "/" + _sanitize_file_name(port_name) + "/" + _single_io_file_name


def _generate_output_file_name(port_name: str) -> str:
    from . import _components as me  # module attr may be swapped (components_local_output_dir_context)

    return me._outputs_dir + "/" + _sanitize_file_name(port_name) + "/" + _single_io_file_name


def load_component(filename=None, url=None, text=None):
    if sum(x is not None for x in (filename, url, text)) != 1:
        raise ValueError("Need to specify exactly one source")
    if filename:
        return load_component_from_file(filename)
    if url:
        return load_component_from_url(url)
    return load_component_from_text(text)


def load_component_from_url(url: str):
    """Fetch component.yaml over HTTP(S) (or file://) and create a task factory."""
    if url is None:
        raise TypeError("url must not be None")
    if url.startswith("file://"):
        return load_component_from_file(url[len("file://"):])
    import requests

    resp = requests.get(url, timeout=60)
    resp.raise_for_status()
    digest = hashlib.sha256(resp.content).hexdigest()
    ref = ComponentReference(url=url, digest=digest)
    return _create_task_factory_from_component_text(resp.content, url, ref)


def load_component_from_file(filename: str):
    if filename is None:
        raise TypeError("filename must not be None")
    if filename.endswith(".zip"):
        with zipfile.ZipFile(filename) as z:
            with z.open("component.yaml") as f:
                return _create_task_factory_from_component_text(f, filename)
    with open(filename, "rb") as f:
        return _create_task_factory_from_component_text(f, filename)


def load_component_from_text(text: str):
    if text is None:
        raise TypeError("text must not be None")
    return _create_task_factory_from_component_text(text, None)


def _create_task_factory_from_component_text(text_or_file, component_filename=None, component_ref=None):
    return _create_task_factory_from_component_dict(load_yaml(text_or_file), component_filename, component_ref)


def _create_task_factory_from_component_dict(component_dict, component_filename=None, component_ref=None):
    return _create_task_factory_from_component_spec(ComponentSpec.from_dict(component_dict), component_filename,
                                                    component_ref)


def _try_get_object_by_name(obj_name: str):
    import builtins

    return builtins.__dict__.get(obj_name, obj_name)


# last handler turns a TaskSpec into a runnable object (ContainerOp by default; graph tasks and the
# local runner install their own)
_created_task_transformation_handler = []


def _create_task_factory_from_component_spec(component_spec: ComponentSpec, component_filename=None,
                                             component_ref: ComponentReference | None = None):
    name = component_spec.name or _default_component_name
    doc = "\n".join(x for x in (component_spec.name, component_spec.description) if x)
    inputs = component_spec.inputs or []
    to_py = generate_unique_name_conversion_table([i.name for i in inputs], _sanitize_python_function_name)
    from_py = {v: k for k, v in to_py.items()}
    if component_ref is None:
        component_ref = ComponentReference(name=component_spec.name or component_filename or _default_component_name)
    component_ref._component_spec = component_spec
    valid = (str, int, float, bool, GraphInputArgument, TaskOutputArgument, PipelineParam)

    def create_task(pythonic_arguments: dict):
        arguments = {from_py[k]: (v if isinstance(v, valid) else str(v)) for k, v in pythonic_arguments.items()
                     if v is not None}
        for key, val in list(arguments.items()):
            if isinstance(val, PipelineParam):
                if _config.type_check_enabled():
                    spec = next(i for i in inputs if i.name == key)
                    if val.param_type is not None and not check_types(val.param_type.to_dict_or_str(),
                                                                      "" if spec.type is None else spec.type):
                        raise InconsistentTypeException(
                            f'Component "{name}" is expecting {key} to be type({spec.type}), but the passed argument '
                            f"is type({val.param_type.serialize()})")
                arguments[key] = str(val)
        task = TaskSpec(component_ref=component_ref, arguments=arguments)
        if _created_task_transformation_handler:
            task = _created_task_transformation_handler[-1](task)
        return task

    ordered = [i for i in inputs if i.default is None and not i.optional] + \
              [i for i in inputs if not (i.default is None and not i.optional)]
    params = [_dynamic.KwParameter(
        to_py[p.name], annotation=(_try_get_object_by_name(str(p.type)) if p.type else inspect.Parameter.empty),
        default=p.default if p.default is not None else (None if p.optional else inspect.Parameter.empty))
        for p in ordered]
    f = _dynamic.create_function_from_parameters(create_task, params, documentation=doc, func_name=name,
                                                 func_filename=component_filename)
    f.component_spec = component_spec
    return f


def components_local_output_dir_context(output_dir: str):
    """Context manager swapping the `/outputs` root (host-side execution of component commands)."""
    import contextlib

    from . import _components as me

    @contextlib.contextmanager
    def ctx():
        old = me._outputs_dir
        me._outputs_dir = output_dir
        try:
            yield
        finally:
            me._outputs_dir = old

    return ctx()


_ = os
