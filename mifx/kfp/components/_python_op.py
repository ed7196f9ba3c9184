"""Lightweight components: a self-contained Python function -> component spec / task factory.

Reference: `sdk/python/kfp/components/_python_op.py:40-336` — the function is captured with
cloudpickle and embedded in a `python3 -c` program that parses positional argv (inputs, then output
file paths) and writes each output (NamedTuple fields, or a single `Output`) to its file.
Differences by design: the default base image is a ROCm PyTorch image, the pickle travels base64
encoded, and `bool` inputs are parsed as truth strings ('False' -> False)."""
from __future__ import annotations

import base64
import inspect
import re
import sys
from collections import OrderedDict
from typing import List

from ._components import _create_task_factory_from_component_spec
from ._structures import (ComponentSpec, ContainerImplementation, ContainerSpec, InputSpec, InputValuePlaceholder,
                          OutputPathPlaceholder, OutputSpec)
from ._yaml_utils import dump_yaml

_default_base_image = "rocm/pytorch:latest"


def _python_function_name_to_component_name(name: str) -> str:
    return re.sub(" +", " ", name.replace("_", " ")).strip(" ").capitalize()


def _capture_function_code_using_cloudpickle(func, modules_to_capture: List[str] | None = None) -> str:
    import pickle

    import cloudpickle

    modules_to_capture = modules_to_capture if modules_to_capture is not None else [func.__module__]
    saved = {}
    try:  # capture the function's own module by value instead of by reference
        for m in modules_to_capture:
            if m in sys.modules:
                saved[m] = sys.modules.pop(m)
        blob = cloudpickle.dumps(func, pickle.DEFAULT_PROTOCOL)
    finally:
        sys.modules.update(saved)
    b64 = base64.b64encode(blob).decode()
    return "\n".join([
        "import base64, pickle",
        "try:",
        "    import cloudpickle  # noqa: F401 (needed to unpickle closures)",
        "except ImportError:",
        "    import subprocess, sys",
        '    subprocess.call([sys.executable, "-m", "pip", "install", "cloudpickle", "--quiet"])',
        f"{func.__name__} = pickle.loads(base64.b64decode('{b64}'))",
    ])


def _annotation_to_type_struct(annotation):
    if not annotation or annotation == inspect.Parameter.empty:
        return None
    if isinstance(annotation, type):
        return str(annotation.__name__)
    return str(annotation)


def _func_to_component_spec(func, extra_code: str = "", base_image: str = _default_base_image,
                            modules_to_capture: List[str] | None = None) -> ComponentSpec:
    deco_image = getattr(func, "_component_base_image", None)
    if deco_image is not None:
        if base_image is not _default_base_image and deco_image != base_image:
            raise ValueError(f"base_image ({base_image}) conflicts with the decorator-specified base image metadata "
                             f"({deco_image})")
        base_image = deco_image
    elif base_image is None:
        raise ValueError("base_image cannot be None")
    try:  # resolve string annotations (modules using `from __future__ import annotations`)
        sig = inspect.signature(func, eval_str=True)
    except Exception:  # noqa: BLE001 - unresolvable names keep their string form
        sig = inspect.signature(func)
    types = OrderedDict()
    inputs, outputs, out_names, arguments = [], [], [], []
    for p in sig.parameters.values():
        ts = _annotation_to_type_struct(p.annotation)
        types[p.name] = str(ts)
        arguments.append(InputValuePlaceholder(p.name))
        inputs.append(InputSpec(name=p.name, type=ts,
                                default=str(p.default) if p.default is not inspect.Parameter.empty else None))
    ret = sig.return_annotation
    if hasattr(ret, "_fields"):  # NamedTuple -> one output per field
        ftypes = getattr(ret, "__annotations__", None) or getattr(ret, "_field_types", {}) or {}
        for f in ret._fields:
            outputs.append(OutputSpec(name=f, type=_annotation_to_type_struct(ftypes.get(f))))
            out_names.append(f)
            arguments.append(OutputPathPlaceholder(f))
    elif ret is not None and ret != inspect.Parameter.empty:
        outputs.append(OutputSpec(name="Output", type=_annotation_to_type_struct(ret)))
        out_names.append("output")
        arguments.append(OutputPathPlaceholder("Output"))
    conv = {"int": "int", "float": "float", "bool": "_to_bool"}
    parse_lines = "\n".join(f"    '{n}': {conv.get(t, 'str')}(sys.argv[{i + 1}]),"
                            for i, (n, t) in enumerate(types.items()))
    out_lines = "\n".join(f"    sys.argv[{i + len(types) + 1}]," for i in range(len(out_names)))
    source = f"""{extra_code}
{_capture_function_code_using_cloudpickle(func, modules_to_capture)}
import sys


def _to_bool(s):
    if s.strip().lower() in ('true', 't', 'yes', 'y', '1', 'on'):
        return True
    if s.strip().lower() in ('false', 'f', 'no', 'n', '0', 'off'):
        return False
    raise ValueError('not a boolean: ' + s)


_args = {{
{parse_lines}
}}
_output_files = [
{out_lines}
]
_outputs = {func.__name__}(**_args)
if not hasattr(_outputs, '__getitem__') or isinstance(_outputs, str):
    _outputs = [_outputs]
from pathlib import Path
for _idx, _filename in enumerate(_output_files):
    _p = Path(_filename)
    _p.parent.mkdir(parents=True, exist_ok=True)
    _p.write_text(str(_outputs[_idx]))
"""
    source = re.sub("\n\n\n+", "\n\n", source).strip("\n") + "\n"
    name = getattr(func, "_component_human_name", None) or _python_function_name_to_component_name(func.__name__)
    desc = getattr(func, "_component_description", None) or func.__doc__
    if desc:
        desc = desc.strip() + "\n"
    return ComponentSpec(name=name, description=desc, inputs=inputs, outputs=outputs,
                         implementation=ContainerImplementation(container=ContainerSpec(
                             image=base_image, command=["python3", "-c", source], args=arguments)))


def func_to_component_text(func, extra_code: str = "", base_image: str = _default_base_image,
                           modules_to_capture: List[str] | None = None) -> str:
    return dump_yaml(_func_to_component_spec(func, extra_code, base_image, modules_to_capture).to_dict())


def func_to_component_file(func, output_component_file: str, base_image: str = _default_base_image,
                           extra_code: str = "", modules_to_capture: List[str] | None = None) -> None:
    with open(output_component_file, "w") as f:
        f.write(func_to_component_text(func, extra_code, base_image, modules_to_capture))


def func_to_container_op(func, output_component_file: str | None = None, base_image: str = _default_base_image,
                         extra_code: str = "", modules_to_capture: List[str] | None = None):
    spec = _func_to_component_spec(func, extra_code, base_image, modules_to_capture)
    if output_component_file:
        with open(output_component_file, "w") as f:
            f.write(dump_yaml(spec.to_dict()))
    target = getattr(func, "_component_target_component_file", None)
    if target:
        with open(target, "w") as f:
            f.write(dump_yaml(spec.to_dict()))
    return _create_task_factory_from_component_spec(spec)
