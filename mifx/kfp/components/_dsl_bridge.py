"""TaskSpec -> dsl.ContainerOp: placeholder expansion into command/args, file outputs, env,
metadata annotations/labels (reference: `sdk/python/kfp/components/_dsl_bridge.py:21-175`)."""
from __future__ import annotations

from collections import OrderedDict

from ..dsl._metadata import ComponentMeta, ParameterMeta, _annotation_to_typemeta
from ._components import _default_component_name, _generate_output_file_name
from ._structures import (ConcatPlaceholder, ContainerImplementation, IfPlaceholder, InputPathPlaceholder,
                          InputValuePlaceholder, IsPresentPlaceholder, OutputPathPlaceholder, TaskSpec)


def _strtobool(v: str) -> bool:
    v = v.strip().lower()
    if v in ("y", "yes", "t", "true", "on", "1"):
        return True
    if v in ("n", "no", "f", "false", "off", "0"):
        return False
    raise ValueError(f"invalid truth value {v!r}")


def resolve_command_line(component_spec, arguments: dict):
    """Expand a container component's command/args for the given arguments.
    Returns (command, args, output_paths: OrderedDict[output name -> path])."""
    c = component_spec.implementation.container
    inputs = {i.name: i for i in component_spec.inputs or []}
    output_paths = OrderedDict()
    fixed = c.file_outputs or {}
    for out in component_spec.outputs or []:
        if out.name in fixed:
            output_paths[out.name] = fixed[out.name]

    def part(arg):
        if arg is None:
            return None
        if isinstance(arg, (str, int, float, bool)):
            return str(arg)
        if isinstance(arg, InputValuePlaceholder):
            v = arguments.get(arg.input_name)
            if v is not None:
                return str(v)
            if inputs[arg.input_name].optional:
                return None
            raise ValueError(f"No value provided for input {arg.input_name}")
        if isinstance(arg, InputPathPlaceholder):
            v = arguments.get(arg.input_name)
            if v is not None:
                raise ValueError(f"ContainerOp does not support input artifacts - input {arg.input_name}")
            if inputs[arg.input_name].optional:
                return None
            raise ValueError(f"No value provided for input {arg.input_name}")
        if isinstance(arg, OutputPathPlaceholder):
            fn = _generate_output_file_name(arg.output_name)
            if arg.output_name in output_paths and output_paths[arg.output_name] != fn:
                raise ValueError(f"Conflicting output files specified for port {arg.output_name}: "
                                 f"{output_paths[arg.output_name]} and {fn}")
            output_paths[arg.output_name] = fn
            return fn
        if isinstance(arg, ConcatPlaceholder):
            return "".join(expand(arg.items))
        if isinstance(arg, IfPlaceholder):
            s = arg.if_structure
            cond = part(s.condition)
            ok = bool(cond) and _strtobool(cond)
            node = s.then_value if ok else s.else_value
            if node is None:
                return []
            return expand(node) if isinstance(node, list) else part(node)
        if isinstance(arg, IsPresentPlaceholder):
            return str(arguments.get(arg.input_name) is not None)
        raise TypeError(f"Unrecognized argument type: {arg}")

    def expand(items):
        out = []
        for it in items or []:
            e = part(it)
            if e is None:
                continue
            if isinstance(e, list):
                out.extend(e)
            else:
                out.append(str(e))
        return out

    return expand(c.command), expand(c.args), output_paths


def create_container_op_from_task(task_spec: TaskSpec):
    spec = task_spec.component_ref._component_spec
    if not isinstance(spec.implementation, ContainerImplementation):
        raise TypeError("Only container component tasks can be converted to ContainerOp")
    command, args, output_paths = resolve_command_line(spec, task_spec.arguments or {})
    return _task_object_factory(name=spec.name or _default_component_name, container_image=spec.implementation.
                                container.image, command=command, arguments=args, output_paths=output_paths,
                                env=spec.implementation.container.env, component_spec=spec)


def _create_container_op_from_resolved_task(name: str, container_image: str, command=None, arguments=None,
                                            output_paths=None, env=None, component_spec=None):
    from .. import dsl
    from ..k8s import V1EnvVar
    from ._naming import _sanitize_python_function_name, generate_unique_name_conversion_table

    to_k8s = generate_unique_name_conversion_table(list((output_paths or {}).keys()), _sanitize_python_function_name)
    file_outputs = {to_k8s[n]: p for n, p in (output_paths or {}).items()}
    meta = ComponentMeta(name=component_spec.name, description=component_spec.description)
    for i in component_spec.inputs or []:
        meta.inputs.append(ParameterMeta(name=i.name, description=i.description,
                                         param_type=_annotation_to_typemeta(i.type), default=i.default))
    for o in component_spec.outputs or []:
        meta.outputs.append(ParameterMeta(name=o.name, description=o.description,
                                          param_type=_annotation_to_typemeta(o.type)))
    task = dsl.ContainerOp(name=name, image=container_image, command=command, arguments=arguments,
                           file_outputs=file_outputs)
    task._set_metadata(meta)
    for k, v in (env or {}).items():
        task.container.add_env_variable(V1EnvVar(name=k, value=v))
    if component_spec.metadata:
        for k, v in (component_spec.metadata.annotations or {}).items():
            task.add_pod_annotation(k, v)
        for k, v in (component_spec.metadata.labels or {}).items():
            task.add_pod_label(k, v)
    return task


_task_object_factory = _create_container_op_from_resolved_task
