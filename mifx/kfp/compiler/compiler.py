"""DSL -> Argo Workflow compiler.

Reference semantics: `sdk/python/kfp/compiler/compiler.py:57-693`.
  1. Run the pipeline function inside a `dsl.Pipeline` context with PipelineParam arguments.
  2. Build the group tree (root pipeline group / exit handler / condition / graph; recursive graph
     references behave like leaf tasks).
  3. For every data edge producer -> consumer, find their first *uncommon* ancestors: the value
     leaves the producer through each upstream group's `outputs`, enters each downstream group
     through its `inputs`, and becomes a dependency between the two sibling subtrees.
  4. Emit one DAG template per group (tasks, `when` for conditions, sorted dependencies and
     arguments) and one container/resource template per op; wire onExit, volumes, deadlines and
     image pull secrets; write .yaml / .tar.gz / .zip packages.
"""
from __future__ import annotations

import inspect
import io
import tarfile
import zipfile
from collections import defaultdict

import yaml

from .. import _config, dsl
from ..dsl._metadata import TypeMeta, _extract_pipeline_metadata
from ._k8s_helper import convert_k8s_obj_to_json, sanitize_k8s_name
from ._op_to_template import op_to_template


def _full_name(p) -> str:
    return f"{p.op_name}-{p.name}" if p.op_name else p.name


class _Analysis:
    """Group-tree bookkeeping for one pipeline."""

    def __init__(self, pipeline):
        self.pipeline = pipeline
        self.root = pipeline.groups[0]
        self.paths: dict[str, list[str]] = {}        # op / recursive-group name -> ancestor path (incl. self)
        self.group_paths: dict[str, list[str]] = {}  # non-recursive group name -> path (incl. self)
        self.groups: dict[str, object] = {}          # group name -> group (non-recursive)
        self._walk(self.root, [self.root.name])
        self.groups[self.root.name] = self.root
        self.cond_params = self._condition_params()

    def _walk(self, group, path):
        for g in group.groups:
            if g.recursive_ref:
                self.paths[g.name] = path + [g.name]
                continue
            self.group_paths[g.name] = path + [g.name]
            self.groups[g.name] = g
            self._walk(g, path + [g.name])
        for op in group.ops:
            self.paths[op.name] = path + [op.name]

    def path_of(self, name: str) -> list[str]:
        if name in self.paths:
            return self.paths[name]
        if name in self.group_paths:
            return self.group_paths[name]
        raise ValueError(f"{name} does not exist.")

    def uncommon(self, up: str, down: str) -> tuple[list[str], list[str]]:
        a, b = self.path_of(up), self.path_of(down)
        n = 0
        while n < min(len(a), len(b)) and a[n] == b[n]:
            n += 1
        return a[n:], b[n:]

    def _condition_params(self):
        out = defaultdict(set)

        def walk(group, params):
            if group.type == "condition":
                params = list(params)
                for operand in (group.condition.operand1, group.condition.operand2):
                    if isinstance(operand, dsl.PipelineParam):
                        params.append(operand)
            for op in group.ops:
                out[op.name].update(params)
            for g in group.groups:
                if g.recursive_ref:
                    out[g.name].update(params)
                else:
                    walk(g, params)

        walk(self.root, [])
        return out

    # -------------------------------------------------------------------------------- I/O
    def inputs_outputs(self):
        inputs, outputs = defaultdict(set), defaultdict(set)

        def route(param, consumer_name, skip_last_for_condition=False):
            name = _full_name(param)
            up, down = self.uncommon(param.op_name, consumer_name)
            for i, g in enumerate(down):
                if i == 0:
                    inputs[g].add((name, up[0]))
                elif skip_last_for_condition and i == len(down) - 1:
                    continue
                else:
                    inputs[g].add((name, None))
            for i, g in enumerate(up):
                outputs[g].add((name, None if i == len(up) - 1 else up[i + 1]))

        for op in self.pipeline.ops.values():
            for p in list(op.inputs) + list(self.cond_params[op.name]):
                if p.value:
                    continue
                if p.op_name:
                    route(p, op.name)
                elif not op.is_exit_handler:
                    for g in self.paths[op.name]:
                        inputs[g].add((_full_name(p), None))

        def recursive(group):
            if group.recursive_ref:
                params = [(p, False) for p in group.inputs] + [(p, True) for p in self.cond_params[group.name]]
                for p, is_cond in params:
                    if p.value:
                        continue
                    if p.op_name:
                        route(p, group.name, skip_last_for_condition=is_cond)
                    else:
                        for g in self.paths[group.name]:
                            inputs[g].add((_full_name(p), None))
            for sub in group.groups:
                recursive(sub)

        recursive(self.root)
        return inputs, outputs

    def dependencies(self):
        deps = defaultdict(set)
        for op in self.pipeline.ops.values():
            ups = {p.op_name for p in list(op.inputs) + list(self.cond_params[op.name]) if p.op_name}
            ups |= set(op.dependent_names)
            for u in ups:
                if u not in self.pipeline.ops and u not in self.groups:
                    raise ValueError(f"compiler cannot find the {u}")
                a, b = self.uncommon(u, op.name)
                deps[b[0]].add(a[0])

        def walk(group):
            if group.recursive_ref:
                ups = {p.op_name for p in list(group.inputs) + list(self.cond_params[group.name]) if p.op_name}
            else:
                ups = {d.name for d in group.dependencies}
            for u in ups:
                if u not in self.pipeline.ops and u not in self.group_paths:
                    raise ValueError(f"compiler cannot find the {u}")
                a, b = self.uncommon(u, group.name)
                deps[b[0]].add(a[0])
            for sub in group.groups:
                walk(sub)

        walk(self.root)
        return deps


def _resolve(value, refs) -> str:
    if isinstance(value, dsl.PipelineParam):
        name = _full_name(value)
        tasks = [t for n, t in refs if n == name]
        if tasks and tasks[0] is not None:
            return "{{tasks.%s.outputs.parameters.%s}}" % (tasks[0], name)
        return "{{inputs.parameters.%s}}" % name
    return str(value)


def _group_to_template(group, inputs, outputs, deps) -> dict:
    t = {"name": group.name}
    if inputs.get(group.name):
        t["inputs"] = {"parameters": sorted(({"name": n} for n, _ in inputs[group.name]), key=lambda x: x["name"])}
    if outputs.get(group.name):
        t["outputs"] = {"parameters": sorted(
            ({"name": n, "valueFrom": {"parameter": "{{tasks.%s.outputs.parameters.%s}}" % (d, n)}}
             for n, d in outputs[group.name]), key=lambda x: x["name"])}
    tasks = []
    for sub in list(group.groups) + list(group.ops):
        rec = isinstance(sub, dsl.OpsGroup) and sub.recursive_ref
        target = sub.recursive_ref.name if rec else sub.name
        task = {"name": target, "template": target}
        if isinstance(sub, dsl.OpsGroup) and sub.type == "condition":
            refs = inputs.get(sub.name, [])
            c = sub.condition
            task["when"] = f"{_resolve(c.operand1, refs)} {c.operator} {_resolve(c.operand2, refs)}"
        if deps.get(sub.name):
            task["dependencies"] = sorted(deps[sub.name])
        if inputs.get(sub.name):
            args = []
            for pname, producer in inputs[sub.name]:
                arg_name = pname
                if rec:  # map the recursive call's argument to the referenced graph's parameter name
                    idx = next(i for i, p in enumerate(sub.inputs) if _full_name(p) == pname)
                    arg_name = _full_name(sub.recursive_ref.inputs[idx])
                val = ("{{tasks.%s.outputs.parameters.%s}}" % (producer, pname) if producer
                       else "{{inputs.parameters.%s}}" % pname)
                args.append({"name": arg_name, "value": val})
            task["arguments"] = {"parameters": sorted(args, key=lambda x: x["name"])}
        tasks.append(task)
    t["dag"] = {"tasks": sorted(tasks, key=lambda x: x["name"])}
    return t


class Compiler:
    """`Compiler().compile(pipeline_func, package_path, type_check=True)`."""

    def _create_templates(self, pipeline, op_transformers=None, op_to_templates_handler=None) -> list:
        handler = op_to_templates_handler or (lambda op: [op_to_template(op)])
        for op in pipeline.ops.values():
            for tr in op_transformers or []:
                tr(op)
        an = _Analysis(pipeline)
        inputs, outputs = an.inputs_outputs()
        deps = an.dependencies()
        templates = [_group_to_template(g, inputs, outputs, deps) for g in an.groups.values()]
        for op in pipeline.ops.values():
            templates.extend(handler(op))
        return templates

    @staticmethod
    def _create_volumes(pipeline) -> list:
        seen, vols = set(), []
        for op in pipeline.ops.values():
            for v in op.volumes or []:
                if v["name"] not in seen:
                    seen.add(v["name"])
                    vols.append(v)
        return sorted(vols, key=lambda x: x["name"])

    def _create_pipeline_workflow(self, args, pipeline, op_transformers=None) -> dict:
        params = []
        for a in args:
            p = {"name": a.name}
            if a.value is not None:
                p["value"] = str(a.value)
            params.append(p)
        templates = sorted(self._create_templates(pipeline, op_transformers), key=lambda x: x["name"])
        exit_handler = None
        if pipeline.groups[0].groups and pipeline.groups[0].groups[0].type == "exit_handler":
            exit_handler = pipeline.groups[0].groups[0].exit_op
        volumes = self._create_volumes(pipeline)
        name = pipeline.name or "Pipeline"
        wf = {"apiVersion": "argoproj.io/v1alpha1", "kind": "Workflow", "metadata": {"generateName": name + "-"},
              "spec": {"entrypoint": name, "templates": templates, "arguments": {"parameters": params},
                       "serviceAccountName": "pipeline-runner"}}
        if pipeline.conf.image_pull_secrets:
            wf["spec"]["imagePullSecrets"] = [convert_k8s_obj_to_json(s) for s in pipeline.conf.image_pull_secrets]
        if pipeline.conf.timeout:
            wf["spec"]["activeDeadlineSeconds"] = pipeline.conf.timeout
        if exit_handler:
            wf["spec"]["onExit"] = exit_handler.name
        if volumes:
            wf["spec"]["volumes"] = volumes
        return wf

    @staticmethod
    def _validate_exit_handler(pipeline) -> None:
        def walk(group, seen_ops, handler_exists):
            if group.type == "exit_handler":
                if handler_exists or len(seen_ops) > 1:
                    raise ValueError("Only one global exit_handler is allowed and all ops need to be included.")
                handler_exists = True
            seen_ops.extend(op.name for op in group.ops)
            for g in group.groups:
                walk(g, seen_ops, handler_exists)

        walk(pipeline.groups[0], [], False)

    def _compile(self, pipeline_func) -> dict:
        spec = inspect.getfullargspec(pipeline_func)
        meta = _extract_pipeline_metadata(pipeline_func, validate=_config.type_check_enabled())
        pname = sanitize_k8s_name(meta.name)
        args_list = []
        for arg in spec.args:
            t = next((i.param_type for i in meta.inputs if i.name == arg), TypeMeta())
            args_list.append(dsl.PipelineParam(sanitize_k8s_name(arg), param_type=t))
        with dsl.Pipeline(pname) as p:
            pipeline_func(*args_list)
        self._validate_exit_handler(p)
        with_defaults = [dsl.PipelineParam(sanitize_k8s_name(a)) for a in spec.args]
        if spec.defaults:
            for arg, d in zip(reversed(with_defaults), reversed(spec.defaults)):
                arg.value = d.value if isinstance(d, dsl.PipelineParam) else d
        location = p.conf.artifact_location
        ops = {}
        for op in p.ops.values():
            if location and not getattr(op, "artifact_location", None):
                op.artifact_location = location
            op.name = sanitize_k8s_name(op.name)
            for prm in op.outputs.values():
                prm.name = sanitize_k8s_name(prm.name)
                if prm.op_name:
                    prm.op_name = sanitize_k8s_name(prm.op_name)
            if op.output is not None:
                op.output.name = sanitize_k8s_name(op.output.name)
                op.output.op_name = sanitize_k8s_name(op.output.op_name)
            if op.dependent_names:
                op.dependent_names = [sanitize_k8s_name(n) for n in op.dependent_names]
            if isinstance(op, dsl.ContainerOp) and op.file_outputs is not None:
                op.file_outputs = {sanitize_k8s_name(k): v for k, v in op.file_outputs.items()}
            elif isinstance(op, dsl.ResourceOp) and op.attribute_outputs is not None:
                op.attribute_outputs = {sanitize_k8s_name(k): v for k, v in op.attribute_outputs.items()}
            ops[op.name] = op
        p.ops = ops
        return self._create_pipeline_workflow(with_defaults, p, p.conf.op_transformers)

    def compile_to_workflow(self, pipeline_func, type_check: bool = True) -> dict:
        old = _config.set_type_check(type_check)
        try:
            return self._compile(pipeline_func)
        finally:
            _config.set_type_check(old)

    def compile(self, pipeline_func, package_path: str, type_check: bool = True) -> None:
        wf = self.compile_to_workflow(pipeline_func, type_check)
        text = dump_yaml(wf)
        write_package(text, package_path)


class _NoAliasDumper(yaml.SafeDumper):
    def ignore_aliases(self, data):
        return True


def dump_yaml(obj) -> str:
    return yaml.dump(obj, Dumper=_NoAliasDumper, default_flow_style=False)


def write_package(yaml_text: str, package_path: str) -> None:
    if package_path.endswith((".tar.gz", ".tgz")):
        with tarfile.open(package_path, "w:gz") as tar:
            data = yaml_text.encode()
            info = tarfile.TarInfo("pipeline.yaml")
            info.size = len(data)
            tar.addfile(info, io.BytesIO(data))
    elif package_path.endswith(".zip"):
        with zipfile.ZipFile(package_path, "w") as z:
            zi = zipfile.ZipInfo("pipeline.yaml")
            zi.compress_type = zipfile.ZIP_DEFLATED
            z.writestr(zi, yaml_text)
    elif package_path.endswith((".yaml", ".yml")):
        with open(package_path, "w") as f:
            f.write(yaml_text)
    else:
        raise ValueError(f"The output path {package_path} should end with one of the following formats: "
                         "[.tar.gz, .tgz, .zip, .yaml, .yml]")


def read_package(package_path: str) -> str:
    """Inverse of write_package: the pipeline.yaml text of a compiled package."""
    if package_path.endswith((".tar.gz", ".tgz")):
        with tarfile.open(package_path, "r:gz") as tar:
            members = tar.getmembers()
            if len(members) != 1:
                raise ValueError("expected exactly one file in the pipeline package")
            return tar.extractfile(members[0]).read().decode()
    if package_path.endswith(".zip"):
        with zipfile.ZipFile(package_path) as z:
            names = z.namelist()
            if len(names) != 1:
                raise ValueError("expected exactly one file in the pipeline package")
            return z.read(names[0]).decode()
    with open(package_path) as f:
        return f.read()
