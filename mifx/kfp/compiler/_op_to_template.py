"""Per-op Argo template generation (container and resource templates).

Reference: `sdk/python/kfp/compiler/_op_to_template.py:30-260`: PipelineParams become
`{{inputs.parameters.<full_name>}}`; default optional output artifacts `mlpipeline-ui-metadata`
and `mlpipeline-metrics` (S3 key `runs/{{workflow.uid}}/{{pod.name}}/<name>.tgz` when an artifact
location is set); outputs from file paths (container) or jsonPath (resource); retryStrategy,
activeDeadlineSeconds, nodeSelector, tolerations, pod metadata, sidecars, display name."""
from __future__ import annotations

import re
from collections import OrderedDict

import yaml

from .. import dsl
from ..dsl._artifact_location import ArtifactLocation
from ._k8s_helper import convert_k8s_obj_to_json

DISPLAY_NAME_ANNOTATION = "kubeflow.org/pipelines/task_display_name"


def _process_obj(obj, tmpl: dict):
    if isinstance(obj, str):
        for t in dsl.match_serialized_pipelineparam(obj):
            obj = re.sub(re.escape(t.pattern), lambda _m, v=tmpl[t.pattern]: v, obj)
        return obj
    if isinstance(obj, list):
        return [_process_obj(x, tmpl) for x in obj]
    if isinstance(obj, tuple):
        return tuple(_process_obj(x, tmpl) for x in obj)
    if isinstance(obj, dict):
        return {k: _process_obj(v, tmpl) for k, v in obj.items()}
    if isinstance(obj, dsl.PipelineParam):
        return tmpl.get(str(obj), "{{inputs.parameters.%s}}" % obj.full_name)
    types = getattr(obj, "swagger_types", None) or getattr(obj, "openapi_types", None)
    if isinstance(types, dict):
        for k in types:
            setattr(obj, k, _process_obj(getattr(obj, k), tmpl))
        return convert_k8s_obj_to_json(obj)
    return obj


def _process_base_ops(op):
    tmpl = {(p.pattern or str(p)): "{{inputs.parameters.%s}}" % p.full_name for p in op.inputs}
    for key in op.attrs_with_pipelineparams:
        setattr(op, key, _process_obj(getattr(op, key), tmpl))
    return op


def _parameters_to_json(params) -> list:
    out = [dict(name=p.full_name, value=p.value) if p.value else dict(name=p.full_name) for p in params]
    out.sort(key=lambda x: x["name"])
    return out


def _outputs_to_json(op, outputs: dict, param_outputs: dict, output_artifacts: list) -> dict:
    key = "jsonPath" if isinstance(op, dsl.ResourceOp) else "path"
    params = [{"name": p.full_name, "valueFrom": {key: param_outputs[p.name]}} for p in outputs.values()]
    params.sort(key=lambda x: x["name"])
    ret = {}
    if params:
        ret["parameters"] = params
    if output_artifacts:
        ret["artifacts"] = output_artifacts
    return ret


def op_to_template(op) -> dict:
    processed = _process_base_ops(op)
    if isinstance(op, dsl.ContainerOp):
        paths = OrderedDict(op.output_artifact_paths)
        paths.setdefault("mlpipeline-ui-metadata", "/mlpipeline-ui-metadata.json")
        paths.setdefault("mlpipeline-metrics", "/mlpipeline-metrics.json")
        artifacts = [convert_k8s_obj_to_json(ArtifactLocation.create_artifact_for_s3(
            op.artifact_location, name=n, path=p, key="runs/{{workflow.uid}}/{{pod.name}}/" + n + ".tgz"))
            for n, p in paths.items()]
        for a in artifacts:
            if a["name"] in ("mlpipeline-ui-metadata", "mlpipeline-metrics"):
                a["optional"] = True
        template = {"name": processed.name, "container": convert_k8s_obj_to_json(processed.container)}
        param_outputs = processed.file_outputs
    elif isinstance(op, dsl.ResourceOp):
        artifacts = []
        resource = convert_k8s_obj_to_json(processed.resource)  # a dict once params were substituted
        resource["manifest"] = yaml.dump(convert_k8s_obj_to_json(processed.k8s_resource), default_flow_style=False)
        template = {"name": processed.name, "resource": resource}
        param_outputs = processed.attribute_outputs
    else:
        raise TypeError(f"unsupported op type {type(op).__name__}")
    ins = _parameters_to_json(processed.inputs)
    if ins:
        template["inputs"] = {"parameters": ins}
    template["outputs"] = _outputs_to_json(op, processed.outputs, param_outputs, artifacts)
    if processed.node_selector:
        template["nodeSelector"] = processed.node_selector
    if processed.tolerations:
        template["tolerations"] = processed.tolerations
    if processed.pod_annotations or processed.pod_labels:
        template["metadata"] = {}
        if processed.pod_annotations:
            template["metadata"]["annotations"] = processed.pod_annotations
        if processed.pod_labels:
            template["metadata"]["labels"] = processed.pod_labels
    if processed.num_retries:
        template["retryStrategy"] = {"limit": processed.num_retries}
    if processed.timeout:
        template["activeDeadlineSeconds"] = processed.timeout
    if processed.sidecars:
        template["sidecars"] = processed.sidecars
    if processed.display_name:
        template.setdefault("metadata", {}).setdefault("annotations", {})[DISPLAY_NAME_ANNOTATION] = \
            processed.display_name
    return template


_op_to_template = op_to_template
