"""Argo `resource` templates: ResourceOp, VolumeOp (PVC creation), VolumeSnapshotOp.

Reference: `sdk/python/kfp/dsl/_resource_op.py:22-149`, `_volume_op.py:30-142`,
`_volume_snapshot_op.py:25-126`."""
from __future__ import annotations

import re

from ..k8s import (V1ObjectMeta, V1PersistentVolumeClaim, V1PersistentVolumeClaimSpec, V1ResourceRequirements,
                   V1TypedLocalObjectReference)
from . import _pipeline_param
from ._container_op import BaseOp
from ._pipeline_param import PipelineParam, match_serialized_pipelineparam, sanitize_k8s_name
from ._pipeline_volume import PipelineVolume


class Resource:
    swagger_types = {"action": "str", "merge_strategy": "str", "success_condition": "str",
                     "failure_condition": "str", "manifest": "str"}
    attribute_map = {"action": "action", "merge_strategy": "mergeStrategy", "success_condition": "successCondition",
                     "failure_condition": "failureCondition", "manifest": "manifest"}

    def __init__(self, action=None, merge_strategy=None, success_condition=None, failure_condition=None,
                 manifest=None):
        self.action = action
        self.merge_strategy = merge_strategy
        self.success_condition = success_condition
        self.failure_condition = failure_condition
        self.manifest = manifest


class ResourceOp(BaseOp):
    def __init__(self, k8s_resource=None, action: str = "create", merge_strategy: str | None = None,
                 success_condition: str | None = None, failure_condition: str | None = None,
                 attribute_outputs: dict | None = None, **kwargs):
        super().__init__(**kwargs)
        self.attrs_with_pipelineparams = list(self.attrs_with_pipelineparams) + ["_resource", "k8s_resource",
                                                                                 "attribute_outputs"]
        if k8s_resource is None:
            raise ValueError("You need to provide a k8s_resource.")
        if merge_strategy and action != "apply":
            raise ValueError("You can't set merge_strategy when action != 'apply'")
        if action not in ("create", "delete", "apply", "patch", "replace", "get"):
            raise ValueError(f"invalid action {action}")
        self._resource = Resource(action=action, merge_strategy=merge_strategy, success_condition=success_condition,
                                  failure_condition=failure_condition)
        self.k8s_resource = k8s_resource
        extra = dict(attribute_outputs or {})
        self.attribute_outputs = dict(getattr(self, "attribute_outputs", None) or {})
        self.attribute_outputs.update(extra)
        self.attribute_outputs.setdefault("name", "{.metadata.name}")
        self.attribute_outputs.setdefault("manifest", "{}")
        self.outputs = {n: PipelineParam(n, op_name=self.name) for n in self.attribute_outputs}
        self.output = self.outputs["name"]
        if len(extra) == 1:
            self.output = self.outputs[list(extra)[0]]

    @property
    def resource(self) -> Resource:
        return self._resource


VOLUME_MODE_RWO = ["ReadWriteOnce"]
VOLUME_MODE_RWM = ["ReadWriteMany"]
VOLUME_MODE_ROM = ["ReadOnlyMany"]


def _validate_memory_string(s):
    if re.match(r"^[0-9]+(E|Ei|P|Pi|T|Ti|G|Gi|M|Mi|K|Ki){0,1}$", s) is None:
        raise ValueError('Invalid memory string. Should be an integer, or integer followed by one of '
                         '"E|Ei|P|Pi|T|Ti|G|Gi|M|Mi|K|Ki"')


class VolumeOp(ResourceOp):
    """Creates a PVC; `.volume` is a PipelineVolume mountable by later ops."""

    def __init__(self, resource_name: str | None = None, size: str | None = None, storage_class: str | None = None,
                 modes: list | None = None, annotations: dict | None = None, data_source=None, **kwargs):
        modes = VOLUME_MODE_RWM if modes is None and "k8s_resource" not in kwargs else modes
        self.attribute_outputs = {"size": "{.status.capacity.storage}"}
        if "k8s_resource" in kwargs:
            if resource_name or size or storage_class or modes or annotations:
                raise ValueError("You cannot provide k8s_resource along with other arguments.")
            if not isinstance(kwargs["k8s_resource"], V1PersistentVolumeClaim):
                raise ValueError("k8s_resource in VolumeOp must be an instance of V1PersistentVolumeClaim")
            super().__init__(**kwargs)
            self.volume = PipelineVolume(name=sanitize_k8s_name(self.name), pvc=self.outputs["name"])
            return
        if not size:
            raise ValueError("Please provide size")
        if not match_serialized_pipelineparam(str(size)):
            _validate_memory_string(size)
        if data_source and not isinstance(data_source, (str, PipelineParam, V1TypedLocalObjectReference)):
            raise ValueError("data_source can be one of (str, PipelineParam, V1TypedLocalObjectReference).")
        if data_source and isinstance(data_source, (str, PipelineParam)):
            data_source = V1TypedLocalObjectReference(api_group="snapshot.storage.k8s.io", kind="VolumeSnapshot",
                                                      name=data_source)
        if not match_serialized_pipelineparam(str(resource_name)):
            resource_name = sanitize_k8s_name(resource_name)
        k8s_resource = V1PersistentVolumeClaim(
            api_version="v1", kind="PersistentVolumeClaim",
            metadata=V1ObjectMeta(name="{{workflow.name}}-%s" % resource_name, annotations=annotations),
            spec=V1PersistentVolumeClaimSpec(access_modes=modes, resources=V1ResourceRequirements(
                requests={"storage": size}), storage_class_name=storage_class, data_source=data_source))
        super().__init__(k8s_resource=k8s_resource, **kwargs)
        self.volume = PipelineVolume(name=sanitize_k8s_name(self.name), pvc=self.outputs["name"])


class VolumeSnapshotOp(ResourceOp):
    """Creates a VolumeSnapshot of a PVC; `.snapshot` can seed a new VolumeOp."""

    def __init__(self, resource_name: str | None = None, pvc: str | None = None, snapshot_class: str | None = None,
                 annotations: dict | None = None, volume=None, **kwargs):
        self.attribute_outputs = {"size": "{.status.restoreSize}"}
        kwargs.setdefault("success_condition", "status.readyToUse == true")
        if "k8s_resource" in kwargs:
            if resource_name or pvc or snapshot_class or annotations or volume:
                raise ValueError("You cannot provide k8s_resource along with other arguments.")
            super().__init__(**kwargs)
            self.snapshot = V1TypedLocalObjectReference(api_group="snapshot.storage.k8s.io", kind="VolumeSnapshot",
                                                        name=self.outputs["name"])
            return
        if not (pvc or volume):
            raise ValueError("You must provide a pvc or a volume.")
        if pvc and volume:
            raise ValueError("You can't provide both pvc and volume.")
        deps = []
        if pvc:
            source = V1TypedLocalObjectReference(kind="PersistentVolumeClaim", name=pvc)
        else:
            if getattr(volume, "persistent_volume_claim", None) is None:
                raise ValueError("The volume must be referencing a PVC.")
            deps = list(getattr(volume, "dependent_names", []))
            source = V1TypedLocalObjectReference(kind="PersistentVolumeClaim",
                                                 name=volume.persistent_volume_claim.claim_name)
        if not match_serialized_pipelineparam(str(resource_name)):
            resource_name = sanitize_k8s_name(resource_name)
        k8s_resource = {"apiVersion": "snapshot.storage.k8s.io/v1alpha1", "kind": "VolumeSnapshot",
                        "metadata": V1ObjectMeta(name="{{workflow.name}}-%s" % resource_name, annotations=annotations),
                        "spec": {"source": source}}
        if snapshot_class:
            k8s_resource["spec"]["snapshotClassName"] = snapshot_class
        super().__init__(k8s_resource=k8s_resource, **kwargs)
        self.dependent_names.extend(deps)
        self.snapshot = V1TypedLocalObjectReference(api_group="snapshot.storage.k8s.io", kind="VolumeSnapshot",
                                                    name=self.outputs["name"])


_ = _pipeline_param
