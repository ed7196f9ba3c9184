"""Kubernetes v1 object subsets used by graph-component tasks (`k8sContainerOptions`, `k8sPodOptions`).

Reference surface: `sdk/python/kfp/components/structures/kubernetes/v1.py:14-455` — typed ModelBase
structs (wire names in camelCase) for Container, EnvVar, VolumeMount, ResourceRequirements, probes,
Toleration, Volume (secret / nfs / pvc typed, every other source an opaque mapping) and the Argo subset
of a Pod (metadata annotations/labels + spec deadline/affinity/nodeSelector/tolerations/volumes).

Each struct is declared as one field table: (python name, type hint, default); the wire name is the
camelCase of the python name unless overridden. `_define` builds the ModelBase subclass with a real
typed `__init__` signature so ModelBase's type checks and dict (de)serialisation apply unchanged."""
from __future__ import annotations

import inspect
from typing import Dict, List, Mapping, Optional, Union

from ...modelbase import ModelBase

_REQUIRED = inspect.Parameter.empty


def _camel(name: str) -> str:
    head, *rest = name.split("_")
    return head + "".join(w[:1].upper() + w[1:] for w in rest)


def _define(cls_name: str, fields: list, wire: dict | None = None, doc: str = "") -> type:
    params = [inspect.Parameter("self", inspect.Parameter.POSITIONAL_OR_KEYWORD)]
    hints = {}
    for name, hint, default in fields:
        params.append(inspect.Parameter(name, inspect.Parameter.POSITIONAL_OR_KEYWORD, default=default,
                                        annotation=hint))
        hints[name] = hint
    sig = inspect.Signature(params)

    def __init__(self, *args, **kwargs):
        bound = sig.bind(self, *args, **kwargs)
        bound.apply_defaults()
        ModelBase.__init__(self, dict(bound.arguments))

    __init__.__signature__ = sig
    __init__.__annotations__ = hints
    names = {n: _camel(n) for n, _, _ in fields if _camel(n) != n}
    names.update(wire or {})
    cls = type(cls_name, (ModelBase,), {"__init__": __init__, "_serialized_names": names, "__doc__": doc,
                                        "__module__": __name__})
    __init__.__qualname__ = f"{cls_name}.__init__"
    return cls


_opt = None  # default for every optional field

EnvVar = _define("EnvVar", [("name", str, _REQUIRED), ("value", Optional[str], _opt)])
ExecAction = _define("ExecAction", [("command", List[str], _REQUIRED)])
HTTPGetAction = _define("HTTPGetAction", [("port", Union[int, str], _REQUIRED), ("host", Optional[str], _opt),
                                          ("path", Optional[str], _opt), ("scheme", Optional[str], _opt),
                                          ("http_headers", Optional[List[Mapping]], _opt)])
TCPSocketAction = _define("TCPSocketAction", [("port", Union[int, str], _REQUIRED), ("host", Optional[str], _opt)])
Handler = _define("Handler", [("exec", Optional[ExecAction], _opt), ("http_get", Optional[HTTPGetAction], _opt),
                              ("tcp_socket", Optional[TCPSocketAction], _opt)], wire={"exec": "exec"})
Lifecycle = _define("Lifecycle", [("post_start", Optional[Handler], _opt), ("pre_stop", Optional[Handler], _opt)])
VolumeMount = _define("VolumeMount", [("name", str, _REQUIRED), ("mount_path", str, _REQUIRED),
                                      ("mount_propagation", Optional[str], _opt), ("read_only", Optional[bool], _opt),
                                      ("sub_path", Optional[str], _opt)])
ResourceRequirements = _define("ResourceRequirements", [("limits", Optional[Dict[str, str]], _opt),
                                                        ("requests", Optional[Dict[str, str]], _opt)])
ContainerPort = _define("ContainerPort", [("container_port", int, _REQUIRED), ("host_ip", Optional[str], _opt),
                                          ("host_port", Optional[int], _opt), ("name", Optional[str], _opt),
                                          ("protocol", Optional[str], _opt)], wire={"host_ip": "hostIP"})
VolumeDevice = _define("VolumeDevice", [("device_path", str, _REQUIRED), ("name", str, _REQUIRED)])
Probe = _define("Probe", [("exec", Optional[ExecAction], _opt), ("http_get", Optional[HTTPGetAction], _opt),
                          ("tcp_socket", Optional[TCPSocketAction], _opt),
                          ("failure_threshold", Optional[int], _opt), ("initial_delay_seconds", Optional[int], _opt),
                          ("period_seconds", Optional[int], _opt), ("success_threshold", Optional[int], _opt),
                          ("timeout_seconds", Optional[int], _opt)], wire={"exec": "exec"})
SecurityContext = _define("SecurityContext", [
    ("allow_privilege_escalation", Optional[bool], _opt), ("capabilities", Optional[Mapping], _opt),
    ("privileged", Optional[bool], _opt), ("read_only_root_filesystem", Optional[bool], _opt),
    ("run_as_group", Optional[int], _opt), ("run_as_non_root", Optional[bool], _opt),
    ("run_as_user", Optional[int], _opt), ("se_linux_options", Optional[Mapping], _opt)])
Container = _define("Container", [
    ("image", Optional[str], _opt), ("command", Optional[List[str]], _opt), ("args", Optional[List[str]], _opt),
    ("env", Optional[List[EnvVar]], _opt), ("working_dir", Optional[str], _opt),
    ("lifecycle", Optional[Lifecycle], _opt), ("volume_mounts", Optional[List[VolumeMount]], _opt),
    ("resources", Optional[ResourceRequirements], _opt), ("ports", Optional[List[ContainerPort]], _opt),
    ("volume_devices", Optional[List[VolumeDevice]], _opt), ("name", Optional[str], _opt),
    ("image_pull_policy", Optional[str], _opt), ("liveness_probe", Optional[Probe], _opt),
    ("readiness_probe", Optional[Probe], _opt), ("security_context", Optional[SecurityContext], _opt),
    ("stdin", Optional[bool], _opt), ("stdin_once", Optional[bool], _opt),
    ("termination_message_path", Optional[str], _opt), ("termination_message_policy", Optional[str], _opt),
    ("tty", Optional[bool], _opt)], doc="Container options a task may override (resources, mounts, env, ...).")
Toleration = _define("Toleration", [("effect", Optional[str], _opt), ("key", Optional[str], _opt),
                                    ("operator", Optional[str], _opt), ("toleration_seconds", Optional[int], _opt),
                                    ("value", Optional[str], _opt)])
KeyToPath = _define("KeyToPath", [("key", str, _REQUIRED), ("path", str, _REQUIRED), ("mode", Optional[int], _opt)])
SecretVolumeSource = _define("SecretVolumeSource", [("default_mode", Optional[int], _opt),
                                                    ("items", Optional[List[KeyToPath]], _opt),
                                                    ("optional", Optional[bool], _opt),
                                                    ("secret_name", Optional[str], _opt)])
NFSVolumeSource = _define("NFSVolumeSource", [("path", str, _REQUIRED), ("server", str, _REQUIRED),
                                              ("read_only", Optional[bool], _opt)])
PersistentVolumeClaimVolumeSource = _define("PersistentVolumeClaimVolumeSource", [
    ("claim_name", str, _REQUIRED), ("read_only", Optional[bool], _opt)])

# every volume source other than secret / nfs / pvc is carried as an unvalidated mapping
_OPAQUE_SOURCES = ("aws_elastic_block_store azure_disk azure_file cephfs cinder config_map downward_api empty_dir fc "
                   "flex_volume flocker gce_persistent_disk git_repo glusterfs host_path iscsi "
                   "photon_persistent_disk portworx_volume projected quobyte rbd scale_io storageos "
                   "vsphere_volume").split()
Volume = _define("Volume", [("name", str, _REQUIRED), ("secret", Optional[SecretVolumeSource], _opt),
                            ("nfs", Optional[NFSVolumeSource], _opt),
                            ("persistent_volume_claim", Optional[PersistentVolumeClaimVolumeSource], _opt)]
                 + [(s, Optional[Mapping], _opt) for s in _OPAQUE_SOURCES],
                 wire={"downward_api": "downwardAPI", "scale_io": "scaleIO"})
PodSpecArgoSubset = _define("PodSpecArgoSubset", [
    ("active_deadline_seconds", Optional[int], _opt), ("affinity", Optional[Mapping], _opt),
    ("node_selector", Optional[Dict[str, str]], _opt), ("tolerations", Optional[List[Toleration]], _opt),
    ("volumes", Optional[List[Volume]], _opt)])
ObjectMetaArgoSubset = _define("ObjectMetaArgoSubset", [("annotations", Optional[Dict[str, str]], _opt),
                                                        ("labels", Optional[Dict[str, str]], _opt)])
PodArgoSubset = _define("PodArgoSubset", [("metadata", Optional[ObjectMetaArgoSubset], _opt),
                                          ("spec", Optional[PodSpecArgoSubset], _opt)],
                        doc="The part of a Pod that Argo lets a workflow template set.")
