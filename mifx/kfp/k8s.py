"""Minimal Kubernetes / Argo object models (no `kubernetes` package dependency).

Every model carries `swagger_types` / `attribute_map` like the generated kubernetes-client
models, so pipeline code written against `kubernetes.client` (`V1EnvVar`, `V1Volume`, ...) and the
compiler's JSON conversion work unchanged (reference: `sdk/python/kfp/compiler/_k8s_helper.py:132-183`).
"""
from __future__ import annotations

import re


def _camel(name: str) -> str:
    head, *rest = name.split("_")
    return head + "".join(p[:1].upper() + p[1:] for p in rest)


class K8sModel:
    swagger_types: dict = {}
    attribute_map: dict = {}

    def __init__(self, **kwargs):
        for k in self.swagger_types:
            setattr(self, k, kwargs.pop(k, None))
        if kwargs:
            raise TypeError(f"{type(self).__name__} got unexpected arguments {sorted(kwargs)}")

    def to_dict(self) -> dict:
        from .compiler._k8s_helper import convert_k8s_obj_to_json

        return convert_k8s_obj_to_json(self)

    def __eq__(self, other):
        return type(self) is type(other) and self.__dict__ == other.__dict__

    def __hash__(self):
        return id(self)

    def __repr__(self):
        body = ", ".join(f"{k}={getattr(self, k)!r}" for k in self.swagger_types if getattr(self, k) is not None)
        return f"{type(self).__name__}({body})"


_SPECIAL_KEYS = {"ref": "$ref", "_except": "except", "_continue": "continue", "_from": "from"}


def _model(name: str, fields: str, base=K8sModel, overrides: dict | None = None):
    names = fields.split()
    attr_map = {f: _SPECIAL_KEYS.get(f, _camel(f)) for f in names}
    attr_map.update(overrides or {})
    cls = type(name, (base,), {"swagger_types": {f: "object" for f in names}, "attribute_map": attr_map})
    return cls


V1ObjectMeta = _model("V1ObjectMeta", "annotations cluster_name creation_timestamp deletion_grace_period_seconds "
                      "deletion_timestamp finalizers generate_name generation labels name namespace owner_references "
                      "resource_version self_link uid")
V1LocalObjectReference = _model("V1LocalObjectReference", "name")
V1ObjectReference = _model("V1ObjectReference", "api_version field_path kind name namespace resource_version uid")
V1TypedLocalObjectReference = _model("V1TypedLocalObjectReference", "api_group kind name")
V1SecretKeySelector = _model("V1SecretKeySelector", "key name optional")
V1ConfigMapKeySelector = _model("V1ConfigMapKeySelector", "key name optional")
V1ObjectFieldSelector = _model("V1ObjectFieldSelector", "api_version field_path")
V1ResourceFieldSelector = _model("V1ResourceFieldSelector", "container_name divisor resource")
V1EnvVarSource = _model("V1EnvVarSource", "config_map_key_ref field_ref resource_field_ref secret_key_ref")
V1EnvVar = _model("V1EnvVar", "name value value_from")
V1SecretEnvSource = _model("V1SecretEnvSource", "name optional")
V1ConfigMapEnvSource = _model("V1ConfigMapEnvSource", "name optional")
V1EnvFromSource = _model("V1EnvFromSource", "config_map_ref prefix secret_ref")
V1VolumeMount = _model("V1VolumeMount", "mount_path mount_propagation name read_only sub_path")
V1VolumeDevice = _model("V1VolumeDevice", "device_path name")
V1ContainerPort = _model("V1ContainerPort", "container_port host_ip host_port name protocol")
V1ResourceRequirements = _model("V1ResourceRequirements", "limits requests")
V1Capabilities = _model("V1Capabilities", "add drop")
V1SecurityContext = _model("V1SecurityContext", "allow_privilege_escalation capabilities privileged "
                           "read_only_root_filesystem run_as_group run_as_non_root run_as_user se_linux_options")
V1ExecAction = _model("V1ExecAction", "command")
V1HTTPGetAction = _model("V1HTTPGetAction", "host http_headers path port scheme")
V1TCPSocketAction = _model("V1TCPSocketAction", "host port")
V1Probe = _model("V1Probe", "_exec failure_threshold http_get initial_delay_seconds period_seconds success_threshold "
                 "tcp_socket timeout_seconds", overrides={"_exec": "exec"})
V1Handler = _model("V1Handler", "_exec http_get tcp_socket", overrides={"_exec": "exec"})
V1Lifecycle = _model("V1Lifecycle", "post_start pre_stop")
V1Container = _model("V1Container", "args command env env_from image image_pull_policy lifecycle liveness_probe name "
                     "ports readiness_probe resources security_context stdin stdin_once termination_message_path "
                     "termination_message_policy tty volume_devices volume_mounts working_dir")
V1Toleration = _model("V1Toleration", "effect key operator toleration_seconds value")
V1PersistentVolumeClaimVolumeSource = _model("V1PersistentVolumeClaimVolumeSource", "claim_name read_only")
V1SecretVolumeSource = _model("V1SecretVolumeSource", "default_mode items optional secret_name")
V1ConfigMapVolumeSource = _model("V1ConfigMapVolumeSource", "default_mode items name optional")
V1HostPathVolumeSource = _model("V1HostPathVolumeSource", "path type")
V1EmptyDirVolumeSource = _model("V1EmptyDirVolumeSource", "medium size_limit")
V1NFSVolumeSource = _model("V1NFSVolumeSource", "path read_only server")
V1Volume = _model("V1Volume", "aws_elastic_block_store azure_disk azure_file cephfs cinder config_map downward_api "
                  "empty_dir fc flex_volume flocker gce_persistent_disk git_repo glusterfs host_path iscsi name nfs "
                  "persistent_volume_claim photon_persistent_disk portworx_volume projected quobyte rbd scale_io "
                  "secret storageos vsphere_volume")
V1PersistentVolumeClaimSpec = _model("V1PersistentVolumeClaimSpec", "access_modes data_source resources selector "
                                     "storage_class_name volume_mode volume_name")
V1PersistentVolumeClaim = _model("V1PersistentVolumeClaim", "api_version kind metadata spec status")
V1Secret = _model("V1Secret", "api_version data kind metadata string_data type")
V1PodSpec = _model("V1PodSpec", "containers node_selector restart_policy service_account_name tolerations volumes")
V1Pod = _model("V1Pod", "api_version kind metadata spec status")
V1DeleteOptions = _model("V1DeleteOptions", "api_version grace_period_seconds kind propagation_policy")

# Argo workflow models (argo-models 2.2.1a)
V1alpha1S3Artifact = _model("V1alpha1S3Artifact", "access_key_secret bucket endpoint insecure key region "
                            "secret_key_secret")
V1alpha1Artifact = _model("V1alpha1Artifact", "archive _from global_name mode name optional path s3",
                          overrides={"_from": "from", "global_name": "globalName"})
V1alpha1S3ArtifactRepository = _model("V1alpha1S3ArtifactRepository", "access_key_secret bucket endpoint insecure "
                                      "key_prefix region secret_key_secret")
V1alpha1ArtifactLocation = _model("V1alpha1ArtifactLocation", "artifactory git hdfs http raw s3")

# `client.models` / `models` namespaces used as `kubernetes.client.models.V1EnvVar`
models = type("models", (), {k: v for k, v in dict(globals()).items() if re.match(r"V1", k)})
ApiClient = None
