"""GCP op modifiers (reference: `sdk/python/kfp/gcp.py:18-109`)."""
from __future__ import annotations

import warnings

from .k8s import V1EnvVar, V1SecretVolumeSource, V1Toleration, V1Volume, V1VolumeMount


def use_gcp_secret(secret_name: str = "user-gcp-sa", secret_file_path_in_volume: str = "/user-gcp-sa.json",
                   volume_name: str | None = None, secret_volume_mount_path: str = "/secret/gcp-credentials"):
    """Mount the service-account secret and point GOOGLE_APPLICATION_CREDENTIALS (and the gcloud
    override) at it."""
    if volume_name is None:
        volume_name = "gcp-credentials-" + secret_name
    else:
        warnings.warn("The volume_name parameter is deprecated; volume names are generated automatically.",
                      DeprecationWarning)
    cred_path = secret_volume_mount_path + secret_file_path_in_volume

    def _use_gcp_secret(task):
        return (task.add_volume(V1Volume(name=volume_name, secret=V1SecretVolumeSource(secret_name=secret_name)))
                .add_volume_mount(V1VolumeMount(name=volume_name, mount_path=secret_volume_mount_path))
                .add_env_variable(V1EnvVar(name="GOOGLE_APPLICATION_CREDENTIALS", value=cred_path))
                .add_env_variable(V1EnvVar(name="CLOUDSDK_AUTH_CREDENTIAL_FILE_OVERRIDE", value=cred_path)))

    return _use_gcp_secret


def use_tpu(tpu_cores: int, tpu_resource: str, tf_version: str):
    """Request Cloud TPU cores for the op (annotation + resource limit)."""

    def _set_tpu_spec(task):
        task.add_pod_annotation("tf-version.cloud-tpus.google.com", tf_version)
        task.container.add_resource_limit("cloud-tpus.google.com/{}".format(tpu_resource), str(tpu_cores))
        return task

    return _set_tpu_spec


def use_preemptible_nodepool(toleration: V1Toleration | None = None):
    """Schedule the op onto a GKE preemptible node pool."""
    toleration = toleration or V1Toleration(effect="NoSchedule", key="preemptible", operator="Equal", value="true")

    def _set_preemptible(task):
        task.add_toleration(toleration)
        task.add_node_selector_constraint("cloud.google.com/gke-preemptible", "true")
        return task

    return _set_preemptible
