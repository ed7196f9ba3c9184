"""On-prem op modifier (reference: `sdk/python/kfp/onprem.py:2-22`)."""
from __future__ import annotations

from .k8s import V1PersistentVolumeClaimVolumeSource, V1Volume, V1VolumeMount


def mount_pvc(pvc_name: str = "pipeline-claim", volume_name: str = "pipeline", volume_mount_path: str = "/mnt/pipeline"):
    """Mount an existing PVC into the op."""

    def _mount_pvc(task):
        pvc = V1PersistentVolumeClaimVolumeSource(claim_name=pvc_name)
        task.add_volume(V1Volume(name=volume_name, persistent_volume_claim=pvc))
        task.container.add_volume_mount(V1VolumeMount(mount_path=volume_mount_path, name=volume_name))
        return task

    return _mount_pvc
