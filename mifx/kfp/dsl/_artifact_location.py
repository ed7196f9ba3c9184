"""S3/Minio artifact repository descriptor for op output artifacts.

Reference: `sdk/python/kfp/dsl/_artifact_location.py:20-152` (`ArtifactLocation.s3`,
`create_artifact_for_s3`; artifact key `runs/{{workflow.uid}}/{{pod.name}}/<name>.tgz`)."""
from __future__ import annotations

from ..k8s import (V1alpha1Artifact, V1alpha1ArtifactLocation, V1alpha1S3Artifact, V1SecretKeySelector)


def _dict_to_secret(d) -> V1SecretKeySelector | None:
    if isinstance(d, dict) and d.get("name") and d.get("key"):
        return V1SecretKeySelector(name=d.get("name"), key=d.get("key"), optional=d.get("optional"))
    return d or V1SecretKeySelector(key="", optional=True)  # Argo wants the selector even when unused


class ArtifactLocation:
    @staticmethod
    def s3(bucket: str | None = None, endpoint: str | None = None, insecure: bool = False, region: str | None = None,
           access_key_secret=None, secret_key_secret=None) -> V1alpha1ArtifactLocation:
        return V1alpha1ArtifactLocation(s3=V1alpha1S3Artifact(
            bucket=bucket, endpoint=endpoint, insecure=insecure, region=region,
            access_key_secret=_dict_to_secret(access_key_secret), secret_key_secret=_dict_to_secret(secret_key_secret)))

    @staticmethod
    def create_artifact_for_s3(artifact_location, name: str, path: str, key: str, **kwargs) -> V1alpha1Artifact:
        if isinstance(artifact_location, dict):  # already converted to JSON by param substitution
            s3 = artifact_location.get("s3")
            if not s3:
                return V1alpha1Artifact(name=name, path=path, **kwargs)
            s3 = V1alpha1S3Artifact(bucket=s3.get("bucket"), endpoint=s3.get("endpoint"), insecure=s3.get("insecure"),
                                    region=s3.get("region"),
                                    access_key_secret=_dict_to_secret(s3.get("accessKeySecret")),
                                    secret_key_secret=_dict_to_secret(s3.get("secretKeySecret")))
        elif not artifact_location or not getattr(artifact_location, "s3", None):
            return V1alpha1Artifact(name=name, path=path, **kwargs)
        else:
            s3 = artifact_location.s3
        return V1alpha1Artifact(name=name, path=path, s3=V1alpha1S3Artifact(
            bucket=s3.bucket, endpoint=s3.endpoint, insecure=s3.insecure, region=s3.region,
            access_key_secret=s3.access_key_secret, secret_key_secret=s3.secret_key_secret, key=key), **kwargs)
