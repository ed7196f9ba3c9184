"""AWS op modifier (reference: `sdk/python/kfp/aws.py:14-59`)."""
from __future__ import annotations

from .k8s import V1EnvVar, V1EnvVarSource, V1SecretKeySelector


def _secret_env(name: str, secret_name: str, key: str) -> V1EnvVar:
    return V1EnvVar(name=name, value_from=V1EnvVarSource(secret_key_ref=V1SecretKeySelector(name=secret_name, key=key)))


def use_aws_secret(secret_name: str = "aws-secret", aws_access_key_id_name: str = "AWS_ACCESS_KEY_ID",
                   aws_secret_access_key_name: str = "AWS_SECRET_ACCESS_KEY"):
    """Expose AWS credentials from a k8s secret as AWS_ACCESS_KEY_ID / AWS_SECRET_ACCESS_KEY."""

    def _use_aws_secret(task):
        return (task.add_env_variable(_secret_env("AWS_ACCESS_KEY_ID", secret_name, aws_access_key_id_name))
                .add_env_variable(_secret_env("AWS_SECRET_ACCESS_KEY", secret_name, aws_secret_access_key_name)))

    return _use_aws_secret
