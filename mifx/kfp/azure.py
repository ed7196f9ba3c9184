"""Azure op modifier (reference: `sdk/python/kfp/azure.py:14-75`)."""
from __future__ import annotations

from .aws import _secret_env

_AZ_KEYS = ("AZ_SUBSCRIPTION_ID", "AZ_TENANT_ID", "AZ_CLIENT_ID", "AZ_CLIENT_SECRET")


def use_azure_secret(secret_name: str = "azcreds"):
    """Expose the Azure service-principal secret keys as environment variables."""

    def _use_azure_secret(task):
        for k in _AZ_KEYS:
            task = task.add_env_variable(_secret_env(k, secret_name, k))
        return task

    return _use_azure_secret
