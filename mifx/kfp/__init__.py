"""Pipelines SDK with the KFP 0.1.x surface: `dsl`, `compiler`, `components`, `Client`, op modifiers
(`gcp`, `aws`, `azure`, `onprem`, `amd`) and host-local execution (`local`).

Reference: `sdk/python/kfp/__init__.py`. `import mifx.kfp as kfp` is the intended spelling;
`mifx.kfp.compat.install()` additionally registers `kfp` / `kubernetes.client` module aliases so
unmodified KFP pipeline files run against this implementation."""
from . import components, dsl  # noqa: F401
from ._client import Client  # noqa: F401
from ._config import *  # noqa: F401,F403
