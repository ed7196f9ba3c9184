"""Module aliases so unmodified KFP-0.1 pipeline files run on this SDK.

`install()` registers `kfp`, `kfp.dsl`, `kfp.compiler`, `kfp.components`, `kfp.gcp`, ... as aliases
of `mifx.kfp.*`, and — only when the real `kubernetes` package is not importable — a small
`kubernetes` / `kubernetes.client` / `kubernetes.client.models` stand-in backed by `mifx.kfp.k8s`
(reference pipelines do `from kubernetes import client as k8s_client`)."""
from __future__ import annotations

import importlib
import importlib.util
import sys
import types

_SUBMODULES = ("dsl", "dsl.types", "compiler", "components", "gcp", "aws", "azure", "onprem", "amd", "notebook",
               "_client", "_config", "local", "cli", "cli.cli", "cli.run",
               "compiler._k8s_helper", "compiler._op_to_template", "compiler.compiler", "compiler.main",
               "compiler._component_builder", "components._components", "components._python_op",
               "components._structures", "components._yaml_utils", "components._naming",
               "components._dsl_bridge", "components.modelbase", "components._component_store",
               "dsl._metadata", "dsl._pipeline_param", "dsl._container_op", "dsl._ops_group", "dsl._pipeline",
               "dsl._component", "dsl._resource_op", "dsl._pipeline_volume", "dsl._artifact_location")


def _install_kubernetes_stub() -> None:
    from . import k8s

    models = types.ModuleType("kubernetes.client.models")
    for name in dir(k8s):
        if name.startswith(("V1", "V1alpha1", "V1beta1")):
            setattr(models, name, getattr(k8s, name))
    client = types.ModuleType("kubernetes.client")
    client.__dict__.update({k: v for k, v in models.__dict__.items() if not k.startswith("__")})
    client.models = models
    kube = types.ModuleType("kubernetes")
    kube.client = client
    kube.__mifx_stub__ = True
    sys.modules.update({"kubernetes": kube, "kubernetes.client": client, "kubernetes.client.models": models})


def install(kubernetes: bool = True) -> None:
    import mifx.kfp as root

    sys.modules["kfp"] = root
    for sub in _SUBMODULES:
        mod = importlib.import_module("mifx.kfp." + sub)
        sys.modules["kfp." + sub] = mod
    if kubernetes and importlib.util.find_spec("kubernetes") is None and "kubernetes" not in sys.modules:
        _install_kubernetes_stub()
