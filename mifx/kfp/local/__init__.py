"""Execution of compiled pipelines (the Argo controller's role): on this host, or one Pod per step on a Kubernetes
cluster (`kube.KubeStepRunner`)."""
from .executor import LocalWorkflowExecutor, WorkflowError, evaluate_when, run_workflow  # noqa: F401
