"""Host-local execution of compiled pipelines (offline stand-in for the Argo controller)."""
from .executor import LocalWorkflowExecutor, WorkflowError, evaluate_when, run_workflow  # noqa: F401
