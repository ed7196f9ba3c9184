"""Pipeline orchestration: artifacts/channels, components, Pipeline, LocalDagRunner (+ Airflow and
Kubeflow runners in their own modules)."""
from .artifact import Artifact, Channel, csv_input, external_input  # noqa: F401
from .component import BaseComponent, BaseExecutor, ChannelParameter, ComponentSpec, ExecutionParameter  # noqa: F401
from .pipeline import CycleError, Pipeline, sqlite_metadata_connection_config, topological_sort  # noqa: F401
from .runner import LocalDagRunner, RunResult  # noqa: F401
from .dag_runners import AirflowDagRunner, KubeflowDagRunner, KubeflowDagRunnerConfig  # noqa: F401,E402
