"""Experiment tracking with the MLflow file-store API surface (reference: `notebooks/mlflow/mlflow-wine.ipynb`
cell 2: set_tracking_uri('file://...'), set_experiment, start_run, log_param, log_metric,
sklearn.log_model). Runs, params, metrics (with steps/timestamps), tags and artifacts are plain
files, so the directory is browsable and diff-able; torch models are logged as safetensors via
`mifx.serving.saved_model`, other models with joblib (files this library writes itself)."""
from .store import (ActiveRun, FileStore, active_run, create_experiment, end_run, get_experiment_by_name,  # noqa: F401
                    get_run, get_tracking_uri, log_artifact, log_metric, log_metrics, log_model, log_param,
                    log_params, search_runs, set_experiment, set_tag, set_tracking_uri, start_run)
