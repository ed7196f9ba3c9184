"""Remote-training helper with the `fairing.config` surface used by the reference samples
(`kubeflow-pipelines/fairing/fairing_tf.py:60-64`, `fairing_xgboost.py:84-87`):

    from mifx import fairing
    fairing.config.set_builder('append', base_image='rocm/pytorch:latest', registry='my-registry', push=False)
    train = fairing.config.fn(train)     # or: fairing.config.set_model(Model()); fairing.config.run()
    train()

Backends: 'local' deployer runs the function / `model.train()` in a child process (cloudpickle);
'job' deployer builds a context (Dockerfile on the chosen base image + the pickled callable), optionally
builds it with kaniko (`mifx.kfp.compiler._component_builder`) and submits a k8s Job requesting AMD
GPUs through kubectl. `job_manifest()` exposes the Job spec for inspection."""
from .config import Config, config  # noqa: F401
