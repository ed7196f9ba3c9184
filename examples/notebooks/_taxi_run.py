"""Runs the local Chicago-taxi TFX-style pipeline (examples/taxi/taxi_pipeline_local.py) so the
analysis notebooks (04, 06, 07) have artifacts, lineage and several model versions to inspect."""
from __future__ import annotations

import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.abspath(os.path.join(HERE, "..", "..")))
sys.path.insert(0, os.path.abspath(os.path.join(HERE, "..", "taxi")))

from _data import taxi_csvs  # noqa: E402
from taxi_pipeline_local import create_pipeline  # noqa: E402

from mifx.orchestration import LocalDagRunner  # noqa: E402


def run_taxi_pipeline(root: str, rows: int = 3000, train_steps: list[int] | tuple = (200,), batch_size: int = 40):
    """One pipeline run per entry of `train_steps` (same data; runs after the first re-use cached
    upstream components). Returns (metadata db path, pipeline name, [RunResult])."""
    data_dir = os.path.join(root, "data")
    train_csv, _ = taxi_csvs(os.path.join(root, "csv"), rows, rows // 2)
    os.makedirs(data_dir, exist_ok=True)
    dst = os.path.join(data_dir, "data.csv")
    if not os.path.exists(dst):
        with open(train_csv) as src, open(dst, "w") as out:
            out.write(src.read())
    results = []
    for steps in train_steps:
        p = create_pipeline("taxi", os.path.join(root, "pipelines"), data_dir, os.path.join(root, "serving_model", "taxi"),
                            train_steps=steps, eval_steps=max(1, steps // 2), metadata_db_root=os.path.join(root, "metadata"),
                            batch_size=batch_size)
        results.append(LocalDagRunner(max_parallel=2).run(p))
    return os.path.join(root, "metadata", "taxi", "metadata.db"), "taxi", results
