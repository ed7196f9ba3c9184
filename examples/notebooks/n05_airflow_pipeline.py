"""Notebook 05_Airflow_ML_Pipelines (reference `notebooks/05_Airflow_ML_Pipelines.ipynb` L11: unpause the
`taxi` DAG in the Airflow UI and trigger a run). With mifx the same 9-component taxi pipeline is handed to
`AirflowDagRunner`: it writes the DAG file Airflow would schedule (schedule_interval None, start_date
2019-01-01 as in `airflow-dags/taxi_pipeline.py:59-62`) and "triggers" it -- through Airflow when it is
importable, otherwise in-process via the LocalDagRunner with the same component semantics."""
from __future__ import annotations

import argparse
import os
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.abspath(os.path.join(HERE, "..", "..")))
sys.path.insert(0, os.path.abspath(os.path.join(HERE, "..", "taxi")))
sys.path.insert(0, HERE)

from _data import taxi_csvs  # noqa: E402
from taxi_pipeline_local import create_pipeline  # noqa: E402

from mifx.orchestration.dag_runners import AirflowDagRunner  # noqa: E402


def main(argv=None) -> dict:
    ap = argparse.ArgumentParser()
    ap.add_argument("--workdir", default=os.path.join(tempfile.gettempdir(), "mifx_n05"))
    ap.add_argument("--rows", type=int, default=3000)
    ap.add_argument("--train-steps", type=int, default=200)
    a = ap.parse_args(argv)
    root = os.path.abspath(a.workdir)
    data_dir = os.path.join(root, "data")
    os.makedirs(data_dir, exist_ok=True)
    train_csv, _ = taxi_csvs(os.path.join(root, "csv"), a.rows, a.rows // 2)
    with open(train_csv) as src, open(os.path.join(data_dir, "data.csv"), "w") as dst:
        dst.write(src.read())
    factory_args = {"pipeline_name": "taxi", "pipeline_root": os.path.join(root, "pipelines"), "data_root": data_dir,
                    "serving_model_dir": os.path.join(root, "serving_model", "taxi"),
                    "train_steps": a.train_steps, "eval_steps": max(1, a.train_steps // 2),
                    "metadata_db_root": os.path.join(root, "metadata")}
    pipeline = create_pipeline(**factory_args)
    runner = AirflowDagRunner({"schedule_interval": None, "start_date": (2019, 1, 1)})
    dag_file = runner.write_dag(os.path.join(root, "dags", "taxi_pipeline.py"), pipeline,
                                "taxi_pipeline_local:create_pipeline", factory_args)
    print("DAG file:", dag_file)
    result = runner.run(pipeline, "taxi_pipeline_local:create_pipeline", factory_args)  # "unpause + trigger"
    print("run:", result)
    return {"dag_file": dag_file, "result": result}


if __name__ == "__main__":
    main()
