"""Small TFX-style pipeline factory used by the Kubeflow/Airflow runner tests."""
import csv
import os

from mifx.components import CsvExampleGen, SchemaGen, StatisticsGen
from mifx.data.synthetic import TAXI_COLUMNS, synthetic_taxi_csv_rows
from mifx.orchestration import Pipeline, csv_input


def create_pipeline(root: str, rows: int = 300):
    data = os.path.join(root, "data")
    os.makedirs(data, exist_ok=True)
    path = os.path.join(data, "data.csv")
    if not os.path.exists(path):
        with open(path, "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(TAXI_COLUMNS)
            for r in synthetic_taxi_csv_rows(rows, seed=3):
                w.writerow(["" if r[c] is None else r[c] for c in TAXI_COLUMNS])
    gen = CsvExampleGen(input_base=csv_input(data))
    stats = StatisticsGen(input_data=gen.outputs["examples"])
    schema = SchemaGen(stats=stats.outputs["output"])
    return Pipeline("tfx_mini", os.path.join(root, "pipeline_root"), [gen, stats, schema], enable_cache=True,
                    metadata_db_root=os.path.join(root, "metadata.db"))
