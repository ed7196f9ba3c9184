"""Chicago-Taxi end-to-end pipeline on mifx (LocalDagRunner; Airflow/Kubeflow runners optional).

Same 9-component DAG as the reference Airflow pipeline (`airflow-dags/taxi_pipeline.py:68-135`):
CsvExampleGen -> StatisticsGen -> SchemaGen -> ExampleValidator -> Transform -> Trainer ->
Evaluator (sliced by trip_start_hour) -> ModelValidator -> Pusher, with caching and an MLMD
sqlite store at <root>/metadata/<pipeline>/metadata.db.

    python examples/taxi/taxi_pipeline_local.py --data <csv dir> --root /tmp/taxi [--train-steps 10000]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..")))

from mifx.components import (CsvExampleGen, EvalArgs, Evaluator, ExampleValidator, FeatureSlicingSpec,  # noqa: E402
                             ModelValidator, Pusher, PushDestination, SchemaGen, SingleSlicingSpec, StatisticsGen,
                             TrainArgs, Trainer, Transform)
from mifx.components.proto import Filesystem  # noqa: E402
from mifx.orchestration import LocalDagRunner, Pipeline, csv_input  # noqa: E402

MODULE_FILE = os.path.join(os.path.dirname(os.path.abspath(__file__)), "taxi_module.py")


def create_pipeline(pipeline_name: str, pipeline_root: str, data_root: str, serving_model_dir: str,
                    train_steps: int = 10000, eval_steps: int = 5000, enable_cache: bool = True,
                    metadata_db_root: str | None = None, batch_size: int = 40, log_root: str | None = None,
                    num_gpus: int = 1, transform_workers: int = 0) -> Pipeline:
    """num_gpus > 1: the Trainer runs data-parallel, one rank per GPU, batch_size examples per rank per step.
    transform_workers > 1: Transform analyzes and transforms sharded over that many worker processes (the
    reference's Beam DirectRunner workers; mifx.transform.parallel)."""
    examples = csv_input(data_root)
    example_gen = CsvExampleGen(input_base=examples)
    statistics_gen = StatisticsGen(input_data=example_gen.outputs.examples)
    infer_schema = SchemaGen(stats=statistics_gen.outputs.output)
    validate_stats = ExampleValidator(stats=statistics_gen.outputs.output, schema=infer_schema.outputs.output)
    transform = Transform(input_data=example_gen.outputs.examples, schema=infer_schema.outputs.output,
                          module_file=MODULE_FILE, num_workers=transform_workers)
    trainer = Trainer(module_file=MODULE_FILE, transformed_examples=transform.outputs.transformed_examples,
                      schema=infer_schema.outputs.output, transform_output=transform.outputs.transform_output,
                      train_args=TrainArgs(num_steps=train_steps), eval_args=EvalArgs(num_steps=eval_steps),
                      custom_config={"batch_size": batch_size, "num_gpus": num_gpus})
    model_analyzer = Evaluator(examples=example_gen.outputs.examples, model_exports=trainer.outputs.output,
                               feature_slicing_spec=FeatureSlicingSpec(
                                   specs=[SingleSlicingSpec(column_for_slicing=["trip_start_hour"])]))
    model_validator = ModelValidator(examples=example_gen.outputs.examples, model=trainer.outputs.output)
    pusher = Pusher(model_export=trainer.outputs.output, model_blessing=model_validator.outputs.blessing,
                    push_destination=PushDestination(filesystem=Filesystem(base_directory=serving_model_dir)))
    return Pipeline(pipeline_name=pipeline_name, pipeline_root=pipeline_root,
                    components=[example_gen, statistics_gen, infer_schema, validate_stats, transform, trainer,
                                model_analyzer, model_validator, pusher],
                    enable_cache=enable_cache, metadata_db_root=metadata_db_root,
                    additional_pipeline_args={"logger_args": {"log_root": log_root or os.path.join(pipeline_root, "logs"),
                                                              "log_level": "INFO"}})


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--data", required=True)
    ap.add_argument("--root", default="/tmp/mifx_taxi")
    ap.add_argument("--train-steps", type=int, default=10000)
    ap.add_argument("--eval-steps", type=int, default=5000)
    ap.add_argument("--batch-size", type=int, default=40)
    ap.add_argument("--parallel", type=int, default=2)
    ap.add_argument("--num-gpus", type=int, default=1, help="data-parallel Trainer ranks (one per GPU)")
    ap.add_argument("--transform-workers", type=int, default=0, help="sharded Transform worker processes")
    a = ap.parse_args(argv)
    p = create_pipeline("taxi", os.path.join(a.root, "pipelines"), a.data, os.path.join(a.root, "serving_model", "taxi"),
                        a.train_steps, a.eval_steps, metadata_db_root=os.path.join(a.root, "metadata"),
                        batch_size=a.batch_size, num_gpus=a.num_gpus, transform_workers=a.transform_workers)
    res = LocalDagRunner(max_parallel=a.parallel).run(p)
    for cid, r in res.components.items():
        print(f"{cid:>20}: {r.state:9s} exec={r.execution_id} {r.seconds:.2f}s")


if __name__ == "__main__":
    main()
