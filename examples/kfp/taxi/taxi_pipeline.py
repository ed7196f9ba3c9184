"""KFP taxi-cab classification pipeline on this framework (reference:
`kubeflow-pipelines/taxi/taxi-cab-classification-pipeline.py:31-133`).

validate -> transform -> train (HIP taxi DNN) -> analyze + predict -> confusion matrix + ROC -> deploy,
each step mounting the shared output volume (`onprem.mount_pvc`) and requesting an MI355X for the
trainer (`amd.use_amd_gpus`). Compile with `python examples/kfp/taxi/taxi_pipeline.py --output x.yaml`
or run on this host with `--run-local` (the local Argo-equivalent executor)."""
from __future__ import annotations

import argparse
import os
import sys

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..", "..")))

from mifx import kfp_components  # noqa: E402
from mifx.kfp import amd, compiler, dsl, onprem  # noqa: E402

tfdv_op = kfp_components.load("tfdv")
tft_op = kfp_components.load("tft")
train_op = kfp_components.load("dnntrainer")
tfma_op = kfp_components.load("tfma")
predict_op = kfp_components.load("predict")
cm_op = kfp_components.load("confusion_matrix")
roc_op = kfp_components.load("roc")
deploy_op = kfp_components.load("deployer")


# data-parallel dnntrainer ranks (one per GPU of the trainer pod); set by --num-gpus before compiling
NUM_GPUS = 1


@dsl.pipeline(name="TFX Taxi Cab Classification Pipeline Example",
              description="Example pipeline that does classification with model analysis.")
def taxi_cab_classification(output="/mnt", project="taxi-cab-classification-pipeline",
                            column_names="/mnt/taxi/column-names.json", key_columns="trip_start_timestamp",
                            train="/mnt/taxi/train.csv", evaluation="/mnt/taxi/eval.csv", mode="local",
                            preprocess_module="/mnt/taxi/preprocessing.py", learning_rate=0.1,
                            hidden_layer_size="1500", steps=3000, analyze_slice_column="trip_start_hour",
                            platform="onprem"):
    output_template = str(output) + "/{{workflow.uid}}/{{pod.name}}/data"
    target_lambda = "lambda x: (x['target'] > x['fare'] * 0.2)"
    target_class_lambda = "lambda x: 1 if (x['target'] > x['fare'] * 0.2) else 0"
    server_name = "taxi-cab-classification-model-{{workflow.uid}}"

    validation = tfdv_op(inference_data=train, validation_data=evaluation, column_names=column_names,
                         key_columns=key_columns, project=project, mode=mode, validation_output=output_template)
    preprocess = tft_op(training_data_file_pattern=train, evaluation_data_file_pattern=evaluation,
                        schema=validation.outputs["schema"], project=project, mode=mode,
                        preprocessing_module=preprocess_module, transformed_data_dir=output_template)
    training = train_op(transformed_data_dir=preprocess.output, schema=validation.outputs["schema"],
                        learning_rate=learning_rate, hidden_layer_size=hidden_layer_size, steps=steps, target="tips",
                        preprocessing_module=preprocess_module, training_output_dir=output_template,
                        num_gpus=NUM_GPUS)
    analysis = tfma_op(model=training.output, evaluation_data=evaluation, schema=validation.outputs["schema"],
                       project=project, mode=mode, slice_columns=analyze_slice_column,
                       analysis_results_dir=output_template)
    prediction = predict_op(data_file_pattern=evaluation, schema=validation.outputs["schema"], target_column="tips",
                            model=training.output, mode=mode, project=project, predictions_dir=output_template)
    cm = cm_op(predictions=prediction.output, target_lambda=target_lambda, output_dir=output_template)
    roc = roc_op(predictions_dir=prediction.output, target_lambda=target_class_lambda, output_dir=output_template)
    deploy = deploy_op(model_dir=str(training.output) + "/export/export", server_name=server_name,
                       cluster_name=project, pvc_name="users-pvc", service_type="NodePort",
                       output_dir=output_template)
    training.apply(amd.use_amd_gpus(NUM_GPUS))
    for step in (validation, preprocess, training, analysis, prediction, cm, roc, deploy):
        step.apply(onprem.mount_pvc("users-pvc", "local-storage", output))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--output", default="taxi-cab-classification-pipeline.yaml")
    ap.add_argument("--run-local", action="store_true")
    ap.add_argument("--data-dir", default=None, help="dir with train.csv, eval.csv, column-names.json")
    ap.add_argument("--work-dir", default="/tmp/mifx_kfp_taxi")
    ap.add_argument("--steps", type=int, default=3000)
    ap.add_argument("--hidden", default="1500")
    ap.add_argument("--num-gpus", type=int, default=1, help="data-parallel dnntrainer ranks (GPUs of its pod)")
    a = ap.parse_args(argv)
    global NUM_GPUS
    NUM_GPUS = a.num_gpus
    compiler.Compiler().compile(taxi_cab_classification, a.output)
    print(f"compiled -> {a.output}")
    if not a.run_local:
        return None
    import yaml

    from mifx.kfp.local import LocalWorkflowExecutor

    data = os.path.abspath(a.data_dir)
    with open(a.output) as f:
        wf = yaml.safe_load(f)
    env = dict(os.environ, PYTHONPATH=os.path.abspath(os.path.join(os.path.dirname(__file__), "..", "..", "..")))
    args = {"output": os.path.abspath(a.work_dir), "column_names": os.path.join(data, "column-names.json"),
            "train": os.path.join(data, "train.csv"), "evaluation": os.path.join(data, "eval.csv"),
            "preprocess_module": os.path.join(os.path.dirname(os.path.abspath(__file__)), "preprocessing.py"),
            "steps": a.steps, "hidden_layer_size": a.hidden}
    st = LocalWorkflowExecutor(wf, os.path.join(a.work_dir, "run"), args, env=env).run()
    print(f"workflow {st['phase']} {st['message']}")
    return st


if __name__ == "__main__":
    main()
