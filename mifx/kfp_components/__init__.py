"""Reusable pipeline components (component.yaml specs) backed by `python3 -m mifx.kfp_components.<module>`.

`load(name)` returns the KFP task factory of a component; `write_specs(dir)` writes the
component.yaml files (the reference loads the equivalent specs by URL,
`taxi-cab-classification-pipeline.py:21-28`)."""
from __future__ import annotations

import os

import yaml

IMAGE = "mifx/mifx-rocm:latest"

# name -> (module, step, description, inputs [(name, type, default|None)], outputs [(name, type)])
_TAXI = {
    "tfdv": ("Data validation (TFDV-equivalent): statistics, column schema, anomalies",
             [("inference_data", "String", None), ("validation_data", "String", None),
              ("column_names", "String", None), ("key_columns", "String", ""), ("project", "String", ""),
              ("mode", "String", "local"), ("validation_output", "String", None)],
             [("schema", "String"), ("validation_result", "String")]),
    "tft": ("Transform (TFT-equivalent): analyze on train, apply to train/eval",
            [("training_data_file_pattern", "String", None), ("evaluation_data_file_pattern", "String", None),
             ("schema", "String", None), ("project", "String", ""), ("mode", "String", "local"),
             ("preprocessing_module", "String", None), ("transformed_data_dir", "String", None)],
            [("transformed_data_dir", "String")]),
    "dnntrainer": ("Taxi DNN trainer (HIP gather + sparse Adagrad on MI355X)",
                   [("transformed_data_dir", "String", None), ("schema", "String", None),
                    ("learning_rate", "Float", "0.1"), ("hidden_layer_size", "String", "1500"),
                    ("steps", "Integer", "3000"), ("target", "String", "tips"),
                    ("preprocessing_module", "String", ""), ("training_output_dir", "String", None),
                    ("batch_size", "Integer", "32"), ("num_gpus", "Integer", "1")],
                   [("training_output_dir", "String")]),
    "tfma": ("Model analysis (TFMA-equivalent): overall + sliced accuracy/AUC/loss",
             [("model", "String", None), ("evaluation_data", "String", None), ("schema", "String", None),
              ("project", "String", ""), ("mode", "String", "local"), ("slice_columns", "String", ""),
              ("analysis_results_dir", "String", None)],
             [("analysis_results_dir", "String")]),
    "predict": ("Batch prediction",
                [("data_file_pattern", "String", None), ("schema", "String", None), ("target_column", "String", "tips"),
                 ("model", "String", None), ("mode", "String", "local"), ("project", "String", ""),
                 ("predictions_dir", "String", None), ("batch_size", "Integer", "32")],
                [("predictions_dir", "String")]),
    "confusion_matrix": ("Confusion matrix (KFP UI metadata + accuracy metric)",
                         [("predictions", "String", None), ("target_lambda", "String", ""),
                          ("target_column", "String", "target"), ("output_dir", "String", None)],
                         [("accuracy", "Float")]),
    "roc": ("ROC curve (KFP UI metadata + AUC metric)",
            [("predictions_dir", "String", None), ("target_lambda", "String", ""),
             ("target_column", "String", "target"), ("output_dir", "String", None)],
            [("auc", "Float")]),
    "deployer": ("Serving deployment manifests for mifx.serving.server",
                 [("model_dir", "String", None), ("server_name", "String", None), ("cluster_name", "String", ""),
                  ("pvc_name", "String", ""), ("service_type", "String", "ClusterIP"), ("apply", "Integer", "0"),
                  ("output_dir", "String", "/tmp/deploy")],
                 [("manifest", "String")]),
}


def spec_dict(name: str) -> dict:
    desc, inputs, outputs = _TAXI[name]
    args = []
    for n, _t, d in inputs:
        args += [f"--{n}", {"inputValue": n}]
    for n, _t in outputs:
        args += [f"--{n}_out", {"outputPath": n}]
    return {
        "name": name.replace("_", " ").capitalize(),
        "description": desc,
        "inputs": [dict({"name": n, "type": t}, **({"default": d} if d is not None else {})) for n, t, d in inputs],
        "outputs": [{"name": n, "type": t} for n, t in outputs],
        "implementation": {"container": {"image": IMAGE, "command": ["python3", "-m", "mifx.kfp_components.taxi", name],
                                         "args": args}},
    }


def spec_text(name: str) -> str:
    return yaml.safe_dump(spec_dict(name), sort_keys=False)


def load(name: str):
    from ..kfp import components

    return components.load_component_from_text(spec_text(name))


def write_specs(out_dir: str) -> list[str]:
    paths = []
    for name in _TAXI:
        d = os.path.join(out_dir, name)
        os.makedirs(d, exist_ok=True)
        p = os.path.join(d, "component.yaml")
        with open(p, "w") as f:
            f.write(spec_text(name))
        paths.append(p)
    return paths


NAMES = tuple(_TAXI)
