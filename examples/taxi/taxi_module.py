"""Chicago-Taxi user module for the mifx Transform and Trainer components.

Same feature engineering and model as the reference user module (`airflow-dags/taxi_utils.py`):
z-score the 3 dense floats, vocab (top 1000 + 10 OOV) the 2 string features, 10-quantile buckets
for the 4 lat/lon columns, pass the 7 categorical ints through, label = tips > 0.2 * fare (0 when
fare is missing); Wide&Deep with hidden units [100, 70, 48, 34] and batch 40, checkpoints every 999
steps, final exporter 'chicago-taxi' + eval export for the Evaluator.
"""
import numpy as np

import mifx.transform as mt
from mifx.io import dataset
from mifx.models import wide_deep as wdm
from mifx.trainer.estimator import EvalSpec, FinalExporter, RunConfig, TrainSpec, WideDeepEstimator

DENSE_FLOAT_FEATURE_KEYS = wdm.DENSE_FLOAT_FEATURE_KEYS
VOCAB_FEATURE_KEYS = wdm.VOCAB_FEATURE_KEYS
BUCKET_FEATURE_KEYS = wdm.BUCKET_FEATURE_KEYS
CATEGORICAL_FEATURE_KEYS = wdm.CATEGORICAL_FEATURE_KEYS
LABEL_KEY, FARE_KEY = wdm.LABEL_KEY, wdm.FARE_KEY
xf = wdm.transformed_name


def preprocessing_fn(inputs):
    out = {}
    for key in DENSE_FLOAT_FEATURE_KEYS:
        out[xf(key)] = mt.scale_to_z_score(mt.fill_in_missing(inputs[key]))
    for key in VOCAB_FEATURE_KEYS:
        out[xf(key)] = mt.compute_and_apply_vocabulary(mt.fill_in_missing(inputs[key]), top_k=wdm.VOCAB_SIZE,
                                                       num_oov_buckets=wdm.OOV_SIZE, vocab_filename=key)
    for key in BUCKET_FEATURE_KEYS:
        out[xf(key)] = mt.bucketize(mt.fill_in_missing(inputs[key]), wdm.FEATURE_BUCKET_COUNT)
    for key in CATEGORICAL_FEATURE_KEYS:
        out[xf(key)] = mt.fill_in_missing(inputs[key]).astype(np.int64)
    fare = mt.to_float(inputs[FARE_KEY])  # missing -> NaN (vectorised)
    tips = mt.fill_in_missing(inputs[LABEL_KEY]).astype(np.float64)
    out[xf(LABEL_KEY)] = np.where(np.isnan(fare), 0, tips > 0.2 * np.nan_to_num(fare)).astype(np.int64)
    return out


def _input_fn(files, device=None):
    """Transformed examples -> HBM-resident packed records (uint8 [N, 32])."""
    import torch

    cols = dataset.table_to_numpy(dataset.read_split(files[0]))
    rec = wdm.pack_transformed_columns(cols)
    t = torch.from_numpy(rec.view(np.uint8).reshape(-1, 32).copy())
    return t.to(device) if device else t


def trainer_fn(hparams, schema):
    first_dnn_layer_size, num_dnn_layers, dnn_decay_factor = 100, 4, 0.7
    train_batch_size = int((hparams.custom_config or {}).get("batch_size", 40))
    eval_batch_size = 40
    run_config = RunConfig(save_checkpoints_steps=999, keep_checkpoint_max=1, device=hparams.device)
    run_config = run_config.replace(model_dir=hparams.serving_model_dir)
    est = WideDeepEstimator(run_config, hidden_units=[max(2, int(first_dnn_layer_size * dnn_decay_factor ** i))
                                                      for i in range(num_dnn_layers)],
                            warm_start_from=hparams.warm_start_from, batch_size=train_batch_size,
                            eval_batch_size=eval_batch_size)
    dev = est.device
    serving_receiver = lambda: {"kind": "raw_examples", "transform_output": hparams.transform_output,  # noqa: E731
                                "raw_feature_spec": {f.name: f.type for f in schema.feature if f.name != LABEL_KEY}}
    eval_receiver = lambda: {"kind": "eval", "transform_output": hparams.transform_output,  # noqa: E731
                             "label_key": xf(LABEL_KEY)}
    return {
        "estimator": est,
        "train_spec": TrainSpec(lambda: _input_fn(hparams.train_files, dev), max_steps=hparams.train_steps),
        "eval_spec": EvalSpec(lambda: _input_fn(hparams.eval_files, dev), steps=hparams.eval_steps,
                              exporters=[FinalExporter("chicago-taxi", serving_receiver)], name="chicago-taxi-eval"),
        "eval_input_receiver_fn": eval_receiver,
    }
